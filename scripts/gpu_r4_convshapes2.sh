#!/bin/bash
# Config-2 ResNet-101 layer-2/3/4 GEMM shapes (fwd / dx / dw of the bottleneck convolutions at
# bs 128) per tile configuration (CAPK_GEMM_CFG; 0 = the library's choice), graph-replayed.
set -u
OUT=gpurun_out/r4conv2
mkdir -p $OUT
M2=100352; M3=25088; M4=6272
S="l2_c1_fwd:$M2:128:512:fwd,l2_c2_fwd:$M2:128:1152:fwd,l2_c3_fwd:$M2:512:128:fwd"
S="$S,l2_c1_dx:$M2:512:128:dx,l2_c2_dcol:$M2:1152:128:dx,l2_c3_dx:$M2:128:512:dx"
S="$S,l2_c1_dw:$M2:128:512:dw,l2_c2_dw:$M2:128:1152:dw,l2_c3_dw:$M2:512:128:dw"
S="$S,l3_c1_fwd:$M3:256:1024:fwd,l3_c2_fwd:$M3:256:2304:fwd,l3_c3_fwd:$M3:1024:256:fwd"
S="$S,l3_c1_dx:$M3:1024:256:dx,l3_c2_dcol:$M3:2304:256:dx,l3_c3_dx:$M3:256:1024:dx"
S="$S,l3_c1_dw:$M3:256:1024:dw,l3_c2_dw:$M3:256:2304:dw,l3_c3_dw:$M3:1024:256:dw"
S="$S,l4_c1_fwd:$M4:512:2048:fwd,l4_c2_fwd:$M4:512:4608:fwd,l4_c3_fwd:$M4:2048:512:fwd"
S="$S,l4_c1_dx:$M4:2048:512:dx,l4_c2_dcol:$M4:4608:512:dx,l4_c3_dx:$M4:512:2048:dx"
S="$S,l4_c1_dw:$M4:512:2048:dw,l4_c2_dw:$M4:512:4608:dw,l4_c3_dw:$M4:2048:512:dw"
S="$S,l1_c1_dw:401408:64:256:dw,l1_c3_dw:401408:256:64:dw"
export GEMM_SHAPES="$S" GEMM_GRAPH=1 GEMM_ITERS=10
for c in ${CFGS:-0 1 2 4}; do
  echo "== cfg $c" | tee -a $OUT/status
  CAPK_GEMM_CFG=$c timeout -k 10 300 python tools/gemm_bench.py > $OUT/cfg$c.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/cfg$c.log; exit $rc; }
done
python - <<'PY'
import re
cf = {}
for c in "0124":
    try:
        for l in open(f"gpurun_out/r4conv2/cfg{c}.log"):
            m = re.match(r"(\S+)\s+M=.*?(\d+\.\d+) us", l)
            if m: cf.setdefault(m.group(1), {})[c] = float(m.group(2))
    except FileNotFoundError:
        pass
print(f"{'shape':14s} " + " ".join(f"cfg{c:>6s}" for c in "0124"))
for k, v in cf.items():
    print(f"{k:14s} " + " ".join(f"{v.get(c, float('nan')):9.1f}" for c in "0124"))
PY
