# beam-5 LM head (1280 x 50304 x 768, bias epilogue) per forced tile configuration, graph-replayed
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 0 5 6 1 7 9; do
  CAPK_GEMM_CFG=$c GEMM_GRAPH=1 GEMM_SHAPES=lmhead_beam:1280:50304:768:fwd timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -v amdgpu | sed "s/^/cfg=$c: /" >> gpurun_out/lmhead_sweep.txt
done
