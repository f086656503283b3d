#!/bin/bash
# fixed vs per-K-tile cost of the small ring GEMMs: M=1280, N=768, K sweep, no split-K, graph-timed:
# 2-deep ring (cfg 1), 4-deep ring with per-tile fragment reads (cfg 7, CAPK_GEMM_PIPE=0) and with
# the next tile's fragments read under the MFMAs (cfg 7, PIPE)
SH=${KSWEEP_SHAPES:-k64:1280:768:64:fwd,k256:1280:768:256:fwd,k768:1280:768:768:fwd,k1536:1280:768:1536:fwd,k3072:1280:768:3072:fwd,n3072k768:1280:3072:768:fwd,n2304k768:1280:2304:768:fwd}
for r in 1 2; do
  for v in "1 0" "7 0" "7 1"; do
    set -- $v
    CAPK_GEMM_CFG=$1 CAPK_GEMM_PIPE=$2 CAPK_GEMM_MAXSPLIT=1 GEMM_GRAPH=1 GEMM_SHAPES=$SH timeout -k 10 120 python tools/gemm_bench.py | sed "s/^/cfg$1 pipe$2: /" || exit 1
  done
done
