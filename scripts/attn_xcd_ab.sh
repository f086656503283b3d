#!/bin/bash
# attention kernels under CAPK_ATTN_XCD=0 / 1, alternated (tools/attn_bench.py, HIP events),
# with and without the Infinity Cache flush between calls
for f in 1 0; do
  for x in 0 1 0 1; do
    CAPK_ATTN_XCD=$x ATTN_FLUSH=$f ATTN_ONLY=${ATTN_ONLY:-dec_cross,dstep_self,dstep_cross5} timeout -k 10 120 python tools/attn_bench.py | sed "s/^/flush$f xcd$x: /" || exit 1
  done
done
