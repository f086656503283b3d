#!/bin/bash
set -u
OUT=gpurun_out/r4s26
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_attention.py tests/test_gpu_model.py tests/test_gpu_plugins.py tests/test_gpu_qformer.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="base:CAPK_ATTN_WAVES=0 w8:CAPK_ATTN_WAVES=8 nocs:CAPK_COLSUM_STREAM=0" REPS=2 bash scripts/gpu_r4_envab.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
CAPK_ATTN_WAVES=0 timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bal -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --beam-batch 0 > $OUT/prof_bal.log 2>&1 || exit $?
CAPK_ATTN_WAVES=8 timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_w8 -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --beam-batch 0 > $OUT/prof_w8.log 2>&1 || exit $?
for v in bal w8; do echo "== $v"; grep -h "attn_fwd_bf16<64\|attn_bwd_q_bf16<64\|attn_bwd_kv_bf16<64" $OUT/prof_$v/run_kernel_stats.csv | cut -d, -f1-4; done
