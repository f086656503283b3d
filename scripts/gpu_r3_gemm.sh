#!/bin/bash
# gemm8q bring-up: GEMM parity tests (both 256x256 kernels + the default dispatch), then
# per-shape graph-timed throughput of cfg 5 (gemm8p) vs cfg 6 (gemm8q) on the config-3 shapes,
# and cfg 6 built with every store aimed at one L2-resident tile (CAPK_DIAG_L2STORE).
set -u
OUT=gpurun_out/r3gemm
mkdir -p $OUT
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
run() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-22}; ok_rc $rc || exit $rc; }
CFG=6 run sweep 200 python tools/gemm_sweep_check.py
TAILN=12 run tests 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_kernels.py -k "gemm or linear or layouts or items or epilogue or split or fused" -q -rf --timeout 120 --timeout-method thread
export GEMM_GRAPH=1 GEMM_ONLY=${SHAPES:-vit_qkv_fwd,vit_o_fwd,vit_fc1_fwd_gelu_deriv,vit_fc1_fwd_plain,vit_fc2_fwd,vit_qkv_dx,vit_fc1_dx,vit_fc2_dx_gelu_deriv,vit_o_dw,vit_fc1_dw,vit_qkv_dw,lm_head_fwd,lm_head_dw,dec_kv_fwd,bf16_big}
CAPK_GEMM_CFG=5 run bench_cfg5 300 python tools/gemm_bench.py
CAPK_GEMM_CFG=6 run bench_cfg6 300 python tools/gemm_bench.py
CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/libcapk_l2st.so CAPK_GEMM_CFG=6 run bench_cfg6_l2st 300 python tools/gemm_bench.py
