#!/bin/bash
# Round-4 session: attention / kernel tests, the overlapped-epilogue GEMM build's tests and
# rates, the GEMM timestamp trace, attention-backward slicing A/B.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q -s --timeout 280 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_attention.py tests/test_gpu_beam.py::test_transformer_beam5_config3_bf16_vs_fp32 > gpurun_out/t17a.log 2>&1
rc=$?; grep -a "bf16 beam-5\|passed\|failed\|FAILED" gpurun_out/t17a.log | head; [ $rc -le 1 ] || exit $rc
CAPK_LIB_PATH=image-captioning-ml-project_amd/capk/libcapk_diag_exp_epiovl.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/t17b.log 2>&1
rc=$?; tail -2 gpurun_out/t17b.log; [ $rc -eq 0 ] || exit $rc
GX_VARIANTS="exp_epiovl" bash scripts/gpu_r4_gemmexp.sh || exit $?
CAPK_LIB_PATH=image-captioning-ml-project_amd/capk/libcapk_diag_trace.so timeout -k 10 300 python tools/gemm_trace.py > gpurun_out/t17trace.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/t17trace.log | tail -12; [ $rc -eq 0 ] || exit $rc
VARIANTS="s0:CAPK_ATTN_BWD_SLICE=0 s64:CAPK_ATTN_BWD_SLICE=64" bash scripts/gpu_r4_envab.sh
