#!/bin/bash
mkdir -p gpurun_out/sweep
CFG=6 timeout -k 5 200 python tools/gemm_sweep_check.py > gpurun_out/sweep/s6.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/sweep/s6.log | grep -v "^ok" | tail -10
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_kernels.py -k "gemm or linear or layouts or items or epilogue or split or fused" -q -rf --timeout 120 --timeout-method thread > gpurun_out/sweep/t.log 2>&1; rc=$?; tail -12 gpurun_out/sweep/t.log; exit $rc
