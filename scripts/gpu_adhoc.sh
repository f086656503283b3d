set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -x -v -rf --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1
rc=$?; echo "fp8 tests rc=$rc"; tail -5 gpurun_out/fp8_tests.log
[ $rc -eq 0 ] || exit $rc
GEMM_ONLY=f8_clip_qkv,f8_clip_fc1,f8_clip_fc2,f8_gpt2_fc1,f8_lm_head,f8_lm_head_beam5,f8_big,bf16_big,f8_quant_x,vit_qkv_fwd,lm_head_fwd \
  timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/gemm_f8.log 2>&1
rc=$?; echo "gemm rc=$rc"; cat gpurun_out/gemm_f8.log
