set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_checkpoint.py tests/test_gpu_model.py tests/test_gpu_config4.py tests/test_gpu_scst.py -q -rf --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1
echo "rc=$?"; tail -30 gpurun_out/t2.log
