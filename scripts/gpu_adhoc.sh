set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_data.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/td.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/td.log | tail -8
