set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_qformer.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/tq.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|assert|Key" gpurun_out/tq.log | tail -12
