set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_resnet.py tests/test_gpu_lstm.py -x -v -rf --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/t2.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload config2 --steps 5 --warmup 2 > gpurun_out/bench2.log 2>&1
rc=$?; echo "bench2 rc=$rc"; tail -1 gpurun_out/bench2.log | cut -c1-2500
