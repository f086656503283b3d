set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
PROF_TAG=prof_r2 PROF_SECS=300 PROF_CMD="bench.py --steps 3 --warmup 2 --no-cpu-baseline --beam-batch 0" bash scripts/gpu_profile.sh
