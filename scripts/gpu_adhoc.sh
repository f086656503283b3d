set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload config2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench2.log 2>&1
rc=$?; echo "bench2 rc=$rc"; tail -1 gpurun_out/bench2.log | cut -c1-400
