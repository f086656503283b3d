set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload config5 --steps 3 --warmup 2 --beam-reps 3 --no-cpu-baseline > gpurun_out/bench5.log 2>&1
rc=$?; echo "bench5 rc=$rc"; tail -1 gpurun_out/bench5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['beam5']['value'], d['beam5']['ms_per_batch'])"
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['beam5']['value'], d['beam5']['ms_per_batch'])"
