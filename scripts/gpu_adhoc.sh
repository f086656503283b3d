set -u
mkdir -p gpurun_out
S=dec256_cattn,dec256_cproj,dec256_fc,dec256_proj2,dec1280_cattn,dec1280_cproj,dec1280_fc,dec1280_proj2,tdec1280_qkv,tdec1280_fc1,tdec1280_fc2
GEMM_GRAPH=1 GEMM_ONLY=$S GEMM_ITERS=50 timeout -k 10 120 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu
timeout -k 10 600 python -u bench.py --workload config5 --steps 3 --warmup 2 --beam-reps 3 --no-cpu-baseline > gpurun_out/bench5.log 2>&1
rc=$?; echo "bench5 rc=$rc"; tail -1 gpurun_out/bench5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['beam5']['value'], d['beam5']['ms_per_batch'])"
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['beam5']['value'], d['beam5']['ms_per_batch'])"
timeout -k 10 600 python -u bench.py --workload config2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench2.log 2>&1
rc=$?; echo "bench2 rc=$rc"; tail -1 gpurun_out/bench2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
