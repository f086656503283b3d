set -u
mkdir -p gpurun_out/ab2
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_resnet.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2/t.log 2>&1; rc=$?; tail -1 gpurun_out/ab2/t.log; [ $rc -eq 0 ] || exit $rc
CAPK_GEMM_MAXSPLIT=16 timeout -k 10 300 python bench.py --workload config2 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/ab2/c2_16.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload config2 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/ab2/c2_new.log 2>&1 || exit $?
grep '^{' gpurun_out/ab2/c2_16.log | cut -c1-200
grep '^{' gpurun_out/ab2/c2_new.log | cut -c1-200
