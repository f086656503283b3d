#!/bin/bash
# BatchNorm / ResNet parity tests, then the config-2 bench (twice) and a short profile.
set -u
mkdir -p gpurun_out/bn
timeout -k 10 400 python -u -m pytest tests/test_gpu_resnet.py tests/test_gpu_legacy.py tests/test_gpu_lstm.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bn/t.log 2>&1; rc=$?; tail -1 gpurun_out/bn/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload config2 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/bn/c2_$i.log 2>&1 || exit $?
  echo "config2 run $i: $(grep '^{' gpurun_out/bn/c2_$i.log | cut -c1-150)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bn/prof -o run -- python3 bench.py --workload config2 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/bn/prof.log 2>&1 || exit $?
echo prof ok
