set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "ring_configs or product_ln or slab" > gpurun_out/s64_tests.log 2>&1
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_beam.py tests/test_gpu_graphs.py tests/test_gpu_lstm.py >> gpurun_out/s64_tests.log 2>&1
for v in 0 1; do
  CAPK_SLAB_S64=$v $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_slab_$v -o run -- python tools/beam_bench.py --reps 2 > gpurun_out/prof_slab_$v.log 2>&1
done
for i in 1 2; do for v in 0 1; do
  CAPK_SLAB_S64=$v $T 240 python tools/beam_bench.py --reps 3 | sed "s/^/SLAB_S64=$v: /" >> gpurun_out/slab_beam_ab.txt
done; done
