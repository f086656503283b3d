set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_beam.py tests/test_gpu_graphs.py > gpurun_out/beam_tests.log 2>&1
for L in libcapk.so libcapk_bhead.so; do
  CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$L -o run -- python tools/beam_bench.py --reps 3 > gpurun_out/prof_$L.log 2>&1
done
