set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_beam.py tests/test_gpu_graphs.py tests/test_gpu_kernels.py -k "beam or graph or xdec or cross or attention" > gpurun_out/xdec_tests.log 2>&1
LIBS="libcapk_ahead.so" ATTN_ONLY=dec_cross,dstep_cross5 $T 300 bash scripts/attn_lib_ab.sh > gpurun_out/xdec_attn_ab.txt 2>&1
for L in libcapk.so libcapk_ahead.so libcapk_bhead.so; do
  CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/$L $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$L -o run -- python tools/beam_bench.py --reps 3 > gpurun_out/prof_$L.log 2>&1
done
for r in 1 2; do for L in libcapk.so libcapk_ahead.so; do
  CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/$L $T 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --beam-batch 0 2>/dev/null | sed "s/^/$L: /" >> gpurun_out/xdec_train_ab.txt
done; done
