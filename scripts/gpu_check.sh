#!/bin/bash
# Quick GPU check of the tree: -m gpu suite, smoke, config-3 bench.  Each GPU step has its
# own time limit; a crash-type exit ends the session.
set -u
OUT=gpurun_out/chk
mkdir -p $OUT
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  tail -3 $OUT/$name.log | cut -c1-300
  ok_rc $rc || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
for step in "$@"; do
  case $step in
    sweep) CFG=6 run sweep 200 python tools/gemm_sweep_check.py ;;
    gemmtests) run gemmtests 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_kernels.py -q -rf --timeout 120 --timeout-method thread ;;
    gemm5) CAPK_GEMM_8Q=0 GEMM_GRAPH=1 GEMM_ONLY=${SHAPES:-vit_qkv_fwd,vit_o_fwd,vit_fc1_fwd_plain,vit_fc1_fwd_gelu_deriv,vit_fc2_fwd,vit_qkv_dx,vit_fc1_dx,vit_fc2_dx_gelu_deriv,vit_o_dw,vit_fc1_dw,vit_qkv_dw,lm_head_fwd,lm_head_dw,bf16_4k,bf16_8k} run gemm5 300 python tools/gemm_bench.py ;;
    gemm6) CAPK_GEMM_8Q=1 GEMM_GRAPH=1 GEMM_ONLY=${SHAPES:-vit_qkv_fwd,vit_o_fwd,vit_fc1_fwd_plain,vit_fc1_fwd_gelu_deriv,vit_fc2_fwd,vit_qkv_dx,vit_fc1_dx,vit_fc2_dx_gelu_deriv,vit_o_dw,vit_fc1_dw,vit_qkv_dw,lm_head_fwd,lm_head_dw,bf16_4k,bf16_8k} run gemm6 300 python tools/gemm_bench.py ;;
    gemmpf) for pf in ${PFS:-0 3 4 6}; do CAPK_GEMM_PF=$pf CAPK_GEMM_8Q=1 GEMM_GRAPH=1 GEMM_ONLY=${SHAPES:-vit_qkv_fwd,vit_o_fwd,vit_fc1_fwd_plain,vit_fc2_fwd,vit_qkv_dx,vit_fc1_dx,vit_fc2_dx_gelu_deriv,lm_head_fwd,bf16_4k} run gemmpf$pf 200 python tools/gemm_bench.py; done ;;
    bench3p) CAPK_GEMM_8Q=0 run bench_config3_8p 480 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --beam-batch 0 ;;
    diag) for d in ${DIAGS:-nostore row0}; do CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/libcapk_diag_$d.so CAPK_GEMM_8Q=1 GEMM_GRAPH=1 GEMM_ONLY=${SHAPES:-vit_qkv_fwd,vit_o_fwd,vit_fc1_fwd_plain,vit_fc1_fwd_gelu_deriv,vit_fc2_fwd,vit_qkv_dx,lm_head_fwd,bf16_4k} run diag_$d 200 python tools/gemm_bench.py; done ;;
    vit) run vit 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_config4.py tests/test_gpu_fp8.py tests/test_gpu_kernels.py tests/test_gpu_gemm.py -q -rf --timeout 240 --timeout-method thread ;;
    scst) run scst 600 python -u -m pytest tests/test_gpu_scst.py tests/test_gpu_config4.py tests/test_gpu_plugins.py -q -rf --timeout 240 --timeout-method thread ;;
    decsweep) for c in ${CFGS:-1 2 3 4}; do CAPK_GEMM_CFG=$c GEMM_GRAPH=1 GEMM_ONLY=dec256_cattn,dec256_cproj,dec256_fc,dec256_proj2,dec1280_cattn,dec1280_cproj,dec1280_fc,dec1280_proj2,tdec1280_qkv,tdec1280_fc1,tdec1280_fc2 run dec_cfg$c 200 python tools/gemm_bench.py; done
             for ms in ${SPLITS:-1 2 4}; do CAPK_GEMM_MAXSPLIT=$ms GEMM_GRAPH=1 GEMM_ONLY=dec256_cattn,dec256_cproj,dec256_fc,dec256_proj2,dec1280_cattn,dec1280_cproj,dec1280_fc,dec1280_proj2 run dec_split$ms 200 python tools/gemm_bench.py; done ;;
    plugins) run plugins 400 python -u -m pytest tests/test_gpu_plugins.py tests/test_gpu_checkpoint.py -q -rf --timeout 240 --timeout-method thread ;;
    tests) run tests 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread ;;
    smoke) run smoke 240 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench3) run bench_config3 480 python bench.py --steps 10 --warmup 3 ;;
    bench2) run bench_config2 420 python bench.py --workload config2 --steps 8 --warmup 3 ;;
    bench5) run bench_config5 480 python bench.py --workload config5 --steps 5 --warmup 2 ;;
    prof5) run prof5 480 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o run -- python bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline --beam-batch 0 ;;
    prof2) run prof2 480 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof2 -o run -- python bench.py --workload config2 --steps 3 --warmup 2 --no-cpu-baseline ;;
    prof3) run prof3 480 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof3 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --beam-batch 0 ;;
  esac
done
exit 0
