set -u
export GEMM_SHAPES="dx768_197:50432:768:768:dx,dx3072_197:50432:768:3072:dx,fc1g_197:50432:3072:768:fwd_gelu_deriv,fc1p_197:50432:3072:768:fwd,r257:65792:256:768:fwd"
echo "--- SPT on"; timeout -k 10 200 python tools/gemm_bench.py || exit $?
echo "--- SPT off"; CAPK_GEMM_SPT=0 timeout -k 10 200 python tools/gemm_bench.py || exit $?
echo "--- SPT no hand-off (diag)"; CAPK_LIB_PATH=image-captioning-ml-project_amd/capk/libcapk_diag_sptnoho.so timeout -k 10 200 python tools/gemm_bench.py || exit $?
