set -u
export GEMM_SHAPES="dx768_197:50432:768:768:dx,dx3072_197:50432:768:3072:dx,dx2304_197:50432:768:2304:dx,res768_197:50432:768:768:fwd_res,res3072_197:50432:768:3072:fwd_res,fc1g_197:50432:3072:768:fwd_gelu_deriv,qkv_197:50432:2304:768:fwd,lmfwd:5120:50304:768:fwd"
echo "--- SPT on"; timeout -k 10 200 python tools/gemm_bench.py || exit $?
echo "--- SPT off"; CAPK_GEMM_SPT=0 timeout -k 10 200 python tools/gemm_bench.py || exit $?
