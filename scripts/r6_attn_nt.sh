set -u
OUT=gpurun_out/r6; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python tools/attn_sweep.py --mode 1 > $OUT/attn_sweep.txt 2>&1 || exit $?
cat $OUT/attn_sweep.txt | grep -v amdgpu
for r in 1 2; do for nt in 0 1; do
  CAPK_GEMM_NT_STORE=$nt GEMM_ONLY=vit_fc1_fwd_gelu_deriv,vit_fc2_dx_gelu_deriv,vit_qkv_fwd,vit_fc2_fwd,vit_o_fwd timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep TFLOP | sed "s/^/nt$nt /" || exit 1
done; done > $OUT/nt_gemm.txt; cat $OUT/nt_gemm.txt
for nt in 0 1; do
  CAPK_GEMM_NT_STORE=$nt GEMM_ONLY=vit_fc1_fwd_gelu_deriv,vit_fc2_dx_gelu_deriv timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/ntfetch$nt -o run -- python3 tools/gemm_bench.py > $OUT/ntfetch$nt.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $OUT/ntfetch$nt --match gemm8q > $OUT/ntfetch$nt.txt 2>&1; grep -A1 "gemm8q" $OUT/ntfetch$nt.txt | cut -c1-300
done
