set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "attention or attn" --timeout 200 --timeout-method thread > gpurun_out/ta.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ta.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1 || exit 1
cat gpurun_out/attn_bench.log
rm -rf gpurun_out/attn_pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d gpurun_out/attn_pmc -o run --output-format csv -- python3 tools/attn_bench.py > gpurun_out/attn_pmc.log 2>&1 || exit 1
echo pmc ok
