#!/bin/bash
# One GPU-box session: parity tests -> smoke -> bench.  Each GPU step has its own
# time limit; a crash-type exit (abort/segv/timeout/kill) ends the session.
set -u
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-kern,model,smoke,bench}
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test failures (no crash)
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  tail -5 $OUT/$name.log
  ok_rc $rc || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
python -c "import torch;print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0).gcnArchName)" | tee $OUT/device.txt
[[ $STEPS == *kern* ]] && run kern 600 python -m pytest tests/test_gpu_kernels.py -q -rf
[[ $STEPS == *beam* ]] && run beam 900 python -m pytest tests/test_gpu_beam.py -q -rf
[[ $STEPS == *lstm* ]] && run lstm 900 python -m pytest tests/test_gpu_lstm.py -q -rf
[[ $STEPS == *scst* ]] && run scst 900 python -m pytest tests/test_gpu_scst.py -q -rf
[[ $STEPS == *resnet* ]] && run resnet 900 python -u -m pytest tests/test_gpu_resnet.py -q -rf --timeout 300 --timeout-method thread
[[ $STEPS == *legacy* ]] && run legacy 900 python -u -m pytest tests/test_gpu_legacy.py -q -rf --timeout 300 --timeout-method thread
[[ $STEPS == *cfg4* ]] && run cfg4 900 python -m pytest tests/test_gpu_config4.py -q -rf
[[ $STEPS == *dp* ]] && run dp 300 python -u -m pytest tests/test_gpu_dp.py -q -rf --timeout 240 --timeout-method thread
[[ $STEPS == *model* ]] && run model 900 python -m pytest tests/test_gpu_model.py -q -rf
[[ $STEPS == *gemm* ]] && run gemm 300 python tools/gemm_bench.py
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 900 python bench.py --steps ${BSTEPS:-5} --warmup 2
exit 0
