#!/bin/bash
# A/B of the ViT/CLIP weight-gradient side stream (CAPK_DW_STREAM) plus the training-path GPU tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_config4.py tests/test_gpu_plugins.py \
  tests/test_gpu_fp8.py tests/test_gpu_checkpoint.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dw_tests.log 2>&1
rc=$?; tail -2 gpurun_out/dw_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  CAPK_DW_STREAM=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --beam-batch 0 > gpurun_out/dw_$v.log 2>&1 || exit $?
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/dw_{v}.log") if l.startswith("{")][-1])
print("DW_STREAM", v, d["value"], d["ms_per_step"], d.get("final_loss"))
PY
done
