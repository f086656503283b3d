#!/bin/bash
# LSTM step GEMM shapes (config 2): default split-K vs none vs forced configs, graph-timed.
set -o pipefail
mkdir -p gpurun_out
for ms in 0 1 2 4; do
  for cfg in "" 3 4; do
    echo "== MAXSPLIT=$ms CFG=$cfg"
    env ${cfg:+CAPK_GEMM_CFG=$cfg} $( [ $ms -gt 0 ] && echo CAPK_GEMM_MAXSPLIT=$ms ) GEMM_GRAPH=1 GEMM_ONLY=lstm_gates_fwd,lstm_dh_dx GEMM_ITERS=50 \
      timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -v Warning | tail -3 || exit $?
  done
done
