#!/bin/bash
# config-3 bench under the default environment and each knob of ENVS (one run each, the default
# repeated between knobs), same box: re-checks the tuned defaults on the final tree.
OUT=gpurun_out/r6
mkdir -p $OUT
B3="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --beam-batch 0"
i=0
for E in ${ENVS}; do
  i=$((i + 1))
  timeout -k 10 300 $B3 > $OUT/sweep_def_$i.log 2>&1 || { echo "default $i failed"; exit 1; }
  echo "default $(grep -o '"value": [0-9.]*' $OUT/sweep_def_$i.log | head -1)"
  env $E timeout -k 10 300 $B3 > $OUT/sweep_env_$i.log 2>&1 || { echo "$E failed"; exit 1; }
  echo "$E $(grep -o '"value": [0-9.]*' $OUT/sweep_env_$i.log | head -1)"
done
