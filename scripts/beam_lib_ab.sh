#!/bin/bash
# beam-5 (tools/beam_bench.py) per library (libcapk.so vs $LIBS), alternated, 3 rounds
for r in 1 2 3; do
  for L in libcapk.so ${LIBS}; do
    CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/$L timeout -k 10 240 python tools/beam_bench.py --reps 3 | sed "s/^/$L: /" || exit 1
  done
done
