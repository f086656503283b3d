#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no counters, no sys-trace).
set -u
OUT=gpurun_out/${PROF_TAG:-prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 ${PROF_SECS:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 ${PROF_CMD:-bench.py --steps ${BSTEPS:-3} --warmup 2 --no-cpu-baseline} > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "rocprof rc=$rc"
find $OUT -name "*stats*" | head
exit $rc
