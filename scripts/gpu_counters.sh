#!/bin/bash
# PMC counter passes (one --pmc group per rocprofv3 run, kernel-trace only) over a command.
set -u
OUT=gpurun_out/${PROF_TAG:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i [$grp] rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; [ $rc -gt 1 ] && [ $rc -ne 255 ] && exit $rc; }
done < ${PMC_GROUPS:-scripts/pmc_groups.txt}
exit 0
