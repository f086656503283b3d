#!/bin/bash
# Kernel-time profiles (rocprofv3 --kernel-trace --stats) of the beam-5 leg alone and of the
# config-5 SCST update, on this tree.
set -u
OUT=gpurun_out/r3prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-3} | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
[[ ${S:-beam,c5} == *beam* ]] && run beam 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/beam -o run -- python3 tools/beam_bench.py --reps 2
[[ ${S:-beam,c5} == *c5* ]] && run c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5 -o run -- python3 bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline --beam-batch 0
for d in beam c5; do f=$(find $OUT/$d -name "*kernel_stats.csv" 2>/dev/null | head -1); [ -n "$f" ] && { echo "## $d"; python3 tools/kstats.py $f 1 25; }; done
exit 0
