#!/bin/bash
# Round-3 closing evidence on one GPU box, all from this tree: -m gpu suite -> smoke -> bench
# lines (config 3 with beam-5, config 5, config 2) -> rocprofv3 kernel-trace/stats of the
# config-3 / config-5 / config-2 benches -> FETCH_SIZE / WRITE_SIZE passes over the config-3
# bench (GEMM traffic -> profiles/round3/gemm_traffic.json via tools/pmc_traffic.py) -> SQ/LDS/
# MFMA passes.  Every GPU step has its own time limit; a crash-type exit ends the session.
set -u
OUT=gpurun_out/r3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  tail -3 $OUT/$name.log | cut -c1-300
  ok_rc $rc || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
S=${STEPS_R3:-tests,smoke,bench3,bench5,bench2,prof3,prof5,prof2,traffic,sq}
[[ $S == *tests* ]] && run tests 700 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
[[ $S == *smoke* ]] && run smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
[[ $S == *bench3* ]] && run bench_config3 480 python bench.py --steps 10 --warmup 3
[[ $S == *bench5* ]] && run bench_config5 480 python bench.py --workload config5 --steps 5 --warmup 2
[[ $S == *bench2* ]] && run bench_config2 420 python bench.py --workload config2 --steps 8 --warmup 3
[[ $S == *prof3* ]] && run prof3 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof3 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --beam-batch 0
[[ $S == *prof5* ]] && run prof5 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o run -- python3 bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline --beam-batch 0
[[ $S == *prof2* ]] && run prof2 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof2 -o run -- python3 bench.py --workload config2 --steps 3 --warmup 2 --no-cpu-baseline
if [[ $S == *traffic* ]]; then
  run fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0
  run write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0
  python3 tools/pmc_traffic.py $OUT/fetch $OUT/write --out $OUT/gemm_traffic.json --cmd "python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0" > /dev/null
fi
if [[ $S == *sq* ]]; then
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    case $grp in FETCH_SIZE|WRITE_SIZE) continue ;; esac
    i=$((i+1))
    run sq$i 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/sq$i -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0
  done < scripts/pmc_groups.txt
fi
exit 0
