#!/bin/bash
# Round-4 GPU session driver: STEPS=comma list of named steps; every GPU step runs under its
# own time limit and a crash-type exit (not 0/1) ends the call.  Logs under gpurun_out/r4.
set -u
OUT=gpurun_out/r4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/status
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/status
  grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-4} | cut -c1-400
  ok_rc $rc || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
PYT="python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread"
S=${STEPS:-tests}
[[ ,$S, == *,tsel,* ]] && run tsel 600 $PYT ${TESTS}
[[ ,$S, == *,tests,* ]] && run tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
[[ ,$S, == *,smoke,* ]] && run smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
if [[ ,$S, == *,traffic,* ]]; then  # GEMM bytes per launch for bench.py's roofline.traffic (-> profiles/round4/gemm_traffic.json)
  run fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0
  run write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0
  python3 tools/pmc_traffic.py $OUT/fetch $OUT/write --out $OUT/gemm_traffic.json --cmd "python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0" > /dev/null
  # later bench steps of this call read the fresh file (the box's copy of the tree)
  cp $OUT/gemm_traffic.json profiles/round4/gemm_traffic.json
fi
[[ ,$S, == *,bench3,* ]] && run bench_config3 480 python bench.py --steps 10 --warmup 3
[[ ,$S, == *,bench3q,* ]] && run bench_config3q 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --beam-batch 0
[[ ,$S, == *,bench5,* ]] && run bench_config5 480 python bench.py --workload config5 --steps 5 --warmup 2
[[ ,$S, == *,bench2,* ]] && run bench_config2 420 python bench.py --workload config2 --steps 8 --warmup 3
[[ ,$S, == *,prof3,* ]] && run prof3 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof3 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --beam-batch 0
[[ ,$S, == *,prof5,* ]] && run prof5 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o run -- python3 bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline --beam-batch 0
[[ ,$S, == *,prof2,* ]] && run prof2 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof2 -o run -- python3 bench.py --workload config2 --steps 3 --warmup 2 --no-cpu-baseline
[[ ,$S, == *,gemmb,* ]] && run gemmb 400 python tools/gemm_bench.py ${GEMMB_ARGS:-}
[[ ,$S, == *,extra,* ]] && run extra ${EXTRA_SECS:-300} ${EXTRA}
exit 0
