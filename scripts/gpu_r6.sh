#!/bin/bash
# Round-6 GPU session driver: STEPS=comma list of named steps; every GPU step runs under its
# own time limit and a crash-type exit (not 0/1) ends the call.  Logs under gpurun_out/r6.
set -u
OUT=gpurun_out/r6
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
B3="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --beam-batch 0"
S=${STEPS:-tests}
[[ ,$S, == *,tsel,* ]] && run tsel 600 bash -c "$PYT ${TESTS}"
[[ ,$S, == *,tests,* ]] && run tests 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
[[ ,$S, == *,smoke,* ]] && run smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
[[ ,$S, == *,gemmab,* ]] && run gemmab ${GEMMAB_SECS:-400} python -u tools/gemm_ab.py
if [[ ,$S, == *,clock,* ]]; then  # effective clock per GEMM dispatch (GRBM_GUI_ACTIVE / 8 / wall)
  GEMM_ONLY= GEMM_SHAPES=${CLOCK_SHAPES:-qkv4:201728:2304:768:fwd,fc1g4:201728:3072:768:fwd_gelu_deriv,fc2dx4:201728:3072:768:dx_gelu_deriv,fc2f4:201728:768:3072:fwd,qkvdw4:201728:2304:768:dw,b4k:4096:4096:4096:fwd,b8k:8192:8192:8192:fwd} \
  run clock 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/clock -o run -- python3 tools/gemm_bench.py
  python3 tools/clock_probe.py $OUT/clock > $OUT/clock_table.txt; head -30 $OUT/clock_table.txt
fi
if [[ ,$S, == *,fetch,* ]]; then  # FETCH_SIZE per GEMM shape under each raster (CAPK_GEMM_GROUP)
  for g in ${FETCH_GROUPS:-0 -1}; do
    CAPK_GEMM_GROUP=$g run fetch_g$g 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch_g$g -o run -- python3 tools/gemm_bench.py
    python3 tools/pmc_summary.py $OUT/fetch_g$g --match gemm8q > $OUT/fetch_g$g.txt 2>&1 || true
  done
fi
if [[ ,$S, == *,benchab,* ]]; then  # config-3 bench under two environments, ABAB (same box)
  for i in 1 2; do
    env ${ENV_A:-CAPK_GEMM_GROUP=0} timeout -k 10 300 $B3 > $OUT/benchab_A$i.log 2>&1 || { echo "A$i failed"; tail -5 $OUT/benchab_A$i.log; exit 1; }
    echo "A$i $(grep -o '"value": [0-9.]*' $OUT/benchab_A$i.log | head -1)"
    env ${ENV_B:-CAPK_GEMM_GROUP=-1} timeout -k 10 300 $B3 > $OUT/benchab_B$i.log 2>&1 || { echo "B$i failed"; tail -5 $OUT/benchab_B$i.log; exit 1; }
    echo "B$i $(grep -o '"value": [0-9.]*' $OUT/benchab_B$i.log | head -1)"
  done
fi
if [[ ,$S, == *,libtest,* ]]; then  # GEMM tests on every library of LIBS (diagnostic / experimental builds)
  for L in ${LIBS}; do
    CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/$L run libtest_$L 300 $PYT tests/test_gpu_gemm.py
  done
fi
if [[ ,$S, == *,libab,* ]]; then  # tools/gemm_bench.py per library, libraries alternated, 2 rounds
  for r in 1 2; do
    for L in libcapk.so ${LIBS}; do
      CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/$L GEMM_GRAPH=1 run libab_${L}_$r 200 python -u tools/gemm_bench.py
    done
  done
  for L in libcapk.so ${LIBS}; do echo "== $L"; grep -h TFLOP $OUT/libab_${L}_*.log | sort | awk '{print}'; done > $OUT/libab_table.txt
fi
if [[ ,$S, == *,libbench,* ]]; then  # config-3 bench per library, alternated, 2 rounds
  for r in 1 2; do
    for L in libcapk.so ${LIBS}; do
      CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/$L $B3 > $OUT/libbench_${L}_$r.log 2>&1 || { echo "$L failed"; tail -5 $OUT/libbench_${L}_$r.log; exit 1; }
      echo "$L $r $(grep -o '"value": [0-9.]*' $OUT/libbench_${L}_$r.log | head -1)"
    done
  done
fi
if [[ ,$S, == *,lnab,* ]]; then  # tools/ln_bench.py per library, libraries alternated, 2 rounds
  for r in 1 2; do
    for L in libcapk.so ${LIBS}; do
      CAPK_LIB_PATH=$PWD/image-captioning-ml-project_amd/capk/$L run lnab_${L}_$r 120 python -u tools/ln_bench.py
    done
  done
  for L in libcapk.so ${LIBS}; do echo "== $L"; cat $OUT/lnab_${L}_*.log | grep us; done > $OUT/lnab_table.txt
fi
if [[ ,$S, == *,traffic,* ]]; then  # GEMM bytes per launch for bench.py's roofline.traffic (-> profiles/round6/gemm_traffic.json)
  TC="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --beam-batch 0"
  run fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- $TC
  run write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- $TC
  python3 tools/pmc_traffic.py $OUT/fetch $OUT/write --out $OUT/gemm_traffic.json --cmd "$TC" > /dev/null && \
    mkdir -p profiles/round6 && cp $OUT/gemm_traffic.json profiles/round6/gemm_traffic.json
fi
[[ ,$S, == *,hiptrace,* ]] && run hiptrace 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $OUT/hiptrace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --beam-batch 0
[[ ,$S, == *,profbeam,* ]] && run profbeam 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profbeam -o run -- python3 tools/beam_bench.py --reps 2
if [[ ,$S, == *,beamab,* ]]; then  # beam-5 (tools/beam_bench.py) under two environments, ABAB (same box)
  for i in 1 2; do
    env ${ENV_A:-CAPK_RING_GROUP=0} timeout -k 10 240 python tools/beam_bench.py --reps 3 > $OUT/beamab_A$i.log 2>&1 || { echo "beam A$i failed"; tail -5 $OUT/beamab_A$i.log; exit 1; }
    echo "A$i $(grep -h 'captions/s' $OUT/beamab_A$i.log)"
    env ${ENV_B:-CAPK_RING_GROUP=-1} timeout -k 10 240 python tools/beam_bench.py --reps 3 > $OUT/beamab_B$i.log 2>&1 || { echo "beam B$i failed"; tail -5 $OUT/beamab_B$i.log; exit 1; }
    echo "B$i $(grep -h 'captions/s' $OUT/beamab_B$i.log)"
  done
fi
[[ ,$S, == *,bench3,* ]] && run bench_config3 480 python bench.py --steps 10 --warmup 3
[[ ,$S, == *,bench3q,* ]] && run bench_config3q 300 $B3
[[ ,$S, == *,bench5,* ]] && run bench_config5 480 python bench.py --workload config5 --steps 5 --warmup 2
[[ ,$S, == *,bench2,* ]] && run bench_config2 420 python bench.py --workload config2 --steps 8 --warmup 3
[[ ,$S, == *,prof3,* ]] && run prof3 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof3 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --beam-batch 0
[[ ,$S, == *,prof5,* ]] && run prof5 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o run -- python3 bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline --beam-batch 0
[[ ,$S, == *,prof2,* ]] && run prof2 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof2 -o run -- python3 bench.py --workload config2 --steps 3 --warmup 2 --no-cpu-baseline
if [[ ,$S, == *,pmcattn,* ]]; then  # PMC groups (scripts/pmc_groups.txt) over the ViT attention kernels
  PROF_TAG=r6/pmcattn ATTN_ONLY=${ATTN_ONLY:-vit} timeout -k 10 900 bash scripts/gpu_counters.sh python3 tools/attn_bench.py || exit $?
  python3 tools/pmc_summary.py $OUT/pmcattn/p* --match attn_ > $OUT/pmcattn.txt 2>&1; head -60 $OUT/pmcattn.txt
fi
[[ ,$S, == *,attnb,* ]] && run attnb 300 python tools/attn_bench.py
[[ ,$S, == *,gemmb,* ]] && run gemmb 400 python tools/gemm_bench.py ${GEMMB_ARGS:-}
[[ ,$S, == *,extra,* ]] && run extra ${EXTRA_SECS:-300} ${EXTRA}
exit 0
