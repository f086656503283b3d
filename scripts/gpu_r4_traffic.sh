#!/bin/bash
# Counter reconciliation: every tools/traffic_calib.py case under FETCH_SIZE, WRITE_SIZE and
# TCC hit / miss passes (one process per case and pass), then tools/traffic_table.py.
set -u
OUT=gpurun_out/r4traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 60 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
for c in ${CASES:-copy1g fill1g read1g qkv_fwd fc1_gelu_deriv fc2_fwd_res o_dx fc2_dx_dsum lm_fwd qkv_dw}; do
  for p in ${PASSES:-FETCH_SIZE WRITE_SIZE TCC_HIT_sum,TCC_MISS_sum}; do
    pn=$(echo $p | tr ',' '_')
    timeout -s KILL 90 rocprofv3 --pmc $(echo $p | tr ',' ' ') --kernel-trace --output-format csv -d $OUT/$c/$pn -o run -- python3 tools/traffic_calib.py --case $c > $OUT/$c.$pn.log 2>&1
    rc=$?
    echo "$c $pn rc=$rc"
    [ $rc -eq 0 ] || { tail -5 $OUT/$c.$pn.log; exit $rc; }
  done
done
python3 tools/traffic_table.py $OUT > $OUT/table.md && cat $OUT/table.md
exit 0
