# Write log: age-weighted head shares (sk3/sk5/sk6) and a rotating issue
# priority (rot: equal shares, rotsk3: with sk3's weights) vs the strided equal
# shares (s0); per-wave clocks of sk3 and rot.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
V=build/variants
timeout -k 10 400 python -u scripts/log_ab.py $V/libcurvecrc_s0.so $V/libcurvecrc_sk3.so $V/libcurvecrc_sk5.so $V/libcurvecrc_sk6.so $V/libcurvecrc_rot.so $V/libcurvecrc_rotsk3.so > $R/gpurun_out/o_ab_full.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/o_ab_full.log; exit 1; }
tail -6 $R/gpurun_out/o_ab_full.log
for t in ltr3 ltrrot; do
timeout -k 10 300 python -u scripts/trace_log.py $V/libcurvecrc_$t.so > $R/gpurun_out/o_trace_$t.log 2>&1 || { echo TRFAIL; tail -20 $R/gpurun_out/o_trace_$t.log; exit 1; }
tail -1 $R/gpurun_out/o_trace_$t.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$t', {k: d[k] for k in ('block_end_us_p1_p50_p90_max','block_end_us_mean','end_us_median_by_wave_slot')})"
done
echo done
