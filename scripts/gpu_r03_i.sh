# Write log, shipped kernel: timing ablations (wrong results, timing only):
# (the ablations take the generic merge path: gen = the same without them)
# 1 no row stores, 3 no page loads, 4 no CRC chain, 5 no data loads or stores.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_ship.so $V/libcurvecrc_gen.so $V/libcurvecrc_abl1.so $V/libcurvecrc_abl3.so $V/libcurvecrc_abl4.so $V/libcurvecrc_abl5.so > $R/gpurun_out/i_abl.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/i_abl.log; exit 1; }
tail -6 $R/gpurun_out/i_abl.log
echo done
