# Write log: changed rows stored under uniform branches (sbr) instead of
# out-of-range offsets for the unchanged ones (ship).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_ship.so $V/libcurvecrc_sbr.so > $R/gpurun_out/j_ab.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/j_ab.log; exit 1; }
tail -2 $R/gpurun_out/j_ab.log
echo done
