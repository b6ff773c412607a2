# Write log: cache-policy bits of the full-mode row loads (2 = nontemporal, shipped; 0, 1, 3).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_ra2.so $V/libcurvecrc_ra0.so $V/libcurvecrc_ra1.so $V/libcurvecrc_ra3.so > $R/gpurun_out/ac_ab.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/ac_ab.log; exit 1; }
tail -4 $R/gpurun_out/ac_ab.log
echo done
