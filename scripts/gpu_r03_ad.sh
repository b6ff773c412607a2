# Write log: page-kernel workgroups per CU (1 shipped; 2 or 3 = the later ones
# start where CUs free up: block-granular balancing, at the cost of an LDS fill
# and a metadata batch per extra workgroup).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_bp1.so $V/libcurvecrc_bp2.so $V/libcurvecrc_bp3.so > $R/gpurun_out/ad_ab.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/ad_ab.log; exit 1; }
tail -3 $R/gpurun_out/ad_ab.log
timeout -k 10 300 python -u scripts/log_ab.py --delta $V/libcurvecrc_bp1.so $V/libcurvecrc_bp2.so > $R/gpurun_out/ad_abd.log 2>&1 || { echo ABDFAIL; tail -20 $R/gpurun_out/ad_abd.log; exit 1; }
tail -2 $R/gpurun_out/ad_abd.log
echo done
