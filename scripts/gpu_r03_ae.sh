# Write log: age weights around the shipped 33/27/22/18 with the 8 x table
# (w35 = 35/27/21/17, w31 = 31/27/23/19, w34b = 34/28/21/17), full and delta.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_w33.so $V/libcurvecrc_w35.so $V/libcurvecrc_w31.so $V/libcurvecrc_w34b.so > $R/gpurun_out/ae_ab.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/ae_ab.log; exit 1; }
tail -4 $R/gpurun_out/ae_ab.log
timeout -k 10 300 python -u scripts/log_ab.py --delta $V/libcurvecrc_w33.so $V/libcurvecrc_w35.so $V/libcurvecrc_w31.so $V/libcurvecrc_w34b.so > $R/gpurun_out/ae_abd.log 2>&1 || { echo ABDFAIL; tail -20 $R/gpurun_out/ae_abd.log; exit 1; }
tail -4 $R/gpurun_out/ae_abd.log
echo done
