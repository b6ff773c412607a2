# Write log: a dynamic tail of 1/DIV of the heads in chunks of K heads (one
# counter) after the age-weighted static shares, vs none (d0 = shipped).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
V=build/variants
timeout -k 10 400 python -u scripts/log_ab.py $V/libcurvecrc_d0.so $V/libcurvecrc_d16k4.so $V/libcurvecrc_d32k2.so $V/libcurvecrc_d8k4.so $V/libcurvecrc_d16k8.so > $R/gpurun_out/q_ab.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/q_ab.log; exit 1; }
tail -5 $R/gpurun_out/q_ab.log
echo done
