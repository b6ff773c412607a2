# Verify-on-read and WAL replay: static shares weighted toward the YOUNGER wave
# of each SIMD (W0/W1 = oldest/younger: 48/52, 45/55, 40/60) vs equal (age0);
# the other direction lost at every weight (profiles/reads_wal_age_ab_r03p.txt).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
V=build/variants
timeout -k 10 400 python -u scripts/reads_ab.py $V/libcurvecrc_age0.so $V/libcurvecrc_i48.so $V/libcurvecrc_i45.so $V/libcurvecrc_i40.so > $R/gpurun_out/s_reads.log 2>&1 || { echo RFAIL; tail -20 $R/gpurun_out/s_reads.log; exit 1; }
tail -4 $R/gpurun_out/s_reads.log
AB_ROUNDS=16 timeout -k 10 400 python -u scripts/wal_sched_ab.py $V/libcurvecrc_age0.so@flat $V/libcurvecrc_i48.so@flat $V/libcurvecrc_i45.so@flat $V/libcurvecrc_i40.so@flat > $R/gpurun_out/s_wal.log 2>&1 || { echo WFAIL; tail -20 $R/gpurun_out/s_wal.log; exit 1; }
grep median $R/gpurun_out/s_wal.log
echo done
