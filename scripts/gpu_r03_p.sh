# Verify-on-read and WAL replay: static shares weighted by SIMD age (AgeSplit;
# W0/W1 = the oldest / younger wave of each SIMD) vs equal shares (age0).
# Parity of the read / WAL / range tests on the shipped weights, then
# interleaved A/B of the weight settings on both paths.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "verify or read or wal or range or chunk_hash or geometr" > $R/gpurun_out/p_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/p_tests.log; exit 1; }
tail -1 $R/gpurun_out/p_tests.log
V=build/variants
timeout -k 10 400 python -u scripts/reads_ab.py $V/libcurvecrc_age0.so $V/libcurvecrc_a52.so $V/libcurvecrc_a55.so $V/libcurvecrc_a60.so $V/libcurvecrc_a65.so > $R/gpurun_out/p_reads.log 2>&1 || { echo RFAIL; tail -20 $R/gpurun_out/p_reads.log; exit 1; }
tail -5 $R/gpurun_out/p_reads.log
AB_ROUNDS=16 timeout -k 10 400 python -u scripts/wal_sched_ab.py $V/libcurvecrc_age0.so@flat $V/libcurvecrc_a52.so@flat $V/libcurvecrc_a55.so@flat $V/libcurvecrc_a60.so@flat $V/libcurvecrc_a65.so@flat > $R/gpurun_out/p_wal.log 2>&1 || { echo WFAIL; tail -20 $R/gpurun_out/p_wal.log; exit 1; }
grep median $R/gpurun_out/p_wal.log
echo done
