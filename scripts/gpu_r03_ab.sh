# Write log: hash table >= 8 x pieces (in-tree build) -- parity of the
# write-log tests, host layer and integrity, then A/B vs 4 x, full and delta.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_host_cpp.py tests/test_integrity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "log or partial or write or host or integrity" > $R/gpurun_out/ab_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/ab_tests.log; exit 1; }
tail -1 $R/gpurun_out/ab_tests.log
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_tf4.so $V/libcurvecrc_tf8.so > $R/gpurun_out/ab2_ab.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/ab2_ab.log; exit 1; }
tail -2 $R/gpurun_out/ab2_ab.log
timeout -k 10 300 python -u scripts/log_ab.py --delta $V/libcurvecrc_tf4.so $V/libcurvecrc_tf8.so > $R/gpurun_out/ab2_abd.log 2>&1 || { echo ABDFAIL; tail -20 $R/gpurun_out/ab2_abd.log; exit 1; }
tail -2 $R/gpurun_out/ab2_abd.log
echo done
