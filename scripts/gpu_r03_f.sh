# Write log: a page with several pieces gets its list (third link + the first
# two descriptors) through the previous step's edge loads.  Parity of the
# write-log tests (both modes) and the C++ host layer, then interleaved A/B
# against the previous build (new2) and the same code without the prefetch (lp0).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_host_cpp.py -m gpu -x -q --timeout 200 --timeout-method thread -k "log or partial or write or host" > $R/gpurun_out/f_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/f_tests.log; exit 1; }
tail -1 $R/gpurun_out/f_tests.log
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_new2.so $V/libcurvecrc_lp.so $V/libcurvecrc_lp0.so > $R/gpurun_out/f_ab_full.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/f_ab_full.log; exit 1; }
tail -3 $R/gpurun_out/f_ab_full.log
timeout -k 10 300 python -u scripts/log_ab.py --delta $V/libcurvecrc_new2.so $V/libcurvecrc_lp.so > $R/gpurun_out/f_ab_delta.log 2>&1 || { echo ABDFAIL; tail -20 $R/gpurun_out/f_ab_delta.log; exit 1; }
tail -2 $R/gpurun_out/f_ab_delta.log
echo done
