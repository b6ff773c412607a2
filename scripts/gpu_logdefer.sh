# Write log: pages with several pieces deferred past the pipeline (lean
# pipeline registers) -- parity of every write-log test and the C++ host layer,
# then interleaved A/B against the previous build, full and delta.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_host_cpp.py tests/test_stream_c3.py tests/test_wal.py -m gpu -x -q --timeout 200 --timeout-method thread -k "log or partial or write or host or wal" > $R/gpurun_out/defer_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/defer_tests.log; exit 1; }
tail -1 $R/gpurun_out/defer_tests.log
timeout -k 10 300 python -u scripts/log_ab.py build/variants/libcurvecrc_cur.so build/variants/libcurvecrc_defer.so > $R/gpurun_out/defer_ab.log 2>&1 || { echo LOGABFAIL; tail -20 $R/gpurun_out/defer_ab.log; exit 1; }
tail -3 $R/gpurun_out/defer_ab.log
timeout -k 10 300 python -u scripts/log_ab.py --delta build/variants/libcurvecrc_cur.so build/variants/libcurvecrc_defer.so > $R/gpurun_out/defer_ab_delta.log 2>&1 || { echo LOGABDFAIL; tail -20 $R/gpurun_out/defer_ab_delta.log; exit 1; }
tail -3 $R/gpurun_out/defer_ab_delta.log
echo done
