# Write log: heads cut among a workgroup's waves by SIMD age (weights W0..W3 for
# the oldest .. youngest wave of each SIMD) vs the strided equal shares (s0).
# Parity of the write-log tests (shipped weights), interleaved A/B of the
# weight settings (full and delta), then the per-wave clocks of the shipped weights.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_host_cpp.py -m gpu -x -q --timeout 200 --timeout-method thread -k "log or partial or write or host" > $R/gpurun_out/n_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/n_tests.log; exit 1; }
tail -1 $R/gpurun_out/n_tests.log
V=build/variants
timeout -k 10 400 python -u scripts/log_ab.py $V/libcurvecrc_s0.so $V/libcurvecrc_eq.so $V/libcurvecrc_sk1.so $V/libcurvecrc_sk2.so $V/libcurvecrc_sk3.so $V/libcurvecrc_sk4.so > $R/gpurun_out/n_ab_full.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/n_ab_full.log; exit 1; }
tail -6 $R/gpurun_out/n_ab_full.log
timeout -k 10 300 python -u scripts/log_ab.py --delta $V/libcurvecrc_s0.so $V/libcurvecrc_sk2.so $V/libcurvecrc_sk3.so > $R/gpurun_out/n_ab_delta.log 2>&1 || { echo ABDFAIL; tail -20 $R/gpurun_out/n_ab_delta.log; exit 1; }
tail -3 $R/gpurun_out/n_ab_delta.log
timeout -k 10 300 python -u scripts/trace_log.py $V/libcurvecrc_ltr.so > $R/gpurun_out/n_trace.log 2>&1 || { echo TRFAIL; tail -20 $R/gpurun_out/n_trace.log; exit 1; }
tail -1 $R/gpurun_out/n_trace.log
echo done
