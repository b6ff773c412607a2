# Write log: rarely used kernel arguments re-read from the kernarg segment
# where used (ca: in-tree build) instead of kept live across the page loop
# (ca0).  Parity of the write-log tests (both modes), host layer and
# integrity, then A/B full and delta.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_host_cpp.py tests/test_integrity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "log or partial or write or host or integrity" > $R/gpurun_out/u_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/u_tests.log; exit 1; }
tail -1 $R/gpurun_out/u_tests.log
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_ca0.so $V/libcurvecrc_ca.so > $R/gpurun_out/u_ab.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/u_ab.log; exit 1; }
tail -2 $R/gpurun_out/u_ab.log
timeout -k 10 300 python -u scripts/log_ab.py --delta $V/libcurvecrc_ca0.so $V/libcurvecrc_ca.so > $R/gpurun_out/u_abd.log 2>&1 || { echo ABDFAIL; tail -20 $R/gpurun_out/u_abd.log; exit 1; }
tail -2 $R/gpurun_out/u_abd.log
echo done
