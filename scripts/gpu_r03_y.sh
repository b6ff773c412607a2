# Verify on read: page counts computed inside the rocPRIM scan's input (rvf,
# the in-tree build: no count launch) vs the separate count kernel (rvf0).
# Every read / verify GPU test on the in-tree build, then interleaved A/B.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "verify or read" > $R/gpurun_out/y_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/y_tests.log; exit 1; }
tail -1 $R/gpurun_out/y_tests.log
V=build/variants
timeout -k 10 400 python -u scripts/reads_ab.py $V/libcurvecrc_rvf0.so $V/libcurvecrc_rvf.so > $R/gpurun_out/y_ab.log 2>&1 || { echo RFAIL; tail -20 $R/gpurun_out/y_ab.log; exit 1; }
tail -2 $R/gpurun_out/y_ab.log
echo done
