# Page kernel: dynamic-tail chunk size (64 pages shipped, 32) and tail share
# (1/16 shipped, 1/12): step and page-kernel time, and the spread of the
# page-kernel launches (the bench's kernel_spread_pct), in the scan step.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
V=build/variants
timeout -k 10 400 python -u scripts/pool_ab.py $V/libcurvecrc_p64.so $V/libcurvecrc_p32.so $V/libcurvecrc_p32d12.so $V/libcurvecrc_p64d12.so > $R/gpurun_out/x_ab.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/x_ab.log; exit 1; }
tail -4 $R/gpurun_out/x_ab.log
echo done
