# quick GPU check used during development: targeted tests + write-log profile
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_host_cpp.py tests/test_pool_native.py -m gpu -x -v --timeout 120 --timeout-method thread -k "beyond_4gib or partial or write_log or host_layer or pool" > gpurun_out/t3.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t3.log; exit 1; }
tail -2 gpurun_out/t3.log
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_log -o run --output-format csv -- python3 $R/scripts/prof_log.py > $R/gpurun_out/prof_log.log 2>&1 || exit 1
grep "ms per" $R/gpurun_out/prof_log.log
