# Write-log path on the GPU: its parity tests, then timing (events) in both
# modes, then a rocprofv3 kernel trace of the whole call.  Each step bounded.
set -u
R=$(pwd)
TAG=${1:-r02}
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "partial or write_log or beyond or hot" > $R/gpurun_out/log_tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/log_tests_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/log_tests_$TAG.log
timeout -k 10 200 python -u scripts/prof_log.py --reps 8 || exit 1
timeout -k 10 200 python -u scripts/prof_log.py --reps 8 --delta || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_log_$TAG
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_log_$TAG -o run --output-format csv -- python3 $R/scripts/prof_log.py > $R/gpurun_out/prof_log_$TAG.log 2>&1 || { echo LOGPROFFAIL; exit 1; }
grep "ms per" $R/gpurun_out/prof_log_$TAG.log
echo done
