# all -m gpu tests, the default bench line, then write-log A/B of the in-tree
# build against the given variants
set -u
R=$(pwd)
TAG=${TAG:-chk}
mkdir -p $R/gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $R/gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/gpu_tests_$TAG.log
timeout -k 10 400 python -u bench.py > $R/gpurun_out/bench_$TAG.log 2>&1 || { echo BENCHFAIL; tail -30 $R/gpurun_out/bench_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/bench_$TAG.log > $R/gpurun_out/bench_$TAG.json
L="curve_amd/libcurvecrc.so"
for v in "$@"; do L="$L build/variants/libcurvecrc_$v.so"; done
[ $# -gt 0 ] && { timeout -k 10 200 python -u scripts/log_ab.py $L || exit 1; }
echo done
