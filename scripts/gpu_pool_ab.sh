# all -m gpu tests, then the scan-step A/B (scripts/pool_ab.py) of the in-tree
# build against build/variants/<v>, then the default bench line
set -u
R=$(pwd)
TAG=${TAG:-pab}
mkdir -p $R/gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $R/gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/gpu_tests_$TAG.log
L="curve_amd/libcurvecrc.so"
for v in "$@"; do L="$L build/variants/libcurvecrc_$v.so"; done
timeout -k 10 200 python -u scripts/pool_ab.py $L || exit 1
timeout -k 10 400 python -u bench.py > $R/gpurun_out/bench_$TAG.log 2>&1 || { echo BENCHFAIL; tail -30 $R/gpurun_out/bench_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/bench_$TAG.log > $R/gpurun_out/bench_$TAG.json
echo done
