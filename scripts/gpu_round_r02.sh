# Round evidence, part 1: every -m gpu test, the default bench line, a
# rocprofv3 kernel-trace/stats profile of the bench.  Each GPU step has its own
# time limit; the first failure ends the script.  usage: gpu_round_r02.sh TAG
set -u
R=$(pwd)
TAG=${1:-r02}
mkdir -p $R/gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -30 $R/gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/gpu_tests_$TAG.log
timeout -k 10 400 python -u bench.py > $R/gpurun_out/bench_$TAG.log 2>&1 || { echo BENCHFAIL; tail -30 $R/gpurun_out/bench_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/bench_$TAG.log > $R/gpurun_out/bench_$TAG.json
bash $R/scripts/gpu_profile.sh $TAG 20 || { echo PROFFAIL; exit 1; }
echo done
