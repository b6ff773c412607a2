# The -m gpu tests only (each bounded), then the host C++ binary's GPU cases.
set -u
R=$(pwd)
TAG=${1:-r02}
mkdir -p $R/gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $R/gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTFAIL; tail -60 $R/gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/gpu_tests_$TAG.log
echo done
