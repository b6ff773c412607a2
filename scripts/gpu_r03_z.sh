# Round-3 final evidence of the shipped tree: every -m gpu test, smoke(), the
# 2-rank gloo rehearsal with rank 1's native comm init failing, the driver's
# bench line, a kernel trace + stats of the bench (rocprofv3), kernel traces of
# the write log alone (full, delta) and its PMC passes (HBM bytes, SQ mix).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $R/gpurun_out/z_tests.log 2>&1 || { echo TESTFAIL; tail -40 $R/gpurun_out/z_tests.log; exit 1; }
tail -1 $R/gpurun_out/z_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $R/gpurun_out/z_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $R/gpurun_out/z_smoke.log; exit 1; }
tail -1 $R/gpurun_out/z_smoke.log
BENCH_DIST_BACKEND=gloo CC_INJECT_COMM_INIT_FAIL_RANK=1 timeout -k 10 300 python bench.py --gpus 2 --chunks 64 --steps 5 --warmup 2 --comm-timeout-ms 5000 --stream-chunks-per-rank 32 > $R/gpurun_out/z_gloo2.log 2>&1 || { echo GLOOFAIL; tail -30 $R/gpurun_out/z_gloo2.log; exit 1; }
tail -1 $R/gpurun_out/z_gloo2.log > $R/gpurun_out/z_gloo2.json
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/z_bench.log 2>&1 || { echo BENCHFAIL; tail -30 $R/gpurun_out/z_bench.log; exit 1; }
tail -1 $R/gpurun_out/z_bench.log > $R/gpurun_out/z_bench.json
bash scripts/gpu_profile.sh r03z 20 || { echo PROFFAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
for mode in full delta; do
  extra=""; [ $mode = delta ] && extra="--delta"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_log_r03z_$mode -o run --output-format csv -- python3 $R/scripts/prof_log.py --reps 10 $extra > $R/gpurun_out/prof_log_r03z_$mode.log 2>&1 || { echo LOGTRACEFAIL; exit 1; }
done
cd $R
bash scripts/gpu_pmc_log.sh _r03z || exit 1
bash scripts/gpu_pmc_log.sh _r03z_delta --delta || exit 1
echo done
