# Round evidence on the final code: -m gpu tests, bench line, kernel-trace
# profile of the bench, PMC traffic passes, write-log / WAL traces, then a
# 2-rank rehearsal of the multi-GPU bench flow on the one GPU (gloo).
set -u
R=$(pwd)
TAG=${1:-r02f}
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" || { echo SMOKEFAIL; exit 1; }
bash $R/scripts/gpu_round_r02.sh $TAG || exit 1
bash $R/scripts/gpu_round_r02b.sh $TAG || exit 1
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --chunks 512 --stream-chunks-per-rank 200 > $R/gpurun_out/bench_gloo2_$TAG.log 2>&1 || { echo GLOOFAIL; tail -30 $R/gpurun_out/bench_gloo2_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/bench_gloo2_$TAG.log
echo alldone
