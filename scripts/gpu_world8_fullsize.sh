# The driver's N=8 bench command at FULL size (1024 x 16 MiB chunks a rank, default legs), as
# the driver launches it (torch.distributed.run --nproc-per-node 8 ... bench.py --gpus 8 --steps 20
# --warmup 5), on the one-GPU box: BENCH_DIST_BACKEND=gloo, all 8 ranks on cuda:0 (128 GiB of
# pools in the 288 GB of HBM).  Checks the N>1 flow end to end at the real sizes (time, memory,
# every leg); its value is meaningless (8 ranks share one GPU).  A ticker keeps gpurun_out live.
# usage: bash scripts/gpu_world8_fullsize.sh [stub]   (stub: CURVE_AMD_LIB = the stub-RCCL test build,
# so the ranks take the NATIVE digest exchange, tests/native/rccl_stub.cpp)
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
( while sleep 30; do date +%T >> $R/gpurun_out/world8_full_tick.txt; done ) &
TICK=$!
EXTRA=""
TAG=world8_full
if [ "${1:-}" = stub ]; then EXTRA="CURVE_AMD_LIB=$R/build/stub/libcurvecrc_stubrccl.so"; TAG=world8_full_stub; fi
P=$(python3 -c "import socket; s=socket.socket(); s.bind(('127.0.0.1',0)); print(s.getsockname()[1])")
env BENCH_DIST_BACKEND=gloo $EXTRA timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port $P bench.py --gpus 8 --steps 20 --warmup 5 \
    > $R/gpurun_out/$TAG.log 2>&1
rc=$?
kill $TICK
grep '^{' $R/gpurun_out/$TAG.log > $R/gpurun_out/$TAG.json
echo "rc=$rc"
exit $rc
