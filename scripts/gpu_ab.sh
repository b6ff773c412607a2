# Interleaved in-process A/B of the in-tree libcurvecrc against variant builds
# (make -C curve_amd/csrc variant NAME=<v> DEFS=...), after the parity tests of
# the path on the in-tree build.  Every step bounded; the first failure ends the call.
# usage (from the repo root, through gpurun): bash scripts/gpu_ab.sh PATH v1 [v2 ...]
#   PATH: log (write log, full + delta) | page (page kernel) | pool (whole scan
#         step) | reads (verify on read) | wal (WAL replay ranges)
set -u
P=$1; shift
mkdir -p gpurun_out
case $P in
  log) K="write_log or partial or resident" ;;
  page|pool) K="page or pool or scan or golden" ;;
  reads) K="verify or read" ;;
  wal) K="range or wal or bufs or chunk_hash" ;;
  *) echo "unknown path $P"; exit 2 ;;
esac
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" \
    > gpurun_out/ab_${P}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_${P}_tests.log; [ $rc = 0 ] || exit 1
L="curve_amd/libcurvecrc.so"
for v in "$@"; do L="$L build/variants/libcurvecrc_$v.so"; done
case $P in
  log) timeout -k 10 300 python -u scripts/log_ab.py $L && timeout -k 10 300 python -u scripts/log_ab.py --delta $L ;;
  page) timeout -k 10 300 python -u scripts/ab_bench.py $L ;;
  pool) timeout -k 10 300 python -u scripts/pool_ab.py $L ;;
  reads) timeout -k 10 300 python -u scripts/reads_ab.py $L ;;
  wal) timeout -k 10 300 python -u scripts/wal_ab.py $L ;;
esac
