# Tail schedules of the verify-on-read and WAL range kernels: their parity
# tests on the in-tree build, then interleaved A/B of the previous build (base),
# the in-tree build and larger tails through 8 per-XCD heads (w8d16: WAL 1/16;
# w8d8: WAL and verify 1/8).
set -u
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "verify or range or wal or read or tail or stream or files" 2>&1 | tail -1 || exit 1
timeout -k 10 200 python -u scripts/reads_ab.py build/variants/libcurvecrc_base.so curve_amd/libcurvecrc.so build/variants/libcurvecrc_w8d8.so || exit 1
AB_ROUNDS=14 timeout -k 10 250 python -u scripts/wal_sched_ab.py build/variants/libcurvecrc_base.so@flat curve_amd/libcurvecrc.so@flat build/variants/libcurvecrc_w8d16.so@flat build/variants/libcurvecrc_w8d8.so@flat || exit 1
echo done
