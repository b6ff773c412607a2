# round 4: WAL tail-size / piece-count variants and the write log's global-load row select,
# each against the in-tree build (interleaved in-process A/B)
set -u
timeout -k 10 400 python -u scripts/wal_ab.py curve_amd/libcurvecrc.so build/variants/libcurvecrc_rr4b.so build/variants/libcurvecrc_d16.so build/variants/libcurvecrc_d16h8.so build/variants/libcurvecrc_d20.so > gpurun_out/wal_ab_tail.txt 2>&1 || { tail -5 gpurun_out/wal_ab_tail.txt; exit 1; }
cat gpurun_out/wal_ab_tail.txt | grep "^wal"
bash scripts/gpu_ab.sh log gsel || exit 1
