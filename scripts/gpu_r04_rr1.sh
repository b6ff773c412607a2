# round 4: one static piece a wave (and its tail size / chunk size) on random and equal WAL entry sizes;
# verify-on-read tail size / chunk size
set -u
L="curve_amd/libcurvecrc.so build/variants/libcurvecrc_rr1.so build/variants/libcurvecrc_rr1d20.so build/variants/libcurvecrc_rr1d48.so build/variants/libcurvecrc_rr1b8.so"
timeout -k 10 500 python -u scripts/wal_ab.py $L > gpurun_out/wal_ab_rr1b.txt 2>&1 || { tail -5 gpurun_out/wal_ab_rr1b.txt; exit 1; }
timeout -k 10 500 python -u scripts/wal_ab.py --fixed 67584 $L >> gpurun_out/wal_ab_rr1b.txt 2>&1 || { tail -5 gpurun_out/wal_ab_rr1b.txt; exit 1; }
grep "^wal" gpurun_out/wal_ab_rr1b.txt
timeout -k 10 400 python -u scripts/reads_ab.py curve_amd/libcurvecrc.so build/variants/libcurvecrc_rvd32.so build/variants/libcurvecrc_rvs64.so build/variants/libcurvecrc_rvd8.so > gpurun_out/reads_ab_tail.txt 2>&1 || { tail -5 gpurun_out/reads_ab_tail.txt; exit 1; }
grep "libcurvecrc" gpurun_out/reads_ab_tail.txt
