# round 4: verify on read in one launch (in-kernel tile counts) vs the count + scan + verify
# path of build/variants/libcurvecrc_r4pre.so; then the range path's tests and A/B again
set -u
bash scripts/gpu_ab.sh reads r4pre || exit 1
bash scripts/gpu_ab.sh wal r4pre || exit 1
timeout -k 10 400 python -u scripts/wal_ab.py curve_amd/libcurvecrc.so build/variants/libcurvecrc_rr1.so build/variants/libcurvecrc_rr1d20.so > gpurun_out/wal_ab_rr1.txt 2>&1 || { tail -5 gpurun_out/wal_ab_rr1.txt; exit 1; }
grep "^wal" gpurun_out/wal_ab_rr1.txt
