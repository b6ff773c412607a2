# Write log: hash-table size >= 4 (shipped), 8 or 16 x pieces, now that the
# engine-owned table needs no per-call memset (fewer probe round trips in the insert).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_tf4.so $V/libcurvecrc_tf8.so $V/libcurvecrc_tf16.so > $R/gpurun_out/aa_ab.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/aa_ab.log; exit 1; }
tail -3 $R/gpurun_out/aa_ab.log
echo done
