# Write log: what a lean single-piece kernel could gain -- ablation 6 (multi-piece
# pages not merged: wrong results for those, timing only) at 2 and 3 pages in
# flight per wave, against the shipped build.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u scripts/log_ab.py build/variants/libcurvecrc_cur.so build/variants/libcurvecrc_abl6d2.so build/variants/libcurvecrc_abl6d3.so > $R/gpurun_out/logdepth_ab.log 2>&1 || { echo LOGABFAIL; tail -20 $R/gpurun_out/logdepth_ab.log; exit 1; }
tail -4 $R/gpurun_out/logdepth_ab.log
echo done
