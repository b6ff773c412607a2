# Write log timing ablation: no edge loads (6 of ~39 memory instructions a
# page, mostly out of range) -- does the memory-instruction count matter?
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
V=build/variants
timeout -k 10 300 python -u scripts/log_ab.py $V/libcurvecrc_ship.so $V/libcurvecrc_noedge.so > $R/gpurun_out/v_ab.log 2>&1 || { echo ABFAIL; tail -20 $R/gpurun_out/v_ab.log; exit 1; }
tail -2 $R/gpurun_out/v_ab.log
echo done
