# Write log: per-wave phase clocks of the page kernel (CC_LOG_TRACE=1 build).
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u scripts/trace_log.py build/variants/libcurvecrc_ltr.so > $R/gpurun_out/m_trace.log 2>&1 || { echo TRFAIL; tail -20 $R/gpurun_out/m_trace.log; exit 1; }
tail -3 $R/gpurun_out/m_trace.log
echo done
