# per-wave timeline of the WAL replay kernel: the trace build of a COPY of the
# sources (scripts/patches/range_trace.py), built in-tree under build/variants by the
# caller beforehand (make variant from the patched copy), then scripts/wal_trace.py.
set -u
timeout -k 10 200 python3 scripts/wal_trace.py build/variants/libcurvecrc_rtrace.so --calls 3 > gpurun_out/wal_trace.json 2> gpurun_out/wal_trace.err || { tail -20 gpurun_out/wal_trace.err; exit 1; }
echo trace done
