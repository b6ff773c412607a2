# delta-mode A/B (round 5): the shipped build (rows [row0,row1] chained, lane-parallel shift) vs the
# whole-page chain (kRowChain false), interleaved in one process, then the same under rocprofv3 kernel trace.
set -u
R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 200 python3 scripts/log_ab.py --delta curve_amd/libcurvecrc.so build/variants/libcurvecrc_norowchain.so > gpurun_out/delta_ab.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kid_delta
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/kid_delta -o run --output-format csv -- python3 $R/scripts/log_ab.py --delta $R/curve_amd/libcurvecrc.so $R/build/variants/libcurvecrc_norowchain.so >> $R/gpurun_out/delta_ab.txt 2>&1 || exit 1
python3 $R/scripts/kid_ab.py $R/gpurun_out/kid_delta "log_pages_kernel<16, true>" 96 >> $R/gpurun_out/delta_ab.txt
rm -rf $R/gpurun_out/kid_delta
cat $R/gpurun_out/delta_ab.txt
