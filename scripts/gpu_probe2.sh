set -u
R=$(pwd)
timeout -k 10 60 ./build/buffer_wrap_probe > gpurun_out/buffer_wrap_probe.json || exit 1
cat gpurun_out/buffer_wrap_probe.json
cd /tmp && export TMPDIR=/tmp
for v in insabl; do
  rm -rf $R/gpurun_out/prof_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$v -o run --output-format csv -- python3 $R/scripts/prof_log.py --lib $R/build/variants/libcurvecrc_$v.so > $R/gpurun_out/prof_$v.log 2>&1 || exit 1
  grep "ms per" $R/gpurun_out/prof_$v.log
done
echo done
