# round 4: write log with G pages per wave (scripts/patches/log_group.py variants): the
# write-log parity tests ON the variant library, then the in-process A/B against the in-tree build
set -u
for v in grp2w12; do
  CURVE_AMD_LIB=$(pwd)/build/variants/libcurvecrc_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "write_log or partial" > gpurun_out/grp_tests_$v.log 2>&1
  rc=$?; tail -3 gpurun_out/grp_tests_$v.log; [ $rc = 0 ] || exit 1
done
timeout -k 10 300 python -u scripts/log_ab.py curve_amd/libcurvecrc.so build/variants/libcurvecrc_grp2w12.so build/variants/libcurvecrc_grp4w8.so build/variants/libcurvecrc_grp2w16.so || exit 1
