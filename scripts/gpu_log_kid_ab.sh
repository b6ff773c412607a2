# Write-log A/B under rocprofv3 (kernel time by Kernel_Id, scripts/kid_ab.py), full and delta mode,
# after the write-log GPU tests on the in-tree build.  usage: bash scripts/gpu_log_kid_ab.sh A.so B.so [TAG]
set -u
R=$(pwd)
A=$1; B=$2; TAG=${3:-ab}
mkdir -p $R/gpurun_out
O=$R/gpurun_out/log_kid_$TAG.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "log or partial or write or probe" > $R/gpurun_out/log_kid_tests_$TAG.log 2>&1
rc=$?; tail -2 $R/gpurun_out/log_kid_tests_$TAG.log; [ $rc = 0 ] || exit 1
: > $O
cd /tmp && export TMPDIR=/tmp
for mode in "" "--delta"; do
  rm -rf $R/gpurun_out/kid_l
  echo "## mode ${mode:-full}: $A then $B" >> $O
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kid_l -o run --output-format csv -- python3 $R/scripts/log_ab.py $mode $R/$A $R/$B 2>/dev/null | grep -v "^W2026\|^E2026" >> $O || exit 1
  python3 $R/scripts/kid_ab.py $R/gpurun_out/kid_l log_insert_kernel 96 >> $O
  python3 $R/scripts/kid_ab.py $R/gpurun_out/kid_l log_pages_kernel 96 >> $O
  rm -rf $R/gpurun_out/kid_l
done
cat $O
