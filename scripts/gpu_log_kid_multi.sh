# Write-log A/B of several builds under rocprofv3 (kernel time by Kernel_Id, in load order),
# full mode then delta.  usage: bash scripts/gpu_log_kid_multi.sh TAG A.so B.so [C.so ...]
set -u
R=$(pwd)
TAG=$1; shift
L=""; for x in "$@"; do L="$L $R/$x"; done
mkdir -p $R/gpurun_out
O=$R/gpurun_out/log_kid_$TAG.txt
: > $O
cd /tmp && export TMPDIR=/tmp
for mode in "" "--delta"; do
  rm -rf $R/gpurun_out/kid_m
  echo "## mode ${mode:-full}: $*" >> $O
  timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/kid_m -o run --output-format csv -- python3 $R/scripts/log_ab.py $mode $L 2>/dev/null | grep -v "^W2026\|^E2026" >> $O || exit 1
  python3 $R/scripts/kid_ab.py $R/gpurun_out/kid_m log_pages_kernel 96 >> $O
  rm -rf $R/gpurun_out/kid_m
done
cat $O
