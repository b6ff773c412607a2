# Page-kernel durations of the write-log queue per build under rocprofv3 --kernel-trace
# (scripts/log_queue_ab.py --only queue, then one run --only singles on the in-tree build as the
# no-grouping baseline).  usage: bash scripts/gpu_log_queue_kernels.sh TAG LIB.so [LIB.so ...]
set -u
R=$(pwd)
TAG=$1; shift
O=$R/gpurun_out/log_queue_kernels_$TAG.txt
: > $O
cd /tmp && export TMPDIR=/tmp
run() {  # label, lib, mode
  rm -rf $R/gpurun_out/lqk
  echo "## $1 ($3)" >> $O
  CURVE_AMD_LIB=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/lqk -o run --output-format csv -- python3 $R/scripts/log_queue_ab.py --only $3 --rounds 8 2>/dev/null | grep -v "^W20\|^E20\|amdgpu.ids" >> $O || return 1
  python3 $R/scripts/log_queue_kernels.py $R/gpurun_out/lqk >> $O
  rm -rf $R/gpurun_out/lqk
}
run in-tree $R/curve_amd/libcurvecrc.so singles || exit 1
for L in "$@"; do run $(basename $L) $R/$L queue || exit 1; done
run in-tree $R/curve_amd/libcurvecrc.so queue || exit 1
cat $O
