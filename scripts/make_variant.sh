#!/bin/bash
# A/B and diagnostic builds WITHOUT touching the shipped sources: copies the
# tracked sources of curve_amd/csrc + include to /tmp/var_NAME, edits the COPY of
# kernels.hip, and builds build/variants/libcurvecrc_NAME.so from it.
# usage: scripts/make_variant.sh NAME sed 'SED-EXPR'     (e.g. a constant)
#        scripts/make_variant.sh NAME py  scripts/patches/X.py [ARGS...]   (X.py KERNELS_HIP ARGS...)
set -e
N=$1; KIND=$2; ARG=$3
shift 3
R=$(cd "$(dirname "$0")/.." && pwd)
D=/tmp/var_$N
rm -rf "$D" && mkdir -p "$D"
(cd "$R" && git ls-files curve_amd/csrc include | tar -cf - -T -) | tar -xf - -C "$D"
cp "$R/curve_amd/csrc/kernels.hip" "$D/curve_amd/csrc/kernels.hip"  # the working tree's kernels
case $KIND in
  sed) sed -i "$ARG" "$D/curve_amd/csrc/kernels.hip" ;;
  py) python3 "$R/$ARG" "$D/curve_amd/csrc/kernels.hip" "$@" ;;
  *) echo "kind: sed | py"; exit 2 ;;
esac
if cmp -s "$R/curve_amd/csrc/kernels.hip" "$D/curve_amd/csrc/kernels.hip"; then echo "edit changed nothing"; exit 1; fi
make -C "$D/curve_amd/csrc" variant NAME="$N" -j8 > "$D/build.log" 2>&1 || { tail -20 "$D/build.log"; exit 1; }
mkdir -p "$R/build/variants"
cp "$D/build/variants/libcurvecrc_$N.so" "$R/build/variants/"
echo "built build/variants/libcurvecrc_$N.so"
