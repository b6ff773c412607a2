#!/bin/bash
# Byte-compare the device code of curve_amd/csrc/kernels.hip (+ kernels.h) at a
# git revision with the working tree's.  Both are built with ONE fixed
# compilation-unit id (-cuid): the default id hashes the source text, so any
# edit -- comments included -- changes the __hip_cuid_* symbol and nothing else.
# usage: scripts/hsaco_identity.sh REV      (exit 0 = identical .hip_fatbin)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:?revision}
T=$(mktemp -d)
trap 'rm -rf $T' EXIT
mkdir -p $T/rev
git -C $R show $REV:curve_amd/csrc/kernels.hip > $T/rev/kernels.hip
git -C $R show $REV:curve_amd/csrc/kernels.h > $T/rev/kernels.h
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -w -cuid=curve_kernels"
/opt/rocm/bin/hipcc $F -c $T/rev/kernels.hip -o $T/rev.o
/opt/rocm/bin/hipcc $F -c $R/curve_amd/csrc/kernels.hip -o $T/tree.o
for x in rev tree; do /opt/rocm/llvm/bin/llvm-objcopy --dump-section .hip_fatbin=$T/$x.bin $T/$x.o; done
md5sum $T/rev.bin $T/tree.bin | sed "s|$T/||"
cmp $T/rev.bin $T/tree.bin && echo "device code identical"
