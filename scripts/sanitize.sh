#!/bin/bash
# ASan + UBSan build of the CPU side and the CPU suite under it (VERDICT r3 item 5;
# the reference ships asan/msan configs, .bazelrc:10-24).  Host code only: the
# device kernels are never sanitized (no GPU sanitizer on this pool) and nothing
# built here travels to a GPU box (build/san is in .gpurunignore).
#   1. build/san/libcurvecrc.so  every source of the library, host code sanitized
#      (clang for the .cpp files; hipcc -Xarch_host for the .hip files)
#   2. build/san/libcurvehost.so the C++ host layer (IntegrityService, chunkserver surfaces)
#   3. build/san/parser_fuzz     hostile sidecars and metapages (tests/native/parser_fuzz.cpp)
#   4. build/san/host_test       curve_amd/host/host_test.cpp (its CPU cases without a GPU)
#   5. python -m pytest tests -m "not gpu" on those libraries, the ASan runtime preloaded
# usage: scripts/sanitize.sh [--fuzz-only]
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
ROCM=${ROCM:-/opt/rocm}
CXX="$ROCM/llvm/bin/clang++"
CC="$ROCM/llvm/bin/clang"
HIPCC="$ROCM/bin/hipcc"
S=$R/build/san
mkdir -p $S/obj
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g"
CXXF="-O1 -std=c++17 -fPIC -msse4.2 -mpclmul -Wall $SAN"
RT=$($CXX -print-file-name=libclang_rt.asan-x86_64.so)
[ -f "$RT" ] || RT=$(ls $ROCM/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
cd $R/curve_amd/csrc
$CXX $CXXF -c crc32c_cpu.cpp -o $S/obj/crc32c_cpu.o
$CXX $CXXF -c integrity.cpp -o $S/obj/integrity.o
$CXX $CXXF -c ../host/chunkserver_host.cpp -o $S/obj/chunkserver_host.o
$CXX $CXXF -c ../host/integrity_service.cpp -o $S/obj/integrity_service.o
$CXX $CXXF -c ../host/integrity_capi.cpp -o $S/obj/integrity_capi.o
$CC -O1 -fPIC -msse4.2 -std=c11 $SAN -c ../../oracle/crc32c_oracle.c -o $S/obj/oracle.o
$CXX $CXXF -I$ROCM/include -D__HIP_PLATFORM_AMD__ -c ../../tests/native/parser_fuzz.cpp -o $S/obj/parser_fuzz.o
# 3: the parsers alone, statically sanitized (no library build needed)
$CXX $SAN -o $S/parser_fuzz $S/obj/parser_fuzz.o $S/obj/chunkserver_host.o $S/obj/integrity.o $S/obj/crc32c_cpu.o \
    -L$R/curve_amd -lcurvecrc -Wl,-rpath,$R/curve_amd -lpthread
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 $S/parser_fuzz
[ "${1:-}" = "--fuzz-only" ] && exit 0
# 1 + 2: the libraries
HF="-O1 -std=c++17 -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address,undefined -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer"
for f in engine kernels pool; do
  [ $S/obj/$f.o -nt $f.hip ] && [ $S/obj/$f.o -nt kernels.h ] || $HIPCC $HF -c $f.hip -o $S/obj/$f.o
done
$HIPCC -shared -fPIC --offload-arch=gfx950 -fsanitize=address,undefined -shared-libsan -o $S/libcurvecrc.so \
    $S/obj/crc32c_cpu.o $S/obj/integrity.o $S/obj/engine.o $S/obj/kernels.o $S/obj/pool.o \
    -L$ROCM/lib -lrccl
$CXX -shared $SAN -shared-libsan -o $S/libcurvehost.so $S/obj/chunkserver_host.o $S/obj/integrity_service.o \
    $S/obj/integrity_capi.o -L$S -lcurvecrc -Wl,-rpath,$S -lpthread
# 4: host_test's CPU cases
$CXX $CXXF -shared-libsan -I$ROCM/include -D__HIP_PLATFORM_AMD__ -o $S/host_test ../host/host_test.cpp \
    $S/obj/chunkserver_host.o $S/obj/integrity_service.o $S/obj/oracle.o -L$S -lcurvecrc -L$ROCM/lib -lamdhip64 \
    -Wl,-rpath,$S -Wl,-rpath,$(dirname $RT) -lpthread
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 $S/host_test
# 5: the CPU suite on the sanitized libraries (first: prove those are the ones loaded)
cd $R
export CURVE_AMD_LIB=$S/libcurvecrc.so CURVE_AMD_HOST_LIB=$S/libcurvehost.so LD_PRELOAD=$RT
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:verify_asan_link_order=0 UBSAN_OPTIONS=print_stacktrace=1
python - <<'PY'
from curve_amd import _lib
_lib.lib(), _lib.host_lib()
maps = open("/proc/self/maps").read()
for want in ("build/san/libcurvecrc.so", "build/san/libcurvehost.so", "libclang_rt.asan"):
    assert want in maps, want
print("sanitized libraries loaded:", _lib.LIB_PATH, _lib.HOST_LIB_PATH)
PY
python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider
echo "sanitize: all steps passed"
