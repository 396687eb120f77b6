#!/bin/bash
# the host code of libfmx under AddressSanitizer + UBSan, on the CPU.
# libfmx's host C++ (smoother.cpp, moments.cpp, and the host side of every .hip/.cpp
# translation unit: -Xarch_host) is rebuilt with clang's ASan/UBSan into
# form_amd/ab/libfmx_asan.so; tests/test_moments.py (the host-only fmx_moments_contract,
# the GTSAM seam's "evaluate anywhere" form) runs against it with the ASan runtime
# preloaded, and tests/cpp/test_stage (the staging helpers) is built and run with gcc's
# ASan/UBSan.  The GPU kernels are not instrumented (no GPU sanitizer on this pool).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=${B:-/tmp/fmx_asan_build}
OUT=$ROOT/form_amd/ab/libfmx_asan.so
mkdir -p "$B" "$ROOT/form_amd/ab"
CLANG=/opt/rocm/lib/llvm/bin/clang++
HIPCC=/opt/rocm/bin/hipcc
SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined"
CXXF="-O1 -g -std=c++17 -fPIC -ffp-contract=off -I$ROOT/include"
C=$ROOT/form_amd/csrc
$CLANG $CXXF $SAN -c $C/smoother.cpp -o $B/smoother.o
$CLANG $CXXF $SAN -ffp-contract=fast -c $C/moments.cpp -o $B/moments.o
HS="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
pids=()
for f in extract voxelmap linearize window snapshot; do
  $HIPCC $CXXF $HS --offload-arch=gfx950 -c $C/$f.hip -o $B/$f.o & pids+=($!)
done
$HIPCC $CXXF $HS --offload-arch=gfx950 -DFMX_MATCH_GROUP=1 -DFMX_VM_NS=gl -c $C/voxelmap.hip -o $B/voxelmap_gl.o & pids+=($!)
for f in comm fmx_api; do
  $HIPCC $CXXF $HS -x hip --offload-arch=gfx950 -c $C/$f.cpp -o $B/$f.o & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
$HIPCC -shared -fPIC -rdynamic --offload-arch=gfx950 -fsanitize=address,undefined -shared-libasan -o $OUT $B/*.o -ldl
RT=$($CLANG -print-file-name=libclang_rt.asan-x86_64.so)
cd "$ROOT"
echo "== tests/test_moments.py against $OUT (ASan + UBSan, $RT preloaded)"
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  FMX_LIB=$OUT python -m pytest tests/test_moments.py -q -p no:cacheprovider 2>&1 | tail -5
echo "== tests/cpp/test_stage (gcc ASan + UBSan)"
g++ -O1 -g -std=c++17 -Wall -Wextra -Werror -I$ROOT/include -I$C -pthread -fsanitize=address,undefined \
  -fno-sanitize-recover=undefined -o /tmp/test_stage_asan tests/cpp/test_stage.cpp
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 /tmp/test_stage_asan
echo "== tests/cpp/test_smoother (gcc ASan + UBSan: the window LM, Schur marginal, Cholesky)"
g++ -O1 -g -std=c++17 -Wall -Wextra -Werror -I$C -ffp-contract=off -fsanitize=address,undefined \
  -fno-sanitize-recover=undefined -o /tmp/test_smoother_asan tests/cpp/test_smoother.cpp $C/smoother.cpp
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 /tmp/test_smoother_asan
echo "ASAN-DONE"
