#!/bin/bash
# AddressSanitizer build of libvit_hip.so's HOST code (device code unchanged: GPU ASan is not available on the pool)
# and the host ABI checker (tests/host_abi_check.c) run against it — no GPU needed.  Output: tools/asan/ (git-ignored)
# and the run log on stdout.   usage: bash tools/asan_host_check.sh
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/vision-transformer_amd/csrc
OUT=$ROOT/tools/asan
mkdir -p "$OUT"
SAN="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
OBJS=""
for m in vit_gemm vit_attention vit_norm vit_misc vit_image; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -munsafe-fp-atomics $SAN -c $C/$m.hip -o $OUT/$m.o &
  OBJS="$OBJS $OUT/$m.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $SAN -o $OUT/libvit_hip_asan.so $OBJS
/opt/rocm/lib/llvm/bin/clang -std=c11 -O1 -g -fsanitize=address -fno-omit-frame-pointer -I$ROOT/include $ROOT/tests/host_abi_check.c \
  -o $OUT/host_abi_check $OUT/libvit_hip_asan.so -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$OUT -Wl,-rpath,/opt/rocm/lib
# (clang: the same AddressSanitizer runtime as the hipcc-built library)
# leak checking off: the HIP runtime keeps its allocations until process exit
ASAN_OPTIONS=detect_leaks=0:abort_on_error=0 $OUT/host_abi_check
echo "asan_host_check: OK"
