#!/bin/bash
# Host ASan + UBSan run of the C ABI's CPU-side tests (tests/test_capi_host.py) against
# libnerfmi_san.so (make -C depth-aware-shader-effects-for-nerf_amd sanitize).  CPU only: no GPU
# code runs (the host tests never launch a kernel).  Prints the pytest summary; a sanitizer report
# makes pytest's process exit non-zero.
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/depth-aware-shader-effects-for-nerf_amd
make -C "$PKG" -j8 sanitize > /dev/null || exit 1
RT=$(/opt/rocm/lib/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)
[ -f "$RT" ] || RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
cd "$ROOT"
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  NERFMI_LIB=$PKG/libnerfmi_san.so NERFMI_SANITIZED=1 \
  python -m pytest tests/test_capi_host.py -q -p no:cacheprovider -m "not gpu"
