#!/bin/bash
# AddressSanitizer build of libslx_hip.so's host side: every csrc/*.hip compiled with
# -Xarch_host -fsanitize=address (device code is never sanitized; it is built at -O0 since the argument checks under
# test run before any HIP call), linked with the ASan test driver tests/asan/capi_errors.c.
# Output under simlingo_amd/csrc/build/asan/ (git-ignored).
# usage: tools/asan_build.sh [run]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/simlingo_amd/csrc/build/asan"
CLANG=/opt/rocm/llvm/bin/clang++
mkdir -p "$OUT"
FL=(-x hip --offload-arch=gfx950 -O1 -g -fno-omit-frame-pointer -Xarch_host -fsanitize=address -Xarch_device -O0
    -fPIC -std=c++17
    -I"$ROOT/include" -I"$ROOT/simlingo_amd/csrc" -munsafe-fp-atomics)
objs=()
pids=()
for src in "$ROOT"/simlingo_amd/csrc/*.hip; do
  o="$OUT/$(basename "${src%.hip}").o"
  objs+=("$o")
  if [ ! -f "$o" ] || [ "$src" -nt "$o" ]; then
    # attention.hip issues its LDS DMA by inline asm with SGPR ("s") operands, which device -O0 cannot allocate
    extra=()
    [ "$(basename "$src")" = "attention.hip" ] && extra=(-Xarch_device -O1)
    "$CLANG" "${FL[@]}" "${extra[@]}" -c "$src" -o "$o" &
    pids+=($!)
  fi
done
for p in "${pids[@]:-}"; do [ -n "$p" ] && wait "$p"; done
"$CLANG" -fsanitize=address -fno-gpu-sanitize --hip-link --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib \
  -o "$OUT/libslx_hip_asan.so"
/opt/rocm/llvm/bin/clang -fsanitize=address -fno-gpu-sanitize -fno-omit-frame-pointer -g -I"$ROOT/include" \
  "$ROOT/tests/asan/capi_errors.c" -L"$OUT" -lslx_hip_asan -Wl,-rpath,"$OUT" -Wl,-rpath,/opt/rocm/lib \
  -o "$OUT/capi_errors"
echo "built $OUT/capi_errors"
if [ "${1:-}" = run ]; then
  ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 "$OUT/capi_errors"
fi
