#!/bin/bash
# One HIP translation unit -> host object with an embedded gfx950 code object
# whose assembly went through isa_e64.py (VOP3 lane selects).  The steps are
# hipcc's own (device codegen, lld, clang-offload-bundler, host compile with
# the bundle), with the device stage stopped at assembly and rewritten.
# If any step of that pipeline fails (a toolchain whose assembly the pass
# does not understand, a missing tool), the unit is compiled by plain hipcc
# instead -- the same code without the rewrite -- and a line says so.
# usage: hip_e64.sh <src.hip> <out.o> <hipcc flags...>
set -uo pipefail
src=$1; out=$2; shift 2
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
LLVM=${LLVM:-/opt/rocm/lib/llvm/bin}
ARCH=${ARCH:-gfx950}
base=${out%.o}

e64() {   # every step must succeed (errexit does not apply inside `if`)
  [ -z "${E64_FORCE_FAIL:-}" ] &&   # test hook: exercise the fallback
  "$HIPCC" "$@" --cuda-device-only -S "$src" -o "$base.dev.s" 2> >(grep -v "argument unused during compilation: .--hip-link" >&2) &&
  "$LLVM/clang" -target amdgcn-amd-amdhsa -mcpu=$ARCH -c "$base.dev.s" -o "$base.dev.orig.o" &&
  "$LLVM/llvm-readelf" -s "$base.dev.orig.o" > "$base.dev.sizes" &&
  python3 "$(dirname "$0")/isa_e64.py" "$base.dev.s" "$base.dev.e64.s" "$base.dev.sizes" &&
  "$LLVM/clang" -target amdgcn-amd-amdhsa -mcpu=$ARCH -c "$base.dev.e64.s" -o "$base.dev.o" &&
  "$LLVM/ld.lld" -m elf64_amdgpu --no-undefined -shared -o "$base.hsaco" "$base.dev.o" &&
  "$LLVM/clang-offload-bundler" -type=o -bundle-align=4096 \
    -targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--$ARCH \
    -input=/dev/null -input="$base.hsaco" -output="$base.hipfb" &&
  "$HIPCC" "$@" --cuda-host-only -Xclang -fcuda-include-gpubinary -Xclang "$base.hipfb" -c "$src" -o "$out"
}

if e64 "$@"; then
  echo e64 > "$base.mode"
else
  echo "hip_e64.sh: the rewrite pipeline failed for $src; compiling it with plain hipcc" >&2
  "$HIPCC" "$@" -c "$src" -o "$out" || exit 1
  echo plain > "$base.mode"
fi
