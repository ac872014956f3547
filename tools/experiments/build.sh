#!/usr/bin/env bash
# Builds a timing experiment: tools/experiments/<name>.patch applied to a copy of the product sources
# (akarirender-1_amd/csrc), compiled to tools/experiments/lib/libakr_hip_<name>.so.  The product
# library is never touched; capi.load_library() accepts AKR_HIP_LIB only for a library in lib/.
# Usage (CPU container, before a gpurun):  tools/experiments/build.sh <name> [<name> ...]
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$(cd "$HERE/../.." && pwd)"
mkdir -p "$HERE/lib"
for name in "$@"; do
    patch_file="$HERE/$name.patch"
    [ -f "$patch_file" ] || { echo "no $patch_file" >&2; exit 1; }
    work="$HERE/build/$name"
    rm -rf "$work"
    mkdir -p "$work/akarirender-1_amd"
    cp -r "$ROOT/akarirender-1_amd/csrc" "$work/akarirender-1_amd/csrc"
    rm -f "$work/akarirender-1_amd/csrc/"*.o
    ln -s "$ROOT/include" "$work/include"
    (cd "$work" && patch -s -p1 < "$patch_file")
    make -s -j8 -C "$work/akarirender-1_amd/csrc" OUT="$HERE/lib/libakr_hip_$name.so" "$HERE/lib/libakr_hip_$name.so"
    rm -rf "$work"
    echo "built tools/experiments/lib/libakr_hip_$name.so"
done
