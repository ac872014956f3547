#!/bin/bash
# WRITE_SIZE of the driver's bench command for each library build (spill writes),
# one rocprofv3 --pmc pass per build (AKR_HIP_LIB selects the build; the environment passes through).
# Usage (GPU box): tools/write_ab.sh <tag> <lib.so> [<lib.so> ...]
tag=$1; shift
export TMPDIR=/tmp
for lib in "$@"; do
    name=$(basename "$lib" .so)
    out=gpurun_out/write_$tag/$name
    mkdir -p "$out"
    echo "pass $name"
    AKR_HIP_LIB=$PWD/$lib timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$out" -o run -- \
        python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --side-legs 0 --wavefront-spp 0 > "$out/bench.log" 2>&1 || exit $?
done
echo "write_ab $tag done"
