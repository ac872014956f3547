#!/bin/bash
# One rocprofv3 PMC pass of the headline bench (counters in their own run, --kernel-trace beside them
# only; MI355X_MICROARCH.md §rocprofv3).  Usage: tools/pmc_one.sh <name> "<counters>" [bench args...]
name=$1; counters=$2; shift 2
args=${*:-"--steps 4 --warmup 1 --cpu-baseline 0 --wavefront-spp 0"}
export TMPDIR=/tmp
out=gpurun_out/pmc1_$name
mkdir -p "$out"
timeout -k 10 240 rocprofv3 --pmc $counters --kernel-trace --output-format csv -d "$out" -o run -- \
    python3 bench.py $args > "$out/bench.log" 2>&1
rc=$?
echo "pmc $name rc=$rc"
exit $rc
