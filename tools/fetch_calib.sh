#!/bin/bash
# Counter passes of tools/fetch_calib, each its own rocprofv3 run:
#   kt   kernel trace + stats           fetch  FETCH_SIZE (TCC_BUBBLE / RDREQ / RDREQ_32B)
#   rq   request counts by size         rq2    128-B requests, DRAM-bound requests, L2 hits / misses
# Usage (GPU box, repo root): tools/fetch_calib.sh <tag>; then python3 tools/fetch_calib.py <tag> here.
tag=${1:-calib}
export TMPDIR=/tmp
out=gpurun_out/calib_$tag
bin=tools/bin/fetch_calib
mkdir -p "$out"
timeout -k 10 120 $bin 1 > "$out/plain.log" 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- $bin 1 > "$out/kt.log" 2>&1 || exit $?
pass() {  # name, counters...
    local name=$1; shift
    echo "pass $name: $*"
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$out/$name" -o run -- $bin 1 \
        > "$out/$name.log" 2>&1
}
pass fetch FETCH_SIZE &&
pass rq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum &&
pass rq2 TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum TCC_MISS_sum TCC_HIT_sum &&
echo "calib $tag done"
