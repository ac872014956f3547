#!/bin/bash
# rocprofv3 passes for the headline bench (run on the GPU box, from the repo root):
#   1. kernel trace + stats (per-kernel durations; must agree with bench.py's HIP-event numbers)
#   2. PMC pass: FETCH_SIZE (TCC memory-side reads) in its own run, kernel trace only beside it
#   3. PMC pass: WRITE_SIZE (TCC memory-side writes; FETCH_SIZE and WRITE_SIZE do not fit one pass)
#   4. PMC pass: TCC hit/miss
# Output under gpurun_out/prof_<tag>/ (csv).  Usage: tools/profile.sh <tag> [bench args...]
tag=${1:-r01}; shift
args=${*:-"--steps 4 --warmup 1 --cpu-baseline 0"}
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p "$out"
set -o pipefail
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
    python3 bench.py $args > "$out/kt.log" 2>&1 || exit $?
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$out/pmc_fetch" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > "$out/pmc_fetch.log" 2>&1 || exit $?
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$out/pmc_write" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > "$out/pmc_write.log" 2>&1 || exit $?
timeout -k 10 900 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d "$out/pmc_tcc" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > "$out/pmc_tcc.log" 2>&1 || exit $?
echo "profile $tag done"
