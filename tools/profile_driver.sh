#!/bin/bash
# rocprofv3 passes of the driver's own bench command (bench.py --steps 20 --warmup 5: the 1040-spp
# frame), each pass its own run, with --kernel-trace only beside the counters
# (MI355X_MICROARCH.md §rocprofv3; at most 8 SQ / 4 TCC / 4 TCP counters per pass):
#   kt     kernel trace + stats of the exact driver command (must agree with the line's HIP events)
#   fetch  FETCH_SIZE            write  WRITE_SIZE          tcc  TCC_HIT / TCC_MISS / TCC_REQ
#   sq     wave-time split (WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY) + VALU issue
#   lat    VmemLatency (SQ_INST_LEVEL_VMEM accumulated / SQ_INSTS_VMEM), VMEM reads, TCP->TCC read latency
#   ea     L2 -> fabric read requests in flight (TCC_EA0_RDREQ_LEVEL) and their count: fabric latency
# tools/prof_summary.py <tag> turns gpurun_out/prof_<tag>/ into profiles/<tag>_{summary.md,traffic.json}.
# Usage (GPU box, repo root): tools/profile_driver.sh <tag> [bench args]
tag=${1:-drv}; shift
args=${*:-"--steps 20 --warmup 5"}
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p "$out"
echo "$args" > "$out/args.txt"
run() {  # name, rocprofv3 options...
    local name=$1; shift
    echo "pass $name: $*" | tee -a "$out/progress.txt"
    timeout -k 10 300 rocprofv3 "$@" --kernel-trace --output-format csv -d "$out/$name" -o run -- \
        python3 bench.py $args --cpu-baseline 0 > "$out/$name.log" 2>&1
    local rc=$?
    echo "pass $name rc=$rc" | tee -a "$out/progress.txt"
    return $rc
}
echo "pass kt" | tee -a "$out/progress.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
    python3 bench.py $args > "$out/kt.log" 2>&1 || exit $?
run fetch --pmc FETCH_SIZE &&
run write --pmc WRITE_SIZE &&
run tcc --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum &&
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE &&
run lat --pmc VmemLatency SQ_INSTS_VMEM_RD TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum &&
run ea --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum &&
echo "profile $tag done"
