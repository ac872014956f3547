#!/bin/bash
# rocprofv3 passes of the driver's own bench command (bench.py --steps 20 --warmup 5: the 1040-spp
# frame), each pass its own run, with --kernel-trace only beside the counters
# (MI355X_MICROARCH.md §rocprofv3; at most 8 SQ / 4 TCC / 4 TCP counters per pass):
#   kt     kernel trace + stats of the exact driver command (must agree with the line's HIP events)
#   fetch  FETCH_SIZE            write  WRITE_SIZE          tcc  TCC_HIT / TCC_MISS / TCC_REQ
#   sq     wave-time split (WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY) + VALU issue
#   lat    VmemLatency (SQ_INST_LEVEL_VMEM accumulated / SQ_INSTS_VMEM), VMEM reads, TCP->TCC read latency
#   ea     L2 -> fabric read requests in flight (TCC_EA0_RDREQ_LEVEL) and their count: fabric latency
#   rq     L2 -> fabric read requests by size (32 / 64 / 128 B): with tools/fetch_calib's calibration
#          (profiles/*_fetch_calib.json) these give the read bytes without FETCH_SIZE's blanket factor
#   rq2    128-B requests as FETCH_SIZE counts them (TCC_BUBBLE), DRAM-bound requests, L2 hits / misses
#   ta     texture-address / texture-data unit busy cycles and their stalls on the L1 (TA_BUSY_avr per
#          TA instance against GRBM_GUI_ACTIVE): is the vector memory pipe's address rate the limit?
#   lds    LDS and scalar-memory instructions and their in-flight levels (latency = level / count), the
#          waves' total and waiting cycles: what the non-VMEM waits are
#   mix    instruction mix per wave (VALU / SALU / branch / LDS / VMEM / SMEM)
#   tcp    L1 (TCP) stall cycles (pending misses, data path to TA, tag conflicts) and its accesses
# The counter passes skip the untimed side legs (the CPU baseline, the C2 / C4 legs and the wavefront leg):
# their timed launch is the same, and the passes stay short.
# tools/prof_summary.py <tag> turns gpurun_out/prof_<tag>/ into profiles/<tag>_{summary.md,traffic.json}.
# Usage (GPU box, repo root): [PASSES="rq rq2"] tools/profile_driver.sh <tag> [bench args]
tag=${1:-drv}; shift
args=${*:-"--steps 20 --warmup 5"}
passes=${PASSES:-"kt fetch write tcc sq lat ea rq rq2"}
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p "$out"
echo "$args" > "$out/args.txt"
declare -A PMC=(
    [fetch]="FETCH_SIZE"
    [write]="WRITE_SIZE"
    [tcc]="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"
    [sq]="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
    [lat]="VmemLatency SQ_INSTS_VMEM_RD TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
    [ea]="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum"
    [rq]="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
    [rq2]="TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum TCC_MISS_sum TCC_HIT_sum"
    [lds]="SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD"
    [mix]="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES"
    [ta]="TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
    [tcp]="TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_ACCESSES_sum GRBM_GUI_ACTIVE"
)
for name in $passes; do
    echo "pass $name" | tee -a "$out/progress.txt"
    if [ "$name" = kt ]; then
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
            python3 bench.py $args > "$out/kt.log" 2>&1
    else
        timeout -s KILL 240 rocprofv3 --pmc ${PMC[$name]} --kernel-trace --output-format csv -d "$out/$name" -o run -- \
            python3 bench.py $args --cpu-baseline 0 --side-legs 0 --wavefront-spp 0 > "$out/$name.log" 2>&1
    fi
    rc=$?
    echo "pass $name rc=$rc" | tee -a "$out/progress.txt"
    [ $rc -eq 0 ] || exit $rc
done
echo "profile $tag done"
