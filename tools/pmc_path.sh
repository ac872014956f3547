#!/bin/bash
# rocprofv3 PMC passes of the headline bench for one render form (path kernel or wavefront), each
# pass its own run with --kernel-trace only beside the counters (MI355X_MICROARCH.md §rocprofv3):
#   sq1: wave-time split (SQ_WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY) + VALU issue
#   sq2: instruction mix (SALU / SMEM / VMEM / LDS) and LDS issue stalls
#   fetch / write / tcc: HBM traffic and L2 hit rate (tools/prof_summary.py conventions)
# Usage: tools/pmc_path.sh <tag> <path 0|1> [steps]
tag=${1:-pmc}; path=${2:-1}; steps=${3:-4}
export TMPDIR=/tmp
out=gpurun_out/pmc_${tag}_p${path}
mkdir -p "$out"
args="--steps $steps --warmup 1 --cpu-baseline 0 --path $path"
run() {  # name, counters...
    local name=$1; shift
    echo "pass $name: $*" | tee -a "$out/progress.txt"
    timeout -k 10 200 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$out/$name" -o run -- \
        python3 bench.py $args > "$out/$name.log" 2>&1
    local rc=$?
    echo "pass $name rc=$rc" | tee -a "$out/progress.txt"
    return $rc
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE &&
run sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run tcc TCC_HIT_sum TCC_MISS_sum
