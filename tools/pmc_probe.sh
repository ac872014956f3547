#!/bin/bash
# Extra PMC passes for the traversal kernel (memory pipeline / TLB / issue), each its own run with
# --kernel-trace only beside it, few counters per pass (the hardware rejects large sets).
# Usage: tools/pmc_probe.sh <tag>; output gpurun_out/pmc_<tag>/
tag=${1:-probe}
export TMPDIR=/tmp
out=gpurun_out/pmc_$tag
mkdir -p "$out"
args="--steps 1 --warmup 0 --cpu-baseline 0"
i=0
for set in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM" \
  "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_LDS" \
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
  "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum" \
  "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum" \
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum" \
  "TD_TD_BUSY_sum TD_TC_STALL_sum" ; do
  i=$((i+1))
  echo "pass $i: $set" | tee -a "$out/progress.txt"
  timeout -k 10 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$out/p$i" -o run -- \
      python3 bench.py $args > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc" | tee -a "$out/progress.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
