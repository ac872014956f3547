#!/bin/bash
# Issue-side PMC passes for the traversal kernel: VALU / VMEM / LDS instruction counts and busy
# cycles, plus UTCL1 translation misses.  Each pass its own rocprofv3 run (--kernel-trace beside
# the counters only), few counters per pass.  Usage: tools/pmc_issue.sh <tag>
tag=${1:-issue}
export TMPDIR=/tmp
out=gpurun_out/pmc_$tag
mkdir -p "$out"
args="--steps 1 --warmup 0 --cpu-baseline 0"
i=0
for set in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" \
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
  "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
  "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum" ; do
  i=$((i+1))
  echo "pass $i: $set" | tee -a "$out/progress.txt"
  timeout -k 10 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$out/p$i" -o run -- \
      python3 bench.py $args > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc" | tee -a "$out/progress.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
