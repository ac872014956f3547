#!/bin/bash
# GPU-box session: each GPU step has its own time limit; the script stops at the first step that
# fails (a test failure, a fault, an abort, a segfault or a time limit: a pytest thread timeout
# leaves its kernel running), and never retries.
# Usage: tools/gpu_session.sh "<step-name> <seconds> <command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for spec in "$@"; do
    name="${spec%% *}"; rest="${spec#* }"
    secs="${rest%% *}"; cmd="${rest#* }"
    echo "=== [$name] timeout ${secs}s: $cmd" | tee -a gpurun_out/session.log
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== [$name] rc=$rc after $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then
        echo "=== stopping: step $name ended with rc=$rc" | tee -a gpurun_out/session.log
        exit $rc
    fi
done
exit 0
