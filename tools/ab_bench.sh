#!/bin/bash
# A/B timing of library builds: full-frame bench (N=1) and the emulated rank of an 8-way split.
# Usage: tools/ab_bench.sh <lib.so> [<lib.so> ...]   (product lib: akarirender-1_amd/libakr_hip.so)
for f in "$@"; do
    echo "== $f"
    AKR_HIP_LIB=$PWD/$f timeout -k 10 120 python bench.py --steps 16 --warmup 2 --cpu-baseline 0 $EXTRA 2>/dev/null \
        | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; u=d['roofline'].get('lane_util',{}); print('full', d['value'], 'closest', k['trace_closest']['avg_ms'], 'shadow', k['trace_shadow']['avg_ms'], 'shade', k['shade']['avg_ms'], {m:[round(x,3) for x in v.values()] for m,v in u.items()})" || exit 1
    AKR_HIP_LIB=$PWD/$f timeout -k 10 120 python bench.py --emulate-world 8 --steps 8 --warmup 2 --cpu-baseline 0 $EXTRA 2>/dev/null \
        | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('emu8 ms/step', d['rank_ms_per_step'], 'proj', d['projected_node_Msamples_per_s'], 'closest', k['trace_closest']['avg_ms'], 'shadow', k['trace_shadow']['avg_ms'])" || exit 1
done
