#!/bin/bash
# Bench every library under akarirender-1_amd/variants/ (tuning builds), wide and BVH2 kernels.
for f in akarirender-1_amd/variants/*.so; do
  for wd in ${WIDE_MODES:-1 0}; do
    echo "== $f wide=$wd"
    AKR_HIP_LIB=$PWD/$f timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --wide $wd $EXTRA 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; u=d['roofline'].get('lane_util',{}); print(d['value'], k['trace_closest']['avg_ms'], k['trace_shadow']['avg_ms'], k['shade']['avg_ms'], {m:[round(x,3) for x in v.values()] for m,v in u.items()})" || exit 1
  done
done
