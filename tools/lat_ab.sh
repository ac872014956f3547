#!/bin/bash
# latency_probe.py over several library builds (AKR_HIP_LIB), smaller soup for speed
for f in "$@"; do echo "== $f"; AKR_HIP_LIB=$PWD/$f timeout -k 10 200 python tools/latency_probe.py --reps 3 || exit 1; done
