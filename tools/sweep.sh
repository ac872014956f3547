#!/bin/bash
# Sweep bench flags: tools/sweep.sh "<flags A>" "<flags B>" ...   (full frame + emulated 8-way rank)
for x in "$@"; do echo "== $x"; EXTRA="$x" tools/ab_bench.sh akarirender-1_amd/libakr_hip.so | tail -2 || exit 1; done
