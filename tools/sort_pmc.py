"""Sums the rocprofv3 --pmc counters of the wavefront's trace kernels (closest hit: k_trace<0, ...>,
shadow: k_trace<2, ...>) in each output directory given, one directory per configuration of
tools/sort_probe.py --no-count, and prints the L2 hit rate, the L2 -> fabric read requests and their
bytes (128 B each on gfx950, profiles/r21_fetch_calib.json) per sample pass.

Usage: python tools/sort_pmc.py --spp 8 gpurun_out/pmc_sort_off gpurun_out/pmc_sort_on ..."""
import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path


def sums(d: Path):
    out = {"closest": defaultdict(float), "shadow": defaultdict(float), "sort": defaultdict(float)}
    disp = {"closest": set(), "shadow": set(), "sort": set()}
    for f in d.rglob("*counter_collection.csv"):
        with f.open() as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                kind = ("closest" if "k_trace<0," in k else "shadow" if "k_trace<2," in k
                        else "sort" if "k_sort_" in k else None)
                if kind:
                    out[kind][row["Counter_Name"]] += float(row["Counter_Value"])
                    disp[kind].add(row["Dispatch_Id"])
    return out, {k: len(v) for k, v in disp.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, required=True, help="sample passes the profiled render ran (plus the 2-spp warmup)")
    ap.add_argument("dirs", nargs="+")
    args = ap.parse_args()
    for d in args.dirs:
        s, nd = sums(Path(d))
        rec = {"dir": d, "dispatches": nd}
        for kind in ("closest", "shadow", "sort"):
            c = s[kind]
            hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
            rq = c.get("TCC_EA0_RDREQ_sum", 0.0)
            rec[kind] = {"l2_hit": round(hit / max(1.0, hit + miss), 4),
                         "rdreq_per_pass": rq / args.spp, "read_GB_per_pass": round(128 * rq / args.spp / 1e9, 3),
                         "l2_req_per_pass": (hit + miss) / args.spp}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
