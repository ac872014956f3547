"""Timeline of the GPU work around the longest kernel of a rocprofv3 trace: every kernel dispatch
and memory copy from `--before` ms ahead of it to `--after` ms past its end, with start offsets,
durations and the idle gaps between consecutive operations.  Finds the host-side and launch
overheads a render pays outside its main kernel.

Usage: python tools/timeline.py <rocprofv3 output dir> [--kernel SUBSTRING] [--before 5] [--after 5]"""
import argparse
import csv
import glob
import os


def rows(path, kind):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("Direction") or r.get("Operation") or kind
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, name))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_path", help="anchor: the longest dispatch whose name contains this")
    ap.add_argument("--before", type=float, default=5.0)
    ap.add_argument("--after", type=float, default=5.0)
    args = ap.parse_args()
    ops = []
    for p in glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True):
        ops += rows(p, "kernel")
    for p in glob.glob(os.path.join(args.dir, "**", "*memory_copy_trace.csv"), recursive=True):
        ops += rows(p, "copy")
    ops.sort()
    anchors = [o for o in ops if o[2] == "kernel" and args.kernel in o[3]]
    if not anchors:
        raise SystemExit(f"no dispatch matching {args.kernel!r}")
    a = max(anchors, key=lambda o: o[1] - o[0])
    lo, hi = a[0] - int(args.before * 1e6), a[1] + int(args.after * 1e6)
    prev_end = None
    print(f"anchor: {a[3][:80]} {(a[1] - a[0]) / 1e6:.3f} ms")
    for s, e, kind, name in ops:
        if e < lo or s > hi:
            continue
        gap = "" if prev_end is None else f"gap {(s - prev_end) / 1e3:9.1f} us"
        print(f"{(s - a[0]) / 1e3:12.1f} us  {(e - s) / 1e3:10.1f} us  {gap:18s} {kind:6s} {name[:90]}")
        prev_end = e if prev_end is None else max(prev_end, e)


if __name__ == "__main__":
    main()
