"""Summarise a tools/profile_driver.sh (or tools/profile.sh) run (rocprofv3 csv) into
profiles/<tag>_summary.md, profiles/<tag>_traffic.json and copies of the kernel stats / counter csvs.

HBM bytes: the L2 -> fabric read requests by size (pass `rq`: 32 x RDREQ_32B + 64 x RDREQ_64B +
128 x RDREQ_128B) when the profile has them, else 2 * FETCH_SIZE * 1024.  tools/fetch_calib (profiles/
r21_fetch_calib.json) calibrated both on the traversal's own widths: on gfx950 every fabric read request
is 128 B whatever the access width (64-B nodes, 32-B leaf headers, 48-B triangles, the 128-B leaf
batch), FETCH_SIZE tallies each at 64 B (its 128-B term, TCC_BUBBLE, reads 0), and one isolated record
costs exactly one request per line it covers; so 2 x FETCH_SIZE = 128 x RDREQ for every width.  Reads
to the Infinity Cache are counted too (RDREQ_DRAM = RDREQ): the figure bounds HBM traffic from above.
WRITE_SIZE (KiB) is added unscaled; TCC_MISS * 128 B is printed beside it.

The persistent path kernel renders every spp of its call in one launch, and bench.py launches it
for the warmup, the timed render and an untimed breakdown.  Its record in traffic.json is the
*timed* launch alone: the longest dispatch of that kernel in each pass (the timed render has the
most spp), with `spp` from the bench line (steps x spp_per_step) and every counter of that one
dispatch, so bench.py's roofline reads the launch the driver times.  The
workload key is the bench line's whole `config`, which bench.py matches field for field."""
import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PASSES = ("fetch", "write", "tcc", "sq", "lat", "ea", "rq", "rq2", "pmc_fetch", "pmc_write", "pmc_tcc")


def short(name):
    name = name.replace("void ", "").replace("akr::", "")
    return name.split("(")[0]


def bench_line(log: Path):
    if not log.exists():
        return None
    lines = [l for l in log.read_text().splitlines() if l.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def read_pass(f: Path):
    """{kernel: {dispatch_id: {"dur_ns": ..., counters...}}} of one PMC pass csv."""
    out = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(f)):
        if "akr::" not in r["Kernel_Name"]:
            continue
        k = short(r["Kernel_Name"])
        d = out[k].setdefault(int(r["Dispatch_Id"]), {"dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[k] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"],
                   r["Grid_Size"])
    return out, meta


def is_path_kernel(k):   # the uncounted persistent path kernels (k_path<false, ...>, k_path_defer<false, ...>)
    return k.startswith("k_path") and "<true" not in k


def main(tag):
    src = ROOT / "gpurun_out" / f"prof_{tag}"
    dst = ROOT / "profiles"
    dst.mkdir(exist_ok=True)
    args = (src / "args.txt").read_text().strip() if (src / "args.txt").exists() else "(tools/profile.sh)"
    out = [f"# rocprofv3 summary — {tag}", "", f"Command: `python3 bench.py {args}` under rocprofv3 "
           f"(`tools/profile_driver.sh {tag}`: one pass per counter group, `--kernel-trace` only beside them).", ""]
    ks = list(csv.DictReader(open(src / "kt" / "run_kernel_stats.csv")))
    out += ["## Kernel time (`rocprofv3 --kernel-trace --stats`)", "",
            "| kernel | calls | total ms | avg ms | min ms | max ms | % |", "|---|---|---|---|---|---|---|"]
    for r in ks:
        if "akr::" not in r["Name"]:
            continue
        out.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                   f"{float(r['AverageNs']) / 1e6:.4f} | {float(r['MinNs']) / 1e6:.4f} | {float(r['MaxNs']) / 1e6:.4f} | "
                   f"{float(r['Percentage']):.2f} |")
    kt_line = bench_line(src / "kt.log")
    if kt_line:
        out += ["", "## bench.py line of the kernel-trace pass", "", "```", json.dumps(kt_line), "```"]

    passes, meta = {}, {}
    for sub in PASSES:
        f = src / sub / "run_counter_collection.csv"
        if f.exists():
            passes[sub], m = read_pass(f)
            meta.update(m)
    line = (bench_line(src / "fetch.log") or bench_line(src / "pmc_fetch.log") or bench_line(src / "rq.log")
            or kt_line)
    workload = line["config"] if line else None
    timed_spp = line["steps"] * line["config"].get("spp_per_step", 1) if line else None

    # per kernel: the timed dispatch of a path kernel (longest in each pass), else the mean over dispatches
    kernels = {}
    for k in sorted({k for p in passes.values() for k in p}):
        rec = {"counters": {}}
        for sub, p in passes.items():
            ds = p.get(k)
            if not ds:
                continue
            if is_path_kernel(k):
                d = max(ds.values(), key=lambda x: x["dur_ns"])
                rec.setdefault("timed_dur_ms", []).append(round(d["dur_ns"] / 1e6, 3))
                for c, v in d.items():
                    if c != "dur_ns":
                        rec["counters"][c] = v
            else:
                for c in {c for d in ds.values() for c in d if c != "dur_ns"}:
                    vals = [d[c] for d in ds.values() if c in d]
                    rec["counters"][c] = sum(vals) / len(vals)
                rec["launches_sampled"] = max(rec.get("launches_sampled", 0), len(ds))
        if k in meta:
            rec["grid_threads"] = int(meta[k][5])
        c = rec["counters"]
        if "TCC_EA0_RDREQ_128B_sum" in c:   # requests by size (calibrated, see the docstring)
            rec["read_bytes"] = (32 * c.get("TCC_EA0_RDREQ_32B_sum", 0.0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0.0)
                                 + 128 * c["TCC_EA0_RDREQ_128B_sum"])
            rec["read_bytes_source"] = "32/64/128 x TCC_EA0_RDREQ_{32B,64B,128B} (profiles/r21_fetch_calib.json)"
            if "FETCH_SIZE" in c:
                rec["read_over_fetch_size"] = rec["read_bytes"] / (c["FETCH_SIZE"] * 1024)
        elif "FETCH_SIZE" in c:
            rec["read_bytes"] = 2 * c["FETCH_SIZE"] * 1024
            rec["read_bytes_source"] = "2 x FETCH_SIZE (calibrated: profiles/r21_fetch_calib.json)"
        if "read_bytes" in rec:
            rec["write_bytes"] = c.get("WRITE_SIZE", 0.0) * 1024
            rec["hbm_bytes_per_launch"] = rec["read_bytes"] + rec["write_bytes"]
            if is_path_kernel(k) and timed_spp:
                rec["timed_spp"] = timed_spp
                rec["hbm_bytes_per_spp"] = rec["hbm_bytes_per_launch"] / timed_spp
                rec["read_bytes_per_spp"] = rec["read_bytes"] / timed_spp
        if "TCC_REQ_sum" in c:
            rec["l2_req_bytes_per_launch"] = c["TCC_REQ_sum"] * 128
            if is_path_kernel(k) and timed_spp:
                rec["l2_req_bytes_per_spp"] = rec["l2_req_bytes_per_launch"] / timed_spp
        kernels[k] = rec

    out += ["", "## Per-launch counters (the timed launch for the persistent path kernel; mean per launch otherwise)", "",
            "| kernel | VGPR | AGPR | SGPR | LDS B | scratch | grid | HBM read MB (128 B x requests, or 2x FETCH) | WRITE_SIZE MB | "
            "TCC_MISS x 128 B MB | L2 hit % | TCC_REQ x 128 B GB |", "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for k, rec in kernels.items():
        c = rec["counters"]
        m = meta.get(k, ("",) * 6)
        hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        out.append(f"| {k} | {m[0]} | {m[1]} | {m[2]} | {m[3]} | {m[4]} | {m[5]} | "
                   f"{rec.get('read_bytes', float('nan')) / 1e6:.1f} | {rec.get('write_bytes', float('nan')) / 1e6:.1f} | "
                   f"{miss * 128 / 1e6:.1f} | {100 * hit / max(1.0, hit + miss):.1f} | "
                   f"{c.get('TCC_REQ_sum', float('nan')) * 128 / 1e9:.2f} |")
    path = [k for k in kernels if is_path_kernel(k)]
    for k in path:
        rec, c = kernels[k], kernels[k]["counters"]
        out += ["", f"## The timed `{k}` launch ({rec.get('timed_spp')} spp)", ""]
        out.append(f"- launch duration in each pass (ms): {rec.get('timed_dur_ms')}")
        if "hbm_bytes_per_spp" in rec:
            out.append(f"- HBM (L2 -> fabric) bytes per sample pass: {rec['hbm_bytes_per_spp'] / 1e9:.3f} GB "
                       f"(read {rec['read_bytes'] / rec['timed_spp'] / 1e9:.3f}, write {rec['write_bytes'] / rec['timed_spp'] / 1e9:.3f})")
        if "l2_req_bytes_per_spp" in rec:
            out.append(f"- L2 requests x 128 B per sample pass: {rec['l2_req_bytes_per_spp'] / 1e9:.3f} GB")
        if "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"]
            out.append(f"- wave time: parked in s_waitcnt (SQ_WAIT_ANY) {100 * c['SQ_WAIT_ANY'] / wc:.1f} %, "
                       f"issue-stalled (SQ_WAIT_INST_ANY) {100 * c['SQ_WAIT_INST_ANY'] / wc:.1f} %, issuing (SQ_ACTIVE_INST_ANY) "
                       f"{100 * c['SQ_ACTIVE_INST_ANY'] / wc:.1f} %; VALU active {100 * c['SQ_ACTIVE_INST_VALU'] / wc:.1f} %")
        if "VmemLatency" in c:
            out.append(f"- VmemLatency (issue to return of a VMEM instruction, mean): {c['VmemLatency']:.0f} cycles")
        if "TCP_TCC_READ_REQ_sum" in c and c["TCP_TCC_READ_REQ_sum"]:
            out.append(f"- TCP -> TCC read latency: {c['TCP_TCC_READ_REQ_LATENCY_sum'] / c['TCP_TCC_READ_REQ_sum']:.0f} cycles "
                       f"mean over {c['TCP_TCC_READ_REQ_sum']:.3g} requests")
        if "TCC_EA0_RDREQ_128B_sum" in c:
            out.append(f"- L2 -> fabric read requests by size: 32 B {c.get('TCC_EA0_RDREQ_32B_sum', 0):.4g}, 64 B "
                       f"{c.get('TCC_EA0_RDREQ_64B_sum', 0):.4g}, 128 B {c['TCC_EA0_RDREQ_128B_sum']:.4g} "
                       f"(read bytes {rec['read_bytes'] / 1e12:.3f} TB per launch)")
        if "TCC_EA0_RDREQ_DRAM_sum" in c:
            out.append(f"- requests destined for DRAM (Infinity Cache hits included): {c['TCC_EA0_RDREQ_DRAM_sum']:.4g}; "
                       f"TCC_BUBBLE (FETCH_SIZE's 128-B term): {c.get('TCC_BUBBLE_sum', 0):.4g}")
        if "TCC_EA0_RDREQ_LEVEL_sum" in c and c.get("TCC_EA0_RDREQ_sum"):
            out.append(f"- L2 -> fabric read requests: {c['TCC_EA0_RDREQ_sum']:.3g}, mean in flight x time / count = "
                       f"{c['TCC_EA0_RDREQ_LEVEL_sum'] / c['TCC_EA0_RDREQ_sum']:.0f} cycles per request")
    (dst / f"{tag}_traffic.json").write_text(json.dumps(
        {"tag": tag, "command": f"python3 bench.py {args}", "workload": workload,
         "source": f"rocprofv3 passes of tools/profile_driver.sh {tag} (the raw counter csvs stay under gpurun_out/; "
                   "the per-launch counters the summary uses are in this file)", "kernels": kernels}, indent=1) + "\n")
    (dst / f"{tag}_summary.md").write_text("\n".join(out) + "\n")
    shutil.copy(src / "kt" / "run_kernel_stats.csv", dst / f"{tag}_kernel_stats.csv")
    print((dst / f"{tag}_summary.md").read_text())


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
