"""Summarise a tools/profile.sh run (rocprofv3 csv) into profiles/<tag>_summary.md + copies of the
kernel stats / counter csvs.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB and
reads half the bytes of 128-byte-line traffic on gfx950, so traffic = 2 * FETCH_SIZE * 1024; the
TCC_MISS_sum * 128 B column is printed beside it as the calibration check for this access pattern.
WRITE_SIZE (KiB, exact for 16-B-per-lane stores and float atomics per the guide) is added unscaled.
Also writes profiles/<tag>_traffic.json: HBM bytes per launch per kernel, which bench.py reports as
roofline.traffic when the workload matches."""
import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def short(name):
    name = name.replace("void ", "").replace("akr::", "")
    return name.split("(")[0]


def main(tag):
    src = ROOT / "gpurun_out" / f"prof_{tag}"
    dst = ROOT / "profiles"
    dst.mkdir(exist_ok=True)
    out = [f"# rocprofv3 summary — {tag}", "", f"Command: `tools/profile.sh {tag}` (see tools/profile.sh).", ""]
    ks = list(csv.DictReader(open(src / "kt" / "run_kernel_stats.csv")))
    out += ["## Kernel time (`rocprofv3 --kernel-trace --stats`)", "",
            "| kernel | calls | total ms | avg ms | min ms | max ms | % |", "|---|---|---|---|---|---|---|"]
    for r in ks:
        if "akr::" not in r["Name"]:
            continue
        out.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                   f"{float(r['AverageNs']) / 1e6:.4f} | {float(r['MinNs']) / 1e6:.4f} | {float(r['MaxNs']) / 1e6:.4f} | "
                   f"{float(r['Percentage']):.2f} |")
    pmc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for sub in ("pmc_fetch", "pmc_write", "pmc_tcc"):
        f = src / sub / "run_counter_collection.csv"
        if not f.exists():
            continue
        for r in csv.DictReader(open(f)):
            if "akr::" not in r["Kernel_Name"]:
                continue
            k = short(r["Kernel_Name"])
            pmc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"], r["Grid_Size"])
    out += ["", "## Per-launch counters (separate `--pmc` passes, `--kernel-trace` only beside them)", "",
            "| kernel | VGPR | SGPR | LDS B | scratch | grid | FETCH_SIZE KiB | HBM read MB (2x FETCH) | "
            "WRITE_SIZE MB | TCC_MISS x 128 B MB | L2 hit % |", "|---|---|---|---|---|---|---|---|---|---|---|"]
    traffic = {}
    for k, c in sorted(pmc.items()):
        fs = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"]) if c["FETCH_SIZE"] else float("nan")
        ws = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"]) if c["WRITE_SIZE"] else 0.0
        traffic[k] = {"hbm_bytes_per_launch": 2 * fs * 1024 + ws * 1024, "read_bytes": 2 * fs * 1024,
                      "write_bytes": ws * 1024, "launches_sampled": len(c["FETCH_SIZE"])}
        hit = sum(c["TCC_HIT_sum"]) / max(1, len(c["TCC_HIT_sum"]))
        miss = sum(c["TCC_MISS_sum"]) / max(1, len(c["TCC_MISS_sum"]))
        m = meta[k]
        out.append(f"| {k} | {m[0]} | {m[1]} | {m[2]} | {m[3]} | {m[4]} | {fs:.0f} | {2 * fs * 1024 / 1e6:.1f} | "
                   f"{ws * 1024 / 1e6:.1f} | {miss * 128 / 1e6:.1f} | {100 * hit / max(1.0, hit + miss):.1f} |")
    workload = None
    for log in ("pmc_fetch.log",):
        p = src / log
        if p.exists():
            lines = [l for l in p.read_text().splitlines() if l.startswith("{")]
            if lines:
                line = json.loads(lines[-1])
                workload = line["config"]
                # a persistent path launch renders every spp of its call: bytes per sample pass
                # (bench.py launches warmup W, timed K and an untimed breakdown of min(K, 4) spp)
                K, Wm = line["steps"], line["warmup"]
                spp_total = (Wm if Wm > 0 else 0) + K + min(K, 4)
                for k, t in traffic.items():
                    # not the counting builds (k_path<true, ...>; the second argument is the LDS-table flag)
                    if k.startswith("k_path") and "<true" not in k and t["launches_sampled"]:
                        t["hbm_bytes_per_spp"] = t["hbm_bytes_per_launch"] * t["launches_sampled"] / spp_total
    (dst / f"{tag}_traffic.json").write_text(json.dumps(
        {"tag": tag, "workload": workload, "source": f"profiles/{tag}_pmc_fetch.csv + {tag}_pmc_write.csv",
         "kernels": traffic}, indent=1) + "\n")
    for log in ("kt.log",):
        p = src / log
        if p.exists():
            lines = [l for l in p.read_text().splitlines() if l.startswith("{")]
            if lines:
                out += ["", "## bench.py line of the kernel-trace pass", "", "```", lines[-1], "```"]
    (dst / f"{tag}_summary.md").write_text("\n".join(out) + "\n")
    shutil.copy(src / "kt" / "run_kernel_stats.csv", dst / f"{tag}_kernel_stats.csv")
    for sub in ("pmc_fetch", "pmc_write", "pmc_tcc"):
        f = src / sub / "run_counter_collection.csv"
        if f.exists():
            shutil.copy(f, dst / f"{tag}_{sub}.csv")
    print((dst / f"{tag}_summary.md").read_text())


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
