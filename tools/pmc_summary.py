"""Summarise tools/pmc_path.sh runs: per-launch counters of the traversal kernels, the wave-time
split (parked in s_waitcnt / issue-stalled / issuing; their sum is SQ_WAVE_CYCLES, MI355X_MICROARCH.md
§rocprofv3) and VALU issue, and HBM traffic per launch (2 x FETCH_SIZE KiB + WRITE_SIZE KiB, gfx950
correction as in tools/prof_summary.py).  Writes profiles/<tag>_pmc.md and profiles/<tag>_traffic.json.
Usage: python tools/pmc_summary.py <tag>   (reads gpurun_out/pmc_<tag>_p1 and _p0)"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KERNELS = {"k_path<false>": "path (k_path)", "k_path<false, true>": "path (k_path, LDS tables)",
           "k_path_defer<false, true>": "path (k_path_defer, LDS tables)", "k_trace<0, false, true, true>": "closest (k_trace)",
           "k_trace<2, false, true, true>": "shadow (k_trace)", "k_shade": "shade (k_shade)"}


def short(name):
    return name.replace("void ", "").replace("akr::", "").split("(")[0]


def load(d):
    vals = defaultdict(lambda: defaultdict(list))
    meta = {}
    for sub in ("sq1", "sq2", "fetch", "write", "tcc"):
        f = d / sub / "run_counter_collection.csv"
        if not f.exists():
            continue
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k not in KERNELS:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = {"vgpr": r.get("VGPR_Count"), "lds": r.get("LDS_Block_Size"), "scratch": r.get("Scratch_Size"),
                       "grid": r.get("Grid_Size")}
    return vals, meta


def main(tag):
    out = [f"# PMC summary — {tag}", "", "Collected by `tools/pmc_path.sh {tag} <path>`; per-launch means of each counter.", ""]
    traffic = {}
    workload = None
    for path in (1, 0):
        d = ROOT / "gpurun_out" / f"pmc_{tag}_p{path}"
        if not d.exists():
            continue
        vals, meta = load(d)
        log = d / "fetch.log"
        spp_total = None
        if log.exists():
            lines = [l for l in log.read_text().splitlines() if l.startswith("{")]
            if lines:
                line = json.loads(lines[-1])
                workload = workload or line["config"]
                # k_path launches of bench.py: warmup W spp, timed K, the untimed breakdown min(K, 4)
                K, Wm = line["steps"], line["warmup"]
                spp_total = (Wm if Wm > 0 else 0) + K + min(K, 4)
        out += [f"## render form: {'persistent path kernel' if path else 'wavefront'} (bench --path {path})", "",
                "| kernel | launches | VGPR | LDS B | waves | wave-cycles | parked (WAIT_ANY) | issue-stall (WAIT_INST_ANY) | "
                "issuing (ACTIVE_INST_ANY) | VALU active / wave-cycles | VALU insts / wave | LDS insts / wave | "
                "VMEM rd / wave | VMEM wr / wave | SALU / wave | HBM MB / launch | read MB | write MB | L2 hit % |",
                "|" + "---|" * 19]
        for k, c in vals.items():
            m = lambda n: (sum(c[n]) / len(c[n])) if c.get(n) else float("nan")
            waves = m("SQ_WAVES")
            wc = m("SQ_WAVE_CYCLES")
            hbm = 2 * m("FETCH_SIZE") * 1024 + (m("WRITE_SIZE") * 1024 if c.get("WRITE_SIZE") else 0.0)
            hit, miss = m("TCC_HIT_sum"), m("TCC_MISS_sum")
            traffic[k] = {"hbm_bytes_per_launch": hbm, "read_bytes": 2 * m("FETCH_SIZE") * 1024,
                          "write_bytes": m("WRITE_SIZE") * 1024, "launches_sampled": len(c.get("FETCH_SIZE", []))}
            if k.startswith("k_path") and spp_total:   # one launch renders every spp: bytes per sample pass
                n = len(c.get("FETCH_SIZE", []))
                traffic[k]["hbm_bytes_per_spp"] = hbm * n / spp_total
            out.append(f"| {KERNELS[k]} | {len(c.get('SQ_WAVES', []))} | {meta[k]['vgpr']} | {meta[k]['lds']} | {waves:.0f} | "
                       f"{wc:.3g} | {m('SQ_WAIT_ANY') / wc:.3f} | {m('SQ_WAIT_INST_ANY') / wc:.3f} | "
                       f"{m('SQ_ACTIVE_INST_ANY') / wc:.3f} | {m('SQ_ACTIVE_INST_VALU') / wc:.3f} | "
                       f"{m('SQ_INSTS_VALU') / waves:.3g} | {m('SQ_INSTS_LDS') / waves:.3g} | "
                       f"{m('SQ_INSTS_VMEM_RD') / waves:.3g} | {m('SQ_INSTS_VMEM_WR') / waves:.3g} | "
                       f"{m('SQ_INSTS_SALU') / waves:.3g} | {hbm / 1e6:.1f} | {2 * m('FETCH_SIZE') * 1024 / 1e6:.1f} | "
                       f"{m('WRITE_SIZE') * 1024 / 1e6:.1f} | {100 * hit / (hit + miss):.1f} |")
        out.append("")
    out += ["Fractions are of SQ_WAVE_CYCLES (quad-cycles summed over waves).  A persistent path launch renders "
            "every spp of its render: the bench's launches are the warmup, the timed K-spp render and the "
            "min(K, 4)-spp breakdown pass, and traffic.json's hbm_bytes_per_spp divides by their spp sum.", ""]
    dst = ROOT / "profiles"
    (dst / f"{tag}_pmc.md").write_text("\n".join(out) + "\n")
    (dst / f"{tag}_traffic.json").write_text(json.dumps(
        {"tag": tag, "workload": workload, "source": f"tools/pmc_path.sh {tag}", "kernels": traffic}, indent=1) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "pmc")
