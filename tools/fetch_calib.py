"""Join tools/fetch_calib's pattern lines with its rocprofv3 counter passes (tools/fetch_calib.sh) into
profiles/<tag>_fetch_calib.json and a markdown table.

Per pattern (one kernel instantiation calib<N>, every record read once from a 2 GiB table):
- known bytes: the records' bytes, and the distinct 64-B sectors and 128-B lines they cover;
- counters: FETCH_SIZE (KiB), TCC_EA0_RDREQ (all / 32 B / 64 B / 128 B), TCC_BUBBLE, RDREQ_DRAM, L2 hit / miss;
- fetch_factor = line-or-sector bytes the requests carry (32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B)
  divided by FETCH_SIZE bytes: the factor that replaces FETCH_SIZE's blanket x2 for this access shape.
Usage: python3 tools/fetch_calib.py <tag>  (reads gpurun_out/calib_<tag>/)."""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def counters(f: Path):
    """{kernel 'calib<N>' or 'flush': {counter: value}} (one dispatch per kernel per pass)."""
    out = defaultdict(dict)
    if not f.exists():
        return out
    for r in csv.DictReader(open(f)):
        m = re.search(r"calib<(\d+)>", r["Kernel_Name"])
        k = f"calib<{m.group(1)}>" if m else ("flush" if "flush" in r["Kernel_Name"] else None)
        if k is None:
            continue
        out[k][r["Counter_Name"]] = out[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def request_bytes(c):
    if not all(k in c for k in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")):
        return None
    return 32 * c["TCC_EA0_RDREQ_32B_sum"] + 64 * c["TCC_EA0_RDREQ_64B_sum"] + 128 * c["TCC_EA0_RDREQ_128B_sum"]


def main(tag):
    src = ROOT / "gpurun_out" / f"calib_{tag}"
    pats = [json.loads(l) for l in (src / "plain.log").read_text().splitlines() if l.startswith("{")]
    cs = defaultdict(dict)
    for sub in ("fetch", "rq", "rq2"):
        for k, d in counters(src / sub / "run_counter_collection.csv").items():
            cs[k].update(d)
    rows = []
    for p in pats:
        c = cs.get(p["kernel"], {})
        rec = dict(p)
        rec["counters"] = c
        if "FETCH_SIZE" in c:
            rec["fetch_bytes"] = c["FETCH_SIZE"] * 1024
        rb = request_bytes(c)
        if rb is not None:
            rec["request_bytes"] = rb
            rec["requests_partition"] = (c["TCC_EA0_RDREQ_32B_sum"] + c["TCC_EA0_RDREQ_64B_sum"]
                                         + c["TCC_EA0_RDREQ_128B_sum"]) / max(1.0, c.get("TCC_EA0_RDREQ_sum", 0.0))
            if rec.get("fetch_bytes"):
                rec["fetch_factor"] = rb / rec["fetch_bytes"]
            for kb in ("record_bytes", "sector64_bytes", "line128_bytes"):
                rec[f"request_over_{kb.split('_')[0]}"] = rb / p[kb]
        if rec.get("fetch_bytes"):
            for kb in ("record_bytes", "sector64_bytes", "line128_bytes"):
                rec[f"fetch_over_{kb.split('_')[0]}"] = rec["fetch_bytes"] / p[kb]
        rows.append(rec)
    (ROOT / "profiles").mkdir(exist_ok=True)
    doc = {"tag": tag, "source": f"tools/fetch_calib.hip + tools/fetch_calib.sh (rocprofv3 passes), {src.name}",
           "table_bytes": 2 << 30, "patterns": rows}
    (ROOT / "profiles" / f"{tag}_fetch_calib.json").write_text(json.dumps(doc, indent=1) + "\n")
    md = [f"# FETCH_SIZE calibration — {tag}", "",
          "Every record read once from a 2 GiB table, 256 B apart (no shared lines); `packed` = two 64-B records "
          "per line. Bytes in GB; `req` = 32·RDREQ_32B + 64·RDREQ_64B + 128·RDREQ_128B.", "",
          "| pattern | ms | record GB | sector GB | line GB | FETCH_SIZE GB | req GB | RDREQ 32/64/128 B (M) | BUBBLE (M) | "
          "req/FETCH | req/line | L2 hit % |", "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        c = r["counters"]
        hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        g = lambda x: f"{x / 1e9:.3f}" if x is not None else "–"
        md.append(f"| {r['pattern']} | {r['ms']:.2f} | {g(r['record_bytes'])} | {g(r['sector64_bytes'])} | "
                  f"{g(r['line128_bytes'])} | {g(r.get('fetch_bytes'))} | {g(r.get('request_bytes'))} | "
                  f"{c.get('TCC_EA0_RDREQ_32B_sum', 0) / 1e6:.2f} / {c.get('TCC_EA0_RDREQ_64B_sum', 0) / 1e6:.2f} / "
                  f"{c.get('TCC_EA0_RDREQ_128B_sum', 0) / 1e6:.2f} | {c.get('TCC_BUBBLE_sum', 0) / 1e6:.2f} | "
                  f"{r.get('fetch_factor', float('nan')):.3f} | {r.get('request_over_line128', float('nan')):.3f} | "
                  f"{100 * hit / max(1.0, hit + miss):.1f} |")
    (ROOT / "profiles" / f"{tag}_fetch_calib.md").write_text("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r21")
