"""Where a kernel's spills sit: splits one kernel of a gfx950 assembly listing (hipcc -S
--offload-device-only) into basic blocks, finds the loops from the back edges (a branch to an
earlier label spans the blocks between), and prints per loop its instruction count, its global loads
and its scratch loads/stores, beside the kernel's totals and the metadata (VGPRs, spills, LDS).

Usage: python tools/isa_spills.py <file.s> <kernel symbol substring>"""
import re
import sys


def kernel_body(text, sym):
    starts = [m for m in re.finditer(r"^(_Z\S*):.*$", text, re.M) if sym in m.group(1)]
    if not starts:
        raise SystemExit(f"no kernel matching {sym}")
    m = starts[0]
    end = text.index(".Lfunc_end", m.end())
    return m.group(1), text[m.end():end].splitlines()


def meta(text, name):
    mm = re.search(r"\.name:\s+" + re.escape(name) + r"\s*$", text, re.M)
    if not mm:
        return {}
    i = mm.start()
    j = text.rfind("- .agpr_count:", 0, i)
    k = text.find("- .agpr_count:", i)
    blk = text[j:k if k > 0 else len(text)]
    out = {}
    for k in ("vgpr_count", "vgpr_spill_count", "sgpr_count", "group_segment_fixed_size", "private_segment_fixed_size"):
        mm = re.search(r"\.%s:\s+(\d+)" % k, blk)
        if mm:
            out[k] = int(mm.group(1))
    return out


def main():
    path, sym = sys.argv[1], sys.argv[2]
    text = open(path).read()
    name, body = kernel_body(text, sym)
    labels, insts = {}, []  # insts: (index, text); labels: name -> inst index
    for l in body:
        s = l.strip()
        if re.match(r"^\.LBB\d+_\d+:", s):
            labels[s[:-1].split(":")[0]] = len(insts)
        elif l.startswith("\t") and s and not s.startswith((".", ";")):
            insts.append(s)
    loops = []
    for i, s in enumerate(insts):
        mm = re.match(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", s)
        if mm:
            tgt = mm.group(1) or mm.group(2)
            if tgt in labels and labels[tgt] <= i:
                loops.append((labels[tgt], i))
    count = lambda a, b, pat: sum(1 for s in insts[a:b + 1] if re.search(pat, s))
    print(name, meta(text, name))
    print(f"total: {len(insts)} insts, scratch loads {count(0, len(insts) - 1, r'^scratch_load')}, "
          f"stores {count(0, len(insts) - 1, r'^scratch_store')}")
    for a, b in sorted(set(loops)):
        print(f"loop [{a}, {b}] {b - a + 1:5d} insts  global loads {count(a, b, r'^global_load'):3d}  "
              f"scratch loads {count(a, b, r'^scratch_load'):3d} stores {count(a, b, r'^scratch_store'):3d}  "
              f"ds {count(a, b, r'^ds_'):3d}")


if __name__ == "__main__":
    main()
