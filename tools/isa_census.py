#!/usr/bin/env python3
"""ISA census of render_kernel: static VALU / SALU / v_mov /
SGPR-spill lane moves per loop region of a hipcc -S listing, and the register
counts.  The traversal loop is the Depth=2 loop holding the node step's seven
global_load_dwordx4; the shading round is the rest of the persistent loop.
Usage: python tools/isa_census.py file.s [kernel_symbol]"""
import collections
import re
import sys

DEFAULT = "_ZN3ptk13render_kernelILb0ELb0ELb0ELb0ELb0ELb0ELb0EEEv7KParams"


def census(path, name=DEFAULT):
    s = open(path).read()
    a = s.index(name + ":")
    b = s.index(".Lfunc_end", a)
    blocks, cur = [], None
    for line in s[a:b].splitlines():
        t = line.strip()
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):(.*)$", line)
        if m:
            hdr = re.search(r"Header=BB(\d+_\d+) Depth=(\d)", t)
            own = "Loop Header" in t
            cur = {"label": m.group(1), "loop": ("BB" + hdr.group(1)) if hdr else (m.group(1).lstrip(".L") if own else None),
                   "depth": int(hdr.group(2)) if hdr else (int(re.search(r"Depth=(\d)", t).group(1)) if own else 0),
                   "ops": collections.Counter()}
            blocks.append(cur)
            continue
        if cur is not None and line.startswith("\t") and t and not t.startswith((".", ";")):
            cur["ops"][t.split()[0]] += 1
    # the traversal loop: the depth-2 loop with the most global_load_dwordx4
    loads = collections.Counter()
    for bl in blocks:
        if bl["depth"] == 2:
            loads[bl["loop"]] += bl["ops"]["global_load_dwordx4"]
    trav = loads.most_common(1)[0][0] if loads else None
    regions = collections.defaultdict(collections.Counter)
    for bl in blocks:
        reg = "traversal" if bl["loop"] == trav else ("persistent loop" if bl["depth"] >= 1 else "outside loops")
        regions[reg].update(bl["ops"])
    out = {}
    for reg, c in regions.items():
        valu = sum(n for op, n in c.items() if op.startswith("v_"))
        salu = sum(n for op, n in c.items() if op.startswith("s_"))
        out[reg] = {"valu": valu, "salu": salu, "v_mov": c["v_mov_b32_e32"] + c["v_mov_b64_e32"],
                    "lane_moves": c["v_readlane_b32"] + c["v_writelane_b32"], "cndmask": c["v_cndmask_b32_e32"] + c["v_cndmask_b32_e64"]}
    m = re.search(r"\.name:\s+" + re.escape(name) + r"\b.*?\.sgpr_spill_count:\s+(\d+).*?\.vgpr_count:\s+(\d+).*?\.vgpr_spill_count:\s+(\d+)", s, re.S)
    out["registers"] = {"sgpr_spill": int(m.group(1)), "vgpr": int(m.group(2)), "vgpr_spill": int(m.group(3))} if m else None
    return out


if __name__ == "__main__":
    import json
    r = census(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else DEFAULT)
    for k, v in r.items():
        print(k, json.dumps(v))
