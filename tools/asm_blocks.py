"""Per-basic-block instruction summary of a kernel in a hipcc -S listing
(diagnostics for register/latency work): block label, loop depth comment,
instruction count, memory / spill / wait ops.
Usage: python tools/asm_blocks.py file.s kernel_symbol [min_insts]"""
import collections
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    s = open(path).read()
    a = s.index(name + ":")
    b = s.index(".Lfunc_end", a)
    cur, rows = None, []
    for l in s[a:b].splitlines():
        t = l.strip()
        if re.match(r"^(\.LBB\S+|; %bb\.\d+):", l) or l.startswith("; %bb."):
            cur = [t.split(":")[0], t.split(";")[-1].strip() if "Loop" in t else "", 0, collections.Counter()]
            rows.append(cur)
            continue
        if cur and l.startswith("\t") and not t.startswith((".", ";")):
            cur[2] += 1
            op = t.split()[0]
            if op.startswith(("global_", "ds_", "v_readlane", "v_writelane", "s_waitcnt", "scratch", "s_load",
                              "buffer_", "v_rcp", "v_rsq", "v_sqrt", "v_div", "s_cbranch", "s_branch")):
                cur[3][op] += 1
    for lab, loop, n, c in rows:
        if n >= mn:
            print(f"{lab:12s} {n:5d} {loop:40s} {dict(c)}")


if __name__ == "__main__":
    main()
