#!/usr/bin/env python3
"""Prints the traversal loop (the depth-2 loop holding the most vector loads) of
a render_kernel instantiation from a hipcc -S listing, without implicit-def /
inline-asm marker lines.  Usage: tools/trav_loop.py file.s [kernel_symbol]"""
import collections
import re
import sys

path = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "_ZN3ptk13render_kernelILb0ELb0ELb0ELb0ELb0ELb1ELb0EEEv7KParams"
s = open(path).read()
a = s.index(name + ":")
b = s.index(".Lfunc_end", a)
blocks, cur = [], None
for line in s[a:b].splitlines():
    if re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", line):
        cur = [line]
        blocks.append(cur)
    elif cur is not None:
        cur.append(line)
loads = collections.Counter()
for bl in blocks:
    h = re.search(r"Header=BB(\d+_\d+) Depth=2", bl[0])
    key = h.group(1) if h else (re.match(r"^\.LBB(\d+_\d+)", bl[0]).group(1) if "Loop Header: Depth=2" in bl[0] else None)
    if key:
        loads[key] += sum("global_load_dwordx" in x for x in bl)
trav = loads.most_common(1)[0][0]
for bl in blocks:
    if ("BB" + trav) in bl[0] or bl[0].startswith(".LBB" + trav + ":"):
        for x in bl:
            if "implicit-def" in x or "ASMSTART" in x or "ASMEND" in x:
                continue
            print(x)
