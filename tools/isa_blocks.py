#!/usr/bin/env python3
"""Per-basic-block instruction class counts of a kernel dump (tools/isa.sh)."""
import sys
from collections import Counter, OrderedDict

blocks = OrderedDict()
cur = "entry"
blocks[cur] = Counter()
for ln in open(sys.argv[1]).read().split("\n"):
    t = ln.strip().split()
    if not t or t[0].startswith(";"):
        continue
    op = t[0]
    if op.endswith(":"):
        cur = op[:-1].split("_Z")[0][:14] or "entry"
        blocks[cur] = Counter()
        continue
    if op.startswith("."):
        continue
    c = ("mfma" if op.startswith("v_mfma") else "lds" if op.startswith("ds_") else
         "vmem" if op.startswith(("buffer_", "global_", "flat_", "scratch_")) else
         "wait" if op.startswith("s_waitcnt") else "valu" if op.startswith("v_") else "salu")
    blocks[cur][c] += 1
    if c == "valu":
        blocks[cur]["v:" + op] += 1
detail = len(sys.argv) > 2
for b, c in blocks.items():
    if sum(v for k, v in c.items() if ":" not in k) == 0:
        continue
    print("%-14s mfma %3d valu %4d lds %3d vmem %3d wait %3d salu %3d" % (b, c["mfma"], c["valu"], c["lds"], c["vmem"],
                                                                         c["wait"], c["salu"]))
    if detail and b in sys.argv[2:]:
        for k, v in sorted(((k, v) for k, v in c.items() if k.startswith("v:")), key=lambda x: -x[1]):
            print("      %4d %s" % (v, k[2:]))
