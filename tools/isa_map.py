#!/usr/bin/env python3
"""Compact instruction-class map of a kernel dump (tools/isa_hist.py --dump):
one character per instruction, M = MFMA, v = VALU, d = LDS, g = vector memory,
w = s_waitcnt, s = other scalar; one line per basic block."""
import sys

for ln in open(sys.argv[1]).read().split("\n"):
    t = ln.strip().split()
    if not t or t[0].startswith(";"):
        continue
    op = t[0]
    if op.endswith(":"):
        print("\n" + op.split("_Z")[0][:12], end=" ")
        continue
    if op.startswith("."):
        continue
    c = ("M" if op.startswith("v_mfma") else "d" if op.startswith("ds_") else
         "g" if op.startswith(("buffer_", "global_", "flat_", "scratch_")) else
         "w" if op.startswith("s_waitcnt") else "v" if op.startswith("v_") else "s")
    print(c, end="")
print()
