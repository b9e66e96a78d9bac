#!/usr/bin/env python3
"""Instruction histogram of one kernel in a device assembly file.

  hipcc ... --cuda-device-only -S csrc/kernels_mc.hip -o /tmp/kmc.s
  python3 tools/isa_hist.py /tmp/kmc.s k_pic_mfmaILi6ELi2 [--dump out.s]

Prints the kernel's VGPR/SGPR/LDS/scratch metadata and instruction counts by
class (MFMA, VALU, LDS, global, scalar memory, waits), static counts only.
"""
import re
import sys
from collections import Counter


def main():
    path, pat = sys.argv[1], sys.argv[2]
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    lines = open(path).read().split("\n")
    start = None
    for i, ln in enumerate(lines):
        lab = ln.split(";")[0].rstrip()
        if lab.endswith(":") and not lab.startswith((".", "\t", " ")) and pat in lab:
            start, name = i, lab[:-1]
            break
    if start is None:
        sys.exit("no kernel matching %r" % pat)
    end = start
    while not lines[end].strip().startswith(".Lfunc_end"):
        end += 1
    body = lines[start:end]
    meta = {}
    for ln in lines[end:end + 80]:
        m = re.match(r"\s*\.(amdhsa_next_free_vgpr|amdhsa_next_free_sgpr|amdhsa_group_segment_fixed_size|"
                     r"amdhsa_private_segment_fixed_size|amdhsa_accum_offset)\s+(\d+)", ln)
        if m:
            meta[m.group(1)] = int(m.group(2))
    c = Counter()
    for ln in body:
        t = ln.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        c[t[0]] += 1
    cls = Counter()
    for op, n in c.items():
        if op.startswith("v_mfma"):
            cls["mfma"] += n
        elif op.startswith("ds_"):
            cls["lds"] += n
        elif op.startswith(("global_", "buffer_", "flat_")):
            cls["vmem"] += n
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            cls["smem"] += n
        elif op.startswith("s_waitcnt"):
            cls["waitcnt"] += n
        elif op.startswith("v_"):
            cls["valu"] += n
        elif op.startswith("s_"):
            cls["salu/branch"] += n
    print(name)
    print("meta", meta)
    print("classes", dict(cls), "total", sum(c.values()))
    for op, n in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3].isdigit() else 50):
        print("%6d %s" % (n, op))
    if dump:
        open(dump, "w").write("\n".join(body) + "\n")


if __name__ == "__main__":
    main()
