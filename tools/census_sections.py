#!/usr/bin/env python3
"""Static per-section instruction census of one kernel's IC-iteration loop.

  tools/isa.sh builds the device assembly (/tmp/isa/kmc.s); then
  python3 tools/census_sections.py /tmp/isa/kmc.s k_pic_fftILi2ELi2ELb0ELb1ELb1E [more.s PATTERN ...]

The loop is every block LLVM annotates "in Loop" (plus its header).  Each
instruction is attributed to a section by its opcode family:
  network     v_mfma (the 4-point network / ones-MFMA sums) and ds_bpermute
  fp64        v_{fma,fmac,add,mul}_f64 (DFT-6 pairs, taps, the one-tap epilogue)
  slicer      v_cvt_i32_f64, v_med3_i32, ds_read_u8 / grid reads
  tie         v_min*_u32 / v_cmp_*_u64 / v_cvt_f64_u32 / v_cmp_eq_f64 (candidates + the rare exact branch)
  counts      v_bcnt, v_mad_u32_u24, v_mul_u32_u24, *_dpp adds, v_readlane, v_xor_b32_sdwa
  select      v_cndmask
  copy        v_mov_b64 / v_mov_b32
  int/addr    the other VALU integer ops
  lds         the other ds_*
  scalar      s_* (waits, nops, branches, SALU)
Static counts (one pass through the code, the rare tie branch included): the
per-wave dynamic totals are the PMC census (tools/gpu_census.sh, census.py)."""
import re
import sys
from collections import Counter, OrderedDict

SECTIONS = ("network", "fp64", "slicer", "tie", "counts", "select", "copy", "int/addr", "lds", "scalar")


def section(op, line):
    if op.startswith("v_mfma") or op.startswith("ds_bpermute"):
        return "network"
    if re.match(r"v_(fma|fmac|add|mul)_f64", op):
        return "fp64"
    if op in ("v_cvt_i32_f64", "v_med3_i32") or op.startswith("ds_read_u8"):
        return "slicer"
    if re.match(r"v_min3?_u(32|16)", op) or re.match(r"v_cmp_\w+_u64", op) or op.startswith("v_cvt_f64_u32") or \
            op.startswith("v_cmp_eq_f64") or op.startswith("v_subbrev") or op.startswith("v_max_i32"):
        return "tie"
    if op.startswith(("v_bcnt", "v_mad_u32_u24", "v_mul_u32_u24", "v_readlane")) or "_dpp" in op or \
            (op.startswith("v_xor_b32_sdwa")):
        return "counts"
    if op.startswith("v_cndmask"):
        return "select"
    if op.startswith("v_mov_b64") or op.startswith("v_mov_b32"):
        return "copy"
    if op.startswith("v_"):
        return "int/addr"
    if op.startswith("ds_"):
        return "lds"
    return "scalar"


def census(path, pat):
    lines = open(path).read().split("\n")
    start = None
    for i, ln in enumerate(lines):
        lab = ln.split(";")[0].rstrip()
        if lab.endswith(":") and not lab.startswith((".", "\t", " ")) and pat in lab:
            start = i
            break
    if start is None:
        sys.exit("no kernel matching %r in %s" % (pat, path))
    end = start
    while not lines[end].strip().startswith(".Lfunc_end"):
        end += 1
    body = lines[start:end]
    whole, loop = Counter(), Counter()
    in_loop = False
    for ln in body:
        t = ln.strip()
        if not t:
            continue
        if t.startswith(".LBB") or t.startswith("; %bb."):
            in_loop = "in Loop" in t or "Loop Header" in t
            continue
        if t.startswith((";", ".")):
            continue
        op = t.split()[0]
        sec = section(op, t)
        whole[sec] += 1
        if in_loop:
            loop[sec] += 1
    return whole, loop


def main():
    args = sys.argv[1:]
    rows = OrderedDict()
    for i in range(0, len(args), 2):
        w, lp = census(args[i], args[i + 1])
        rows["%s:%s" % (args[i].split("/")[-1], args[i + 1])] = (w, lp)
    print("| kernel (asm) | part | " + " | ".join(SECTIONS) + " | total |")
    print("|---|---|" + "---|" * (len(SECTIONS) + 1))
    for name, (w, lp) in rows.items():
        for part, c in (("loop", lp), ("kernel", w)):
            print("| %s | %s | %s | %d |" % (name, part, " | ".join(str(c[s]) for s in SECTIONS), sum(c.values())))


if __name__ == "__main__":
    main()
