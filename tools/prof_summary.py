#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into profiles/.

usage: prof_summary.py TAG STATS_DIR FETCH_DIR WRITE_DIR KERNEL_SUBSTR [BENCH_KERNEL] [WORKLOAD] [SQ_DIR]

* copies <STATS_DIR>/**/*_kernel_stats.csv to profiles/<TAG>_kernel_stats.csv
* averages FETCH_SIZE / WRITE_SIZE (KB) per launch of the kernels whose name
  contains KERNEL_SUBSTR and writes profiles/<TAG>_pmc_<BENCH_KERNEL>.json with
  the HBM bytes per launch, using the gfx950 correction of MI355X_MICROARCH.md
  §HBM: FETCH_SIZE counts half of the bytes of a wide (16 B/lane) coalesced
  streaming read, so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
* SQ_DIR (a --pmc pass of SQ_COUNTERS over the same bench command): the
  per-launch means of those counters, from which bench.py derives the
  kernel's limiter (VALU issue, matrix-core busy, wave stall, occupancy).
* stamps the JSON with the source hash of the engine sources (bench.py
  source_hash) and the workload, so bench.py uses it only for that build.
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(pattern):
    f = sorted(glob.glob(pattern, recursive=True), key=os.path.getmtime)
    if not f:
        raise SystemExit("no file matches %s" % pattern)
    return f[-1]


def counter_mean(d, counter, kern):
    vals = []
    for r in csv.DictReader(open(one(os.path.join(d, "**", "*_counter_collection.csv")))):
        if kern in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    return (sum(vals) / len(vals) if vals else None), len(vals)


SQ_COUNTERS = ("GRBM_GUI_ACTIVE", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_MFMA",
               "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU")


def main():
    tag, sdir, fdir, wdir, kern = sys.argv[1:6]
    bench_kernel = sys.argv[6] if len(sys.argv) > 6 else "k_wcontract"
    workload = sys.argv[7] if len(sys.argv) > 7 else "c2"
    sqdir = sys.argv[8] if len(sys.argv) > 8 else None
    from bench import source_hash
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = one(os.path.join(sdir, "**", "*_kernel_stats.csv"))
    shutil.copy(stats, os.path.join(out, tag + "_kernel_stats.csv"))
    avg_ns = None
    for r in csv.DictReader(open(stats)):
        if kern in r["Name"]:
            avg_ns = float(r["AverageNs"])
    fetch, nf = counter_mean(fdir, "FETCH_SIZE", kern)
    write, nw = counter_mean(wdir, "WRITE_SIZE", kern)
    res = {"kernel": bench_kernel, "kernel_name_match": kern, "workload": workload, "source_hash": source_hash(),
           "avg_duration_ns_rocprof": avg_ns, "fetch_size_kb_per_launch": fetch,
           "write_size_kb_per_launch": write, "launches_sampled": [nf, nw],
           "hbm_bytes_per_launch": (2 * fetch + write) * 1024 if fetch is not None and write is not None else None,
           "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE reports half of "
                         "wide coalesced reads, MI355X_MICROARCH.md §HBM)"}
    if sqdir:
        sq = {}
        for c in SQ_COUNTERS:
            v, n = counter_mean(sqdir, c, kern)
            sq[c] = v
        res["sq_per_launch"] = sq
    with open(os.path.join(out, "%s_pmc_%s.json" % (tag, bench_kernel)), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
