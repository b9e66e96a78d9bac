#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into profiles/.

usage: prof_summary.py TAG STATS_DIR FETCH_DIR WRITE_DIR KERNEL_SUBSTR [BENCH_KERNEL] [WORKLOAD] [SQ_DIR]
       prof_summary.py --all TAG STATS_DIR FETCH_DIR WRITE_DIR WORKLOAD [SQ_DIR]

* copies <STATS_DIR>/**/*_kernel_stats.csv to profiles/<TAG>_kernel_stats.csv
* averages FETCH_SIZE / WRITE_SIZE (KB) per launch of the kernels whose name
  contains KERNEL_SUBSTR and writes profiles/<TAG>_pmc_<BENCH_KERNEL>.json with
  the HBM bytes per launch, using the gfx950 correction of MI355X_MICROARCH.md
  §HBM: FETCH_SIZE counts half of the bytes of a wide (16 B/lane) coalesced
  streaming read, so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
* SQ_DIR (a --pmc pass of SQ_COUNTERS over the same bench command): the
  per-launch means of those counters, from which bench.py derives the
  kernel's limiter (VALU issue, matrix-core busy, wave stall, occupancy).
* --all: the same per-launch means for every kernel of the bench, grouped
  by the engine's timing groups (dsce_kernel_time names: k_jakes, tx,
  rx_front, perfect_ic, k_mic_pilot, k_mic_data, k_wcontract, ...), written
  to profiles/<TAG>_pmc_all.json: bench.py puts each group on its roofline
  with them.  A group's value per launch is the sum of its kernels'
  per-dispatch means (each kernel of a group runs once per group launch on
  the FFT-form OFDM path).
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


# rocprof kernel name (substring) -> timing group (dsce_api.hip Timed names)
GROUPS = (("k_jakes", "k_jakes"), ("k_tx_rows", "tx"), ("k_tx_symbols", "tx"), ("k_txrx_fft", "rx_front"),
          ("k_pic_fft", "perfect_ic"), ("k_poly_", "perfect_ic"), ("k_mic_pilot", "k_mic_pilot"),
          ("k_mic_data", "k_mic_data"), ("k_wpair3", "k_wcontract"), ("k_wrow3", "k_wcontract"),
          ("k_wcontract_valu", "k_wcontract"), ("k_pilot_pre", "k_pilot_pre"), ("k_stage", "k_stage"),
          ("k_precode", "k_stage"), ("k_ls", "k_stage"), ("k_detect", "k_stage"))


def short(name):
    n = name.replace("dsce::", "").replace("void ", "")
    return n[:n.index("(")] if "(" in n else n


def group_span(sdir):
    """Mean span (ns) of the i-th k_pic_fft / k_mic_pilot / k_mic_data dispatch
    triple in the stats run's kernel trace: first start to last end."""
    try:
        tr = one(os.path.join(sdir, "**", "*_kernel_trace.csv"))
    except SystemExit:                          # one(): no trace in this run
        return None
    rows = list(csv.DictReader(open(tr)))
    seq = {"k_pic_fft": [], "k_mic_pilot": [], "k_mic_data": []}
    for r in rows:
        n = r["Kernel_Name"]
        for k in seq:
            if k in n:
                seq[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    m = min(len(v) for v in seq.values())
    if not m:
        return None
    spans = [max(seq[k][i][1] for k in seq) - min(seq[k][i][0] for k in seq) for i in range(m)]
    return sum(spans) / len(spans)


def main_all(argv):
    tag, sdir, fdir, wdir, workload = argv[:5]
    sqdir = argv[5] if len(argv) > 5 else None
    from bench import source_hash
    out = os.path.join(ROOT, "profiles")
    stats = one(os.path.join(sdir, "**", "*_kernel_stats.csv"))
    shutil.copy(stats, os.path.join(out, tag + "_kernel_stats.csv"))
    avg = {short(r["Name"]): float(r["AverageNs"]) for r in csv.DictReader(open(stats))}

    def means(d, counter):
        acc = {}
        for r in csv.DictReader(open(one(os.path.join(d, "**", "*_counter_collection.csv")))):
            if r["Counter_Name"] == counter:
                acc.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
        return {k: sum(v) / len(v) for k, v in acc.items()}
    fetch, write = means(fdir, "FETCH_SIZE"), means(wdir, "WRITE_SIZE")
    sq = {c: means(sqdir, c) for c in SQ_COUNTERS} if sqdir else {}
    groups = {}
    for k in sorted(set(fetch) | set(avg)):
        g = next((grp for sub, grp in GROUPS if sub in k), None)
        if g is None:
            continue
        e = groups.setdefault(g, {"kernels": [], "fetch_size_kb_per_launch": 0.0, "write_size_kb_per_launch": 0.0,
                                  "avg_duration_ns_rocprof": 0.0, "sq_per_launch": {c: 0.0 for c in sq}})
        e["kernels"].append(k)
        e["fetch_size_kb_per_launch"] += fetch.get(k, 0.0)
        e["write_size_kb_per_launch"] += write.get(k, 0.0)
        e["avg_duration_ns_rocprof"] += avg.get(k, 0.0)
        for c in sq:
            e["sq_per_launch"][c] += sq[c].get(k, 0.0)
    # the IC group of the FFT-form OFDM path: its members' counters and, from
    # the stats run's kernel trace, the mean span first start -> last end of
    # each (pic, pilot, data) triple
    mem = [g for g in ("perfect_ic", "k_mic_pilot", "k_mic_data") if g in groups]
    if len(mem) == 3 and any("k_pic_fft" in k for k in groups["perfect_ic"]["kernels"]):
        e = {"kernels": sum((groups[g]["kernels"] for g in mem), []), "members": mem}
        for key in ("fetch_size_kb_per_launch", "write_size_kb_per_launch", "avg_duration_ns_rocprof"):
            e[key] = sum(groups[g][key] for g in mem)
        if sq:
            e["sq_per_launch"] = {c: sum(groups[g]["sq_per_launch"][c] for g in mem) for c in sq}
        e["span_ns_rocprof_trace"] = group_span(sdir)
        groups["ic_stages"] = e
    for e in groups.values():
        e["hbm_bytes_per_launch"] = (2 * e["fetch_size_kb_per_launch"] + e["write_size_kb_per_launch"]) * 1024
        if not sq:
            e.pop("sq_per_launch", None)
    res = {"workload": workload, "source_hash": source_hash(), "kernels": groups,
           "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE reports half of "
                         "wide coalesced reads, MI355X_MICROARCH.md §HBM)"}
    with open(os.path.join(out, "%s_pmc_all.json" % tag), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


def main():
    if sys.argv[1] == "--all":
        return main_all(sys.argv[2:])
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
