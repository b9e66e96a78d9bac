#!/usr/bin/env python3
"""Summarise tools/gpu_census.sh: per kernel, the per-launch mean of every
counter collected and the per-wave figures (counter / SQ_WAVES).

usage: census.py gpurun_out/census_TAG [KERNEL_SUBSTR ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    pats = sys.argv[2:] or ["k_pic_fft", "k_mic_data", "k_mic_pilot", "k_txrx_fft", "k_jakes_grp", "k_tx_rows"]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            for p in pats:
                if p in name:
                    acc[p][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for p in pats:
        c = {k: sum(v) / len(v) for k, v in acc[p].items()}
        if not c:
            continue
        waves = c.get("SQ_WAVES")
        print("== %s (%d counters)" % (p, len(c)))
        for k in sorted(c):
            per_wave = c[k] / waves if waves and k.startswith("SQ_INSTS") else None
            print("  %-32s %16.4g %s" % (k, c[k], ("  per wave %10.1f" % per_wave) if per_wave else ""))


if __name__ == "__main__":
    main()
