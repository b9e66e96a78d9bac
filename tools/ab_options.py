#!/usr/bin/env python3
"""In-process A/B of engine kernel options (dsce_set_option), interleaved rounds,
identical error counts required across variants.

usage: tools/ab_options.py SCHEME "name=v,name=v" "name=v" ... [--config default|c5]
       [--batch B] [--reps N] [--rounds K]
An empty variant string "" is the default path.  Prints per variant the best
realisations/s and the per-kernel HIP-event times of that round.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "channel-estimation_amd")]

import numpy as np  # noqa: E402

from dsce.configs import build_setup  # noqa: E402
from dsce.engine import build_engine  # noqa: E402

NAMES = ("k_jakes", "tx", "rx_front", "k_pilot_pre", "k_wcontract", "perfect_ic", "k_stage")


def parse(v):
    out = {}
    for kv in filter(None, v.split(",")):
        k, x = kv.split("=")
        out[k.strip()] = int(x)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scheme")
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--config", default="default")
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--reps", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    S = build_setup(a.config, schemes=(a.scheme,))
    eng = build_engine(S, batch=a.batch)
    defaults = {k: eng.get_option(k) for v in a.variants for k in parse(v)}
    eng.run(3, 0, a.batch)
    res, ref = {}, None
    for _ in range(a.rounds):
        for v in a.variants:
            for k, x in defaults.items():
                eng.set_option(k, x)
            for k, x in parse(v).items():
                eng.set_option(k, x)
            eng.enable_timing(True)
            t = time.perf_counter()
            c = eng.run(7, 0, a.reps)
            dt = time.perf_counter() - t
            kt = {k: round(eng.kernel_time(k)[1], 2) for k in NAMES}
            eng.enable_timing(False)
            res.setdefault(v, []).append((round(a.reps / dt), kt, sorted(eng.path_info(0))))
            if ref is None:
                ref = c
            assert np.array_equal(c, ref), v
    for v, r in res.items():
        print(repr(v), json.dumps(max(r, key=lambda x: x[0])), flush=True)


if __name__ == "__main__":
    main()
