"""Paper configuration (script:42-46 uncommented: FBMC-OQAM 24 x 60, SR = 196 F,
N = 7350, NP = 32, 16 SNR points 10:2:40, VehA 500 km/h, 4 IC iterations):
BER of the auxiliary-symbol scheme against the points digitised from the
reference's published png/Figure3.png and png/Figure5.png.

usage: paper_run.py [--reps N] [--batch B] [--out FILE]"""
import argparse, json, os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, R + '/channel-estimation_amd']
import numpy as np
from dsce.configs import build_setup
from dsce.engine import build_engine
from dsce.published import compare

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--seed", type=int, default=0x5EED0005)
    ap.add_argument("--out", default=None)
    ap.add_argument("--setup-only", action="store_true")
    a = ap.parse_args()
    S = build_setup("paper", schemes=("fbmc_aux",))
    t0 = time.perf_counter()
    eng = build_engine(S, batch=a.batch)
    setup_s = time.perf_counter() - t0
    print(json.dumps({"setup_s": setup_s, "N": S.N, "LK": S.schemes["fbmc_aux"].LK,
                      "work_model": eng.work_model(0)}), flush=True)
    if a.setup_only:
        return
    counts = np.zeros(eng.counter_shape(), dtype=np.int64)
    done, t0 = 0, time.perf_counter()
    while done < a.reps:
        n = min(a.batch, a.reps - done)
        eng.run(a.seed, done, n, counts)
        done += n
        print(json.dumps({"reps": done, "s": round(time.perf_counter() - t0, 1)}), flush=True)
    el = time.perf_counter() - t0
    bits = eng.bits_per_rep(0)
    snr = [float(x) for x in S.snr_db]
    ber = counts[0] / np.array([bits[0], bits[1]], dtype=float)[None, :, None, None] / a.reps
    rows = compare(ber, snr)
    res = {"config": "paper (script:42-46): FBMC-OQAM aux 24x60, N=7350, NP=32, 16 SNR, NrIter 4",
           "reps": a.reps, "seconds": el, "reps_per_s": a.reps / el, "setup_s": setup_s, "snr_db": snr,
           "ber": ber.tolist(), "compare": rows}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    for r in rows:
        print("%-28s %5s %s  gpu %.4f  published %.4f  ratio %.2f" % (r["curve"], r["snr_db"], r.get("stage", ""),
                                                                       r["ber"], r["published"], r["ratio"]))


if __name__ == "__main__":
    main()
