"""In-process A/B of the MMSE contraction variants (interleaved rounds)."""
import os, sys, time, json
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0] = [R, R + '/channel-estimation_amd']
import numpy as np
from dsce.configs import build_setup
from dsce.engine import build_engine
cfg = sys.argv[1] if len(sys.argv) > 1 else 'ofdm'
S = build_setup('default', schemes=(cfg,))
eng = build_engine(S, batch=8192)
eng.enable_timing(True)
res = {}
ref = None
for rnd in range(3):
    for mode in ('mfma', 'valu'):
        os.environ['DSCE_WCONTRACT'] = mode
        n0, t0 = eng.kernel_time('k_wcontract')
        c = eng.run(7, 0, 8192 * 2)
        n1, t1 = eng.kernel_time('k_wcontract')
        res.setdefault(mode, []).append((t1 - t0) / (n1 - n0))
        if ref is None: ref = c
        assert np.array_equal(c, ref), mode
cm, wb = eng.work_model(0)
fl = cm / S.n_iter * 8192 * 8
print(json.dumps({m: {"ms": [round(x, 4) for x in v], "tflops": round(fl / (min(v) * 1e-3) / 1e12, 2)} for m, v in res.items()}))
