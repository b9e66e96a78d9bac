"""Sweep (engine batch, DSCE_SNR_CHUNK) for one scheme; counts must be identical.
usage: _chunk_sweep.py SCHEME B:C [B:C ...] [--reps N]"""
import os, sys, time, json
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0] = [R, R + '/channel-estimation_amd']
import numpy as np
from dsce.configs import build_setup
from dsce.engine import build_engine
args = sys.argv[1:]
reps = 131072
if '--reps' in args: i = args.index('--reps'); reps = int(args[i + 1]); del args[i:i + 2]
scheme, cfgs = args[0], args[1:]
S = build_setup('default', schemes=(scheme,))
names = ('k_jakes', 'tx', 'rx_front', 'k_wcontract', 'perfect_ic', 'k_stage')
ref = None
for cfg in cfgs:
    b, ch = (int(x) for x in cfg.split(':'))
    os.environ['DSCE_SNR_CHUNK'] = str(ch)
    eng = build_engine(S, batch=b)
    eng.run(3, 0, b)
    best = None
    for rnd in range(2):
        eng.enable_timing(True)
        t = time.perf_counter(); c = eng.run(7, 0, reps); dt = time.perf_counter() - t
        kt = {k: round(eng.kernel_time(k)[1], 2) for k in names}
        eng.enable_timing(False)
        if ref is None: ref = c
        assert np.array_equal(c, ref), cfg
        if best is None or reps / dt > best[0]: best = (round(reps / dt), kt)
    print(cfg, json.dumps(best), flush=True)
    del eng
