"""In-process A/B of engine variants selected by an environment variable
(interleaved rounds, identical counts required).  usage: _ab_env.py SCHEME VAR V1 V2 ... [--batch B] [--reps N]"""
import os, sys, time, json
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0] = [R, R + '/channel-estimation_amd']
import numpy as np
from dsce.configs import build_setup
from dsce.engine import build_engine
args = sys.argv[1:]
batch = 16384; reps = 65536
if '--batch' in args: i = args.index('--batch'); batch = int(args[i + 1]); del args[i:i + 2]
if '--reps' in args: i = args.index('--reps'); reps = int(args[i + 1]); del args[i:i + 2]
scheme, var, vals = args[0], args[1], args[2:]
S = build_setup('default', schemes=(scheme,))
eng = build_engine(S, batch=batch)
eng.run(3, 0, batch)
res, ref = {}, None
names = ('k_jakes', 'tx', 'rx_front', 'k_wcontract', 'perfect_ic', 'k_stage')
for rnd in range(3):
    for v in vals:
        os.environ[var] = v
        eng.enable_timing(True)
        t = time.perf_counter(); c = eng.run(7, 0, reps); dt = time.perf_counter() - t
        kt = {k: round(eng.kernel_time(k)[1], 2) for k in names}
        eng.enable_timing(False)
        res.setdefault(v, []).append((round(reps / dt), kt))
        if ref is None: ref = c
        assert np.array_equal(c, ref), v
for v, r in res.items():
    print(v, json.dumps(max(r, key=lambda x: x[0])))
