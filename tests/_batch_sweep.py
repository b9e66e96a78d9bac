"""Throughput vs device batch size and per-scheme throughput (dev script)."""
import os, sys, time, json
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0] = [R, R + '/channel-estimation_amd']
from dsce.configs import build_setup
from dsce.engine import build_engine
out = {}
for scheme, reps in (('ofdm', 65536), ('fbmc_aux', 8192), ('fbmc_cod', 8192)):
    S = build_setup('default', schemes=(scheme,))
    eng = build_engine(S, batch=8192)
    for b in ((2048, 4096, 8192, 16384) if scheme == 'ofdm' else (2048, 8192)):
        eng.set_batch(b)
        eng.run(1, 0, b)
        eng.enable_timing(True)
        t = time.perf_counter(); eng.run(1, 0, reps); dt = time.perf_counter() - t
        kt = {k: round(eng.kernel_time(k)[1], 2) for k in ('k_jakes', 'tx', 'rx_front', 'k_wcontract', 'perfect_ic', 'k_stage')}
        eng.enable_timing(False)
        out['%s_b%d' % (scheme, b)] = {'reps_per_s': round(reps / dt), 'kernels_ms': kt}
        print(scheme, b, out['%s_b%d' % (scheme, b)], flush=True)
    eng.close()
