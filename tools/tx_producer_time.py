"""Time G/Q production at the paper configuration: host mirror (L Modulation()
calls + GetRXMatrix) vs the on-GPU closed form (dsce_tx_matrices, row f1)."""
import os, sys, time, json
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, R + '/channel-estimation_amd']
from dsce.configs import build_setup
from dsce.engine import Engine
S = build_setup('paper', schemes=('fbmc_aux', 'ofdm'))
eng = Engine()
res = {}
for key in ('fbmc_aux', 'ofdm'):
    m = S.schemes[key].extras['modulation']
    t = time.perf_counter(); G = m.GetTXMatrix(); Q = m.GetRXMatrix().conj().T; th = time.perf_counter() - t
    eng.tx_matrices(m)
    t = time.perf_counter(); G2, Q2 = eng.tx_matrices(m); tg = time.perf_counter() - t
    res[key] = {'shape': list(G.shape), 'host_s': th, 'gpu_s_incl_copy_back': tg}
print(json.dumps(res))
