import sys, numpy as np
import harness
from dsce.configs import build_setup
from dsce.engine import build_engine
S = build_setup("c5", schemes=("fbmc_aux",), snr_db=[36.0])
sc = S.schemes["fbmc_aux"]
eng = build_engine(S, batch=64)
mm = harness.oracle_mmse(S, sc)
for var, key, R in ((0, "W", mm["R_est"][0]), (1, "W0", mm["R_noI"][0])):
    wg = eng.W(0, 0, var); wo = mm[key][:, 0]
    scale = np.abs(wo).max(); c = np.linalg.cond(R)
    d = np.abs(wg - wo)
    tol = max(1e-14 * c, 1e-12) * scale
    bad = d > tol
    print(key, 'cond %.3g scale %.3g maxdiff %.3g tol %.3g nbad %d' % (c, scale, d.max(), tol, bad.sum()))
    if bad.any():
        i = np.argsort(-d)[:8]
        for j in i:
            print('   idx', j, 'gpu', wg[j], 'ora', wo[j], '|wo|', abs(wo[j]), 'diff', d[j])
    # relative error estimate vs cond
    print('   maxdiff/(eps*cond*scale) = %.2f' % (d.max() / (2.2e-16 * c * scale)))
rg = eng.correlation(0)
print('R_noI diff', np.abs(rg[2] - mm['R_noI']).max(), 'R_est diff', np.abs(rg[1]-mm['R_est']).max(), 'R_hP', np.abs(rg[0]-mm['R_hP']).max())
