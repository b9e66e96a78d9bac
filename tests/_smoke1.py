import sys, time, numpy as np
import os; R=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0]=[R, R+'/channel-estimation_amd', R+'/tests']
from dsce.configs import build_setup
from dsce.engine import build_engine
S = build_setup('default', schemes=('ofdm',))
t=time.time(); eng = build_engine(S, batch=8192); print('setup s', time.time()-t, flush=True)
c = eng.run(1, 0, 64); print(c[0,:,0,:,:]/ (64*2560))
eng.enable_timing(True)
t=time.time(); c = eng.run(1, 0, 8192*4); dt=time.time()-t
print('reps/s', 8192*4/dt)
for k in ['k_jakes','tx','rx_front','k_wcontract','perfect_ic','k_stage']: print(k, eng.kernel_time(k))
