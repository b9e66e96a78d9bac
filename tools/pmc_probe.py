"""Small C2 OFDM workload for rocprofv3 counter passes: build, warm up, run
two device batches.  usage: pmc_probe.py [batch] [scheme]"""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0] = [R, R + '/channel-estimation_amd']
from dsce.configs import build_setup
from dsce.engine import build_engine
b = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
scheme = sys.argv[2] if len(sys.argv) > 2 else 'ofdm'
eng = build_engine(build_setup('default', schemes=(scheme,)), batch=b)
eng.run(3, 0, b)
eng.run(7, 0, 2 * b)
print('ok')
