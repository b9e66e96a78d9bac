"""Print the structured-MMSE-IC guard values of the C2 OFDM scheme on the GPU."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, "channel-estimation_amd")
import numpy as np
import harness

S = harness.setup("default", schemes=("ofdm",))
for opts in ({}, {"mic_lr": 0}):
    eng = harness.engine(S, batch=256, options=opts)
    eng.run(0x5EED, 0, 256)
    print(opts, sorted(eng.path_info(0)), eng.structured_check(0), flush=True)
    eng.close()
