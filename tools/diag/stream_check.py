"""Counts with the perfect-CSI chain on a second stream equal the one-stream run."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, "channel-estimation_amd")
import numpy as np
import harness

S = harness.setup("default", schemes=("ofdm",))
a = harness.engine(S, batch=512)
b = harness.engine(S, batch=512, options={"pic_stream": 1})
ca = a.run(0x5EED, 0, 2048)
cb = b.run(0x5EED, 0, 2048)
print("equal:", np.array_equal(ca, cb), sorted(b.path_info(0)), flush=True)
a.close()
b.close()
