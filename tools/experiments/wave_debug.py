#!/usr/bin/env python3
"""Debug probes of the wave-tile kernel on the GPU: with QUEST_WAVE_NOOPS=1
every wave pass only loads and stores its tiles, so a stream of diagonal
gates (one pass) must leave the state unchanged."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import quest_amd as qa  # noqa: E402
from helpers import load_state  # noqa: E402
from quest_amd.ops import capi  # noqa: E402
from quest_amd.utils import oracle as O  # noqa: E402

env = qa.Env()
capi.setQuESTTuning("tile_mode", 3)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 18
rng = np.random.default_rng(1)
v = O.random_state(rng, n)
reg = qa.Register(env, n)
load_state(reg, v)
capi.resetQuESTStats()
for q in range(n):
    reg.z(q)
got = reg.to_numpy()
st = capi.getQuESTStats()
print("stats", st)
d = np.abs(got - v)
print("max diff vs input", d.max(), "wrong amps", int((d > 1e-12).sum()), "of", len(v))
bad = np.nonzero(d > 1e-12)[0][:16]
print("first wrong indices", bad.tolist())
if len(bad):
    for i in bad[:4]:
        j = np.nonzero(np.abs(v - got[i]) < 1e-14)[0]
        print(f"  got[{i}] equals input at {j.tolist()[:4]}")
