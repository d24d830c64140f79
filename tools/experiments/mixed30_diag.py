"""Diagnose test_lane_order_tile_map_30q_mixed: which part disagrees."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import quest_amd as qa
from quest_amd.models import random_mixed
from quest_amd.ops import capi

e = qa.Env()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
circ = random_mixed(n, 300, seed=78, high=8)
if len(sys.argv) > 2 and sys.argv[2] == "shadow":
    capi.setQuESTTuning("wave_shadow", 1)


def run(mode):
    capi.setQuESTTuning("tile_mode", mode)
    capi.resetQuESTStats()
    r = qa.Register(e, n)
    r.init_plus()
    circ.apply(r)
    r.sync()
    return r


ref = run(0)
a = run(3)
st = capi.getQuESTStats()
print("shadow checks", st["waveShadowChecks"], "mismatches", st["waveShadowMismatches"], "passes", st["passes"], flush=True)
print("layout moved", sum(1 for i, p in enumerate(capi.getQubitLayout(a.q)) if i != p), flush=True)
print("norm a", a.total_prob(), "norm ref", ref.total_prob(), flush=True)
pa = np.array([a.prob(q, 1) for q in range(n)])
pb = np.array([ref.prob(q, 1) for q in range(n)])
print("marginal maxdiff", np.max(np.abs(pa - pb)), flush=True)
print("amps", [abs(a.amp(i) - ref.amp(i)) for i in (0, 1, 12345, (1 << 29) + 77)], flush=True)
print("inner perm", a.inner(ref), flush=True)
b = qa.Register(e, n)
capi.cloneQureg(b.q, a.q)
print("inner clone (same layout)", a.inner(b), flush=True)
va = b.to_numpy()   # relayout of the clone
print("clone relayout vs amps", abs(va[12345] - ref.amp(12345)), flush=True)
vr = ref.to_numpy()
print("full maxdiff after relayout", np.max(np.abs(va - vr)), flush=True)
