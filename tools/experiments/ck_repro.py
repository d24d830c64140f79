"""Reproduce the r2 non-unitary result: tests/test_gpu.py checkpoint test
(24-qubit random_layered, 2 layers, seed 2) with diagnostics."""
import os, sys, tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import quest_amd as qa
from quest_amd.models import random_layered
from quest_amd.ops import capi

e = qa.Env()
shadow = int(os.environ.get("SHADOW", "0"))
capi.setQuESTTuning("wave_shadow", shadow)
for it in range(int(os.environ.get("ITERS", "1"))):
    r = qa.Register(e, 24)
    r.init_plus()
    capi.resetQuESTStats()
    random_layered(24, 2, seed=2).apply(r)
    r.sync()
    st = capi.getQuESTStats()
    lay = r.layout() if hasattr(r, "layout") else None
    n1 = r.total_prob()
    v = r.to_numpy()
    n2 = float(np.sum(np.abs(v) ** 2))
    with tempfile.TemporaryDirectory() as d:
        r.save(os.path.join(d, "ck"))
        s = qa.Register(e, 24)
        s.load(os.path.join(d, "ck"))
        ip = s.inner(r)
        ip2 = r.inner(r)
        ns = s.total_prob()
        s.close()
    print(f"it {it}: passes {st['passes']} wave {st['wavePasses']} shadow {st['waveShadowChecks']}/"
          f"{st['waveShadowMismatches']} norm(calc) {n1:.15f} norm(numpy) {n2:.15f} <s|r> {ip.real:.15f} "
          f"<r|r> {ip2.real:.15f} norm(s) {ns:.15f}", flush=True)
    r.close()
