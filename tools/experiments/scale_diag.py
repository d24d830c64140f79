import sys, time
sys.path.insert(0, "/root/repo")
import quest_amd as qa
from quest_amd.models import random_layered
from quest_amd.ops import capi
env = qa.Env()
for n in (int(a) for a in sys.argv[1:]):
    r = qa.Register(env, n); r.init_plus(); r.sync()
    c = random_layered(n, 6, seed=34)
    capi.resetQuESTStats(); t0 = time.perf_counter(); c.apply(r); r.sync(); dt = time.perf_counter() - t0
    st = capi.getQuESTStats()
    print(n, "qubits", len(c.gates), "gates", round(1e3 * dt / len(c.gates), 3), "ms/gate", {k: st[k] for k in ("passes", "wavePasses", "waveOps", "waveTransposes")}, flush=True)
    r.close()
