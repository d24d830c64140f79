"""One flush of 8 two-qubit dephasing channels on a 17-qubit density matrix
(2^34 amplitudes; the density17 extra of bench.py): the time of its single
wave pass of 120 diagonal ops, for a rocprofv3 kernel trace."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import quest_amd as qa

n = 17
env = qa.Env()
d = qa.Register(env, n, density=True)
d.init_plus()
d.sync()
for rep in range(3):
    t0 = time.perf_counter()
    for q in range(0, n - 1, 2):
        d.dephase2(q, q + 1, 0.1)
    d.sync()
    print("dephase2 flush %.2f ms" % (1e3 * (time.perf_counter() - t0)), flush=True)
t0 = time.perf_counter()
for q in range(n):
    d.dephase(q, 0.1)
d.sync()
print("dephase flush %.2f ms" % (1e3 * (time.perf_counter() - t0)), flush=True)
