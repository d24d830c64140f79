"""QuEST_PREC=4 (long double) on the host build, as the reference allows it
(QuEST/include/QuEST_precision.h:36-45; QuEST/CMakeLists.txt:66-70 forbids it
on the GPU only): libQuEST_cpu_f128.so, with qreal = long double end to end
(the ctypes binding uses c_longdouble).  The gate, channel and marginal suites
run against the NumPy oracle in a child process bound to that library.  (The
reference's golden .test data hold inputs whose unitarity is only good to
~1e-13, above quad's REAL_EPS = 1e-14, so the golden suite is not run in quad,
and QASM prints parameters with the reference's "%.17Lg".)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHECK = r'''
import ctypes as C
import numpy as np
import quest_amd as qa
from quest_amd.ops import capi
b = capi.binding()
assert capi.getQuEST_PREC() == 4 and b.lib._quest_path.endswith("libQuEST_cpu_f128.so")
assert C.sizeof(b.Complex) == 2 * C.sizeof(C.c_longdouble)
e = qa.Env()
r = qa.Register(e, 3)
third = np.longdouble(1) / 3
re = np.array([third] + [0] * 7, dtype=np.longdouble)
im = np.zeros(8, dtype=np.longdouble)
P = C.POINTER(C.c_longdouble)
capi._call("setAmps", r.q, 0, re.ctypes.data_as(P), im.ctypes.data_as(P), 8)
out = np.empty(8, dtype=np.longdouble)
oi = np.empty(8, dtype=np.longdouble)
capi._call("copyChunkToBuffers", r.q, out.ctypes.data_as(C.c_void_p), oi.ctypes.data_as(C.c_void_p))
assert out[0] == third and out[0] != np.float64(third), out[0]   # more than double's 53 bits survive
print("quad ok")
'''


def test_quad_library_is_long_double():
    env = dict(os.environ, QUEST_PREC="4", QUEST_BACKEND="cpu")
    out = subprocess.run([sys.executable, "-c", CHECK], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0 and "quad ok" in out.stdout, out.stdout[-2000:] + out.stderr[-2000:]


def test_quad_gate_channel_marginal_suites():
    env = dict(os.environ, QUEST_PREC="4", QUEST_BACKEND="cpu")
    out = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                          "tests/test_gates.py", "tests/test_chan2_gates.py", "tests/test_dephase_diag.py",
                          "tests/test_marginals.py", "tests/test_validation.py"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
