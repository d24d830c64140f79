"""The 37-qubit / 8-GPU configuration's per-rank footprint on real HBM, and a
near-capacity distributed run on one GPU.

The reference's distributed layer keeps a full pairStateVec and exchanges
whole chunks (QuEST_cpu_distributed.c:451-479); this design exchanges slices
through bounded buffers instead (router::memoryPlan).  On one MI355X:

* a 34-qubit register (256 GiB, one rank's chunk of 37 qubits on 8 ranks)
  next to the exchange buffers of the 8-rank plan's k = 3 all-to-all (14 x 2
  buffers of 64 MiB), with an RCCL communicator up and the pipelined exchange
  run through those buffers (runFootprintCheck);
* two RCCL ranks sharing the GPU (QUEST_RCCL_SHARED_GPU=1) at 33 local
  qubits each (2 x 128 GiB): a k = 1 swap, the norm and marginals against a
  single-rank 34-qubit run of the same gates.

Reports go to gpurun_out/ when that directory exists (GPU box runs)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")

FOOT = r'''
import quest_amd as qa
from quest_amd.ops import capi
e = qa.Env()
plan = capi.getQuregMemoryPlan(37, 8)
r = qa.Register(e, 34)
r.init_plus()
r.h(33)
r.h(0)
ok, rep = capi.runFootprintCheck(37, 8)
print("REPORT " + rep)
print("PLAN %d %d %d %d" % (plan["state"], plan["exchange"], plan["scratch"], plan["total"]))
print("OK %d NORM %.15f" % (ok, r.total_prob()))
'''

GATES = r'''
import json, os
import quest_amd as qa
from quest_amd.ops import capi
e = qa.Env()
n = 34
r = qa.Register(e, n)
r.init_plus()
r.ry(0, 0.3)
r.ry(33, 0.7)        # a rank qubit on 2 ranks: a k = 1 swap
r.cnot(33, 1)
r.rx(32, 0.5)
r.t(33)
vals = {"norm": r.total_prob(), "p33": r.prob(33, 1), "p0": r.prob(0, 1), "p1": r.prob(1, 1),
        "p32": r.prob(32, 1)}
for i in (0, 5, (1 << 33) + 7):
    a = r.amp(i)
    vals["amp%d" % i] = [a.real, a.imag]
st = capi.getQuESTStats()
vals["swaps"], vals["bytes"] = st["swaps"], st["bytesExchanged"]
vals["ranks"], vals["transport"] = e.num_ranks, capi.getQuESTTransport()
if e.rank == 0:
    print("VALS " + json.dumps(vals))
'''


def _save(name, text):
    if os.path.isdir(OUT):
        with open(os.path.join(OUT, name), "w") as f:
            f.write(text)


@pytest.mark.gpu
def test_37_qubit_per_rank_footprint_on_one_gpu():
    env = dict(os.environ, QUEST_BACKEND="hip")
    out = subprocess.run([sys.executable, "-c", FOOT], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=400)
    _save("footprint_37q_8r.txt", out.stdout + out.stderr[-3000:])
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "OK 1" in out.stdout, out.stdout
    norm = float(out.stdout.split("NORM")[1])
    assert abs(norm - 1) < 1e-10
    rep = [ln for ln in out.stdout.splitlines() if ln.startswith("REPORT")][0]
    assert "exchange through the caller's 14 x 2 buffers" in rep and "WRONG" not in rep, rep


@pytest.mark.gpu
def test_two_rccl_ranks_at_33_local_qubits_on_one_gpu():
    from quest_amd.parallel import spawn_local

    env = {"QUEST_BACKEND": "hip", "QUEST_COMM": "rccl", "QUEST_RCCL_SHARED_GPU": "1", "QUEST_COMM_TIMEOUT": "400",
           "OMP_NUM_THREADS": "1", "PYTHONPATH": ROOT}
    res = spawn_local(["-c", GATES], 2, env_extra=env, timeout=450)
    for r, p in enumerate(res):
        assert p.returncode == 0, f"rank {r}:\n{p.stdout[-2000:]}\n{p.stderr[-3000:]}"
    dist = json.loads([ln for ln in res[0].stdout.splitlines() if ln.startswith("VALS")][0][5:])
    one = subprocess.run([sys.executable, "-c", GATES], cwd=ROOT, env=dict(os.environ, QUEST_BACKEND="hip"),
                         capture_output=True, text=True, timeout=300)
    assert one.returncode == 0, one.stdout[-2000:] + one.stderr[-3000:]
    single = json.loads([ln for ln in one.stdout.splitlines() if ln.startswith("VALS")][0][5:])
    _save("rccl_2x33_vs_1x34.txt", json.dumps({"two_ranks": dist, "one_rank": single}, indent=1))
    assert dist["ranks"] == 2 and dist["transport"].startswith("RCCL"), dist
    assert dist["swaps"] >= 1 and dist["bytes"] > 0, dist
    for k in ("norm", "p33", "p0", "p1", "p32", "amp0", "amp5", "amp%d" % ((1 << 33) + 7)):
        a, b = dist[k], single[k]
        a = a if isinstance(a, list) else [a]
        b = b if isinstance(b, list) else [b]
        assert max(abs(x - y) for x, y in zip(a, b)) < 1e-12, (k, a, b)
