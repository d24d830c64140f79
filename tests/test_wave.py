"""Wave-tile engine (src/core/wave.hpp planner, tools/gen_wave_asm.py
kernel): the host emulation of its plans (QUEST_CPU_PLANNER=3, same lanes /
register slots / transpositions as the GPU kernel) against the NumPy oracle
on CPU, and the assembly kernel itself against the oracle and against the
LDS tile kernel on the GPU."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra, timeout=600):
    env = dict(os.environ, **env_extra)
    return subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_wave_plans_emulated_on_host_every_gate_kind():
    out = _run([os.path.join(ROOT, "tools", "wave_kinds.py"), "--qubits", "15", "--count", "40"],
               {"QUEST_BACKEND": "cpu", "QUEST_CPU_PLANNER": "3"})
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    assert "bad: []" in out.stdout
    # every kind really ran through wave passes
    assert " wave 0 " not in out.stdout, out.stdout


@pytest.mark.parametrize("knobs", [{"QUEST_WAVE_LANE_OPS": "0"}, {"QUEST_WAVE_LANE_ORDER": "0"},
                                   {"QUEST_WAVE_LANE_ORDER": "2"}, {"QUEST_WAVE_CMIN": "7"}])
def test_wave_plan_variants_emulated_on_host(knobs):
    """Planner variants (lane-bit gates off, lane / wave bit assignment
    orders, more always-in-tile bits) give the same states."""
    out = _run([os.path.join(ROOT, "tools", "wave_kinds.py"), "--qubits", "15", "--count", "24",
                "--kinds", "h,x,y,rx,ry,rz,t,cnot,cy,cz,ccompact,mcunitary"],
               dict({"QUEST_BACKEND": "cpu", "QUEST_CPU_PLANNER": "3"}, **knobs))
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    assert "bad: []" in out.stdout


def test_wave_plans_emulated_on_host_random_streams():
    """Random mixed streams (all gate kinds, controls on any bit) and the
    fusion / golden suites through the wave planner."""
    out = _run(["-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", os.path.join(ROOT, "tests", "test_fusion.py"),
                "-k", "not emulated"], {"QUEST_BACKEND": "cpu", "QUEST_CPU_PLANNER": "3"}, timeout=900)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]


@pytest.mark.gpu
def test_wave_kernel_every_gate_kind_gpu():
    out = _run([os.path.join(ROOT, "tools", "wave_kinds.py"), "--qubits", "21", "--count", "40"], {}, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    assert "bad: []" in out.stdout and " wave 0 " not in out.stdout


@pytest.mark.gpu
def test_fp32_wave_kernel_every_gate_kind_gpu():
    """The fp32 wave kernel (--prec 1: one VGPR per value, 32 amplitudes per
    lane, tile bits 0-1 in the 16-byte vector) per gate kind against the
    oracle, in a subprocess bound to the fp32 HIP library."""
    out = _run([os.path.join(ROOT, "tools", "wave_kinds.py"), "--qubits", "22", "--count", "40"],
               {"QUEST_PREC": "1", "QUEST_BACKEND": "hip"}, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    assert "bad: []" in out.stdout and " wave 0 " not in out.stdout


FP32_DENSITY = r'''
import sys
import numpy as np
sys.path.insert(0, "tests")
import quest_amd as qa
from helpers import apply_random_ops, oracle_for, state_of
from quest_amd.utils import oracle as O
env = qa.Env()
n = 10
rng = np.random.default_rng(310)
reg = qa.Register(env, n, density=True)
o = oracle_for(reg, rng)
qa.capi.resetQuESTStats()
apply_random_ops(reg, o, rng, 30)
for k in range(40):
    a = int(rng.integers(n))
    p = float(rng.uniform(0, 0.5))
    pair = [(reg.dephase, o.dephase), (reg.depolarise, o.depolarise), (reg.damping, o.damping)][k % 3]
    pair[0](a, p)
    pair[1](a, p)
    if k % 5 == 0:
        reg.h(a)
        o.apply(O.H, a)
reg.sync()
st = qa.capi.getQuESTStats()
assert st["wavePasses"] > 0 and st["wavePasses"] == st["passes"], st
err = float(np.max(np.abs(state_of(reg) - o.rho)))
print("err", err)
assert err < 2e-6, err
'''


@pytest.mark.gpu
def test_fp32_density_channels_on_wave_engine_gpu():
    """fp32 one-qubit channels (CH1 / CHD, packed math on register pairs)
    and gates on a 10-qubit density matrix on the wave engine, against the
    NumPy oracle to fp32 precision."""
    out = _run(["-c", FP32_DENSITY], {"QUEST_PREC": "1", "QUEST_BACKEND": "hip"}, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]


@pytest.mark.gpu
def test_fp32_wave_matches_fp64_layered_24q_gpu():
    """A 24-qubit random layered circuit on the fp32 wave engine agrees with
    the fp64 library to fp32 precision (and ran on wave passes)."""
    code = ("import numpy as np, quest_amd as qa\n"
            "from quest_amd.models import random_layered\n"
            "e = qa.Env(); r = qa.Register(e, 24); r.init_plus(); qa.capi.resetQuESTStats()\n"
            "random_layered(24, 12, seed=5).apply(r); r.sync()\n"
            "st = qa.capi.getQuESTStats(); assert st['wavePasses'] > 0, st\n"
            "np.save('{out}', r.to_numpy().astype(np.complex128))\n")
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        res = {}
        for prec in ("1", "2"):
            f = os.path.join(d, f"s{prec}.npy")
            out = _run(["-c", code.format(out=f)], {"QUEST_PREC": prec, "QUEST_BACKEND": "hip"}, timeout=300)
            assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
            res[prec] = np.load(f)
        err = np.max(np.abs(res["1"] - res["2"]))
        assert err < 1e-5 * 2 ** -12 * 40, err   # amplitudes ~2^-12, fp32 per-gate rounding


@pytest.mark.gpu
def test_static_ctrl_cnot_handlers_match_generic_gpu():
    """CNOTs with one slot control (both polarities: X gates before them put
    their control bits in the exchange frame) through the fixed-register swk
    handlers give bit-for-bit the state of the generic mask-tested handler
    (QUEST_WAVE_STATIC_CTRL=0): the two only move data."""
    code = ("import numpy as np, quest_amd as qa\n"
            "from quest_amd.models import random_layered\n"
            "e = qa.Env(); r = qa.Register(e, 22); r.init_plus(); qa.capi.resetQuESTStats()\n"
            "random_layered(22, 12, seed=11).apply(r); r.sync()\n"
            "st = qa.capi.getQuESTStats(); assert st['wavePasses'] > 0, st\n"
            "np.save('{out}', r.to_numpy())\n")
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        res = {}
        for v in ("0", "1"):
            f = os.path.join(d, f"s{v}.npy")
            out = _run(["-c", code.format(out=f)], {"QUEST_WAVE_STATIC_CTRL": v, "QUEST_BACKEND": "hip"}, timeout=300)
            assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
            res[v] = np.load(f)
        assert np.array_equal(res["0"], res["1"])
        assert abs(np.vdot(res["1"], res["1"]).real - 1) < 1e-12


@pytest.mark.gpu
def test_wave_kernel_matches_lds_kernel_gpu(env):
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    n = 22
    outs = {}
    for mode in (0, 3):
        capi.setQuESTTuning("tile_mode", mode)
        reg = qa.Register(env, n)
        reg.init_plus()
        capi.resetQuESTStats()
        random_layered(n, 8, seed=5).apply(reg)
        outs[mode] = reg.to_numpy()
        st = capi.getQuESTStats()
        if mode == 3:
            assert st["wavePasses"] > 0
        reg.close()
    capi.setQuESTTuning("tile_mode", 3)
    assert np.max(np.abs(outs[0] - outs[3])) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("n", [24, 25])
def test_looping_grids_match_one_tile_grid_gpu(env, n):
    """Looping wave grids (workgroups that claim tiles from a counter, and
    with a --pfa / --pfl image the next-tile prefetch: tools/gen_wave_asm.py
    dyn_claim / pf_paths) give bit for bit the state of one workgroup per
    tile and of the static stride (QUEST_WAVE_DYNAMIC=0).  24 and 25 qubits:
    2048 / 4096 tiles over 768 resident workgroups (uneven claims)."""
    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    outs = {}
    for name, per, dyn in (("one", 0, 1), ("static", 3, 0), ("default", -1, 1)):
        capi.setQuESTTuning("wave_wg_per_cu", per)
        capi.setQuESTTuning("wave_dynamic", dyn)
        reg = qa.Register(env, n)
        reg.init_plus()
        capi.resetQuESTStats()
        random_layered(n, 10, seed=n).apply(reg)
        outs[name] = reg.to_numpy()
        assert capi.getQuESTStats()["wavePasses"] > 0
        reg.close()
    capi.setQuESTTuning("wave_wg_per_cu", -1)
    capi.setQuESTTuning("wave_dynamic", 1)
    assert np.array_equal(outs["one"], outs["default"])
    assert np.array_equal(outs["one"], outs["static"])
    assert abs(np.vdot(outs["default"], outs["default"]).real - 1) < 1e-12


XFRAME = r'''
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
import quest_amd as qa
from helpers import GATES_1Q, GATES_2Q, GATES_MQ, apply_named, oracle_for, random_qubits

env = qa.Env()
n = 16
rng = np.random.default_rng(int(sys.argv[2]))
r = qa.Register(env, n)
o = oracle_for(r, rng)
names = GATES_1Q + GATES_2Q + GATES_MQ
for step in range(300):
    # an X, then gates that may use its qubit as target, control or phase mask
    q = int(rng.integers(n))
    apply_named(r, o, "x", [q], rng)
    for _ in range(int(rng.integers(1, 4))):
        name = names[rng.integers(len(names))]
        k = 1 if name in GATES_1Q else 2 if name in GATES_2Q else int(rng.integers(2, 5))
        qs = random_qubits(rng, n, k)
        if rng.random() < 0.6 and q not in qs:
            qs[int(rng.integers(k))] = q
        apply_named(r, o, name, qs, rng)
err = np.max(np.abs(r.to_numpy() - o.v))
print("xframe err", err)
assert err < 1e-10, err
'''


CFRAME = r'''
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
import quest_amd as qa
from helpers import GATES_1Q, GATES_2Q, GATES_MQ, apply_named, oracle_for, random_qubits

env = qa.Env()
n = int(sys.argv[3])
rng = np.random.default_rng(int(sys.argv[2]))
r = qa.Register(env, n)
o = oracle_for(r, rng)
names = GATES_1Q + GATES_2Q + GATES_MQ
for step in range(250):
    # a CNOT (deferred as a conditional flip), then gates on / controlled by /
    # phased on its control or target -- X and Y on the control toggle flips
    c, t = random_qubits(rng, n, 2)
    apply_named(r, o, "cnot", [c, t], rng)
    for _ in range(int(rng.integers(1, 4))):
        q = c if rng.random() < 0.5 else t
        if rng.random() < 0.3:
            apply_named(r, o, ["x", "y", "z"][int(rng.integers(3))], [q], rng)
            continue
        name = names[rng.integers(len(names))]
        k = 1 if name in GATES_1Q else 2 if name in GATES_2Q else int(rng.integers(2, 5))
        qs = random_qubits(rng, n, k)
        if q not in qs:
            qs[int(rng.integers(k))] = q
        apply_named(r, o, name, qs, rng)
err = np.max(np.abs(r.to_numpy() - o.v))
print("cframe err", err)
assert err < 1e-10, err
'''


@pytest.mark.parametrize("cframe", ["1", "0"])
def test_conditional_frame_emulated_on_host(cframe):
    """Deferred CNOTs (planWavePass conditional flips): each CNOT followed by
    gates that use its control or target as target, control or phase mask,
    and X / Y / Z on them (a physical X on an exchanged condition bit must
    toggle the flips it conditions -- the 30-qubit GPU failure of round 4), on
    the wave planner's host emulation against the NumPy oracle;
    QUEST_WAVE_CFRAME=0 executes every CNOT."""
    for seed, n in ((1, 16), (2, 20), (3, 20)):
        out = _run(["-c", CFRAME, ROOT, str(seed), str(n)],
                   {"QUEST_BACKEND": "cpu", "QUEST_CPU_PLANNER": "3", "QUEST_WAVE_CFRAME": cframe})
        assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
        assert "cframe err" in out.stdout


@pytest.mark.gpu
def test_conditional_frame_gpu():
    """The conditional-frame stress on the GPU kernel (22 qubits)."""
    out = _run(["-c", CFRAME, ROOT, "4", "22"], {"QUEST_BACKEND": "hip"}, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "cframe err" in out.stdout


@pytest.mark.parametrize("frame", ["1", "0"])
def test_exchange_frame_emulated_on_host(frame):
    """Deferred X gates (planWavePass exchange frame): X on random qubits
    followed by gates that use that qubit as target, control (register, lane
    and wave bits) or phase mask, on the wave planner's host emulation,
    against the NumPy oracle; QUEST_WAVE_XFRAME=0 executes every X."""
    for seed in (1, 2):
        out = _run(["-c", XFRAME, ROOT, str(seed)],
                   {"QUEST_BACKEND": "cpu", "QUEST_CPU_PLANNER": "3", "QUEST_WAVE_XFRAME": frame})
        assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
        assert "xframe err" in out.stdout


@pytest.mark.gpu
def test_exchange_frame_gpu():
    """The exchange-frame stress on the GPU kernel (20 qubits: wave passes),
    against the NumPy oracle."""
    script = XFRAME.replace("n = 16", "n = 20")
    out = _run(["-c", script, ROOT, "3"], {"QUEST_BACKEND": "hip"}, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "xframe err" in out.stdout


RACE = r'''
import sys
import quest_amd as qa
from quest_amd.models import random_layered
e = qa.Env()
r = qa.Register(e, 24)
r.init_plus()
random_layered(24, 2, seed=2).apply(r)
print("norm %.15f" % r.total_prob())
'''


@pytest.mark.parametrize("barrier", [True, False])
def test_emulation_orders_waves_like_the_kernel(barrier):
    """Round-2's GPU-only wrong result (lane order 2: <psi|psi> = 1.0022 on
    the 24-qubit checkpoint circuit) was a race between the waves of a
    workgroup: a relabelling pass without wave-bit transpositions moved tile
    bits held by wave bits, so each wave stored onto addresses another wave
    had not loaded yet.  The emulation now runs such passes wave by wave (the
    worst legal order) unless the plan carries the store barrier: planned as
    in round 2 (QUEST_WAVE_NO_STORE_BARRIER=1) it loses unitarity like the
    kernel did; planned with the barrier it is exact."""
    # QUEST_DIAG_PHASES=0, QUEST_WAVE_CFRAME=0: the round-2 planner's plan of this short queue
    env = {"QUEST_BACKEND": "cpu", "QUEST_CPU_PLANNER": "3", "QUEST_WAVE_LANE_ORDER": "2", "QUEST_DIAG_PHASES": "0",
           "QUEST_WAVE_CFRAME": "0"}
    if not barrier:
        env["QUEST_WAVE_NO_STORE_BARRIER"] = "1"
    out = _run(["-c", RACE], env)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    norm = float(out.stdout.split("norm")[1])
    if barrier:
        assert abs(norm - 1) < 1e-11, norm
    else:
        assert abs(norm - 1) > 1e-3, norm


FRONT = r'''
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import quest_amd as qa
from quest_amd.models import random_layered
from quest_amd.ops import capi
from quest_amd.utils import oracle as O
n = 20
e = qa.Env()
r = qa.Register(e, n)
r.init_plus()
c = random_layered(n, 36, seed=int(sys.argv[2]))
capi.resetQuESTStats()
c.apply(r)
r.sync()
st = capi.getQuESTStats()
o = O.StateVector(n, np.full(1 << n, 2 ** (-n / 2)))
c.apply_oracle(o)
err = np.abs(r.to_numpy() - o.v).max()
print("front gates %d flushes %d passes %d err %.3e" % (len(c.gates), st["flushes"], st["passes"], err))
assert err < 1e-10, err
'''


def _front(backend, seed, front, **extra):
    env = dict({"QUEST_BACKEND": backend, "QUEST_FRONT_FLUSH": front}, **extra)
    if backend == "cpu":
        env["QUEST_CPU_PLANNER"] = "3"
    out = _run(["-c", FRONT, ROOT, str(seed)], env, timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    f = out.stdout.split("front")[1].split()
    return {f[i]: float(f[i + 1]) for i in range(0, len(f), 2)}


@pytest.mark.parametrize("front", ["0", "512", "128"])
def test_front_flush_emulated_on_host(front):
    """Front flushes (QUEST_FRONT_FLUSH: once that many ops are queued, the
    first pass is planned with the whole queue as lookahead and runs while
    the program keeps issuing gates; the rest stays queued in the layout the
    pass leaves): a 20-qubit, 36-layer circuit (~1100 gates: front flushes,
    the queue limit and the final sync) on the wave planner's host emulation
    against the NumPy oracle."""
    d = _front("cpu", 3, front)
    if front != "0":
        assert d["flushes"] > 3, d    # front flushes happened (not just queue-limit + sync)


@pytest.mark.gpu
def test_front_flush_gpu():
    """The same on the GPU kernel."""
    for front in ("512", "128"):
        d = _front("hip", 4, front)
        assert d["flushes"] > 3, d


PHASES = r'''
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import quest_amd as qa
from quest_amd.models.circuits import Circuit, random_mixed
from quest_amd.ops import capi
from quest_amd.utils import oracle as O
n = 18
e = qa.Env()
r = qa.Register(e, n)
r.init_plus()
c = random_mixed(n, 480, seed=int(sys.argv[2]), high=6)
capi.resetQuESTStats()
# short windows (a read every 24 gates), where QUEST_DIAG_PHASES=2 lowers
# the diagonal gates to phase ops
for i in range(0, len(c.gates), 24):
    part = Circuit(n)
    part.gates = c.gates[i:i + 24]
    part.apply(r)
    r.sync()
st = capi.getQuESTStats()
o = O.StateVector(n, np.full(1 << n, 2 ** (-n / 2)))
c.apply_oracle(o)
err = np.abs(r.to_numpy() - o.v).max()
print("phases passes %d err %.3e" % (st["passes"], err))
assert err < 1e-10, err
'''


def _phases(backend, mode, seed):
    env = {"QUEST_BACKEND": backend, "QUEST_DIAG_PHASES": mode}
    if backend == "cpu":
        env["QUEST_CPU_PLANNER"] = "3"
    out = _run(["-c", PHASES, ROOT, str(seed)], env, timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    return int(out.stdout.split("passes")[1].split()[0])


@pytest.mark.parametrize("mode", ["0", "1", "2"])
def test_diagonal_gates_as_phases_emulated_on_host(mode):
    """QUEST_DIAG_PHASES (tiles.cpp phasesFromDiagonals: a unit-modulus
    diagonal gate -- Z, S, T, Rz, phase shifts, their controlled and
    multi-controlled forms -- becomes phase ops that need no tile bit): mixed
    random gates in short windows on the host emulation against the oracle,
    never, always and for short queues (default)."""
    passes = _phases("cpu", mode, 11)
    assert passes > 0


@pytest.mark.gpu
def test_diagonal_gates_as_phases_gpu():
    """The same on the GPU kernel; lowering never costs passes here."""
    never, always = _phases("hip", "0", 12), _phases("hip", "1", 12)
    assert always <= never, (always, never)


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"QUEST_CACHED_STATE_MB": "0"}, {"QUEST_CACHED_STATE_MB": "4096"},
                                 {"QUEST_SYNC_SPIN": "1"}])
def test_unfused_kernel_variants_gpu(env):
    """The unfused direct kernels with non-temporal accesses at every size
    (QUEST_CACHED_STATE_MB=0) and with plain, cache-resident accesses for the
    whole 18-qubit state (4096), and spinning host waits: mixed random gates
    against the oracle."""
    out = _run(["-c", PHASES, ROOT, "13"], dict({"QUEST_BACKEND": "hip", "QUEST_FUSION": "0"}, **env))
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]


def test_cmin_search_emulated_on_host():
    """QUEST_WAVE_CMIN_SEARCH=1 (each window planned with 6 or 7 always-resident
    low positions, whichever gives fewer passes) on the host emulation
    against the NumPy oracle."""
    _front("cpu", 5, "512", QUEST_WAVE_CMIN_SEARCH="1")
