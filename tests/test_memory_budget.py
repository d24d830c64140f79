"""Per-rank memory budget of createQureg (quest_amd.h getQuregMemoryPlan):
the plan's arithmetic for the 37-qubit / 8-GPU configuration, and the
E_OUT_OF_MEMORY refusal with a breakdown when the (overridden) free device
memory is too small -- checked in subprocesses because the override is read
at create time from the environment."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code, **env):
    e = dict(os.environ, QUEST_BACKEND="cpu", PYTHONPATH=ROOT, **env)
    return subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=120, cwd=ROOT)


def test_plan_single_rank():
    from quest_amd.ops import capi

    p = capi.getQuregMemoryPlan(30)
    assert p["state"] == 2 * 8 * (1 << 30)
    assert p["exchange"] == 0
    assert p["total"] == p["state"] + p["exchange"] + p["scratch"]


def test_plan_37_qubits_on_8_ranks_fits_one_mi355x():
    """37 qubits over 8 ranks: 2^34 amplitudes (256 GiB) per rank plus the
    all-to-all slice buffers of a 3-qubit swap: 7 peers x 2 x 2 x 32 MiB.
    The total must stay below one MI355X's 288 GB."""
    from quest_amd.ops import capi

    p = capi.getQuregMemoryPlan(37, 8)
    slice_amps = (256 << 20 >> 2) // 16
    assert p["state"] == 2 * 8 * (1 << 34)  # 256 GiB
    assert p["exchange"] == 2 * 2 * 7 * slice_amps * 2 * 8 == 7 * (1 << 28)  # 1.75 GiB
    assert p["total"] < 288e9
    # one qubit more per GPU does not fit
    assert capi.getQuregMemoryPlan(38, 8)["total"] > 288e9
    # 2 ranks: a one-qubit swap, slices of 256 MiB
    assert capi.getQuregMemoryPlan(31, 2)["exchange"] == 2 * 2 * 1 * (16 << 20) * 2 * 8


def test_create_refuses_when_memory_short():
    code = ("import quest_amd as qa\n"
            "from quest_amd.ops.capi import QuESTError\n"
            "e = qa.Env()\n"
            "try:\n"
            "    qa.Register(e, 26)\n"
            "    print('CREATED')\n"
            "except QuESTError as x:\n"
            "    print('REFUSED', x.code, x.message)\n"
            "r = qa.Register(e, 10)\n"
            "print('SMALL OK', r.num_amps)\n")
    out = _run(code, QUEST_DEVICE_MEM_MB="512")
    assert out.returncode == 0, out.stderr
    assert "REFUSED" in out.stdout and "CREATED" not in out.stdout, out.stdout
    assert "need 1.06 GiB per rank" in out.stdout and "0.50 GiB free" in out.stdout, out.stdout
    assert "SMALL OK 1024" in out.stdout


def test_create_without_handler_exits_with_code():
    code = ("from quest_amd.ops import capi\n"
            "b = capi.binding()\n"
            "b.exit_on_error(True)\n"
            "env = b.lib.createQuESTEnv()\n"
            "b.lib.createQureg(30, env)\n"
            "print('UNREACHABLE')\n")
    out = _run(code, QUEST_DEVICE_MEM_MB="1024")
    assert out.returncode == 30, (out.returncode, out.stdout, out.stderr)
    assert "Out of device memory" in out.stdout and "state 16.00" in out.stdout
