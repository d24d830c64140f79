"""bench.py in the driver's multi-GPU launch shape on ONE GPU (VERDICT r2
item 3): ``python -m torch.distributed.run --nnodes=1 --nproc-per-node 8
--master-addr 127.0.0.1 --master-port P bench.py --gpus 8 ...`` with the
ranks sharing the card through the device-IPC transport, and through RCCL
itself with QUEST_RCCL_SHARED_GPU=1 (RCCL refuses two ranks on one device of
one host; each rank then presents its own host id).  This runs everything the
8-GPU job runs except the xGMI links: torchrun rendezvous, the gloo port agreement in
quest_amd.parallel.init_distributed, the library's TCP bootstrap, amplitude
sharding over 8 ranks (3 rank qubits), all-to-all qubit swaps through the
communication stream, max-over-ranks timing and the rank-0 JSON line."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("ranks", [2, 8])
def test_bench_under_torchrun_ipc(ranks):
    env = dict(os.environ, QUEST_COMM="ipc", QUEST_BACKEND="hip", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "QUEST_BOOTSTRAP_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(ranks),
           "--qubits", "22", "--steps", "4", "--warmup", "1", "--allow-transport"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout   # rank 0 only
    d = json.loads(lines[0])
    n = 22 + {2: 1, 8: 3}[ranks]
    assert d["n_gpus"] == ranks and d["config"]["qubits"] == n
    assert "IPC" in d["config"]["transport"]
    assert d["config"]["swaps"] > 0, d["config"]     # rank qubits were swapped in
    assert d["config"]["norm_error"] < 1e-10
    assert d["value"] > 0 and d["steps"] == 4
    # rank predicates are tags: every rank planned the same passes (round 6)
    assert d["config"]["layout_aligns_max"] == 0, d["config"]


@pytest.mark.parametrize("ranks", [2, 8])
def test_bench_under_torchrun_rccl_shared_gpu(ranks):
    """The same launch with the RCCL transport itself: QUEST_RCCL_SHARED_GPU=1
    gives each rank its own RCCL host id, so RCCL accepts N ranks on one GPU
    and connects them through its network transport (loopback).  bench.py
    takes the RCCL path it takes on 8 GPUs (no --allow-transport): grouped
    ncclSend / ncclRecv all-to-all swaps on the communication stream and
    RCCL scalar collectives."""
    env = dict(os.environ, QUEST_COMM="rccl", QUEST_RCCL_SHARED_GPU="1", QUEST_BACKEND="hip", OMP_NUM_THREADS="1",
               QUEST_COMM_TIMEOUT="150")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "QUEST_BOOTSTRAP_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(ranks),
           "--qubits", "22", "--steps", "4", "--warmup", "1"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    n = 22 + {2: 1, 8: 3}[ranks]
    assert d["n_gpus"] == ranks and d["config"]["qubits"] == n
    assert d["config"]["transport"].startswith("RCCL"), d["config"]["transport"]
    assert "RCCL" in d["config"]["parallelism"]
    assert d["config"]["swaps"] > 0, d["config"]
    assert d["config"]["norm_error"] < 1e-10
    assert d["config"]["layout_aligns_max"] == 0, d["config"]
    assert all("overlapped_passes" in s for s in d["config"]["seeds"]), d["config"]["seeds"]
