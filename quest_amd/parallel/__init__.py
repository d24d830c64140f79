"""Multi-process (one rank per GPU) launch and bootstrap helpers.

The native library bootstraps its RCCL communicator from torchrun-style
environment variables (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR) plus a
rendezvous port (QUEST_BOOTSTRAP_PORT, default MASTER_PORT + 1).  Under
``torch.distributed.run`` the MASTER_PORT is owned by torch's own store, so
:func:`init_distributed` uses torch.distributed (gloo, CPU) as the control
plane to agree on a free port before the library creates its communicator;
all bulk data then moves over RCCL inside the library.
"""
from __future__ import annotations

import os
import socket


def world() -> tuple[int, int, int]:
    r = int(os.environ.get("RANK", "0"))
    w = int(os.environ.get("WORLD_SIZE", "1"))
    lr = int(os.environ.get("LOCAL_RANK", str(r)))
    return r, w, lr


def _free_port() -> int:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def init_distributed(use_torch: bool = True) -> tuple[int, int]:
    """Prepare the environment for ``createQuESTEnv`` in a multi-rank job.

    Returns (rank, world_size).  With world size 1 this is a no-op."""
    rank, size, local = world()
    if size == 1:
        return 0, 1
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("QUEST_BOOTSTRAP_ADDR", os.environ["MASTER_ADDR"])
    if use_torch and "QUEST_BOOTSTRAP_PORT" not in os.environ:
        import torch.distributed as dist

        if not dist.is_initialized():
            dist.init_process_group("gloo", rank=rank, world_size=size)
        obj = [_free_port() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        os.environ["QUEST_BOOTSTRAP_PORT"] = str(obj[0])
    return rank, size


def barrier():
    try:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.barrier()
    except ImportError:  # pragma: no cover
        pass


def allreduce_max(x: float) -> float:
    try:
        import torch
        import torch.distributed as dist

        if dist.is_initialized():
            t = torch.tensor([x], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())
    except ImportError:  # pragma: no cover
        pass
    return x


def shutdown():
    """End of a multi-rank job: every rank meets once more, then the
    torch.distributed control plane goes down in order (a gloo process group
    left to the interpreter's exit can abort a rank in its teardown --
    "terminate called without an active exception")."""
    try:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
    except ImportError:  # pragma: no cover
        pass


def spawn_local(script_args: list[str], nprocs: int, env_extra: dict | None = None, timeout: float = 300,
                python: str | None = None):
    """Run ``python <script_args>`` as `nprocs` local ranks (used by the
    multi-process CPU tests; the analogue of the reference's oversubscribed
    ``mpiexec -n 4``).  Returns the list of CompletedProcess objects."""
    import subprocess
    import sys

    port = _free_port()
    procs = []
    for r in range(nprocs):
        e = dict(os.environ)
        e.update({"RANK": str(r), "WORLD_SIZE": str(nprocs), "LOCAL_RANK": str(r),
                  "MASTER_ADDR": "127.0.0.1", "QUEST_BOOTSTRAP_ADDR": "127.0.0.1",
                  "QUEST_BOOTSTRAP_PORT": str(port)})
        if env_extra:
            e.update(env_extra)
        procs.append(subprocess.Popen([python or sys.executable] + script_args, env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    out = []
    for p in procs:
        try:
            so, se = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        out.append(subprocess.CompletedProcess(p.args, p.returncode, so, se))
    return out
