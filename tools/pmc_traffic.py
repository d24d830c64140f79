#!/usr/bin/env python3
"""Workload for the HBM-traffic counters (tools/pmc_traffic.sh): a
calibration copy of a known byte count, then the unfused kernels and one
wave pass on a 28-qubit state (4 GiB: re + im).

  1. torch copy of a 4 GiB fp64 tensor (reads 4 GiB, writes 4 GiB): the
     counters' scale for a wide streaming read on this GPU;
  2. H on qubits 0 / 2 / 14 and T on 14 (direct kernels, one pass each);
  3. a fused random layer (one wave pass).
The summary (tools/pmc_summary.py --traffic) divides every dispatch's bytes by
the bytes it moves by construction."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import quest_amd as qa
    from quest_amd.models import random_layered
    from quest_amd.ops import capi

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 28
    x = torch.ones(1 << (n + 1), dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    for _ in range(2):
        y.copy_(x)
    torch.cuda.synchronize()
    del x, y
    torch.cuda.empty_cache()
    env = qa.Env()
    r = qa.Register(env, n)
    r.init_plus()
    capi.setGateFusion(0)
    for fn, t in ((r.h, 0), (r.h, 2), (r.h, n // 2), (r.t, n // 2)):
        for _ in range(2):
            fn(t)
        r.sync()
    capi.setGateFusion(1)
    random_layered(n, 1, seed=3).apply(r)
    r.sync()
    print("state bytes", 16 * (1 << n))
    r.close()


if __name__ == "__main__":
    main()
