"""One rank of a distributed-equivalence run:
``python tests/dist_worker.py <scenario> <out.npz>`` (rank 0 writes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    if os.environ.get("QUEST_TEST_STACKS"):
        # debugging a hung rank: every thread's Python stack after N seconds
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["QUEST_TEST_STACKS"]), exit=True)
    import quest_amd as qa
    from scenarios import SCENARIOS

    name, out = sys.argv[1], sys.argv[2]
    env = qa.Env()
    res = SCENARIOS[name](env)
    res["_ranks"] = env.num_ranks
    res["_transport"] = qa.capi.getQuESTTransport()
    # every rank's own counters (a rank other than 0 is the one that would
    # have aligned its layout)
    import json

    st = qa.capi.getQuESTStats()
    with open(f"{out}.rank{env.rank}.json", "w") as f:
        json.dump({k: int(st[k]) for k in ("layoutAligns", "swaps", "passes")}, f)
    if env.rank == 0:
        import numpy as np

        np.savez(out, **{k: np.asarray(v) for k, v in res.items()})
    env.close()


if __name__ == "__main__":
    main()
