"""Tracing (QUEST_TRACE), failure detection (QUEST_COMM_TIMEOUT) and the
statistics counters."""
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def test_trace_events_distributed(tmp_path):
    from quest_amd.parallel import spawn_local

    trace = tmp_path / "trace.jsonl"
    out = str(tmp_path / "o.npz")
    res = spawn_local([os.path.join(HERE, "dist_worker.py"), "random_ops_statevector", out], 2,
                      env_extra={"QUEST_BACKEND": "cpu", "PYTHONPATH": ROOT, "QUEST_TRACE": str(trace)}, timeout=300)
    assert all(p.returncode == 0 for p in res), [p.stderr[-2000:] for p in res]
    evs = [json.loads(line) for line in trace.read_text().splitlines()]
    kinds = {e["ev"] for e in evs}
    assert {"create", "flush", "swap", "destroy"} <= kinds
    assert {e["rank"] for e in evs if e["ev"] != "trace_start"} == {0, 1}
    assert all("monotonic" in e for e in evs if e["ev"] == "trace_start")
    flushes = [e for e in evs if e["ev"] == "flush"]
    assert all(e["ops_fused"] <= e["ops"] and e["passes"] >= 1 for e in flushes)
    swaps = [e for e in evs if e["ev"] == "swap"]
    assert all(e["bytes_sent"] > 0 for e in swaps)


def test_dead_peer_detected_by_timeout(tmp_path):
    """Rank 1 stops responding inside a collective; rank 0 reports it and
    exits after QUEST_COMM_TIMEOUT instead of hanging."""
    import socket

    s = socket.socket()
    s.bind(("", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(2):
        e = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                 QUEST_BOOTSTRAP_ADDR="127.0.0.1", QUEST_BOOTSTRAP_PORT=str(port), QUEST_BACKEND="cpu",
                 PYTHONPATH=ROOT, QUEST_COMM_TIMEOUT="3")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), "hang_rank1",
                                       str(tmp_path / "x.npz")], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    t0 = time.time()
    try:
        _, err = procs[0].communicate(timeout=60)
        assert procs[0].returncode != 0
        assert "no progress from peer rank 1" in err
        assert time.time() - t0 < 50
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.communicate()
