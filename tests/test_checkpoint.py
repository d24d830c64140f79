"""Binary checkpoint / restart (saveQuregCheckpoint / loadQuregCheckpoint):
round trips for state-vectors and density matrices, error codes, and
restoring a checkpoint written by 4 ranks on 1 and 2 ranks (and vice versa)."""
import os
import sys

import numpy as np
import pytest

from quest_amd.ops import capi
from quest_amd.ops.capi import QuESTError

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def test_round_trip_statevector_and_density(env, tmp_path):
    import quest_amd as qa
    from quest_amd.models import random_layered

    r = qa.Register(env, 12)
    r.init_plus()
    random_layered(12, 2, seed=1).apply(r)
    want = r.to_numpy()
    assert r.save(tmp_path / "sv")
    assert (tmp_path / "sv.0").stat().st_size == 64 + 2 * 8 * 4096
    s = qa.Register(env, 12)
    assert s.load(tmp_path / "sv")
    np.testing.assert_array_equal(s.to_numpy(), want)
    s.h(3)  # usable after a load
    d = qa.Register(env, 4, density=True)
    d.init_plus()
    d.damping(1, 0.3)
    d.cnot(1, 2)
    assert d.save(tmp_path / "dm")
    e = qa.Register(env, 4, density=True)
    assert e.load(tmp_path / "dm")
    np.testing.assert_array_equal(e.to_numpy(), d.to_numpy())
    for x in (r, s, d, e):
        x.close()


def test_errors(env, tmp_path):
    import quest_amd as qa

    r = qa.Register(env, 6)
    with pytest.raises(QuESTError) as ei:
        r.load(tmp_path / "missing")
    assert ei.value.code == 17
    r.save(tmp_path / "six")
    other = qa.Register(env, 7)
    with pytest.raises(QuESTError) as ei:
        other.load(tmp_path / "six")
    assert "Checkpoint does not match" in ei.value.message
    dm = qa.Register(env, 3, density=True)  # also 64 amplitudes, but a density matrix
    with pytest.raises(QuESTError):
        dm.load(tmp_path / "six")
    for x in (r, other, dm):
        x.close()


def _run(name, ranks, ckpt, tmp_path):
    from quest_amd.parallel import spawn_local

    out = str(tmp_path / f"{name}_{ranks}.npz")
    res = spawn_local([os.path.join(HERE, "dist_worker.py"), name, out], ranks,
                      env_extra={"QUEST_BACKEND": "cpu", "PYTHONPATH": os.path.dirname(HERE), "QA_CKPT": ckpt},
                      timeout=300)
    for r, p in enumerate(res):
        assert p.returncode == 0, f"rank {r}:\n{p.stdout[-2000:]}\n{p.stderr[-3000:]}"
    with np.load(out, allow_pickle=False) as z:
        return z["state"]


def test_restore_on_other_rank_counts(env, tmp_path, monkeypatch):
    from scenarios import checkpoint_load

    ckpt = str(tmp_path / "four")
    written = _run("checkpoint_save", 4, ckpt, tmp_path)
    assert sorted(os.listdir(tmp_path)).count("four.3") == 1
    monkeypatch.setenv("QA_CKPT", ckpt)
    np.testing.assert_allclose(checkpoint_load(env)["state"], written, atol=0)      # 4 -> 1
    np.testing.assert_allclose(_run("checkpoint_load", 2, ckpt, tmp_path), written, atol=0)  # 4 -> 2
    ckpt2 = str(tmp_path / "two")
    w2 = _run("checkpoint_save", 2, ckpt2, tmp_path)
    np.testing.assert_allclose(w2, written, atol=1e-12)
    np.testing.assert_allclose(_run("checkpoint_load", 4, ckpt2, tmp_path), w2, atol=0)  # 2 -> 4


def test_corrupt_checkpoint_leaves_state_untouched(env, tmp_path):
    """A truncated data file, or a header whose fields are inconsistent
    (ampsPerChunk 0, chunks x ampsPerChunk != total), is refused before the
    register is touched (advisor finding, round 1)."""
    import struct

    import quest_amd as qa

    r = qa.Register(env, 8)
    r.init_plus()
    r.rx(3, 0.7)
    assert r.save(tmp_path / "ok")
    before = r.to_numpy()
    raw = (tmp_path / "ok.0").read_bytes()
    # truncated: header intact, last amplitudes missing
    (tmp_path / "trunc.0").write_bytes(raw[:-8])
    # ampsPerChunk = 0 (offset 32) would divide by zero
    bad = bytearray(raw)
    bad[32:40] = struct.pack("<q", 0)
    (tmp_path / "zero.0").write_bytes(bytes(bad))
    # numChunks = 2 (offset 24) with ampsPerChunk = total
    bad = bytearray(raw)
    bad[24:28] = struct.pack("<i", 2)
    (tmp_path / "chunks.0").write_bytes(bytes(bad))
    s = qa.Register(env, 8)
    s.init_classical(5)
    for name in ("trunc", "zero", "chunks"):
        with pytest.raises(QuESTError):
            s.load(tmp_path / name)
        got = s.to_numpy()
        assert got[5] == 1 and np.count_nonzero(got) == 1, name
    assert s.load(tmp_path / "ok")
    np.testing.assert_array_equal(s.to_numpy(), before)
    r.close()
    s.close()
