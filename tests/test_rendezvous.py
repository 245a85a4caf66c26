"""tritd.rendezvous.StarGroup (bench.py's torch-free rank plumbing, VERDICT r5
next 3a) and the shard-row synthetic generator it feeds (config 5 at N > 1):
CPU only, several processes."""
import multiprocessing as mp
import os
import socket
import time

import numpy as np
import pytest

from conftest import PKG


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q, fail_rank):
    import sys
    import numpy as np
    sys.path.insert(0, PKG)
    from tritd.rendezvous import StarGroup
    try:
        g = StarGroup(rank, world, port, timeout=30)
        out = {}
        g.barrier()
        out["bcast"] = g.broadcast_bytes(b"\x00\x01rccl-id" if rank == 0 else None)
        out["max"] = g.allreduce_max(float(rank) * 1.5)
        out["sum"] = g.allreduce_sum([1.0, float(rank), 0.1 * rank])
        out["gather"] = g.allgather([rank, rank * rank])
        a = np.arange(5, dtype=np.float64) * (rank + 1)
        g.allreduce_f64(a)
        b = np.array([rank, -rank, 0.5], dtype=np.float64)
        g.allreduce_f64(b, "max")
        out["f64"] = (a.tolist(), b.tolist())
        if rank == fail_rank:
            os._exit(3)  # dies without closing anything: the others must not hang
        g.barrier()
        g.close()
        q.put((rank, "ok", out))
    except Exception as e:  # noqa: BLE001
        q.put((rank, "error", repr(e)))


def _run(world, fail_rank=-1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q, fail_rank)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    t0 = time.time()
    while len(res) < world - (1 if fail_rank >= 0 else 0) and time.time() - t0 < 60:
        try:
            r, st, out = q.get(timeout=1)
            res[r] = (st, out)
        except Exception:  # noqa: BLE001
            pass
    for p in ps:
        p.join(30)
        if p.is_alive():
            p.kill()
    return res, time.time() - t0


@pytest.mark.parametrize("world", [2, 3, 5])
def test_star_group_collectives(world):
    res, _ = _run(world)
    assert sorted(res) == list(range(world))
    for r, (st, out) in res.items():
        assert st == "ok", out
        assert out["bcast"] == b"\x00\x01rccl-id"
        assert out["max"] == 1.5 * (world - 1)
        assert out["sum"] == [float(world), float(sum(range(world))),
                              sum(0.1 * k for k in range(world))]
        assert out["gather"] == [[k, k * k] for k in range(world)]
        tot = sum(k + 1 for k in range(world))
        assert out["f64"] == ([float(i * tot) for i in range(5)], [world - 1.0, 0.0, 0.5])


def test_star_group_peer_failure_does_not_hang():
    """A rank that dies mid-run: every other rank's next collective fails
    promptly (closed connection), well before the 30 s deadline."""
    res, dt = _run(3, fail_rank=2)
    assert dt < 25
    for r in (0, 1):
        assert res[r][0] == "error", res


def test_star_group_single_rank_needs_no_socket():
    import sys
    sys.path.insert(0, PKG)
    from tritd.rendezvous import StarGroup
    g = StarGroup(0, 1, 0)
    assert g.broadcast_bytes(b"id") == b"id" and g.allreduce_sum([2.0]) == [2.0]
    assert g.allgather(7) == [7] and g.allreduce_max(3.0) == 3.0
    g.close()


@pytest.mark.parametrize("rows", [(0, 40), (0, 13), (13, 27), (27, 40), (5, 6)])
def test_f32_generator_shard_rows_are_the_full_draws(rows):
    """bench.py's config 5 at N > 1: each rank draws only its mode-1 rows
    (synth.low_rank_plus_outliers_f32(rows=...)); they equal those rows of
    the whole draw bitwise."""
    import sys
    sys.path.insert(0, PKG)
    from tritd import synth
    full = synth.low_rank_plus_outliers_f32(40, 12, 10, 3, chunk=7)
    part = synth.low_rank_plus_outliers_f32(40, 12, 10, 3, chunk=7, rows=rows)
    assert np.array_equal(part["D"], full["D"][rows[0]:rows[1]])
    assert np.array_equal(part["Lstar"], full["Lstar"][rows[0]:rows[1]])
    for k in ("A0", "B0", "C0"):
        assert np.array_equal(part[k], full[k])
