"""Multi-rank path on CPU: world_size 2 over gloo.

The library's collectives are RCCL on the GPU box; here the same mode-1
sharded schedule (oracle/tritd_sharded.py, the algebra solver.cpp runs) is
driven with torch.distributed all_reduce over gloo and must reproduce the
unsharded goldens.  Also covers the host-side shard partition
(tritd.dist.shard_bounds) that bench.py uses.
"""
import os
import socket

import numpy as np
import pytest

from conftest import GOLDEN, ORACLE, PKG, load_golden, rel


def test_shard_bounds_tile_the_mode():
    from tritd.dist import all_bounds, shard_bounds
    for n1 in (1, 7, 30, 512, 513):
        for world in (1, 2, 3, 4, 8):
            if world > n1:
                with pytest.raises(ValueError):
                    shard_bounds(n1, world, 0)
                continue
            b = all_bounds(n1, world)
            sizes = [i1 - i0 for i0, i1 in b]
            assert min(sizes) >= 1 and max(sizes) - min(sizes) <= 1
    assert shard_bounds(512, 8, 3) == (192, 256)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, outdir, kind="admm"):
    import sys
    for p in (PKG, ORACLE):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from tritd.dist import shard_bounds
    import tritd_sharded

    # a file store in the test's directory: no TCP port to race for (`port` unused)
    dist.init_process_group("gloo", init_method="file://" + os.path.join(outdir, "gloo_store"),
                            rank=rank, world_size=world)
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    import json
    opts = json.loads(str(z["opts"]))
    r = int(z["r"])
    D = z["D"] if kind == "admm" else z["X"]
    i0, i1 = shard_bounds(D.shape[0], world, rank)

    def allreduce(x):
        t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64))
        dist.all_reduce(t)
        return t.numpy()

    run = tritd_sharded.sharded_admm if kind == "admm" else tritd_sharded.sharded_als
    res = run(D[i0:i1], i0, i1, r, opts, z["A0"], z["B0"], z["C0"], allreduce)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), i0=i0, i1=i1, **{
        k: v for k, v in res.items() if k != "k"}, k=res["k"])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["g30_r3", "g17x16x20_r8", "g12x10x8_r2_stop"])
def test_sharded_schedule_world2_matches_golden(tmp_path, name):
    import torch.multiprocessing as mp
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), name, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    g = load_golden(name)
    O = np.zeros_like(g["O"])
    E = np.zeros_like(g["E"])
    A = np.zeros_like(g["A"])
    for rank in range(world):
        z = np.load(tmp_path / f"rank{rank}.npz")
        i0, i1 = int(z["i0"]), int(z["i1"])
        O[i0:i1] = z["O"]
        E[i0:i1] = z["E"]
        A[i0:i1] = z["A_rows"]
        assert int(z["k"]) == g["k"]
        assert rel(z["B"], g["B"]) < 1e-8 and rel(z["C"], g["C"]) < 1e-8
        np.testing.assert_allclose(z["errHist"], g["errHist"], rtol=1e-8, atol=1e-13)
    assert rel(A, g["A"]) < 1e-8
    assert rel(O, g["O"]) < 1e-9
    assert rel(E, g["E"]) < 1e-9


# ---------------------------------------------------------------------------
# The library's own communicator schedule (solver.cpp iterate_fused with a
# comm): two all-reduces per iteration, the norm partials per K5 workgroup in
# red1's tail sized to the largest shard, the stop test deferred behind the
# next iteration's speculative M1 .. M2.  Uneven shards whose padded heights
# straddle a multiple of 16 (n1 = 33 on 2 ranks: 17 -> 32 and 16 rows; n1 = 49
# on 3 ranks: 17 / 16 / 16) launch different K5 grids.

def _lib_case(n1, stop):
    import tritd_oracle  # noqa: F401  (path check)
    from tritd import synth
    d = synth.low_rank_plus_outliers(n1, 10, 8, 2, seed=5, init_seed=9)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=30, tol=0.2 if stop else 1e-5)
    return d, opts


def _lib_worker(rank, world, port, n1, stop, clear_tail, outdir):
    import sys
    for p in (PKG, ORACLE):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from tritd.dist import shard_bounds
    import tritd_sharded

    # a file store in the test's directory: no TCP port to race for (`port` unused)
    dist.init_process_group("gloo", init_method="file://" + os.path.join(outdir, "gloo_store"),
                            rank=rank, world_size=world)
    d, opts = _lib_case(n1, stop)
    i0, i1 = shard_bounds(n1, world, rank)

    def allreduce(x, op=dist.ReduceOp.SUM):
        t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64).copy())
        dist.all_reduce(t, op=op)
        return t.numpy()

    res = tritd_sharded.library_admm(d["D"][i0:i1], i0, i1, 2, opts, d["A0"], d["B0"], d["C0"],
                                     allreduce, lambda x: allreduce(x, dist.ReduceOp.MAX),
                                     clear_tail=clear_tail)
    # every all-reduce must have had the same count on every rank: compare
    # the sequences through a max and a min all-reduce of the padded list
    c = np.zeros(4 * 30 + 8)
    c[: len(res["counts"])] = res["counts"]
    cmax = allreduce(c, dist.ReduceOp.MAX)
    cmin = allreduce(c, dist.ReduceOp.MIN)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), i0=i0, i1=i1, same=bool((cmax == cmin).all()),
             nwg=tritd_sharded.k5_workgroups(i1 - i0, 10),
             **{k: v for k, v in res.items() if k not in ("k", "counts")}, k=res["k"])
    dist.barrier()
    dist.destroy_process_group()


def _run_lib(tmp_path, world, n1, stop, clear_tail=True):
    import torch.multiprocessing as mp
    mp.start_processes(_lib_worker, args=(world, _free_port(), n1, stop, clear_tail, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    return [np.load(tmp_path / f"rank{q}.npz") for q in range(world)]


@pytest.mark.parametrize("world,n1,stop", [(2, 33, False), (2, 33, True), (3, 49, False),
                                           (3, 49, True)])
def test_library_schedule_uneven_shards_match_oracle(tmp_path, world, n1, stop):
    import tritd_oracle as orc
    d, opts = _lib_case(n1, stop)
    rA, rB, rC, rO, reh, rE, rk, _ = orc.triple_decomp_ADMM(d["D"], 2, opts, d["A0"], d["B0"],
                                                            d["C0"])
    zs = _run_lib(tmp_path, world, n1, stop)
    assert len({int(z["nwg"]) for z in zs}) > 1, "case must give the ranks different K5 grids"
    assert (rk < 30) == stop
    A = np.zeros_like(rA)
    O = np.zeros_like(rO)
    E = np.zeros_like(rE)
    for z in zs:
        assert bool(z["same"]), "ranks issued all-reduces of different counts"
        i0, i1 = int(z["i0"]), int(z["i1"])
        A[i0:i1], O[i0:i1], E[i0:i1] = z["A_rows"], z["O"], z["E"]
        assert int(z["k"]) == rk
        np.testing.assert_allclose(z["errHist"], reh, rtol=1e-8, atol=1e-13)
        assert rel(z["B"], rB) < 1e-8 and rel(z["C"], rC) < 1e-8
    assert rel(A, rA) < 1e-8 and rel(O, rO) < 1e-9 and rel(E, rE) < 1e-9


def test_library_schedule_needs_the_tail_cleared(tmp_path):
    """Without k_reduce_finish clearing the tail, the pairs past the smaller
    shard's grid keep the previous iteration's sums and errHist goes wrong:
    the uneven case above really exercises the padded tail."""
    import tritd_oracle as orc
    d, opts = _lib_case(33, False)
    *_, reh, _, _, _ = orc.triple_decomp_ADMM(d["D"], 2, opts, d["A0"], d["B0"], d["C0"])
    zs = _run_lib(tmp_path, 2, 33, False, clear_tail=False)
    assert not np.allclose(zs[0]["errHist"], reh[: len(zs[0]["errHist"])], rtol=1e-6)


@pytest.mark.parametrize("name", ["als30_r3", "als20x24x18_r5_stop"])
def test_sharded_als_world2_matches_golden(tmp_path, name):
    """triple_decomp_ALS over 2 gloo ranks (the als.cpp schedule) == unsharded goldens."""
    import torch.multiprocessing as mp
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), name, str(tmp_path), "als"),
                       nprocs=world, join=True, start_method="spawn")
    g = load_golden(name)
    A = np.zeros_like(g["A"])
    for rank in range(world):
        z = np.load(tmp_path / f"rank{rank}.npz")
        i0, i1 = int(z["i0"]), int(z["i1"])
        A[i0:i1] = z["A_rows"]
        assert int(z["k"]) == g["k"]
        assert rel(z["B"], g["B"]) < 1e-8 and rel(z["C"], g["C"]) < 1e-8
        np.testing.assert_allclose(z["errHist"], g["errHist"], rtol=1e-9, atol=1e-14)
    assert rel(A, g["A"]) < 1e-8


def test_allreduce_counts_agree_for_every_partition():
    """Every shard_bounds partition (n1 <= 200, 1..8 ranks) gives every rank the
    same all-reduce counts once red1's norm tail is sized to the largest
    shard's K5 grid (solver.cpp agree_counts), although the per-rank grids
    differ whenever the padded shard heights straddle a multiple of 16."""
    import tritd_sharded
    from tritd.dist import all_bounds
    n2, n3, RP = 10, 8, 16
    straddles = 0
    for n1 in range(1, 201):
        for world in range(1, 9):
            if world > n1:
                continue
            grids = [tritd_sharded.k5_workgroups(i1 - i0, n2) for i0, i1 in all_bounds(n1, world)]
            tail = max(grids)
            counts = {(n2 * RP + RP * RP + 2 * tail, ((n3 + 15) // 16 * 16) * RP) for _ in grids}
            assert len(counts) == 1
            straddles += len(set(grids)) > 1
    assert straddles > 0  # the max is needed: some partitions give the ranks different grids
