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

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
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
