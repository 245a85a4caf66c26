"""Host side of the multi-GPU path: one process per GPU, mode-1 shards
(SURVEY.md §8e).

Each rank owns rows i in [i0, i1) of D (and of O, E, Y_L, Y_O, T, A^).
B^ and C^ are replicated.  Per iteration libtritd issues two RCCL
all-reduces on its own stream (M2 | A^TA with the previous iteration's
residual-norm partials in its tail, then M3); the only host-side collective is the broadcast of the 128-byte RCCL unique id
at start-up, done here over torch.distributed.
"""
from __future__ import annotations


def shard_bounds(n1: int, world: int, rank: int):
    """Balanced contiguous mode-1 ranges: the first n1 % world ranks get one
    extra row.  Every rank gets at least one row: world must be <= n1."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    if world > n1:
        raise ValueError("more ranks than mode-1 rows")
    base, extra = divmod(n1, world)
    i0 = rank * base + min(rank, extra)
    return i0, i0 + base + (1 if rank < extra else 0)


def all_bounds(n1: int, world: int):
    b = [shard_bounds(n1, world, r) for r in range(world)]
    # ranges must tile [0, n1) without gaps/overlap
    assert b[0][0] == 0 and b[-1][1] == n1
    assert all(b[k][1] == b[k + 1][0] for k in range(world - 1))
    return b


def make_comm(torch_dist, rank: int, world: int, device: int):
    """Create libtritd's RCCL communicator: rank 0 draws the unique id, the
    torch.distributed group (any backend) broadcasts it."""
    from .api import Comm
    uid = [Comm.unique_id() if rank == 0 else None]
    torch_dist.broadcast_object_list(uid, src=0)
    return Comm(uid[0], world, rank, device)


def make_host_comm(torch_dist, rank: int, world: int, device: int):
    """libtritd communicator whose all-reduces go through torch.distributed on
    host copies (any backend, e.g. gloo): the library's own multi-rank
    schedule with several ranks on one GPU, where RCCL cannot run."""
    import torch
    from .api import Comm

    def fn(buf, op):
        t = torch.from_numpy(buf)  # shares memory: the reduced values land in buf
        torch_dist.all_reduce(t, op=torch_dist.ReduceOp.MAX if op else torch_dist.ReduceOp.SUM)

    return Comm.host(fn, world, rank, device)
