"""Host-side rendezvous of the one-process-per-GPU path without torch.

libtritd's RCCL communicator needs one thing from the host before its first
all-reduce: every rank must hold the same 128-byte unique id (SURVEY.md §8e;
`tritd_comm_unique_id` / `tritd_comm_create`).  The benchmark additionally
needs a barrier around its timed region, a max over the ranks' times and a
gather of per-rank figures.  `StarGroup` provides exactly these over TCP on
one node: rank 0 holds a listening socket, the other ranks connect to it,
and every collective is a gather to rank 0 followed by a broadcast back.

Rank processes that use it never import torch, so libtritd binds the system
`/opt/rocm` HIP runtime and RCCL — the stack every GPU test runs on — and not
the copies bundled with torch.  The listening
socket is created by the launcher (bench.py's rank parent, which may use
torch.distributed on the CPU to publish its port) and inherited by rank 0's
worker as a file descriptor, so no port is ever chosen and re-bound.

Every receive has a deadline, and a peer that exits closes its socket: a
failing rank makes the others fail promptly instead of hanging in a
collective.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time

DEFAULT_TIMEOUT = 900.0


def _send(sock, obj):
    data = json.dumps(obj).encode()
    sock.sendall(struct.pack("<I", len(data)) + data)


def _recv_exact(sock, n, deadline):
    buf = bytearray()
    while len(buf) < n:
        left = deadline - time.monotonic()
        if left <= 0:
            raise TimeoutError("rendezvous: peer did not answer in time")
        sock.settimeout(left)
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous: peer closed the connection (a rank failed?)")
        buf += chunk
    return bytes(buf)


def _recv(sock, timeout):
    deadline = time.monotonic() + timeout
    (n,) = struct.unpack("<I", _recv_exact(sock, 4, deadline))
    return json.loads(_recv_exact(sock, n, deadline).decode())


class StarGroup:
    """`world` ranks on one host; rank 0 is the hub.  Collectives take and
    return JSON-serialisable values (bytes travel as hex)."""

    def __init__(self, rank: int, world: int, port: int, listen_fd: int | None = None,
                 host: str = "127.0.0.1", timeout: float = DEFAULT_TIMEOUT):
        if not 0 <= rank < world:
            raise ValueError("bad rank/world")
        self.rank, self.world, self.timeout = rank, world, timeout
        self.peers = []
        self.sock = None
        self._seq = 0
        if world == 1:
            return
        if rank == 0:
            if listen_fd is not None:
                ls = socket.socket(fileno=listen_fd)
            else:
                ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
                ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                ls.bind((host, port))
                ls.listen(world)
            ls.settimeout(timeout)
            peers = {}
            try:
                while len(peers) < world - 1:
                    c, _ = ls.accept()
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    hello = _recv(c, timeout)
                    r = int(hello["rank"])
                    if not 0 < r < world or r in peers or hello.get("world") != world:
                        raise RuntimeError("rendezvous: bad hello %r" % (hello,))
                    peers[r] = c
            finally:
                ls.close()
            self.peers = [peers[r] for r in range(1, world)]
        else:
            deadline = time.monotonic() + timeout
            while True:
                try:
                    s = socket.create_connection((host, port), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            _send(s, {"rank": rank, "world": world})
            self.sock = s

    @classmethod
    def from_env(cls, timeout: float = DEFAULT_TIMEOUT):
        """RANK / WORLD_SIZE, TRITD_RDZV_PORT, and on rank 0 the inherited
        listening socket TRITD_RDZV_FD (bench.py's rank parent sets them)."""
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        port = int(os.environ.get("TRITD_RDZV_PORT", "0"))
        fd = os.environ.get("TRITD_RDZV_FD")
        return cls(rank, world, port, int(fd) if fd and rank == 0 else None, timeout=timeout)

    # -- collectives ------------------------------------------------------
    def _exchange(self, value, combine):
        """Gather `value` to rank 0, apply combine(list in rank order), return
        the result on every rank."""
        self._seq += 1
        if self.world == 1:
            return combine([value])
        if self.rank == 0:
            vals = [value]
            for r, p in enumerate(self.peers, start=1):
                m = _recv(p, self.timeout)
                if m.get("seq") != self._seq:
                    raise RuntimeError("rendezvous: rank %d out of step (%r vs %d)"
                                       % (r, m.get("seq"), self._seq))
                vals.append(m["v"])
            out = combine(vals)
            for p in self.peers:
                _send(p, {"seq": self._seq, "v": out})
            return out
        _send(self.sock, {"seq": self._seq, "v": value})
        m = _recv(self.sock, self.timeout)
        if m.get("seq") != self._seq:
            raise RuntimeError("rendezvous: hub out of step")
        return m["v"]

    def barrier(self):
        self._exchange(None, lambda vs: None)

    def broadcast_bytes(self, data: bytes | None) -> bytes:
        """rank 0's `data` on every rank."""
        h = self._exchange(data.hex() if self.rank == 0 else None, lambda vs: vs[0])
        return bytes.fromhex(h)

    def allreduce_max(self, x: float) -> float:
        return float(self._exchange(float(x), max))

    def allreduce_sum(self, xs):
        """elementwise sum of equal-length lists of floats, in rank order"""
        def comb(vs):
            out = [0.0] * len(vs[0])
            for v in vs:
                for q, a in enumerate(v):
                    out[q] += a
            return out
        return self._exchange([float(a) for a in xs], comb)

    def allgather(self, value):
        return self._exchange(value, list)

    def allreduce_f64(self, buf, op="sum"):
        """In-place sum (rank order) or max of a float64 numpy array over the
        ranks, as raw bytes (the host transport's all-reduces: ~0.6 M doubles
        per call at config 5, which JSON would turn into megabytes of text)."""
        import numpy as np
        self._seq += 1
        if self.world == 1:
            return buf
        hdr = struct.Struct("<QQ")  # seq, nbytes
        data = np.ascontiguousarray(buf, dtype=np.float64)

        def send(sock, arr):
            b = arr.tobytes()
            sock.sendall(hdr.pack(self._seq, len(b)) + b)

        def recv(sock):
            deadline = time.monotonic() + self.timeout
            seq, n = hdr.unpack(_recv_exact(sock, hdr.size, deadline))
            if seq != self._seq or n != data.nbytes:
                raise RuntimeError("rendezvous: peer out of step (%d/%d bytes %d/%d)"
                                   % (seq, self._seq, n, data.nbytes))
            return np.frombuffer(_recv_exact(sock, n, deadline), dtype=np.float64)

        if self.rank == 0:
            acc = data.copy()
            for p in self.peers:
                v = recv(p)
                if op == "max":
                    np.maximum(acc, v, out=acc)
                else:
                    acc += v
            for p in self.peers:
                send(p, acc)
        else:
            send(self.sock, data)
            acc = recv(self.sock)
        buf[...] = acc.reshape(buf.shape)
        return buf

    def close(self):
        for p in self.peers:
            p.close()
        if self.sock is not None:
            self.sock.close()
        self.peers, self.sock = [], None


def make_comm(group: StarGroup, device: int):
    """libtritd's RCCL communicator, its unique id drawn by rank 0 and
    broadcast through the group."""
    from .api import Comm
    uid = group.broadcast_bytes(Comm.unique_id() if group.rank == 0 else None)
    return Comm(uid, group.world, group.rank, device)


def make_host_comm(group: StarGroup, device: int):
    """libtritd's host transport with the group's all-reduces (sum / max of
    float64 buffers): the multi-rank schedule with ranks sharing a GPU."""
    from .api import Comm

    def fn(buf, op):
        group.allreduce_f64(buf, "max" if op else "sum")

    return Comm.host(fn, group.world, group.rank, device)
