"""Collectives of the multi-GPU path, without PyTorch.

One process per GPU, launched by any launcher that sets RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_ADDR / MASTER_PORT (torchrun, or a plain loop).  The
reference has no collective at all -- its per-contig workers return through
multiprocessing.Pool pickling (bwt.py:3894-3912); here ranks exchange only
small count vectors (bwtmi.dist.write_sharded), so two transports suffice:

  RcclComm   ncclAllReduce over xGMI, bound in libbwtmi (bwtmi_comm_*); the
             128-byte RCCL id travels over the TCP rendezvous below
  HostComm   the same reductions over the rendezvous sockets themselves (a
             star through rank 0): CPU tests, and rehearsals with more ranks
             than GPUs

Rendezvous: rank 0 listens on MASTER_ADDR:(MASTER_PORT + 1) -- MASTER_PORT
itself belongs to the launcher's store -- or on BWTMI_RDZV_PORT.
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import List, Optional

import numpy as np

from . import _lib

_I64, _F64 = 0, 1
SUM, MAX = 0, 1


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _recv_exact(s: socket.socket, n: int) -> bytes:
    out = bytearray()
    while len(out) < n:
        b = s.recv(n - len(out))
        if not b:
            raise ConnectionError("rendezvous peer closed the connection")
        out += b
    return bytes(out)


def _send_msg(s: socket.socket, payload: bytes) -> None:
    s.sendall(struct.pack("<q", len(payload)) + payload)


def _recv_msg(s: socket.socket) -> bytes:
    (n,) = struct.unpack("<q", _recv_exact(s, 8))
    return _recv_exact(s, n)


class Rendezvous:
    """Star of TCP connections to rank 0 (kept open for HostComm)."""

    def __init__(self, world: int, rank: int, addr: Optional[str] = None, port: Optional[int] = None,
                 timeout: float = 300.0):
        self.world, self.rank = world, rank
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            port = int(os.environ.get("BWTMI_RDZV_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
        self.peers: List[Optional[socket.socket]] = [None] * world
        self.up: Optional[socket.socket] = None
        if world == 1:
            return
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(world)
            srv.settimeout(timeout)
            try:
                for _ in range(world - 1):
                    conn, _ = srv.accept()
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    (r,) = struct.unpack("<i", _recv_exact(conn, 4))
                    if not 0 < r < world or self.peers[r] is not None:
                        raise ConnectionError(f"rendezvous: unexpected rank {r}")
                    self.peers[r] = conn
            finally:
                srv.close()
        else:
            t0 = time.time()
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=10.0)
                    break
                except OSError:
                    if time.time() - t0 > timeout:
                        raise
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(None)
            s.sendall(struct.pack("<i", rank))
            self.up = s

    def bcast(self, payload: bytes) -> bytes:
        """rank 0's payload on every rank."""
        if self.world == 1:
            return payload
        if self.rank == 0:
            for s in self.peers[1:]:
                _send_msg(s, payload)
            return payload
        return _recv_msg(self.up)

    def gather(self, payload: bytes) -> List[bytes]:
        """every rank's payload, on rank 0 (others get [])."""
        if self.world == 1:
            return [payload]
        if self.rank == 0:
            return [payload] + [_recv_msg(s) for s in self.peers[1:]]
        _send_msg(self.up, payload)
        return []

    def close(self) -> None:
        for s in self.peers:
            if s is not None:
                s.close()
        if self.up is not None:
            self.up.close()
        self.peers, self.up = [None] * self.world, None


class HostComm:
    """All-reduce through rank 0 over the rendezvous sockets."""

    kind = "host"

    def __init__(self, rdzv: Rendezvous):
        self.r = rdzv
        self.world, self.rank = rdzv.world, rdzv.rank

    def allreduce(self, arr: np.ndarray, op: int = SUM) -> np.ndarray:
        a = np.ascontiguousarray(arr)
        if self.world == 1:
            return a.copy()
        parts = self.r.gather(a.tobytes())
        if self.rank == 0:
            acc = a.copy()
            for b in parts[1:]:
                x = np.frombuffer(b, dtype=a.dtype).reshape(a.shape)
                acc = acc + x if op == SUM else np.maximum(acc, x)
            out = acc.tobytes()
        else:
            out = b""
        return np.frombuffer(self.r.bcast(out), dtype=a.dtype).reshape(a.shape).copy()

    def barrier(self) -> None:
        self.allreduce(np.zeros(1, dtype=np.int64))

    def close(self) -> None:
        self.r.close()


class RcclComm:
    """ncclAllReduce on the rank's GPU (libbwtmi bwtmi_comm_*)."""

    kind = "rccl"

    def __init__(self, rdzv: Rendezvous, device: int):
        import ctypes as C
        self.world, self.rank, self.device = rdzv.world, rdzv.rank, device
        uid = C.create_string_buffer(128)
        if self.rank == 0:
            _lib.check(_lib.lib().bwtmi_comm_unique_id(uid))
        raw = rdzv.bcast(uid.raw)
        uid = C.create_string_buffer(raw, 128)
        self.h = C.c_void_p()
        _lib.check(_lib.lib().bwtmi_comm_init(device, self.world, self.rank, uid, C.byref(self.h)))
        rdzv.close()

    def allreduce(self, arr: np.ndarray, op: int = SUM) -> np.ndarray:
        a = np.array(arr, copy=True, order="C")
        if a.dtype == np.int64:
            dt = _I64
        elif a.dtype == np.float64:
            dt = _F64
        else:
            raise TypeError(f"allreduce of {a.dtype} (int64 / float64 only)")
        if a.size:
            _lib.check(_lib.lib().bwtmi_comm_allreduce(self.h, a.ctypes.data, a.size, dt, op))
        return a

    def barrier(self) -> None:
        self.allreduce(np.zeros(1, dtype=np.int64))

    def close(self) -> None:
        if self.h:
            _lib.lib().bwtmi_comm_free(self.h)
            self.h = None


def allgather_words(c, words: np.ndarray) -> List[np.ndarray]:
    """Every rank's int64 vector, in rank order, through two sum all-reduces
    (sizes, then each rank's words at its offset of a zeroed buffer)."""
    w = np.ascontiguousarray(words, dtype=np.int64)
    if c is None or c.world == 1:
        return [w.copy()]
    sizes = np.zeros(c.world, dtype=np.int64)
    sizes[c.rank] = w.size
    sizes = c.allreduce(sizes)
    off = np.concatenate([[0], np.cumsum(sizes)])
    buf = np.zeros(int(off[-1]), dtype=np.int64)
    buf[off[c.rank]:off[c.rank + 1]] = w
    buf = c.allreduce(buf)
    return [buf[off[r]:off[r + 1]] for r in range(c.world)]


_COMM = None


def get(transport: Optional[str] = None):
    """The process's communicator (created once).  transport: "rccl", "host",
    or None = BWTMI_COMM, else rccl when this process sees a GPU."""
    global _COMM
    if _COMM is not None:
        return _COMM
    rank, world, local = env_rank()
    transport = transport or os.environ.get("BWTMI_COMM")
    if transport is None:
        try:
            transport = "rccl" if _lib.device_count() > 0 else "host"
        except Exception:
            transport = "host"
    rdzv = Rendezvous(world, rank)
    _COMM = RcclComm(rdzv, local) if transport == "rccl" else HostComm(rdzv)
    return _COMM


def allgather_bytes(comm, blob: bytes) -> List[bytes]:
    """Every rank's bytes on every rank: sizes by one all-reduce, the payloads by
    a second one over a zero-padded int64 buffer (each rank fills its slot)."""
    world, rank = comm.world, comm.rank
    sizes = np.zeros(world, dtype=np.int64)
    sizes[rank] = len(blob)
    sizes = comm.allreduce(sizes)
    words = [(int(s) + 7) // 8 for s in sizes]
    off = np.concatenate([[0], np.cumsum(words)]).astype(np.int64)
    buf = np.zeros(max(1, int(off[-1])), dtype=np.int64)
    if blob:
        padded = blob + b"\0" * (words[rank] * 8 - len(blob))
        buf[off[rank]:off[rank] + words[rank]] = np.frombuffer(padded, dtype=np.int64)
    buf = comm.allreduce(buf)
    raw = buf.tobytes()
    return [raw[off[r] * 8: off[r] * 8 + int(sizes[r])] for r in range(world)]


def close() -> None:
    global _COMM
    if _COMM is not None:
        _COMM.close()
        _COMM = None
