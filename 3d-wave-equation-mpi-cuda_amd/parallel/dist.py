"""torch.distributed integration.

* :func:`init_from_env` — one process per GPU, torchrun env (RANK / WORLD_SIZE / LOCAL_RANK /
  MASTER_ADDR / MASTER_PORT), ``nccl`` (= RCCL on ROCm) on GPUs, ``gloo`` on CPU.
* :func:`rccl_transport` — the native halo transport: torch.distributed only carries the
  128-byte RCCL unique id; the time loop then runs in C++ with ncclSend/ncclRecv groups on
  the solver's comm stream (no Python in the loop).
* :class:`TorchHostTransport` — a host-memory transport over torch.distributed point-to-
  point (gloo), used by the OpenMP backend for multi-process CPU runs and tests; it is the
  process-level equivalent of the reference's MPI_Sendrecv chain (mpi_new.cpp:201-238).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch
import torch.distributed as dist

from .._native import load


def env_rank() -> tuple[int, int, int]:
    r = int(os.environ.get("RANK", "0"))
    w = int(os.environ.get("WORLD_SIZE", "1"))
    lr = int(os.environ.get("LOCAL_RANK", str(r)))
    return r, w, lr


def init_from_env(backend: str | None = None) -> tuple[int, int, int]:
    """Initialise the default process group from torchrun-style env (idempotent)."""
    rank, world, local = env_rank()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, world, local


def broadcast_bytes(b: bytes | None, src: int = 0, group=None) -> bytes:
    obj = [b]
    dist.broadcast_object_list(obj, src=src, group=group)
    return obj[0]


def rccl_transport(device: int | None = None, group=None):
    """Native RCCL transport for this rank; the unique id travels via torch.distributed."""
    C = load()
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if device is None:
        device = torch.cuda.current_device()
    uid = C.rccl_unique_id() if rank == 0 else None
    uid = broadcast_bytes(uid, 0, group)
    return C.RcclTransport(rank, world, uid, device)


def _host_view(addr: int, nbytes: int) -> torch.Tensor:
    buf = (ctypes.c_uint8 * nbytes).from_address(addr)
    return torch.from_numpy(np.ctypeslib.as_array(buf))


_SIGN = np.uint64(1 << 63)


class TorchHostTransport:
    """Factory for a native ``Transport`` backed by torch.distributed p2p on host memory."""

    def __new__(cls, group=None):
        C = load()

        class _T(C.Transport):
            def __init__(self, g):
                C.Transport.__init__(self)
                self.g = g

            def name(self):
                return "torch." + dist.get_backend(self.g)

            def rank(self):
                return dist.get_rank(self.g)

            def size(self):
                return dist.get_world_size(self.g)

            def device(self):
                return False

            def exchange(self, sends, recvs, stream):
                ops = []
                for peer, tag, addr, nb in recvs:
                    ops.append(dist.irecv(_host_view(addr, nb), src=peer, group=self.g, tag=tag))
                for peer, tag, addr, nb in sends:
                    ops.append(dist.isend(_host_view(addr, nb), dst=peer, group=self.g, tag=tag))
                for w in ops:
                    w.wait()

            def allreduce_max_u64(self, addr, n, stream):
                # order-preserving keys: flip the sign bit so signed max == unsigned max
                a = np.ctypeslib.as_array((ctypes.c_uint64 * n).from_address(addr))
                t = torch.from_numpy((a ^ _SIGN).view(np.int64).copy())
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.g)
                a[:] = t.numpy().view(np.uint64) ^ _SIGN

            def allreduce_max_host(self, values):
                t = torch.tensor(values, dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.g)
                return t.tolist()

            def barrier(self):
                dist.barrier(group=self.g)

        return _T(group)
