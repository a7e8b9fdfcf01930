"""torch.distributed integration.

* :func:`init_from_env` — one process per GPU, torchrun env (RANK / WORLD_SIZE / LOCAL_RANK /
  MASTER_ADDR / MASTER_PORT), ``nccl`` (= RCCL on ROCm) on GPUs, ``gloo`` on CPU.
* :func:`rccl_transport` — the native halo transport: torch.distributed only carries the
  128-byte RCCL unique id; the time loop then runs in C++ with ncclSend/ncclRecv groups on
  the solver's comm stream (no Python in the loop).
* :class:`TorchHostTransport` — a host-memory transport over torch.distributed point-to-
  point (gloo), used by the OpenMP backend for multi-process CPU runs and tests; it is the
  process-level equivalent of the reference's MPI_Sendrecv chain (mpi_new.cpp:201-238).
* :class:`TorchStagedTransport` — a *device* transport that stages faces through host
  memory over gloo. Slow, but lets P processes share one GPU (RCCL refuses duplicate GPUs),
  which is how the multi-process HIP path is tested on a single MI355X — the role MPS
  oversubscription plays in the reference (README.txt:44, cuda_sol.cpp:519).

Both Python transports default to ``fifo=True``: every message travels with tag 0, so
messages between a pair of ranks match strictly in posting order — the semantics of
tag-less ncclSend/ncclRecv. A solver whose per-peer message order were inconsistent
between sender and receiver would fail the multi-process tests here, not only on RCCL.
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


def init_from_env(backend: str | None = None, force: bool = False) -> tuple[int, int, int]:
    """Initialise the default process group from torchrun-style env (idempotent).
    A single-process world is only initialised with ``force`` (no group is needed)."""
    rank, world, local = env_rank()
    if (world > 1 or force) and not dist.is_initialized():
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


def rccl_transport(device: int | None = None, group=None, overlap: str = "auto"):
    """Native RCCL transport for this rank; the unique id travels via torch.distributed. The
    communicator's CTA budget follows the run's overlap mode (C.rccl_max_ctas: RCCL's own budget
    for off and auto, a cap when overlap is forced on and the interior sweep runs beside the halo)."""
    C = load()
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if device is None:
        device = torch.cuda.current_device()
    uid = C.rccl_unique_id() if rank == 0 else None
    uid = broadcast_bytes(uid, 0, group)
    return C.RcclTransport(rank, world, uid, device, C.rccl_max_ctas(overlap))


def _host_view(addr: int, nbytes: int) -> torch.Tensor:
    buf = (ctypes.c_uint8 * nbytes).from_address(addr)
    return torch.from_numpy(np.ctypeslib.as_array(buf))


_SIGN = np.uint64(1 << 63)


class TorchHostTransport:
    """Factory for a native ``Transport`` backed by torch.distributed p2p on host memory."""

    def __new__(cls, group=None, fifo: bool = True):
        C = load()

        class _T(C.Transport):
            def __init__(self, g):
                C.Transport.__init__(self)
                self.g = g
                self.fifo = fifo

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
                    ops.append(dist.irecv(_host_view(addr, nb), src=peer, group=self.g,
                                          tag=0 if self.fifo else tag))
                for peer, tag, addr, nb in sends:
                    ops.append(dist.isend(_host_view(addr, nb), dst=peer, group=self.g,
                                          tag=0 if self.fifo else tag))
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


class TorchStagedTransport:
    """Factory for a device ``Transport``: D2H -> gloo p2p -> H2D (testing/bring-up only)."""

    def __new__(cls, group=None, fifo: bool = True):
        C = load()

        class _S(C.Transport):
            def __init__(self, g):
                C.Transport.__init__(self)
                self.g = g
                self.fifo = fifo

            def name(self):
                return "staged." + dist.get_backend(self.g)

            def rank(self):
                return dist.get_rank(self.g)

            def size(self):
                return dist.get_world_size(self.g)

            def device(self):
                return True

            def exchange(self, sends, recvs, stream):
                C.hip_stream_sync(stream)
                sbufs = []
                for peer, tag, addr, nb in sends:
                    h = np.empty(nb, dtype=np.uint8)
                    C.hip_memcpy(h.ctypes.data, addr, nb, stream)
                    sbufs.append((peer, tag, torch.from_numpy(h)))
                rbufs = [(addr, nb, torch.empty(nb, dtype=torch.uint8)) for _, _, addr, nb in recvs]
                tg = (lambda tag: 0) if self.fifo else (lambda tag: tag)
                ops = [dist.irecv(t, src=peer, group=self.g, tag=tg(tag))
                       for (peer, tag, _, _), (_, _, t) in zip(recvs, rbufs)]
                ops += [dist.isend(t, dst=peer, group=self.g, tag=tg(tag)) for peer, tag, t in sbufs]
                for w in ops:
                    w.wait()
                for addr, nb, t in rbufs:
                    C.hip_memcpy(addr, t.numpy().ctypes.data, nb, stream)

            def allreduce_max_u64(self, addr, n, stream):
                h = np.empty(n, dtype=np.uint64)
                C.hip_memcpy(h.ctypes.data, addr, n * 8, stream)
                t = torch.from_numpy((h ^ _SIGN).view(np.int64).copy())
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.g)
                out = t.numpy().view(np.uint64) ^ _SIGN
                C.hip_memcpy(addr, out.ctypes.data, n * 8, stream)

            def allreduce_max_host(self, values):
                t = torch.tensor(values, dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.g)
                return t.tolist()

            def barrier(self):
                dist.barrier(group=self.g)

        return _S(group)


def make_transport(kind: str, backend: str = "hip", overlap: str = "auto"):
    """'rccl' (native, one GPU per rank), 'staged' (device via gloo), 'gloo' (host, CPU)."""
    if kind == "rccl":
        return rccl_transport(torch.cuda.current_device(), overlap=overlap)
    if kind == "staged":
        return TorchStagedTransport()
    if kind in ("gloo", "host"):
        return TorchHostTransport()
    raise ValueError(f"unknown transport {kind}")
