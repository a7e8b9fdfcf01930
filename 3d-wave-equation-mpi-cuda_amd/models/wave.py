"""Solver front-end: a problem description plus a runner over the native backends.

``WaveProblem`` mirrors the reference CLI (``prog N Np Lx Ly Lz [T] [timesteps]``,
mpi_new.cpp:382-393) and its physics (mpi_new.cpp:396-405); ``WaveSolver`` runs it on the
HIP backend (MI355X) or the OpenMP oracle, single rank, simulated ranks, or one rank of a
torch.distributed job.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Any

from .._native import load

PI_REF = 3.1415926535  # the reference CPU programs' truncated pi (mpi_new.cpp:23)
CFL_LIMIT = 1.0 / math.sqrt(3.0)


def _len_arg(v) -> str:
    if isinstance(v, str):
        return v
    return repr(float(v))


@dataclass
class WaveProblem:
    N: int
    Lx: Any = "pi"
    Ly: Any = "pi"
    Lz: Any = "pi"
    T: float = 1.0
    timesteps: int = 20
    dtype: str = "fp64"
    pi: str = "ref"
    ic: str = "ref"
    scheme: str = "leapfrog"  # "delta": increment form (u^n = u^{n-1} + d^n), fp32 accuracy
    math: str = "exact"       # "fma": coef/h^2 folded into FMAs (temporal-blocking kernels)

    def _pi(self) -> float:
        return PI_REF if self.pi == "ref" else math.pi

    def lengths(self) -> tuple[float, float, float]:
        p = self._pi()
        return tuple(p if v == "pi" else float(v) for v in (self.Lx, self.Ly, self.Lz))

    @property
    def courant(self) -> float:
        p = self._pi()
        a = math.sqrt(1 / (4 * p * p))
        tau = self.T / self.timesteps
        return a * tau / (min(self.lengths()) / self.N)

    def stable(self) -> bool:
        return self.courant <= CFL_LIMIT

    def min_stable_timesteps(self) -> int:
        """Smallest K with C <= 1/sqrt(3) (the reference never checks)."""
        p = self._pi()
        a = math.sqrt(1 / (4 * p * p))
        return math.ceil(a * self.T * self.N / (min(self.lengths()) * CFL_LIMIT))

    @property
    def points(self) -> int:
        return (self.N + 1) ** 3

    def args(self, Np: int = 1, **opts) -> list[str]:
        a = [str(self.N), str(Np), _len_arg(self.Lx), _len_arg(self.Ly), _len_arg(self.Lz),
             repr(float(self.T)), str(self.timesteps),
             "--dtype", self.dtype, "--pi", self.pi, "--ic", self.ic, "--scheme", self.scheme,
             "--math", self.math]
        for k, v in opts.items():
            if v is None or v is False:
                continue
            flag = "--" + k.replace("_", "-")
            if v is True:
                a.append(flag)
            elif isinstance(v, (list, tuple)):
                a += [flag, ",".join(str(x) for x in v)]
            else:
                a += [flag, str(v)]
        return a


@dataclass
class RunResult:
    N: int
    timesteps: int
    nprocs: int
    dims: list
    dtype: str
    backend: str
    kernel: str
    transport: str
    courant: float
    max_abs: list
    max_rel: list
    total_ms: float
    init_ms: float
    loop_ms: float
    exchange_ms: float
    comm_ms: float
    solve_ms: list
    mpts_per_s: float
    mpts_per_s_best: float
    aborted: bool
    abort_layer: int
    abort_reason: str
    report: str
    json: str
    extra: dict = field(default_factory=dict)

    @property
    def linf_abs(self) -> float:
        return self.max_abs[-1]

    @classmethod
    def from_dict(cls, d: dict) -> "RunResult":
        names = set(cls.__dataclass_fields__) - {"extra"}
        kw = {k: d[k] for k in names if k in d}
        return cls(**kw, extra={k: v for k, v in d.items() if k not in names})


class WaveSolver:
    """Run a :class:`WaveProblem`.

    backend   "hip" (MI355X kernels) or "cpu" (OpenMP oracle)
    ranks     >0: simulate that many ranks in this process (loopback transport)
    overlap   True / False / "auto" (time the first two solves on and off, keep the faster)
    graph     "auto" | "on" | "off": replay the IC + time loop as one hipGraph
    transport a native transport (``parallel.rccl_transport()`` / ``TorchHostTransport``)
              making this process one rank of a distributed job
    model_link "GBPS[,LAT_US]": every halo exchange also waits its busiest link's modelled time
              (overlap rehearsals on one GPU, --model-link)
    """

    def __init__(self, problem: WaveProblem, backend: str = "hip", *, ranks: int = 0,
                 dims=None, overlap=True, kernel: str = "auto", chunk: int = 0,
                 transport=None, Np: int | None = None, threads: int = 0, fmt: str = "none",
                 out_dir: str | None = None, check_every: int = 0, fault: str | None = None,
                 checkpoint_every: int = 0, checkpoint_dir: str | None = None,
                 resume: str | None = None, profile: bool = False, device: int | None = None,
                 graph: str = "auto", model_link: str | None = None):
        self.problem = problem
        self.backend = backend
        self.transport = transport
        self.Np = Np if Np is not None else (transport.size() if transport is not None else max(1, ranks))
        ov = overlap if isinstance(overlap, str) else ("on" if overlap else "off")
        self.opts = dict(ranks=ranks or None, dims=dims, overlap=ov, kernel=kernel,
                         chunk=chunk or None, threads=threads or None, format=fmt,
                         out_dir=out_dir, check_every=check_every or None, fault=fault,
                         checkpoint_every=checkpoint_every or None,
                         checkpoint_dir=checkpoint_dir, resume=resume, profile=profile,
                         device=device, graph=graph if backend == "hip" else None,
                         model_link=model_link if backend == "hip" else None, quiet=True)

    def args(self, **extra) -> list[str]:
        o = dict(self.opts)
        o.update(extra)
        return self.problem.args(self.Np, **o)

    def solve_field(self, layer: int | None = None):
        """One solve, then layer K (default) or K-1 as a NumPy array of the global grid
        ((N+1)^3, float64) when every rank lives in this process, else this process's blocks
        (dicts with rank / off / ext / data) — the reference's print_layer debug aid (C30)."""
        import numpy as np

        C = load()
        a = self.args()
        sess = C.Session(a, self.backend, self.transport)
        res = RunResult.from_dict(sess.solve(a))
        blocks = sess.field(self.problem.timesteps if layer is None else layer)
        if len(blocks) != res.nprocs:
            return res, blocks
        n1 = self.problem.N + 1
        g = np.zeros((n1, n1, n1))
        for b in blocks:
            (i0, j0, k0), (ni, nj, nk) = b["off"], b["ext"]
            g[i0:i0 + ni, j0:j0 + nj, k0:k0 + nk] = np.asarray(b["data"]).reshape(ni, nj, nk)
        return res, g

    def run(self, repeat: int = 1, warmup: int = 0, write: bool = False, root: bool = True) -> RunResult:
        C = load()
        a = self.args(repeat=repeat, warmup=warmup or None)
        d = C.run(a, self.backend, self.transport, write, root)
        return RunResult.from_dict(d)
