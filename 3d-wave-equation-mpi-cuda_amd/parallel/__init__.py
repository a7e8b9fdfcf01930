"""Parallelism: 3-D domain decomposition (native topology) and transports.

Strategies: P1 spatial 3-D block decomposition with face halos, P3 GPU
kernels, P4 ranks x GPU, P5 simulated ranks (``ranks=P`` loopback), P6 RCCL p2p halos,
P7 max-reduction of the per-layer errors.
"""
from .topology import dims_create, topology  # noqa: F401


def __getattr__(name):
    if name in ("init_from_env", "rccl_transport", "TorchHostTransport", "env_rank",
                "broadcast_bytes", "TorchStagedTransport", "make_transport"):
        from . import dist as _d

        return getattr(_d, name)
    raise AttributeError(name)
