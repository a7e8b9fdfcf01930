"""Cartesian decomposition queries, answered by the native topology (csrc/topology.cpp).

Semantics of MPI_Dims_create + MPI_Cart_create(periods={1,0,0}, reorder=false) +
Cart_shift as used by the reference (mpi_new.cpp:409-433).
"""
from __future__ import annotations

from .._native import load


def dims_create(nprocs: int, dims=(0, 0, 0)) -> list[int]:
    return load().dims_create(int(nprocs), list(dims))


def topology(N: int, nprocs: int, rank: int, dims=(0, 0, 0)) -> dict:
    """Decomposition of rank ``rank``: dims, coords, ext (X,Y,Z), off (x0,y0,z0),
    nbr[axis] = [minus, plus] (-1 = none), compute/error/owned boxes (local indices),
    and the halo message plan (axis, side, peer, tag, count)."""
    return load().topology(int(N), int(nprocs), int(rank), list(dims))
