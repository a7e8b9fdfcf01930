"""Console entry points (pyproject.toml [project.scripts]) for the native programs.

``wave3d-solve N Np Lx Ly Lz [T] [timesteps] [options]`` runs the MI355X program and
``wave3d-cpu ...`` the OpenMP oracle, both with the reference's command line
(mpi_new.cpp:382-393). The program runs as a child process (this process never touches the
GPU) and its exit code is returned.
"""
from __future__ import annotations

import subprocess
import sys

from ._native import program


def _run(name: str, argv: list[str] | None) -> int:
    return subprocess.call([program(name)] + list(sys.argv[1:] if argv is None else argv))


def solve_main(argv: list[str] | None = None) -> int:
    return _run("wave3d", argv)


def cpu_main(argv: list[str] | None = None) -> int:
    return _run("wave3d_cpu", argv)


if __name__ == "__main__":
    sys.exit(solve_main())
