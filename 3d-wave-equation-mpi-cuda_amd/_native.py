"""Loader for the in-tree native extension ``_wave3d_C`` (C++/HIP runtime, pybind11).

``torch`` is imported first on purpose: the extension links ``libamdhip64.so.7`` and
``librccl.so.1`` by soname, so inside a torch process it binds to the HIP runtime and RCCL
that torch already loaded instead of pulling in a second copy of either.

There is no Python fallback for the solver or the kernels: if the extension is missing
this raises, so a GPU run can never silently degrade to an eager/PyTorch path.
"""
from __future__ import annotations

import glob
import importlib.util
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(PKG_DIR, "build")

_C = None


def extension_path() -> str | None:
    hits = sorted(glob.glob(os.path.join(PKG_DIR, "_wave3d_C*.so")))
    return hits[0] if hits else None


def build(jobs: int = 8, arch: str = "gfx950", quiet: bool = True) -> None:
    """Compile libwave3d, the programs and the Python binding for ``arch`` (in-tree)."""
    cmd = ["make", "-C", PKG_DIR, f"-j{jobs}", f"ARCH={arch}", f"PYTHON={sys.executable}"]
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("wave3d native build failed:\n" + out.stdout[-4000:] + out.stderr[-8000:])
    if not quiet:
        print(out.stdout)


def load():
    """Import and return the native module (raises ImportError if it is not built)."""
    global _C
    if _C is not None:
        return _C
    import torch  # noqa: F401  (see module docstring: shared HIP runtime / RCCL)

    path = extension_path()
    if path is None:
        raise ImportError(
            "wave3d native extension _wave3d_C is not built; run "
            f"`make -C {PKG_DIR}` or `python -c 'import wave3d; wave3d.build()'`"
        )
    spec = importlib.util.spec_from_file_location("wave3d._wave3d_C", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["wave3d._wave3d_C"] = mod
    _C = mod
    return mod


def program(name: str) -> str:
    """Absolute path of a built program (``wave3d`` or ``wave3d_cpu``)."""
    p = os.path.join(BUILD_DIR, name)
    if not os.path.exists(p):
        raise FileNotFoundError(f"{p} not built; run `make -C {PKG_DIR}`")
    return p
