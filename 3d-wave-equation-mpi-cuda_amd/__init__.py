"""wave3d — MI355X-native 3-D acoustic wave-equation solver.

Capabilities of ``aleksgri/3D-wave-equation-MPI-CUDA`` (periodic-x / Dirichlet-y,z leapfrog
with the 7-point Laplacian, per-layer L-inf error against the analytic solution, the
``prog N Np Lx Ly Lz [T] [timesteps]`` CLI and ``output_N{N}_Np{Np}.txt`` report), rebuilt
for AMD Instinct MI355X:

* ``csrc/``     C++17/HIP runtime: topology, hand-written CDNA4 kernels, RCCL transport,
                OpenMP oracle, checkpointing, report writer (``libwave3d.so``,
                programs ``build/wave3d`` and ``build/wave3d_cpu``).
* ``models/``   problem definitions, the solver front-end and benchmark presets.
* ``ops/``      tensor-level access to the HIP kernels plus PyTorch reference ops.
* ``parallel/`` torch.distributed bootstrap of the native RCCL transport, gloo transport.
* ``utils/``    report parsing, golden values, timing helpers.
"""
from ._native import build, load as load_native, program, PKG_DIR  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # lazy: keep `import wave3d` cheap and free of torch/HIP until something is used
    if name in ("WaveProblem", "WaveSolver", "RunResult"):
        from .models import wave

        return getattr(wave, name)
    if name == "presets":
        from .models import presets

        return presets
    raise AttributeError(name)
