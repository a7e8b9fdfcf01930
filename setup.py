"""Installs the framework directory 3d-wave-equation-mpi-cuda_amd/ as the package ``wave3d``
(its name is not a Python identifier). Build the native parts in-tree first:
``python -c "import __graft_entry__ as g; g.build()"``; the .so files and programs are
shipped as package data."""
from setuptools import setup

PKG = "3d-wave-equation-mpi-cuda_amd"
setup(
    name="wave3d",
    version="0.2.0",
    description="MI355X-native 3-D acoustic wave-equation solver (CDNA4 HIP kernels, RCCL halos)",
    python_requires=">=3.10",
    install_requires=["numpy", "torch"],
    package_dir={"wave3d": PKG},
    packages=["wave3d", "wave3d.models", "wave3d.ops", "wave3d.parallel", "wave3d.utils"],
    package_data={"wave3d": ["_wave3d_C*.so", "build/libwave3d.so", "build/wave3d", "build/wave3d_cpu"]},
    entry_points={"console_scripts": ["wave3d-solve = wave3d.cli:solve_main",
                                      "wave3d-cpu = wave3d.cli:cpu_main"]},
)
