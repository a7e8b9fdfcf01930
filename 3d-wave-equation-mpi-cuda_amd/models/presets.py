"""Benchmark/validation configurations (BASELINE.json "configs").

The reference defaults (T=1, K=20) are unstable for N >= 256 with L = pi (C > 1/sqrt(3),
SURVEY §4.2.3), so every GPU config uses a stable K.
"""
from __future__ import annotations

from .wave import WaveProblem

# Reference numbers measured on the survey host, Mpoints/s.
BASELINE_MPTS = {512: 138.5, 1024: 159.8, 128: 96.7}
# Accuracy goldens: final-layer L-inf abs for L=pi, T=1.
GOLDEN_LINF = {
    (32, 20): 1.75963e-04,
    (64, 20): 4.22698e-05,
    (128, 20): 8.81051e-06,
    (256, 40): 2.20262e-06,
    (512, 100): 6.03381e-07,
    (1024, 100): 8.04265e-08,
}

CONFIGS = {
    # N=128^3 fp64 single-process OpenMP (openmp_sol path, plumbing)
    "cpu128": dict(problem=WaveProblem(128, timesteps=20), backend="cpu", Np=8, dims=None),
    # N=512^3 fp64 on one MI355X
    "gpu512": dict(problem=WaveProblem(512, timesteps=100), backend="hip", Np=1, dims=None),
    # N=512^3 fp64 on 2 MI355X, slab decomposition (2x1x1)
    "gpu512x2": dict(problem=WaveProblem(512, timesteps=100), backend="hip", Np=2, dims=[2, 1, 1]),
    # config 4's grid on 4 MI355X (MPI_Dims_create(4) = 2x2x1; bench.py --gpus 4)
    "gpu1024x4": dict(problem=WaveProblem(1024, timesteps=100), backend="hip", Np=4, dims=[2, 2, 1]),
    # N=1024^3 fp64 on 8 MI355X, 2x2x2 blocks (6-face deep halos, interior/shell overlap)
    "gpu1024x8": dict(problem=WaveProblem(1024, timesteps=100), backend="hip", Np=8, dims=[2, 2, 2]),
    # N=2048^3 fp32 on 8 MI355X; the increment form (profiles/fp32_scheme_r4.txt: 6.3x lower
    # L-inf than fp32 leapfrog, and 3 % faster on the tb3 sweep)
    "gpu2048x8_fp32": dict(problem=WaveProblem(2048, timesteps=200, dtype="fp32", scheme="delta"), backend="hip",
                           Np=8, dims=None),
}


def default_scheme(dtype: str) -> str:
    """Time-stepping form for a precision. fp64: the reference's leapfrog (bitwise parity with
    its error tables). fp32: the increment form u^n = u^{n-1} + d^n, d^n = d^{n-1} + a2 tau^2
    lap u^{n-1} — the same scheme in exact arithmetic, without leapfrog's 2u - u cancellation that
    sets the fp32 error floor (mpi_new.cpp:338); measured 3.2x (N=512) / 6.3x (N=2048) lower
    L-inf at +3 % throughput on the tb3 sweep (profiles/fp32_scheme_r4.txt; round 2, tb2:
    profiles/fp32_accuracy_r2.txt)."""
    return "leapfrog" if dtype == "fp64" else "delta"


# bench.py --gpus n: the BASELINE.json config for that GPU count, each backed by a golden
# L-inf (decomposition-invariant: the reference's errors are identical for every P).
#   1: config 2 (N=512, one GPU)              2: config 3 (N=512, 2x1x1 slabs)
#   4: config 4's grid on MPI_Dims_create(4)  8: config 4 (N=1024, 2x2x2 blocks)
# 1 -> 8 is weak scaling (1025^3/8 ~= 513^3 nodes per GPU); 2 and 4 are strong-scaling points
# of the 512^3 and 1024^3 grids.
BENCH_BY_GPUS = {
    1: dict(N=512, dims=None, scaling="weak", config="gpu512"),
    2: dict(N=512, dims=[2, 1, 1], scaling="strong", config="gpu512x2"),
    4: dict(N=1024, dims=[2, 2, 1], scaling="strong", config="gpu1024x4"),
    8: dict(N=1024, dims=[2, 2, 2], scaling="weak", config="gpu1024x8"),
}


def bench_plan(n_gpus: int) -> dict:
    """Global N, decomposition, scaling kind and golden of the benchmark at n_gpus."""
    if n_gpus in BENCH_BY_GPUS:
        p = dict(BENCH_BY_GPUS[n_gpus])
    else:
        p = dict(N=weak_scaling_N(n_gpus), dims=None, scaling="weak", config=f"weak{n_gpus}")
    p["golden"] = GOLDEN_LINF.get((p["N"], 100))
    return p


def weak_scaling_N(n_gpus: int, base_N: int = 512) -> int:
    """Global N keeping (N+1)^3 / n_gpus ~= (base_N+1)^3 (per-GPU work fixed)."""
    if n_gpus <= 1:
        return base_N
    if n_gpus == 8 and base_N == 512:
        return 1024  # the BASELINE 8-GPU config (1025^3 / 8 = 134.6M vs 513^3 = 135.0M)
    return round((base_N + 1) * n_gpus ** (1.0 / 3.0)) - 1


def bench_problem(n_gpus: int, timesteps: int = 100, dtype: str = "fp64") -> WaveProblem:
    return WaveProblem(weak_scaling_N(n_gpus), timesteps=timesteps, dtype=dtype)


def default_math(backend: str, dtype: str) -> str:
    """Stencil arithmetic of the benchmark. The GPU runs the FMA form (coef/h^2 folded; the
    fp64 sweep is issue-bound, and it lets three-layer blocking beat two-layer: 364k vs 316-323k
    Mpts/s at N=512 fp64 with the same 9-digit L-inf, profiles/math_fma_r3.txt); the CPU
    oracle keeps the reference's exact operation order. `--math exact` reproduces the
    reference's printed tables bit for bit on the GPU too."""
    return "fma" if backend == "hip" else "exact"
