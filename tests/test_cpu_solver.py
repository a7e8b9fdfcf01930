"""OpenMP oracle: goldens (Appendix C), decomposition invariance, bitwise agreement with the
plain-PyTorch solve, fp32, checkpoint/resume, fault detection."""
import os

import pytest


def _solve(prob, **kw):
    import wave3d

    kw.setdefault("threads", 4)
    return wave3d.WaveSolver(prob, "cpu", **kw).run()


def _fmt(r):
    from wave3d.utils import fmt6

    return [(fmt6(a), fmt6(b)) for a, b in zip(r.max_abs, r.max_rel)]


@pytest.mark.parametrize("ranks", [0, 2, 4, 8])
def test_golden_table_n32(C, ranks):
    import wave3d
    from wave3d.utils import GOLDEN_N32_K20

    assert _fmt(_solve(wave3d.WaveProblem(32, timesteps=20), ranks=ranks)) == GOLDEN_N32_K20


@pytest.mark.parametrize("key", [(64, 20), (128, 20)])
def test_golden_final(C, key):
    import wave3d
    from wave3d.utils import GOLDEN_FINAL

    N, K = key
    assert _fmt(_solve(wave3d.WaveProblem(N, timesteps=K), threads=8))[-1] == GOLDEN_FINAL[key]


def test_spot_values(C):
    import wave3d
    from wave3d.utils import GOLDEN_SPOTS

    for (N, K, ic), spots in GOLDEN_SPOTS.items():
        if N > 128:
            continue
        got = _fmt(_solve(wave3d.WaveProblem(N, timesteps=K, ic=ic), threads=8))
        for layer, v in spots.items():
            assert got[layer] == v


@pytest.mark.parametrize("ranks,dims", [(2, None), (3, None), (4, None), (6, None), (8, None),
                                        (4, (1, 2, 2)), (4, (1, 1, 4)), (2, (1, 2, 1))])
def test_decomposition_invariance(C, ranks, dims):
    """The shifted IC exercises the periodic seams; every decomposition,
    including dims[0]=1 (local periodic wrap) must give identical per-layer errors."""
    import wave3d

    p = wave3d.WaveProblem(27, Lx=1.3, Ly="pi", Lz=2.1, timesteps=11, ic="shifted")
    base = _solve(p)
    r = _solve(p, ranks=ranks, dims=dims)
    assert r.max_abs == base.max_abs and r.max_rel == base.max_rel


def test_bitwise_equal_to_torch_reference(C):
    import wave3d
    from wave3d.ops import reference

    for ic, phase in (("ref", 0.0), ("shifted", 0.7)):
        r = _solve(wave3d.WaveProblem(24, Lx=1.1, Ly="pi", Lz=1.9, timesteps=9, ic=ic))
        a, b, _ = reference.solve(24, 9, L=(1.1, "pi", 1.9), phase=phase)
        assert r.max_abs == a and r.max_rel == b


def test_delta_scheme_bitwise_equal_to_torch_reference(C):
    """Increment form (--scheme delta) of the OpenMP oracle == the PyTorch delta solve."""
    import wave3d
    from wave3d.ops import reference

    for ic, phase in (("ref", 0.0), ("shifted", 0.7)):
        r = _solve(wave3d.WaveProblem(24, Lx=1.1, Ly="pi", Lz=1.9, timesteps=9, ic=ic, scheme="delta"))
        a, b, _ = reference.solve(24, 9, L=(1.1, "pi", 1.9), phase=phase, scheme="delta")
        assert r.max_abs == a and r.max_rel == b and r.extra["scheme"] == "delta"
        # decomposition invariance holds for the increment form too
        m = _solve(wave3d.WaveProblem(24, Lx=1.1, Ly="pi", Lz=1.9, timesteps=9, ic=ic, scheme="delta"),
                   ranks=4)
        assert m.max_abs == r.max_abs and m.max_rel == r.max_rel


def test_delta_scheme_fp32_accuracy(C):
    """fp32 with the increment form stays at the fp64 error (the leapfrog's 2u - u cancellation
    is gone); plain fp32 leapfrog is ~80x worse here (N=128, K=400)."""
    import wave3d

    p = dict(timesteps=400)
    e64 = _solve(wave3d.WaveProblem(128, **p)).max_abs[-1]
    lf32 = _solve(wave3d.WaveProblem(128, dtype="fp32", **p)).max_abs[-1]
    d32 = _solve(wave3d.WaveProblem(128, dtype="fp32", scheme="delta", **p)).max_abs[-1]
    assert d32 < 1.2 * e64 and lf32 > 20 * d32


def test_fp32_close_to_fp64(C):
    import wave3d

    a = _solve(wave3d.WaveProblem(48, timesteps=20))
    b = _solve(wave3d.WaveProblem(48, timesteps=20, dtype="fp32"))
    assert b.dtype == "fp32"
    assert b.max_abs[-1] == pytest.approx(a.max_abs[-1], rel=0.05)


def test_checkpoint_resume_bitwise(C, tmp_path):
    import wave3d

    p = wave3d.WaveProblem(20, timesteps=14, ic="shifted")
    full = _solve(p, ranks=4)
    _solve(p, ranks=4, checkpoint_every=6, checkpoint_dir=str(tmp_path))
    res = _solve(p, ranks=4, resume=str(tmp_path))
    assert res.extra["resumed_from"] == 12
    assert res.max_abs == full.max_abs and res.max_rel == full.max_rel
    # a different configuration is refused
    with pytest.raises(Exception):
        _solve(wave3d.WaveProblem(20, timesteps=15), ranks=4, resume=str(tmp_path))


def test_checkpoint_resume_delta_scheme(C, tmp_path):
    """The increment form checkpoints d^n with u^n and resumes bitwise; a leapfrog run refuses
    those files (the header records the scheme)."""
    import wave3d

    p = wave3d.WaveProblem(20, timesteps=14, ic="shifted", dtype="fp32", scheme="delta")
    full = _solve(p, ranks=2)
    _solve(p, ranks=2, checkpoint_every=6, checkpoint_dir=str(tmp_path))
    res = _solve(p, ranks=2, resume=str(tmp_path))
    assert res.extra["resumed_from"] == 12
    assert res.max_abs == full.max_abs and res.max_rel == full.max_rel
    with pytest.raises(Exception):
        _solve(wave3d.WaveProblem(20, timesteps=14, ic="shifted", dtype="fp32"), ranks=2,
               resume=str(tmp_path))


def test_checkpoint_records_math_mode(C, tmp_path):
    """The header records --math: an fma run neither resumes from an exact run's
    checkpoints nor prunes them, and the exact run still resumes bitwise afterwards."""
    import wave3d

    d = str(tmp_path)
    exact = wave3d.WaveProblem(20, timesteps=14, ic="shifted")
    fma = wave3d.WaveProblem(20, timesteps=14, ic="shifted", math="fma")
    full = _solve(exact, ranks=2)
    _solve(exact, ranks=2, checkpoint_every=6, checkpoint_dir=d)
    for r in range(2):
        assert C.checkpoint_layers(d, r) == [6, 12]
    with pytest.raises(Exception):
        _solve(fma, ranks=2, resume=d)
    # an fma run checkpointing into the same directory leaves the exact files alone
    _solve(fma, ranks=2, checkpoint_every=5, checkpoint_dir=d)
    for r in range(2):
        assert C.checkpoint_layers(d, r) == [5, 6, 10, 12]
    res = _solve(exact, ranks=2, resume=d)
    assert res.extra["resumed_from"] == 12
    assert res.max_abs == full.max_abs and res.max_rel == full.max_rel
    resf = _solve(fma, ranks=2, resume=d)
    assert resf.extra["resumed_from"] == 10 and resf.extra["math"] == "fma"


def test_checkpoint_generations_and_agreed_resume(C, tmp_path):
    """Two complete generations per rank are kept; a rank whose newest file is missing (a crash
    while writing it) makes every rank resume from the newest layer they all have."""
    import wave3d

    p = wave3d.WaveProblem(20, timesteps=14, ic="shifted")
    full = _solve(p, ranks=3)
    d = str(tmp_path)
    _solve(p, ranks=3, checkpoint_every=3, checkpoint_dir=d)
    for r in range(3):
        assert C.checkpoint_layers(d, r) == [9, 12]
    os.remove(os.path.join(d, "ckpt_r1_L12.bin"))  # rank 1 died writing layer 12
    res = _solve(p, ranks=3, resume=d)
    assert res.extra["resumed_from"] == 9
    assert res.max_abs == full.max_abs and res.max_rel == full.max_rel
    os.remove(os.path.join(d, "ckpt_r2_L9.bin"))  # no layer common to every rank any more
    with pytest.raises(Exception, match="common"):
        _solve(p, ranks=3, resume=d)


def test_checkpoint_stale_files_of_other_runs(C, tmp_path):
    """A directory still holding higher-layer files of other runs (a longer K, another N, and
    the same configuration run further before) neither makes pruning delete this run's
    checkpoints nor makes resume pick a stale file (files are matched on the header)."""
    import shutil

    import wave3d

    d = str(tmp_path)
    other = tmp_path / "other"
    # a longer run (K=30) and another N leave layers 24/27 and 12 behind for ranks 0..2
    _solve(wave3d.WaveProblem(20, timesteps=30, ic="shifted"), ranks=3, checkpoint_every=3, checkpoint_dir=str(other))
    _solve(wave3d.WaveProblem(22, timesteps=14, ic="shifted"), ranks=3, checkpoint_every=12,
           checkpoint_dir=str(other / "n22"))
    for f in os.listdir(other):
        if f.endswith(".bin"):
            shutil.copy(other / f, tmp_path / f)
    for f in os.listdir(other / "n22"):
        shutil.copy(other / "n22" / f, tmp_path / ("x" + f))  # different names must not matter
    # the same configuration once left layer 13 behind; this run checkpoints layers 6 and 12:
    # writing 6 removes the superseded 13 (it would otherwise outrank this run's files)
    p = wave3d.WaveProblem(20, timesteps=14, ic="shifted")
    _solve(p, ranks=3, checkpoint_every=13, checkpoint_dir=d)
    for r in range(3):
        assert C.checkpoint_layers(d, r) == [13, 24, 27]
    full = _solve(p, ranks=3)
    _solve(p, ranks=3, checkpoint_every=6, checkpoint_dir=d)
    for r in range(3):
        assert C.checkpoint_layers(d, r) == [6, 12, 24, 27]  # K=30's two newest survive untouched
    res = _solve(p, ranks=3, resume=d)
    assert res.extra["resumed_from"] == 12
    assert res.max_abs == full.max_abs and res.max_rel == full.max_rel


def test_checkpoint_agreed_resume_multiprocess(C, tmp_path):
    """The same agreement across processes (gloo host transport, 2 ranks): rank 1's newest
    checkpoint is missing, both processes resume from layer 9 and reproduce the full run."""
    from test_dist import torchrun

    args = ["20", "1", "pi", "pi", "pi", "1", "14", "--ic", "shifted", "--threads", "1"]
    d = str(tmp_path)
    full = torchrun(2, ["--backend", "cpu", "--transport", "gloo"], args)
    torchrun(2, ["--backend", "cpu", "--transport", "gloo"],
             args + ["--checkpoint-every", "3", "--checkpoint-dir", d])
    assert C.checkpoint_layers(d, 0) == [9, 12] and C.checkpoint_layers(d, 1) == [9, 12]
    os.remove(os.path.join(d, "ckpt_r1_L12.bin"))
    res = torchrun(2, ["--backend", "cpu", "--transport", "gloo"], args + ["--resume", d])
    assert res["resumed_from"] == 9
    assert res["max_abs"] == full["max_abs"] and res["max_rel"] == full["max_rel"]


def test_fault_injection_detected(C):
    import wave3d

    p = wave3d.WaveProblem(16, timesteps=10)
    r = _solve(p, check_every=1, fault="nan:0:3")
    assert r.aborted and r.abort_layer == 4 and "non-finite" in r.abort_reason
    clean = _solve(p, ranks=2)
    bad = _solve(p, ranks=2, fault="drop_face:1:4")
    assert bad.max_abs[-1] > 10 * clean.max_abs[-1]


def test_divergence_abort(C):
    import wave3d

    # C = 1.3 > 1/sqrt(3): the reference silently reports 6.9e7
    p = wave3d.WaveProblem(64, timesteps=20, T=8.0)
    assert p.courant > 1.2
    r = _solve(p, check_every=1)
    assert r.aborted


def test_reference_laplacian_exact_on_quadratics():
    import torch

    from wave3d.ops import reference

    n = 9
    x = torch.arange(n, dtype=torch.float64)
    X, Y, Z = torch.meshgrid(x, x, x, indexing="ij")
    u = 0.5 * X * X + 1.5 * Y * Y - Z * Z + 3 * X * Y
    lap = reference.laplace7(u, 1.0, 1.0, 1.0)
    assert torch.allclose(lap, torch.full_like(lap, 1.0 + 3.0 - 2.0), atol=1e-12)


def test_field_dump_matches_torch_reference(C, cpu_prog, tmp_path):
    """Final-layer field access (print_layer analogue): OpenMP ranks, the .npy dump and the
    plain-PyTorch solve agree bit for bit."""
    import subprocess

    import numpy as np
    import torch

    import wave3d
    from wave3d.ops import reference as R

    N, K = 18, 7
    p = wave3d.WaveProblem(N, timesteps=K, ic="shifted")
    res, g = wave3d.WaveSolver(p, "cpu", ranks=3).solve_field()
    _, _, uK = R.solve(N, K, phase=0.7)
    ref = uK[1:N + 2].numpy()
    assert g.shape == (N + 1,) * 3
    assert np.array_equal(g, ref)
    path = str(tmp_path / "u.npy")
    subprocess.run([cpu_prog] + p.args(1) + ["--ranks", "2", "--dump", path, "--format", "none",
                                              "--quiet"], check=True, cwd=tmp_path)
    assert np.array_equal(np.load(path), ref)


@pytest.mark.parametrize("scheme,dtype", [("leapfrog", "fp64"), ("delta", "fp64"), ("leapfrog", "fp32"),
                                          ("delta", "fp32")])
def test_fma_math_oracle(C, scheme, dtype):
    """--math fma on the OpenMP oracle (the HIP kernels' FMA form, node for node): L-inf abs
    equal to the exact form's within rounding (fp64: 6 significant digits, as printed), the
    same on any decomposition bit for bit."""
    import wave3d

    p = wave3d.WaveProblem(24, Lx=1.3, Ly="pi", Lz=2.0, timesteps=17, ic="shifted", scheme=scheme, dtype=dtype)
    ex = _solve(p)
    p.math = "fma"
    fm = _solve(p)
    assert fm.extra["math"] == "fma" and ex.extra["math"] == "exact"
    if dtype == "fp64":
        assert [f"{a:.6g}" for a in fm.max_abs] == [f"{a:.6g}" for a in ex.max_abs]
    else:
        assert fm.max_abs[-1] == pytest.approx(ex.max_abs[-1], rel=2e-2)
    assert _solve(p, ranks=4).max_abs == fm.max_abs


def test_fma_leapfrog_keeps_reference_goldens(C):
    """The fp64 --math fma leapfrog in 9 operations (stencil_math leap_fm: scaled neighbour pairs
    minus the scaled centre, the leapfrog's 2c - u2 kept), shared by the OpenMP oracle and every
    HIP kernel, keeps the reference's printed L-inf abs table at N=32 K=20 (6 digits; the max
    relative error sits at the rounding noise next to f's zero plane)."""
    import wave3d
    from wave3d.utils import GOLDEN_N32_K20

    r = _solve(wave3d.WaveProblem(32, timesteps=20, math="fma"))
    assert r.extra["math"] == "fma"
    for (a, r_), (ga, gr) in zip(_fmt(r), GOLDEN_N32_K20):
        assert a == ga and float(r_) == pytest.approx(float(gr), rel=1e-2)
