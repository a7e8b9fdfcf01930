"""End-to-end HIP solver tests on one MI355X: goldens, decomposition invariance (simulated
ranks, with and without the interior/shell overlap), CPU/GPU bitwise agreement, fp32,
checkpoint/resume, fault detection, the CLI program."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu


def _solve(prob, backend="hip", **kw):
    import wave3d

    return wave3d.WaveSolver(prob, backend, **kw).run()


def _fmt(r):
    from wave3d.utils import fmt6

    return [(fmt6(a), fmt6(b)) for a, b in zip(r.max_abs, r.max_rel)]


@pytest.mark.parametrize("kernel", ["march", "naive", "flat", "auto", "march8", "tb2", "tb2r4", "tb2r4w8", "tb2r2w16", "tb3", "tb2r2w8k2", "tb2r2w16k2"])
def test_golden_n32(C, kernel):
    import wave3d
    from wave3d.utils import GOLDEN_N32_K20

    r = _solve(wave3d.WaveProblem(32, timesteps=20), kernel=kernel)
    assert r.backend == "hip" and r.kernel == {"march": "march4", "auto": "tb4"}.get(kernel, kernel)
    assert _fmt(r) == GOLDEN_N32_K20


@pytest.mark.parametrize("kernel", ["auto", "march2", "naive"])
@pytest.mark.parametrize("ranks,overlap", [(2, True), (2, False), (4, True), (8, True), (8, False), (3, True)])
def test_decomposition_invariance(C, ranks, overlap, kernel):
    """auto = temporal blocking (2-deep halos), march2/naive = single-step (6-face halos), all
    on the MPI_Dims_create decomposition (2x2x2 at 8 ranks) as in the reference."""
    import wave3d

    p = wave3d.WaveProblem(40, Lx=1.3, Ly="pi", Lz=2.0, timesteps=15, ic="shifted")
    base = _solve(p, kernel="march2")
    r = _solve(p, ranks=ranks, overlap=overlap, kernel=kernel)
    assert r.transport == "loopback"
    assert r.dims == C.dims_create(ranks, [0, 0, 0])
    assert r.max_abs == base.max_abs and r.max_rel == base.max_rel


def test_cpu_gpu_bitwise(C):
    import wave3d

    p = wave3d.WaveProblem(37, Lx=1.7, Ly=2.2, Lz="pi", timesteps=12, ic="shifted")
    g = _solve(p)
    c = _solve(p, backend="cpu", threads=4)
    assert g.max_abs == c.max_abs and g.max_rel == c.max_rel


def test_spots_and_shifted(C):
    import wave3d
    from wave3d.utils import GOLDEN_SPOTS

    for (N, K, ic), spots in GOLDEN_SPOTS.items():
        if N > 128:
            continue
        got = _fmt(_solve(wave3d.WaveProblem(N, timesteps=K, ic=ic)))
        for layer, val in spots.items():
            assert got[layer] == val, (N, K, ic, layer)


def test_n512_golden(C):
    import wave3d
    from wave3d.utils import GOLDEN_SPOTS

    got = _fmt(_solve(wave3d.WaveProblem(512, timesteps=100)))
    for layer, val in GOLDEN_SPOTS[(512, 100, "ref")].items():
        assert got[layer] == val


def test_fp32_close(C):
    import wave3d

    p64 = wave3d.WaveProblem(64, timesteps=20)
    p32 = wave3d.WaveProblem(64, timesteps=20, dtype="fp32")
    a, b = _solve(p64), _solve(p32)
    assert b.max_abs[-1] == pytest.approx(a.max_abs[-1], rel=0.05)


@pytest.mark.parametrize("kernel", ["auto", "tb3", "march2"])
@pytest.mark.parametrize("K", [12, 13])
def test_checkpoint_resume(C, tmp_path, kernel, K):
    import wave3d

    p = wave3d.WaveProblem(30, timesteps=K, ic="shifted")
    full = _solve(p, ranks=2, kernel=kernel)
    d = str(tmp_path)
    _solve(p, ranks=2, checkpoint_every=5, checkpoint_dir=d, kernel=kernel)
    # a checkpoint is written at the end of a sweep holding a multiple of 5 (not the last one):
    # layer 10 for single steps; three-layer sweeps (tb3: layers 1-3, 4-6, 7-9, 10-12, then a
    # single step for K=13): layer 6 at K=12 and 12 at K=13; four-layer sweeps of the fp64 auto
    # kernel (tb4: 1-4, 5-8, 9-12, then a single step for K=13): 8 at K=12 and 12 at K=13
    layers = sorted(int(f[len("ckpt_r0_L"):-4]) for f in os.listdir(d) if f.startswith("ckpt_r0_L"))
    want = {"march2": {12: 10, 13: 10}, "tb3": {12: 6, 13: 12}, "auto": {12: 8, 13: 12}}[kernel][K]
    assert layers and layers[-1] == want
    res = _solve(p, ranks=2, resume=d, kernel=kernel)
    assert res.extra["resumed_from"] == layers[-1]
    assert res.max_abs == full.max_abs and res.max_rel == full.max_rel


def test_fault_detection(C):
    import wave3d

    p = wave3d.WaveProblem(24, timesteps=10)
    r = _solve(p, check_every=1, fault="nan:0:4")
    # the NaN is written after the sweep holding layer 4 and seen by the next sweep's fused
    # errors: layer 5 with two-layer sweeps, up to 8 with the four-layer sweeps of the fp64 auto (tb4)
    assert r.aborted and 4 <= r.abort_layer <= 8
    ok = _solve(p, check_every=1)
    assert not ok.aborted
    bad = _solve(p, ranks=2, fault="drop_face:1:4")  # an exchanged layer for tb2 and march2
    assert bad.max_abs[-1] > 10 * ok.max_abs[-1]


def test_program_cli_matches_cpu(C, gpu_prog, cpu_prog, tmp_path):
    for prog in (gpu_prog, cpu_prog):
        subprocess.run([prog, "32", "1", "pi", "pi", "pi", "1", "20", "--format", "new",
                        "--out-dir", str(tmp_path), "--out-name", os.path.basename(prog) + ".txt"],
                       check=True, capture_output=True, timeout=120)
    a = open(tmp_path / "wave3d.txt").read().splitlines()
    b = open(tmp_path / "wave3d_cpu.txt").read().splitlines()
    ea = [l for l in a if l.startswith("max abs")]
    eb = [l for l in b if l.startswith("max abs")]
    assert ea == eb and len(ea) == 21
    assert a[0].startswith("grids initialized in") and a[1].startswith("numerical solution calculated in")


def test_session_reuse(C):
    import wave3d

    p = wave3d.WaveProblem(32, timesteps=20)
    s = wave3d.WaveSolver(p, "hip")
    args = s.args()
    sess = C.Session(args, "hip", None)
    r1 = sess.solve(args)
    r2 = sess.solve(args)
    assert r1["max_abs"] == r2["max_abs"]


@pytest.mark.parametrize("kernel", ["tb2", "tb2r4"])
@pytest.mark.parametrize("N,K,L,ic", [(37, 12, (1.7, 2.2, "pi"), "shifted"),
                                      (30, 13, ("pi", "pi", "pi"), "shifted"),
                                      (21, 1, (1.0, 1.3, 0.9), "ref"),
                                      (70, 9, ("pi", 1.5, "pi"), "ref"),
                                      (12, 6, ("pi", "pi", "pi"), "shifted")])
def test_temporal_blocking_bitwise(C, kernel, N, K, L, ic):
    """Two layers per sweep (redundant ring evaluation, periodic seam alias) must reproduce the
    OpenMP oracle bit for bit, for even and odd K."""
    import wave3d

    p = wave3d.WaveProblem(N, Lx=L[0], Ly=L[1], Lz=L[2], timesteps=K, ic=ic)
    g = _solve(p, kernel=kernel)
    c = _solve(p, backend="cpu", threads=4)
    assert g.kernel == kernel
    assert g.max_abs == c.max_abs and g.max_rel == c.max_rel


def test_temporal_blocking_fp32_and_resume(C, tmp_path):
    import wave3d

    p32 = wave3d.WaveProblem(48, timesteps=20, dtype="fp32")
    a, b = _solve(p32), _solve(p32, kernel="tb2")
    assert b.max_abs[-1] == pytest.approx(a.max_abs[-1], rel=1e-3)
    p = wave3d.WaveProblem(26, timesteps=14, ic="shifted")
    full = _solve(p, kernel="tb2")
    _solve(p, kernel="tb2", checkpoint_every=6, checkpoint_dir=str(tmp_path))
    res = _solve(p, kernel="tb2", resume=str(tmp_path))
    assert res.extra["resumed_from"] == 12
    assert res.max_abs == full.max_abs and res.max_rel == full.max_rel


@pytest.mark.parametrize("ranks,overlap,kernel", [(2, True, "tb2"), (3, True, "tb2r4"), (4, False, "tb2"),
                                                  (8, True, "tb2r4"), (2, False, "tb2r8")])
def test_temporal_blocking_slabs_loopback(C, ranks, overlap, kernel):
    """Multi-rank temporal blocking (x slabs, 2-deep halos + seam alias plane) on simulated
    ranks, with and without the interior/shell overlap: bitwise equal to one rank."""
    import wave3d

    for K in (9, 10):
        p = wave3d.WaveProblem(45, Lx=1.3, Ly="pi", Lz=2.0, timesteps=K, ic="shifted")
        base = _solve(p, backend="cpu", threads=4)
        r = _solve(p, ranks=ranks, overlap=overlap, kernel=kernel, dims=[ranks, 1, 1])
        assert r.dims == [ranks, 1, 1] and r.kernel == kernel
        assert r.max_abs == base.max_abs and r.max_rel == base.max_rel


@pytest.mark.parametrize("kernel", ["march2", "march2p", "march4p", "naive", "tb2"])
def test_fp32_bitwise_vs_cpu(C, kernel):
    """fp32 kernels (incl. the packed-fp32 v_pk_* variants) reproduce the OpenMP fp32
    oracle's per-layer errors bit for bit (shifted IC exercises the periodic seam)."""
    import wave3d

    p = wave3d.WaveProblem(40, timesteps=12, dtype="fp32", ic="shifted")
    ref = _solve(p, "cpu")
    got = _solve(p, kernel=kernel)
    assert got.kernel == kernel
    assert got.max_abs == ref.max_abs and got.max_rel == ref.max_rel
    multi = _solve(p, kernel=kernel, ranks=3) if kernel != "tb2" else _solve(p, kernel=kernel, ranks=2)
    assert multi.max_abs == ref.max_abs and multi.max_rel == ref.max_rel


@pytest.mark.parametrize("kernel,ranks", [("auto", 0), ("march2", 0), ("march2", 3), ("tb2", 2)])
def test_graph_replay_matches_direct(C, kernel, ranks):
    """hipGraph replay of the whole solve (incl. loopback halo copies and the overlap
    stream joins) gives the same errors as direct launches, solve after solve."""
    import wave3d

    p = wave3d.WaveProblem(36, timesteps=11, ic="shifted")
    d = _solve(p, kernel=kernel, ranks=ranks, graph="off")
    g = wave3d.WaveSolver(p, "hip", kernel=kernel, ranks=ranks, graph="on").run(repeat=3)
    assert not d.extra["graph"] and g.extra["graph"]
    assert g.max_abs == d.max_abs and g.max_rel == d.max_rel


@pytest.mark.parametrize("dims,overlap", [((2, 2, 2), True), ((1, 2, 2), True), ((2, 1, 2), False),
                                          ((1, 1, 3), True), ((2, 2, 1), False), ((1, 3, 1), True)])
def test_temporal_blocking_3d_decomposition(C, dims, overlap):
    """Temporal blocking on y/z splits: x planes in place, then y rows and z columns (2-deep
    for D, 1-deep for C) over the full extent of the axes exchanged before — edges without
    diagonal messages. Bitwise equal to the OpenMP oracle."""
    import wave3d

    P = dims[0] * dims[1] * dims[2]
    for K in (8, 9):
        p = wave3d.WaveProblem(29, Lx=1.3, Ly="pi", Lz=2.0, timesteps=K, ic="shifted")
        base = _solve(p, backend="cpu", threads=4)
        r = _solve(p, ranks=P, dims=list(dims), overlap=overlap, kernel="tb2r2w8")
        assert r.dims == list(dims) and r.kernel == "tb2r2w8"
        assert r.max_abs == base.max_abs and r.max_rel == base.max_rel


def test_temporal_blocking_3d_fp32_resume(C, tmp_path):
    import wave3d

    p = wave3d.WaveProblem(26, timesteps=13, ic="shifted", dtype="fp32")
    base = _solve(p, backend="cpu", threads=4)
    full = _solve(p, ranks=8, dims=[2, 2, 2])
    assert full.max_abs == base.max_abs and full.max_rel == base.max_rel
    _solve(p, ranks=8, dims=[2, 2, 2], checkpoint_every=4, checkpoint_dir=str(tmp_path))
    res = _solve(p, ranks=8, dims=[2, 2, 2], resume=str(tmp_path))
    assert res.extra["resumed_from"] == 12
    assert res.max_abs == full.max_abs and res.max_rel == full.max_rel


@pytest.mark.parametrize("kernel", ["tb3", "tb3r2w4", "tb3r4w4", "tb3r1w16", "tb3r1w8"])
@pytest.mark.parametrize("K", [9, 10, 11])
def test_tb3_single_rank_bitwise(C, kernel, K):
    """Three-layer temporal blocking (C never stored, seam partner planes from k_seam_c) with
    two-layer / single-step tails: bitwise equal to the OpenMP oracle (shifted IC)."""
    import wave3d

    p = wave3d.WaveProblem(40, Lx=1.3, Ly="pi", Lz=2.0, timesteps=K, ic="shifted")
    base = _solve(p, backend="cpu", threads=4)
    r = _solve(p, kernel=kernel)
    assert r.kernel == kernel
    assert r.max_abs == base.max_abs and r.max_rel == base.max_rel


@pytest.mark.parametrize("ranks,dims,overlap", [(2, None, True), (3, None, False), (4, None, True),
                                                (8, [2, 2, 2], True), (4, [1, 2, 2], False),
                                                (2, [1, 1, 2], True)])
def test_tb3_multi_rank_bitwise(C, ranks, dims, overlap):
    import wave3d

    for K in (10, 12):
        p = wave3d.WaveProblem(47, Lx=1.3, Ly="pi", Lz=2.0, timesteps=K, ic="shifted")
        base = _solve(p, backend="cpu", threads=4)
        for kernel in ("tb3", "tb3r1w8"):
            r = _solve(p, ranks=ranks, dims=dims, overlap=overlap, kernel=kernel)
            assert r.kernel == kernel
            assert r.max_abs == base.max_abs and r.max_rel == base.max_rel


def test_tb3_fp32_resume_and_fault(C, tmp_path):
    import wave3d

    p32 = wave3d.WaveProblem(44, timesteps=13, dtype="fp32", ic="shifted")
    base = _solve(p32, backend="cpu", threads=4)
    r = _solve(p32, kernel="tb3")
    assert r.max_abs == base.max_abs and r.max_rel == base.max_rel
    p = wave3d.WaveProblem(40, timesteps=14, ic="shifted")
    full = _solve(p, kernel="tb3", ranks=2)
    _solve(p, kernel="tb3", ranks=2, checkpoint_every=6, checkpoint_dir=str(tmp_path))
    res = _solve(p, kernel="tb3", ranks=2, resume=str(tmp_path))
    assert res.extra["resumed_from"] == 12
    assert res.max_abs == full.max_abs and res.max_rel == full.max_rel
    bad = _solve(p, kernel="tb3", ranks=2, fault="nan:1:5", check_every=1)
    assert bad.aborted


@pytest.mark.parametrize("kernel,ranks,layer", [("auto", 0, None), ("march2", 3, None), ("tb3", 2, None),
                                                ("tb2", 4, 10), ("flat", 0, None)])
def test_field_bitwise_vs_cpu(C, kernel, ranks, layer):
    """The final field itself (not only the error maxima) is bitwise equal to the oracle."""
    import numpy as np

    import wave3d

    p = wave3d.WaveProblem(33, timesteps=11, ic="shifted")
    _, ref = wave3d.WaveSolver(p, "cpu", threads=4).solve_field(layer)
    _, got = wave3d.WaveSolver(p, "hip", kernel=kernel, ranks=ranks).solve_field(layer)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("kernel,ranks,dims,overlap", [
    ("auto", 0, None, True), ("tb2", 0, None, True), ("tb2r4", 0, None, True),
    ("auto", 2, [2, 1, 1], True), ("tb2", 3, [3, 1, 1], False), ("auto", 8, [2, 2, 2], True),
    ("tb2", 4, [1, 2, 2], False), ("tb3", 0, None, True), ("tb3r1w8", 0, None, True),
    ("tb3", 2, [2, 1, 1], True), ("tb3", 8, [2, 2, 2], True), ("tb3r1w8", 4, [1, 2, 2], False)])
def test_delta_scheme_matches_cpu(C, dtype, kernel, ranks, dims, overlap):
    """Increment form on the HIP temporal-blocking path (u and d levels in the ring; tb3: the D
    level carries d^{m+2}; two-layer / single-step tails) == the OpenMP oracle's increment form,
    bit for bit, for K = 10, 11, 12, one rank, x slabs and 3-D blocks, with and without overlap."""
    import wave3d

    for K in (10, 11, 12):
        p = wave3d.WaveProblem(29, Lx=1.3, Ly="pi", Lz=2.0, timesteps=K, ic="shifted", dtype=dtype,
                               scheme="delta")
        ref = _solve(p, backend="cpu", threads=4)
        got = _solve(p, kernel=kernel, ranks=ranks, dims=dims, overlap=overlap)
        assert got.extra["scheme"] == "delta"
        assert got.max_abs == ref.max_abs and got.max_rel == ref.max_rel


def test_delta_scheme_fp32_accuracy_gpu(C):
    """fp32 increment form at the fp64 error where fp32 leapfrog is far off (N=128, K=400)."""
    import wave3d

    e64 = _solve(wave3d.WaveProblem(128, timesteps=400)).linf_abs
    lf = _solve(wave3d.WaveProblem(128, timesteps=400, dtype="fp32")).linf_abs
    d = _solve(wave3d.WaveProblem(128, timesteps=400, dtype="fp32", scheme="delta")).linf_abs
    assert d < 1.2 * e64 and lf > 20 * d


@pytest.mark.parametrize("ranks,dims", [(0, None), (2, [2, 1, 1]), (8, [2, 2, 2])])
def test_delta_scheme_checkpoint_resume(C, tmp_path, ranks, dims):
    """Increment form on the HIP sweep: checkpoint (d^n, u^n) after layer 12, resume, equal to
    the uninterrupted run bit for bit (and to the OpenMP oracle)."""
    import wave3d

    p = wave3d.WaveProblem(29, Lx=1.3, Ly="pi", Lz=2.0, timesteps=16, ic="shifted", dtype="fp32",
                           scheme="delta")
    ref = _solve(p, backend="cpu", threads=4)
    full = _solve(p, ranks=ranks, dims=dims)
    _solve(p, ranks=ranks, dims=dims, checkpoint_every=6, checkpoint_dir=str(tmp_path))
    res = _solve(p, ranks=ranks, dims=dims, resume=str(tmp_path))
    assert res.extra["resumed_from"] == 12

    def diff(r):  # layers whose maxima differ from the oracle's
        return [n for n in range(len(ref.max_abs))
                if (r.max_abs[n], r.max_rel[n]) != (ref.max_abs[n], ref.max_rel[n])]

    assert diff(full) == [], f"uninterrupted run vs oracle, layers {diff(full)}"
    assert diff(res) == [], f"resumed run vs oracle, layers {diff(res)}"


@pytest.mark.parametrize("kernel", ["tb2r2w8", "tb2r2w8k2"])
def test_tile_orders_bitwise(C, kernel):
    """The XCD-band (default), j-fastest and k-fastest tile orders of the temporal-blocking
    sweep give the same per-layer error maxima, bit for bit (N=129: 8 tile rows, so the band
    order is active). The order is read once per process (WAVE3D_TILE_ORDER): one subprocess
    each."""
    import json
    import sys

    code = ("import json, wave3d; r = wave3d.WaveSolver(wave3d.WaveProblem(129, timesteps=20), "
            f"'hip', kernel='{kernel}').run(); print(json.dumps([r.max_abs, r.max_rel]))")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for order in ("band", "j", "k"):
        env = dict(os.environ, WAVE3D_TILE_ORDER=order)
        p = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                           text=True, timeout=120)
        assert p.returncode == 0, p.stderr[-2000:]
        out[order] = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["band"] == out["j"] == out["k"]


def test_loop_copy_sdma_bitwise(C):
    """Simulated ranks' loopback halo copies on the DMA engines (WAVE3D_LOOP_COPY=sdma,
    hipMemcpyDeviceToDeviceNoCU) give the same per-layer errors as HIP's copy kernels, bit for
    bit, on 2x1x1 and 2x2x2 with overlap off and on (read once per process: one subprocess each)."""
    import json
    import sys

    code = ("import json, wave3d; p = wave3d.WaveProblem(48, timesteps=13, ic='shifted'); "
            "out = [wave3d.WaveSolver(p, 'hip', ranks=P, dims=d, overlap=o).run() "
            "for P, d in ((2, [2, 1, 1]), (8, [2, 2, 2])) for o in (False, True)]; "
            "print(json.dumps([[r.max_abs, r.max_rel] for r in out]))")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for mode in ("blit", "sdma"):
        env = dict(os.environ, WAVE3D_LOOP_COPY=mode)
        p = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                           text=True, timeout=120)
        assert p.returncode == 0, p.stderr[-2000:]
        out[mode] = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["blit"] == out["sdma"]
    assert all(r == out["blit"][0] for r in out["blit"])


def test_fp32_auto_is_tb4_bitwise(C):
    """fp32 leapfrog "auto" runs four-layer blocking (tb4, k_tbn r2w8): bitwise equal to the
    OpenMP fp32 oracle on one rank and on a 2x2x1 decomposition with overlap (4-deep halos)."""
    import wave3d

    p = wave3d.WaveProblem(40, timesteps=13, dtype="fp32", ic="shifted")
    ref = _solve(p, "cpu")
    got = _solve(p)
    assert got.kernel == "tb4"
    assert got.max_abs == ref.max_abs and got.max_rel == ref.max_rel
    multi = _solve(p, ranks=4, dims=[2, 2, 1], overlap=True)
    assert multi.kernel == "tb4"
    assert multi.max_abs == ref.max_abs and multi.max_rel == ref.max_rel


@pytest.mark.parametrize("math_,want", [("fma", "tb4"), ("exact", "tb3")])
def test_fp32_delta_auto_kernel(C, math_, want):
    """The fp32 increment form's "auto" sweep: tb4 with --math fma (two workgroups per CU since
    round 5, 872-878k vs tb3 787-790k at N=512, profiles/deep_sweeps_r5.txt step 13), tb3 in
    exact arithmetic; both at the OpenMP oracle's max abs errors."""
    import wave3d

    p = wave3d.WaveProblem(29, Lx=1.3, Ly="pi", Lz=2.0, timesteps=13, ic="shifted", dtype="fp32",
                           scheme="delta", math=math_)
    ref = _solve(p, backend="cpu", threads=4)
    got = _solve(p)
    assert got.kernel == want and got.extra["scheme"] == "delta"
    assert got.max_abs == ref.max_abs


@pytest.mark.parametrize("kernel,scheme", [("tb2", "leapfrog"), ("tb3", "leapfrog"), ("march2", "leapfrog"),
                                           ("tb2", "delta")])
@pytest.mark.parametrize("dims", ["2,2,2", "1,2,2"])
@pytest.mark.parametrize("K", [40, 41])
@pytest.mark.parametrize("halo", ["direct", "rounds"])
def test_overlap_concurrent_interior_bitwise(C, kernel, scheme, dims, K, halo):
    """Overlap on a grid large enough that the tile-aligned interior is non-empty (N=160: the
    interior sweep really runs concurrently with the shells on the comm stream), on the 3-D
    block decompositions, odd and even K: bitwise equal to the OpenMP oracle."""
    import wave3d

    p = wave3d.WaveProblem(160, Lx=1.3, Ly="pi", Lz=2.0, timesteps=K, ic="shifted", scheme=scheme)
    assert p.stable()
    d = [int(x) for x in dims.split(",")]
    s = wave3d.WaveSolver(p, "hip", ranks=d[0] * d[1] * d[2], dims=d, overlap=True, kernel=kernel)
    s.opts["halo"] = halo
    r = s.run()
    assert r.extra["overlap"] is True and r.extra["overlap_interior"] > 0
    ref = _solve(p, backend="cpu", threads=8)
    assert r.max_abs == ref.max_abs and r.max_rel == ref.max_rel


@pytest.mark.parametrize("kernel", ["tb3", "tb3r1w8", "tb2r2w8"])
def test_fma_math_goldens(C, kernel):
    """--math fma keeps the reference's printed error tables (6 significant digits) at N=32 and
    the headline N=512 K=100 L-inf, though it is not bitwise with the exact form."""
    import wave3d
    from wave3d.utils import GOLDEN_N32_K20, GOLDEN_SPOTS

    r = wave3d.WaveSolver(wave3d.WaveProblem(32, timesteps=20), "hip", kernel=kernel)
    r.opts["math"] = "fma"
    res = r.run()
    assert res.extra["math"] == "fma"
    # L-inf abs: the reference's 6 digits on every layer. The max relative error is set by the
    # nodes next to f's zero plane (sin(PI_ref) ~ 9e-11), where |u - f| is at the rounding noise
    # of the stencil: any other rounding order moves it in the 3rd-4th digit
    for (a, r_), (ga, gr) in zip(_fmt(res), GOLDEN_N32_K20):
        assert a == ga and float(r_) == pytest.approx(float(gr), rel=1e-2)
    r = wave3d.WaveSolver(wave3d.WaveProblem(512, timesteps=100), "hip", kernel=kernel)
    r.opts["math"] = "fma"
    got = _fmt(r.run())
    for layer, (a, _) in GOLDEN_SPOTS[(512, 100, "ref")].items():
        assert got[layer][0] == a


@pytest.mark.parametrize("kernel", ["tb3", "tb2r2w8"])
@pytest.mark.parametrize("ranks,dims", [(8, [2, 2, 2]), (2, [2, 1, 1]), (4, [1, 2, 2])])
def test_fma_math_decomposition_invariance(C, kernel, ranks, dims):
    """Every node's FMA-form arithmetic is the same on any decomposition (rings recomputed with
    the same operations, seam C planes by the same formula): bitwise equal to one rank."""
    import wave3d

    p = wave3d.WaveProblem(64, Lx=1.3, Ly="pi", Lz=2.0, timesteps=29, ic="shifted")
    assert p.stable()
    one = wave3d.WaveSolver(p, "hip", kernel=kernel)
    one.opts["math"] = "fma"
    many = wave3d.WaveSolver(p, "hip", kernel=kernel, ranks=ranks, dims=dims, overlap=True)
    many.opts["math"] = "fma"
    a, b = one.run(), many.run()
    assert a.max_abs == b.max_abs and a.max_rel == b.max_rel


@pytest.mark.parametrize("kernel,scheme,dtype", [("auto", "leapfrog", "fp64"), ("tb3", "leapfrog", "fp64"),
                                                 ("tb2r2w8", "leapfrog", "fp64"), ("march4", "leapfrog", "fp64"),
                                                 ("naive", "leapfrog", "fp64"), ("auto", "delta", "fp32"),
                                                 ("auto", "leapfrog", "fp32"), ("tb2r2w8", "delta", "fp64")])
@pytest.mark.parametrize("ranks", [1, 8])
def test_fma_math_matches_oracle(C, kernel, scheme, dtype, ranks):
    """--math fma on every kernel family against the OpenMP oracle's FMA form: the values — and
    so the per-layer max abs errors — bit for bit (same operations per node); the max relative
    error within rounding of the reference's quotient (RelMax, device_common.hpp)."""
    import wave3d

    p = wave3d.WaveProblem(48, Lx=1.3, Ly="pi", Lz=2.0, timesteps=23, ic="shifted", scheme=scheme, dtype=dtype,
                           math="fma")
    g = _solve(p, kernel=kernel, ranks=ranks if ranks > 1 else 0, overlap=True)
    c = _solve(p, backend="cpu", threads=8)
    assert g.extra["math"] == "fma" and c.extra["math"] == "fma"
    assert g.max_abs == c.max_abs
    for a, b in zip(g.max_rel, c.max_rel):
        assert a == pytest.approx(b, rel=1e-9 if dtype == "fp64" else 1e-4)


# ---- four-layer temporal blocking (k_tbn, depth 4) -------------------------------------------
@pytest.mark.parametrize("K", [9, 10, 11, 12, 13])
@pytest.mark.parametrize("math_", ["exact", "fma"])
def test_tb4_single_rank_bitwise(C, K, math_):
    """Four layers per sweep (two in registers, seam partners of two layers from the two-stage
    seam pre-kernel, periodic self-wrap of depth 3 / 4) with three-, two-layer and single-step
    tails: bitwise equal to the OpenMP oracle (shifted IC: the periodic seam is exercised)."""
    import wave3d

    p = wave3d.WaveProblem(40, Lx=1.3, Ly="pi", Lz=2.0, timesteps=K, ic="shifted", math=math_)
    base = _solve(p, backend="cpu", threads=4)
    r = _solve(p, kernel="tb4")
    assert r.kernel == "tb4" and r.extra["math"] == math_
    assert r.max_abs == base.max_abs
    if math_ == "exact":
        assert r.max_rel == base.max_rel
    else:
        for a, b in zip(r.max_rel, base.max_rel):
            assert a == pytest.approx(b, rel=1e-9)


@pytest.mark.parametrize("ranks,dims,overlap", [(2, None, True), (3, None, False), (4, None, True),
                                                (8, [2, 2, 2], True), (8, [2, 2, 2], False),
                                                (4, [1, 2, 2], False), (2, [1, 1, 2], True)])
def test_tb4_multi_rank_bitwise(C, ranks, dims, overlap):
    """Simulated ranks (loopback halos of depth 4 / 3, seam alias planes on x splits) with and
    without the interior/shell overlap: bitwise equal to the OpenMP oracle."""
    import wave3d

    for K in (12, 14):
        p = wave3d.WaveProblem(47, Lx=1.3, Ly="pi", Lz=2.0, timesteps=K, ic="shifted")
        base = _solve(p, backend="cpu", threads=4)
        r = _solve(p, ranks=ranks, dims=dims, overlap=overlap, kernel="tb4")
        assert r.kernel == "tb4"
        assert r.max_abs == base.max_abs and r.max_rel == base.max_rel


def test_tb4_resume_fault_and_goldens(C, tmp_path):
    """Checkpoint / resume across four-layer sweeps (resume re-plans the level ring), fault
    detection, the N=32 golden table and the headline N=512 K=100 L-inf with --math fma."""
    import wave3d
    from wave3d.utils import GOLDEN_N32_K20, GOLDEN_SPOTS

    p = wave3d.WaveProblem(40, timesteps=17, ic="shifted")
    full = _solve(p, kernel="tb4", ranks=2)
    _solve(p, kernel="tb4", ranks=2, checkpoint_every=6, checkpoint_dir=str(tmp_path))
    res = _solve(p, kernel="tb4", ranks=2, resume=str(tmp_path))
    assert res.extra["resumed_from"] == 12
    assert res.max_abs == full.max_abs and res.max_rel == full.max_rel
    bad = _solve(p, kernel="tb4", ranks=2, fault="nan:1:5", check_every=1)
    assert bad.aborted
    assert _fmt(_solve(wave3d.WaveProblem(32, timesteps=20), kernel="tb4")) == GOLDEN_N32_K20
    got = _fmt(_solve(wave3d.WaveProblem(512, timesteps=100, math="fma"), kernel="tb4"))
    for layer, (a, _) in GOLDEN_SPOTS[(512, 100, "ref")].items():
        assert got[layer][0] == a


@pytest.mark.parametrize("dims", ["2,2,2", "1,2,2"])
@pytest.mark.parametrize("K", [40, 42])
def test_tb4_overlap_concurrent_interior_bitwise(C, dims, K):
    """N=160 with a non-empty tile-aligned interior on 3-D block decompositions: the overlapped
    four-layer sweeps are bitwise equal to the OpenMP oracle."""
    import wave3d

    p = wave3d.WaveProblem(160, Lx=1.3, Ly="pi", Lz=2.0, timesteps=K, ic="shifted")
    d = [int(x) for x in dims.split(",")]
    r = _solve(p, ranks=d[0] * d[1] * d[2], dims=d, overlap=True, kernel="tb4")
    assert r.extra["overlap"] is True and r.extra["overlap_interior"] > 0
    ref = _solve(p, backend="cpu", threads=8)
    assert r.max_abs == ref.max_abs and r.max_rel == ref.max_rel


@pytest.mark.parametrize("math", ["exact", "fma"])
@pytest.mark.parametrize("ranks,dims,overlap", [(0, None, True), (2, [2, 1, 1], True), (8, [2, 2, 2], True),
                                                (4, [1, 2, 2], False), (3, [3, 1, 1], False)])
def test_tb4_delta_fp32_matches_cpu(C, math, ranks, dims, overlap):
    """The fp32 increment form on four-layer sweeps (k_tbn DELTA: d rides in registers from layer
    to layer, the sweep stores d and u of its last layer; the seam stages keep layer m's d at the
    partner planes for stage 2) == the OpenMP oracle's increment form bit for bit, K = 10..13
    (tb3 / tb2 / single-step tails), one rank, x slabs and 3-D blocks, with and without overlap
    (--math fma: the values and max abs errors bit for bit, the relative error within ulps)."""
    import wave3d

    for K in (10, 11, 12, 13):
        p = wave3d.WaveProblem(29, Lx=1.3, Ly="pi", Lz=2.0, timesteps=K, ic="shifted", dtype="fp32",
                               scheme="delta", math=math)
        ref = _solve(p, backend="cpu", threads=4)
        got = _solve(p, kernel="tb4", ranks=ranks, dims=dims, overlap=overlap)
        assert got.kernel == "tb4" and got.extra["scheme"] == "delta"
        assert got.max_abs == ref.max_abs
        if math == "exact":
            assert got.max_rel == ref.max_rel
        else:  # --math fma: the relative error from reciprocal tables, within ulps (RelMax)
            assert got.max_rel == pytest.approx(ref.max_rel, rel=1e-5)


def test_tb4_delta_fp32_resume_and_accuracy(C, tmp_path):
    """Checkpoint / resume of the fp32 increment form across four-layer sweeps (the d level is the
    sweep's first stored slot), bitwise with the uninterrupted run; the N=128 K=400 accuracy of
    the increment form (at the fp64 error, where fp32 leapfrog is far off) holds on tb4."""
    import wave3d

    p = wave3d.WaveProblem(40, timesteps=17, ic="shifted", dtype="fp32", scheme="delta")
    full = _solve(p, kernel="tb4", ranks=2)
    _solve(p, kernel="tb4", ranks=2, checkpoint_every=6, checkpoint_dir=str(tmp_path))
    res = _solve(p, kernel="tb4", ranks=2, resume=str(tmp_path))
    assert res.extra["resumed_from"] == 12
    assert res.max_abs == full.max_abs and res.max_rel == full.max_rel
    e64 = _solve(wave3d.WaveProblem(128, timesteps=400)).linf_abs
    d = _solve(wave3d.WaveProblem(128, timesteps=400, dtype="fp32", scheme="delta"), kernel="tb4").linf_abs
    assert d < 1.2 * e64


def test_tb4_delta_fp64_is_refused(C):
    """The fp64 increment form has no four-layer instantiation (register budget): asking for it
    fails with a message, the auto kernel keeps tb3 / tb2 there."""
    import wave3d

    p = wave3d.WaveProblem(24, timesteps=8, scheme="delta")
    with pytest.raises(Exception, match="increment form"):
        _solve(p, kernel="tb4")
    assert _solve(p).kernel != "tb4"


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
@pytest.mark.parametrize("math_", ["exact", "fma"])
def test_tb4_repeat_solves_identical(C, dtype, math_):
    """The LDS-DMA four-layer sweeps give the same per-layer errors on every solve of a session
    (a counted-wait mistake — e.g. the first sweep, which stages no B — shows up as a solve that
    differs), and fp64 the OpenMP oracle's bit for bit. N=200 tiles every tile row and column
    with partial last tiles; 8 sweeps include the first."""
    import wave3d

    p = wave3d.WaveProblem(200, timesteps=33, ic="shifted", dtype=dtype, math=math_)
    s = wave3d.WaveSolver(p, "hip", kernel="tb4")
    runs = [s.run() for _ in range(5)]
    for r in runs[1:]:
        assert r.max_abs == runs[0].max_abs and r.max_rel == runs[0].max_rel
    if dtype == "fp64":
        c = _solve(p, backend="cpu", threads=8)
        assert runs[0].max_abs == c.max_abs
