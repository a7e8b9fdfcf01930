"""Isolated temporal-blocking sweeps (k_tb2, k_tb3) vs the plain-PyTorch oracle.

One launch on random fields: C = u^m and D = u^{m+1} (tb3: C errors only, D, E) over boxes
that cross 64-lane k tiles, TJ-row j tiles and short i chunks, with a Dirichlet column inside
the ring (C = 0 outside ``cdom``). The oracle chains ``reference.stencil_field`` per layer on
the whole grid (ops/reference.py). fp64 must be bitwise equal (values and fused error
maxima); fp32 within a few ulps (same rounded operations, reference on the CPU).
The end-to-end solves are covered against the OpenMP oracle in test_gpu_solver.py.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
COEF = dict(hx2=0.011, hy2=0.013, hz2=0.017)
CT = (-0.83, 0.47, 0.21)
COEFS = (3.1e-4, 2.9e-4, 2.7e-4)


def _rand(shape, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g, dtype=torch.float64).to(dtype)


def _tables(n, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    return [(torch.rand(n, generator=g, dtype=torch.float64) * 2 - 1).to(dtype) for _ in range(3)]


def _mask(shape, G, cdom):
    """j/k inside cdom (logical) as a tensor-index mask."""
    m = torch.zeros(shape, dtype=torch.bool)
    _, _, j0, j1, k0, k1 = cdom
    m[:, j0 + G - 1:j1 + G, k0 + G - 1:k1 + G] = True
    return m


def _sl(box, G):
    i0, i1, j0, j1, k0, k1 = box
    o = G - 1
    return (slice(i0 + o, i1 + o + 1), slice(j0 + o, j1 + o + 1), slice(k0 + o, k1 + o + 1))


def _check(got, exp, dtype):
    if dtype == torch.float64:
        assert torch.equal(got, exp)
    else:
        torch.testing.assert_close(got, exp, rtol=4e-6, atol=4e-6)


def _check_err(err, vals, box, ei, tx, ty, tz, ct, dtype):
    from wave3d.ops import kernels, reference

    i0, i1, j0, j1, k0, k1 = box
    f = reference.analytic(tx[ei[0]:ei[1] + 1], ty[j0:j1 + 1], tz[k0:k1 + 1],
                           torch.tensor(ct, dtype=dtype).item())
    ea, er = reference.max_errors(vals[ei[0] - i0:ei[1] - i0 + 1].double(), f.double())
    (ga, gr, bad), = kernels.decode_err(err)
    if dtype == torch.float64:
        assert ga == ea and gr == er
    else:
        assert math.isclose(ga, ea, rel_tol=1e-5) and math.isclose(gr, er, rel_tol=1e-4)
    assert not bad


CASES = [
    # (X, Y, Z), boxes, cdom (j/k part used), chunk
    ((9, 40, 131), [(2, 8, 3, 37, 60, 130)], (1, 9, 1, 40, 1, 130), 3),
    ((9, 40, 131), [(1, 9, 1, 40, 1, 130)], (1, 9, 1, 40, 1, 130), 0),
    ((12, 21, 70), [(1, 2, 1, 21, 1, 69), (3, 12, 5, 9, 2, 66)], (1, 12, 1, 21, 1, 69), 4),
    ((7, 9, 11), [(1, 7, 2, 8, 2, 10)], (1, 7, 2, 8, 2, 10), 0),
]


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("first", [False, True])
@pytest.mark.parametrize("rows,waves,kw", [(2, 4, 1), (2, 8, 1), (4, 4, 1), (2, 8, 2), (2, 16, 2)])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_tb2_sweep_matches_reference(C, dtype, first, rows, waves, kw, case):
    from wave3d.ops import kernels, reference

    (X, Y, Z), boxes, cdom, chunk = CASES[case]
    G = 2
    shape = (X + 2 * G, Y + 2 * G, Z + 2 * G)
    A, B = _rand(shape, dtype, 1), _rand(shape, dtype, 2)
    tx, ty, tz = _tables(max(shape), dtype, 3)
    dA, dB, dC, dD = A.to(DEV), B.to(DEV), torch.full(shape, -7.0, dtype=dtype, device=DEV), \
        torch.full(shape, -9.0, dtype=dtype, device=DEV)
    errC, errD = kernels.new_err(1), kernels.new_err(1)
    ei = (boxes[0][0], boxes[0][1])
    if len(boxes) > 1:  # errors over every box's rows: use one shared i range
        ei = (min(b[0] for b in boxes), max(b[1] for b in boxes))
    kernels.tb_sweep(dA, dB, dC, dD, boxes, first=first, cdom=cdom, err_i=ei, tx=tx.to(DEV),
                     ty=ty.to(DEV), tz=tz.to(DEV), coefs_c=(*COEF.values(), COEFS[0], CT[0]),
                     coefs_d=(*COEF.values(), COEFS[1], CT[1]), err_c=errC, err_d=errD,
                     rows=rows, waves=waves, chunk=chunk, kwaves=kw)
    torch.cuda.synchronize()
    cast = lambda v: torch.tensor(v, dtype=dtype).item()  # noqa: E731
    h = {k: cast(v) for k, v in COEF.items()}
    Cf, Df = reference.chained_layers(A, B, 2, first=first, mask=_mask(shape, G, cdom),
                                      coefs=[cast(COEFS[0]), cast(COEFS[1])], **h)
    gC, gD = dC.cpu(), dD.cpu()
    touched = torch.zeros(shape, dtype=torch.bool)
    for b in boxes:
        s = _sl(b, G)
        _check(gC[s], Cf[s], dtype)
        _check(gD[s], Df[s], dtype)
        touched[s] = True
    assert bool((gC[~touched] == -7.0).all()) and bool((gD[~touched] == -9.0).all())
    if len(boxes) == 1:
        _check_err(errC, gC[_sl(boxes[0], G)], boxes[0], ei, tx, ty, tz, CT[0], dtype)
        _check_err(errD, gD[_sl(boxes[0], G)], boxes[0], ei, tx, ty, tz, CT[1], dtype)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("first", [False, True])
@pytest.mark.parametrize("rows,waves", [(2, 8), (2, 4), (1, 16), (1, 8)])
@pytest.mark.parametrize("case", [0, 2, 3])
def test_tb3_sweep_matches_reference(C, dtype, first, rows, waves, case):
    from wave3d.ops import kernels, reference

    (X, Y, Z), boxes, cdom, chunk = CASES[case]
    G = 3
    shape = (X + 2 * G, Y + 2 * G, Z + 2 * G)
    A, B = _rand(shape, dtype, 4), _rand(shape, dtype, 5)
    tx, ty, tz = _tables(max(shape), dtype, 6)
    dD, dE = torch.full(shape, -7.0, dtype=dtype, device=DEV), torch.full(shape, -9.0, dtype=dtype, device=DEV)
    errs = [kernels.new_err(1) for _ in range(3)]
    ei = (min(b[0] for b in boxes), max(b[1] for b in boxes))
    co = [(*COEF.values(), COEFS[q], CT[q]) for q in range(3)]
    kernels.tb3_sweep(A.to(DEV), B.to(DEV), dD, dE, boxes, first=first, cdom=cdom, err_i=ei,
                      tx=tx.to(DEV), ty=ty.to(DEV), tz=tz.to(DEV), coefs_c=co[0], coefs_d=co[1],
                      coefs_e=co[2], err_c=errs[0], err_d=errs[1], err_e=errs[2], rows=rows,
                      waves=waves, chunk=chunk)
    torch.cuda.synchronize()
    cast = lambda v: torch.tensor(v, dtype=dtype).item()  # noqa: E731
    h = {k: cast(v) for k, v in COEF.items()}
    Cf, Df, Ef = reference.chained_layers(A, B, 3, first=first, mask=_mask(shape, G, cdom),
                                          coefs=[cast(c) for c in COEFS], **h)
    gD, gE = dD.cpu(), dE.cpu()
    for b in boxes:
        s = _sl(b, G)
        _check(gD[s], Df[s], dtype)
        _check(gE[s], Ef[s], dtype)
    if len(boxes) == 1:
        s = _sl(boxes[0], G)
        for err, vals, q in ((errs[0], Cf[s], 0), (errs[1], gD[s], 1), (errs[2], gE[s], 2)):
            _check_err(err, vals, boxes[0], ei, tx, ty, tz, CT[q], dtype)


def test_tb_sweep_shape_checks(C):
    from wave3d.ops import kernels

    G = 2
    shape = (5 + 2 * G, 6 + 2 * G, 7 + 2 * G)
    u = torch.zeros(shape, dtype=torch.float64, device=DEV)
    t = torch.zeros(max(shape), dtype=torch.float64, device=DEV)
    e = kernels.new_err(1)
    kw = dict(first=False, cdom=(1, 5, 1, 6, 1, 7), err_i=(1, 5), tx=t, ty=t, tz=t,
              coefs_c=(1, 1, 1, 1, 1), coefs_d=(1, 1, 1, 1, 1), err_c=e, err_d=e)
    with pytest.raises(ValueError):
        kernels.tb_sweep(u, u, u, u, (0, 5, 1, 6, 1, 7), **kw)   # i outside the owned region
    with pytest.raises(ValueError):
        kernels.tb_sweep(u, u, u, u, (1, 5, 1, 6, 1, 7), rows=3, waves=4, **kw)  # no such tile


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("first", [False, True])
@pytest.mark.parametrize("rows,waves,kw", [(2, 4, 1), (2, 8, 1), (4, 4, 1), (2, 8, 2)])
@pytest.mark.parametrize("case", [0, 2, 3])
def test_tb2_delta_sweep_matches_reference(C, dtype, first, rows, waves, kw, case):
    """Increment form: the C level receives d^{m+1}, D receives u^{m+1}; errors of u^m, u^{m+1}."""
    from wave3d.ops import kernels, reference

    (X, Y, Z), boxes, cdom, chunk = CASES[case]
    G = 2
    shape = (X + 2 * G, Y + 2 * G, Z + 2 * G)
    A = _rand(shape, dtype, 7)
    Dm1 = (_rand(shape, dtype, 8) - 0.5) * 1e-3  # increments are small
    tx, ty, tz = _tables(max(shape), dtype, 9)
    dC = torch.full(shape, -7.0, dtype=dtype, device=DEV)
    dD = torch.full(shape, -9.0, dtype=dtype, device=DEV)
    errC, errD = kernels.new_err(1), kernels.new_err(1)
    ei = (min(b[0] for b in boxes), max(b[1] for b in boxes))
    kernels.tb_sweep(A.to(DEV), Dm1.to(DEV), dC, dD, boxes, first=first, cdom=cdom, err_i=ei,
                     tx=tx.to(DEV), ty=ty.to(DEV), tz=tz.to(DEV),
                     coefs_c=(*COEF.values(), COEFS[0], CT[0]), coefs_d=(*COEF.values(), COEFS[1], CT[1]),
                     err_c=errC, err_d=errD, rows=rows, waves=waves, chunk=chunk, delta=True,
                     kwaves=kw)
    torch.cuda.synchronize()
    cast = lambda v: torch.tensor(v, dtype=dtype).item()  # noqa: E731
    h = {k: cast(v) for k, v in COEF.items()}
    Cf, Df, dn = reference.chained_delta(A, Dm1, first=first, mask=_mask(shape, G, cdom),
                                         coefs=[cast(COEFS[0]), cast(COEFS[1])], **h)
    gC, gD = dC.cpu(), dD.cpu()
    for b in boxes:
        s = _sl(b, G)
        _check(gC[s], dn[s], dtype)
        _check(gD[s], Df[s], dtype)
    if len(boxes) == 1:
        s = _sl(boxes[0], G)
        _check_err(errC, Cf[s], boxes[0], ei, tx, ty, tz, CT[0], dtype)
        _check_err(errD, gD[s], boxes[0], ei, tx, ty, tz, CT[1], dtype)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("first", [False, True])
@pytest.mark.parametrize("rows,waves", [(2, 8), (1, 16), (1, 8)])
@pytest.mark.parametrize("case", [0, 2, 3])
def test_tb3_fma_sweep_close_to_reference(C, dtype, first, rows, waves, case):
    """--math fma: the same three-layer sweep with coef/h^2 folded into FMAs. Not bitwise (the
    reference's operation order is not kept), so within a few ulps of the chained oracle."""
    from wave3d.ops import kernels, reference

    (X, Y, Z), boxes, cdom, chunk = CASES[case]
    G = 3
    shape = (X + 2 * G, Y + 2 * G, Z + 2 * G)
    A, B = _rand(shape, dtype, 4), _rand(shape, dtype, 5)
    tx, ty, tz = _tables(max(shape), dtype, 6)
    dD, dE = torch.full(shape, -7.0, dtype=dtype, device=DEV), torch.full(shape, -9.0, dtype=dtype, device=DEV)
    errs = [kernels.new_err(1) for _ in range(3)]
    ei = (min(b[0] for b in boxes), max(b[1] for b in boxes))
    # the FMA sweep keeps one coefficient triple for the non-first layers (as in a solve, where
    # every layer but the Taylor start has the same a2 tau^2)
    coefs = (COEFS[0] if first else COEFS[1], COEFS[1], COEFS[1])
    co = [(*COEF.values(), coefs[q], CT[q]) for q in range(3)]
    kernels.tb3_sweep(A.to(DEV), B.to(DEV), dD, dE, boxes, first=first, cdom=cdom, err_i=ei,
                      tx=tx.to(DEV), ty=ty.to(DEV), tz=tz.to(DEV), coefs_c=co[0], coefs_d=co[1],
                      coefs_e=co[2], err_c=errs[0], err_d=errs[1], err_e=errs[2], rows=rows,
                      waves=waves, chunk=chunk, fma=True)
    torch.cuda.synchronize()
    h = {k: float(v) for k, v in COEF.items()}
    Cf, Df, Ef = reference.chained_layers(A.double(), B.double(), 3, first=first, mask=_mask(shape, G, cdom),
                                          coefs=list(coefs), **h)
    tol = dict(rtol=1e-12, atol=1e-12) if dtype == torch.float64 else dict(rtol=2e-5, atol=2e-5)
    gD, gE = dD.cpu(), dE.cpu()
    for b in boxes:
        s = _sl(b, G)
        torch.testing.assert_close(gD[s].double(), Df[s], **tol)
        torch.testing.assert_close(gE[s].double(), Ef[s], **tol)
    if len(boxes) == 1:  # the fused error keys of all three layers
        s = _sl(boxes[0], G)
        for err, vals, q in ((errs[0], Cf[s], 0), (errs[1], Df[s], 1), (errs[2], Ef[s], 2)):
            _check_err_fma(err, vals, boxes[0], ei, tx, ty, tz, CT[q], dtype)


def _check_err_fma(err, vals, box, ei, tx, ty, tz, ct, dtype):
    """--math fma error keys vs the fp64 oracle: |u - f| to 1e-12 relative, |u - f|/|f| (taken as
    |d| * 1/|sx sy| * 1/|sz| / |ct| in the sweep) to 1e-9; fp32 to its rounding."""
    from wave3d.ops import kernels, reference

    i0, i1, j0, j1, k0, k1 = box
    f = reference.analytic(tx[ei[0]:ei[1] + 1].double(), ty[j0:j1 + 1].double(), tz[k0:k1 + 1].double(),
                           float(torch.tensor(ct, dtype=dtype).item()))
    ea, er = reference.max_errors(vals[ei[0] - i0:ei[1] - i0 + 1].double(), f)
    (ga, gr, bad), = kernels.decode_err(err)
    ra, rr = (1e-12, 1e-9) if dtype == torch.float64 else (1e-5, 1e-4)
    assert math.isclose(ga, ea, rel_tol=ra) and math.isclose(gr, er, rel_tol=rr)
    assert not bad


TBN_CASES = [
    # (X, Y, Z), boxes, cdom, chunk — as CASES, with a box that starts past the first plane and
    # chunks short enough that every work item runs its prologue / epilogue planes
    ((11, 40, 131), [(2, 10, 3, 37, 60, 130)], (1, 11, 1, 40, 1, 130), 3),
    ((11, 40, 131), [(1, 11, 1, 40, 1, 130)], (1, 11, 1, 40, 1, 130), 0),
    ((13, 21, 70), [(1, 2, 1, 21, 1, 69), (3, 13, 5, 9, 2, 66)], (1, 13, 1, 21, 1, 69), 5),
    ((9, 9, 11), [(1, 9, 2, 8, 2, 10)], (1, 9, 2, 8, 2, 10), 0),
    # one- and two-plane work items: shorter than the steady window's start (only checked planes)
    ((11, 40, 131), [(2, 10, 3, 37, 60, 130)], (1, 11, 1, 40, 1, 130), 1),
    ((11, 40, 131), [(1, 11, 1, 40, 1, 130)], (1, 11, 1, 40, 1, 130), 2),
]


@pytest.mark.parametrize("first", [False, True])
@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("case", range(len(TBN_CASES)))
def test_tbn_depth3_bitwise_equal_to_tb3(C, first, fma, case):
    """The generic deep sweep at depth 3 is the three-layer sweep: k_tbn<3> and k_tb3 on the
    same fields give bitwise identical D, E and error keys (fp64, exact and --math fma)."""
    from wave3d.ops import kernels

    (X, Y, Z), boxes, cdom, chunk = TBN_CASES[case]
    G, dtype = 4, torch.float64
    shape = (X + 2 * G, Y + 2 * G, Z + 2 * G)
    A, B = _rand(shape, dtype, 14).to(DEV), _rand(shape, dtype, 15).to(DEV)
    tx, ty, tz = (t.to(DEV) for t in _tables(max(shape), dtype, 16))
    ei = (min(b[0] for b in boxes), max(b[1] for b in boxes))
    coefs = (COEFS[0] if first or not fma else COEFS[1], COEFS[1], COEFS[2] if not fma else COEFS[1])
    co = [(*COEF.values(), coefs[q], CT[q]) for q in range(3)]
    outs = []
    for tbn in (False, True):
        dD, dE = (torch.full(shape, v, dtype=dtype, device=DEV) for v in (-7.0, -9.0))
        errs = [kernels.new_err(1) for _ in range(3)]
        kw = dict(first=first, cdom=cdom, err_i=ei, tx=tx, ty=ty, tz=tz, rows=2, waves=8, chunk=chunk,
                  ghost=G, fma=fma)
        if tbn:
            kernels.tbn_sweep(A, B, dD, dE, boxes, depth=3, coefs=co, errs=errs, **kw)
        else:
            kernels.tb3_sweep(A, B, dD, dE, boxes, coefs_c=co[0], coefs_d=co[1], coefs_e=co[2], err_c=errs[0],
                              err_d=errs[1], err_e=errs[2], **kw)
        torch.cuda.synchronize()
        outs.append((dD.cpu(), dE.cpu(), [e.cpu() for e in errs]))
    (d0, e0, k0), (d1, e1, k1) = outs
    assert torch.equal(d0, d1) and torch.equal(e0, e1)
    for a, b in zip(k0, k1):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("first", [False, True])
@pytest.mark.parametrize("case", range(len(TBN_CASES)))
def test_tbn_depth4_sweep_matches_reference(C, dtype, first, case):
    """Four layers per sweep (k_tbn<4>, exact arithmetic): the stored layers u^{m+2}, u^{m+3} and
    the error keys of all four layers against the chained plain-PyTorch oracle — bitwise in fp64;
    nodes outside the boxes untouched."""
    from wave3d.ops import kernels, reference

    (X, Y, Z), boxes, cdom, chunk = TBN_CASES[case]
    G = 4
    shape = (X + 2 * G, Y + 2 * G, Z + 2 * G)
    A, B = _rand(shape, dtype, 24), _rand(shape, dtype, 25)
    tx, ty, tz = _tables(max(shape), dtype, 26)
    c4 = (3.1e-4, 2.9e-4, 2.7e-4, 2.6e-4)
    ct4 = (-0.83, 0.47, 0.21, -0.66)
    dO0, dO1 = (torch.full(shape, v, dtype=dtype, device=DEV) for v in (-7.0, -9.0))
    errs = [kernels.new_err(1) for _ in range(4)]
    ei = (min(b[0] for b in boxes), max(b[1] for b in boxes))
    co = [(*COEF.values(), c4[q], ct4[q]) for q in range(4)]
    kernels.tbn_sweep(A.to(DEV), B.to(DEV), dO0, dO1, boxes, depth=4, first=first, cdom=cdom, err_i=ei,
                      tx=tx.to(DEV), ty=ty.to(DEV), tz=tz.to(DEV), coefs=co, errs=errs, chunk=chunk)
    torch.cuda.synchronize()
    cast = lambda v: torch.tensor(v, dtype=dtype).item()  # noqa: E731
    h = {k: cast(v) for k, v in COEF.items()}
    L = reference.chained_layers(A, B, 4, first=first, mask=_mask(shape, G, cdom), coefs=[cast(c) for c in c4], **h)
    g0, g1 = dO0.cpu(), dO1.cpu()
    touched = torch.zeros(shape, dtype=torch.bool)
    for b in boxes:
        s = _sl(b, G)
        _check(g0[s], L[2][s], dtype)
        _check(g1[s], L[3][s], dtype)
        touched[s] = True
    assert bool((g0[~touched] == -7.0).all()) and bool((g1[~touched] == -9.0).all())
    if len(boxes) == 1:
        s = _sl(boxes[0], G)
        for q in range(4):
            _check_err(errs[q], L[q][s], boxes[0], ei, tx, ty, tz, ct4[q], dtype)


@pytest.mark.parametrize("first", [False, True])
@pytest.mark.parametrize("case", range(len(TBN_CASES)))
def test_tbn_depth4_delta_fp32_matches_reference(C, first, case):
    """The fp32 increment form on four-layer sweeps (k_tbn DELTA, exact arithmetic): O0 = d of the
    last layer, O1 = u of the last layer, and the error keys of all four layers, against the
    chained plain-PyTorch increment-form oracle; nodes outside the boxes untouched."""
    from wave3d.ops import kernels, reference

    dtype = torch.float32
    (X, Y, Z), boxes, cdom, chunk = TBN_CASES[case]
    G = 4
    shape = (X + 2 * G, Y + 2 * G, Z + 2 * G)
    A = _rand(shape, dtype, 31)
    Dm1 = (_rand(shape, dtype, 32) - 0.5) * 1e-3  # increments are small
    tx, ty, tz = _tables(max(shape), dtype, 33)
    c4 = (3.1e-4, 2.9e-4, 2.7e-4, 2.6e-4)
    ct4 = (-0.83, 0.47, 0.21, -0.66)
    dO0, dO1 = (torch.full(shape, v, dtype=dtype, device=DEV) for v in (-7.0, -9.0))
    errs = [kernels.new_err(1) for _ in range(4)]
    ei = (min(b[0] for b in boxes), max(b[1] for b in boxes))
    co = [(*COEF.values(), c4[q], ct4[q]) for q in range(4)]
    kernels.tbn_sweep(A.to(DEV), Dm1.to(DEV), dO0, dO1, boxes, depth=4, first=first, cdom=cdom, err_i=ei,
                      tx=tx.to(DEV), ty=ty.to(DEV), tz=tz.to(DEV), coefs=co, errs=errs, chunk=chunk, delta=True)
    torch.cuda.synchronize()
    cast = lambda v: torch.tensor(v, dtype=dtype).item()  # noqa: E731
    h = {k: cast(v) for k, v in COEF.items()}
    L, dl = reference.chained_delta_layers(A, Dm1, 4, first=first, mask=_mask(shape, G, cdom),
                                           coefs=[cast(c) for c in c4], **h)
    g0, g1 = dO0.cpu(), dO1.cpu()
    touched = torch.zeros(shape, dtype=torch.bool)
    for b in boxes:
        s = _sl(b, G)
        _check(g0[s], dl[s], dtype)
        _check(g1[s], L[3][s], dtype)
        touched[s] = True
    assert bool((g0[~touched] == -7.0).all()) and bool((g1[~touched] == -9.0).all())
    if len(boxes) == 1:
        s = _sl(boxes[0], G)
        for q in range(4):
            _check_err(errs[q], L[q][s], boxes[0], ei, tx, ty, tz, ct4[q], dtype)


def test_tbn_delta_fp64_unsupported(C):
    """No fp64 increment-form instantiation of k_tbn (register budget): refused up front."""
    from wave3d.ops import kernels

    u = torch.zeros((20, 20, 20), dtype=torch.float64, device=DEV)
    with pytest.raises(ValueError, match="delta=True"):
        kernels.tbn_sweep(u, u, u, u, (1, 12, 1, 12, 1, 12), depth=4, first=False, cdom=(1, 12, 1, 12), err_i=(1, 12),
                          tx=u[0, 0], ty=u[0, 0], tz=u[0, 0], coefs=[(1, 1, 1, 0, 0)] * 4,
                          errs=[kernels.new_err(1) for _ in range(4)], delta=True)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("first", [False, True])
@pytest.mark.parametrize("case", range(len(TBN_CASES)))
def test_tbn_depth4_fma_close_to_reference(C, dtype, first, case):
    """The --math fma four-layer sweep (the fp64 bench kernel) within a few ulps of the fp64
    chained oracle, error keys included."""
    from wave3d.ops import kernels, reference

    (X, Y, Z), boxes, cdom, chunk = TBN_CASES[case]
    G = 4
    shape = (X + 2 * G, Y + 2 * G, Z + 2 * G)
    A, B = _rand(shape, dtype, 34), _rand(shape, dtype, 35)
    tx, ty, tz = _tables(max(shape), dtype, 36)
    c = 2.9e-4
    c4 = (3.1e-4 if first else c, c, c, c)
    ct4 = (-0.83, 0.47, 0.21, -0.66)
    dO0, dO1 = (torch.full(shape, v, dtype=dtype, device=DEV) for v in (-7.0, -9.0))
    errs = [kernels.new_err(1) for _ in range(4)]
    ei = (min(b[0] for b in boxes), max(b[1] for b in boxes))
    co = [(*COEF.values(), c4[q], ct4[q]) for q in range(4)]
    kernels.tbn_sweep(A.to(DEV), B.to(DEV), dO0, dO1, boxes, depth=4, first=first, cdom=cdom, err_i=ei,
                      tx=tx.to(DEV), ty=ty.to(DEV), tz=tz.to(DEV), coefs=co, errs=errs, chunk=chunk, fma=True)
    torch.cuda.synchronize()
    h = {k: float(v) for k, v in COEF.items()}
    L = reference.chained_layers(A.double(), B.double(), 4, first=first, mask=_mask(shape, G, cdom),
                                 coefs=list(c4), **h)
    tol = dict(rtol=1e-12, atol=1e-12) if dtype == torch.float64 else dict(rtol=4e-5, atol=4e-5)
    g0, g1 = dO0.cpu(), dO1.cpu()
    for b in boxes:
        s = _sl(b, G)
        torch.testing.assert_close(g0[s].double(), L[2][s], **tol)
        torch.testing.assert_close(g1[s].double(), L[3][s], **tol)
    if len(boxes) == 1:
        s = _sl(boxes[0], G)
        for q in range(4):
            _check_err_fma(errs[q], L[q][s], boxes[0], ei, tx, ty, tz, ct4[q], dtype)
