"""HIP kernel numerics vs the plain-PyTorch reference (ops/reference.py).

fp64 results must be *bitwise* equal (both sides round every operation in the reference's
order, no FMA contraction); fp32 within a few ulps of the fp32 torch reference.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rand_grid(shape, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(shape, generator=g, dtype=torch.float64).to(dtype).to(DEV)


def _tables(shape, dtype, seed):
    g = torch.Generator().manual_seed(seed + 100)
    return [(torch.rand(n, generator=g, dtype=torch.float64) * 2 - 1).to(dtype).to(DEV) for n in shape]


def _ref_errors(u_box, f_box):
    from wave3d.ops import reference

    return reference.max_errors(u_box.double().cpu(), f_box.double().cpu())


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("kernel", ["march", "naive"])
@pytest.mark.parametrize("first", [False, True])
@pytest.mark.parametrize("shape,box,chunk", [
    ((13, 21, 70), (1, 11, 1, 19, 1, 68), 0),      # whole owned region
    ((13, 21, 70), (2, 10, 3, 17, 2, 66), 3),      # interior sub-box, short chunks
    ((9, 40, 131), (1, 7, 5, 33, 60, 129), 2),     # k box across 64-lane tiles
    ((6, 7, 9), (1, 4, 1, 5, 1, 7), 0),            # tiny
])
def test_step_matches_reference(C, dtype, kernel, first, shape, box, chunk):
    from wave3d.ops import kernels, reference

    u1 = _rand_grid(shape, dtype, 1)
    u2 = _rand_grid(shape, dtype, 2)
    u = torch.full(shape, -7.0, dtype=dtype, device=DEV)
    tx, ty, tz = _tables(shape, dtype, 3)
    hx2, hy2, hz2, coef, ct = 0.011, 0.013, 0.017, 3.1e-4, -0.83
    err = kernels.new_err(1)
    ei = (box[0] + 1, box[1])  # exclude the first box row from the error domain
    kernels.step(u1, u2, u, box, first=first, err_i=ei, tx=tx, ty=ty, tz=tz,
                 coefs=(hx2, hy2, hz2, coef, ct), err=err, kernel=kernel, chunk=chunk)
    torch.cuda.synchronize()
    cast = lambda v: torch.tensor(v, dtype=dtype).item()  # noqa: E731
    exp_box = reference.step(u1.cpu(), u2.cpu(), box, first=first, hx2=cast(hx2), hy2=cast(hy2),
                             hz2=cast(hz2), coef=cast(coef))
    i0, i1, j0, j1, k0, k1 = box
    got = u[i0:i1 + 1, j0:j1 + 1, k0:k1 + 1].cpu()
    if dtype == torch.float64:
        assert torch.equal(got, exp_box)
    else:
        torch.testing.assert_close(got, exp_box, rtol=2e-6, atol=2e-6)
    # nodes outside the box untouched
    mask = torch.ones(shape, dtype=torch.bool)
    mask[i0:i1 + 1, j0:j1 + 1, k0:k1 + 1] = False
    assert bool((u.cpu()[mask] == -7.0).all())
    # fused errors
    f = reference.analytic(tx.cpu(), ty.cpu(), tz.cpu(), cast(ct))
    fb = f[ei[0]:ei[1] + 1, j0:j1 + 1, k0:k1 + 1]
    ea, er = _ref_errors(got[ei[0] - i0:, :, :], fb)
    (ga, gr, bad), = kernels.decode_err(err)
    if dtype == torch.float64:
        assert ga == ea and gr == er
    else:
        assert math.isclose(ga, ea, rel_tol=1e-5) and math.isclose(gr, er, rel_tol=1e-4)
    assert not bad


def test_step_wrap_and_fused_pack(C):
    from wave3d.ops import kernels

    shape = (12, 10, 75)
    dt = torch.float64
    u1, u2 = _rand_grid(shape, dt, 5), _rand_grid(shape, dt, 6)
    u = torch.zeros(shape, dtype=dt, device=DEV)
    tx, ty, tz = _tables(shape, dt, 7)
    nx, ny, nz = shape
    X, Y, Z = nx - 2, ny - 2, nz - 2
    zb = [torch.zeros(X * ny, dtype=dt, device=DEV) for _ in range(2)]
    yb = [torch.zeros(X * nz, dtype=dt, device=DEV) for _ in range(2)]
    box = (1, X, 1, Y, 1, Z)
    err = kernels.new_err(1)
    kernels.step(u1, u2, u, box, first=False, err_i=(2, X - 1), tx=tx, ty=ty, tz=tz,
                 coefs=(0.1, 0.2, 0.3, 0.01, 0.5), err=err, wrap=(X - 1, 0, 2, X + 1),
                 pack=([zb[0], zb[1], yb[0], yb[1]], [1, Z, 1, Y]))
    torch.cuda.synchronize()
    uc = u.cpu()
    assert torch.equal(uc[0, 1:Y + 1, 1:Z + 1], uc[X - 1, 1:Y + 1, 1:Z + 1])
    assert torch.equal(uc[X + 1, 1:Y + 1, 1:Z + 1], uc[2, 1:Y + 1, 1:Z + 1])
    for side, k in ((0, 1), (1, Z)):
        z = zb[side].cpu().view(X, ny)
        assert torch.equal(z[:, 1:Y + 1], uc[1:X + 1, 1:Y + 1, k])
    for side, j in ((0, 1), (1, Y)):
        y = yb[side].cpu().view(X, nz)
        assert torch.equal(y[:, 1:Z + 1], uc[1:X + 1, j, 1:Z + 1])


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_init_kernel(C, dtype):
    from wave3d.ops import kernels, reference

    shape = (8, 9, 70)
    u = torch.zeros(shape, dtype=dtype, device=DEV)
    tx, ty, tz = _tables(shape, dtype, 9)
    err = kernels.new_err(1)
    kernels.init(u, (1, 6, 1, 7, 1, 68), tx=tx, ty=ty, tz=tz, ct0=0.75, err=err, wrap=(5, 0, 2, 7))
    torch.cuda.synchronize()
    f = reference.analytic(tx.cpu(), ty.cpu(), tz.cpu(), torch.tensor(0.75, dtype=dtype).item())
    uc = u.cpu()
    assert torch.equal(uc[1:7, 1:8, 1:69], f[1:7, 1:8, 1:69])
    assert torch.equal(uc[0, 1:8, 1:69], uc[5, 1:8, 1:69])
    assert torch.equal(uc[7, 1:8, 1:69], uc[2, 1:8, 1:69])
    (a, r, bad), = kernels.decode_err(err)
    assert a == 0.0 and r == 0.0 and not bad


def test_faces_roundtrip(C):
    from wave3d.ops import kernels

    shape = (7, 11, 13)
    nx, ny, nz = shape
    u = _rand_grid(shape, torch.float64, 11)
    by = torch.zeros((nx - 2) * nz, dtype=torch.float64, device=DEV)
    bz = torch.zeros((nx - 2) * ny, dtype=torch.float64, device=DEV)
    kernels.faces(u, [(by, 1, 3), (bz, 2, 5)], to_buf=True)
    torch.cuda.synchronize()
    uc = u.cpu()
    assert torch.equal(by.cpu().view(nx - 2, nz)[:, 1:-1], uc[1:nx - 1, 3, 1:-1])
    assert torch.equal(bz.cpu().view(nx - 2, ny)[:, 1:-1], uc[1:nx - 1, 1:-1, 5])
    v = torch.zeros_like(u)
    kernels.faces(v, [(by, 1, 0), (bz, 2, nz - 1)], to_buf=False)
    torch.cuda.synchronize()
    vc = v.cpu()
    assert torch.equal(vc[1:nx - 1, 0, 1:-1], uc[1:nx - 1, 3, 1:-1])
    assert torch.equal(vc[1:nx - 1, 1:-1, nz - 1], uc[1:nx - 1, 1:-1, 5])
    assert float(vc[:, 0, 0].abs().sum()) == 0.0  # corners untouched


def test_zero_faces(C):
    from wave3d.ops import kernels

    shape = (6, 8, 9)
    u = torch.ones(shape, dtype=torch.float64, device=DEV)
    kernels.zero_faces(u, 1 | 8)
    torch.cuda.synchronize()
    uc = u.cpu()
    X, Y, Z = 4, 6, 7
    assert bool((uc[1:X + 1, 1:Y + 1, 1] == 0).all())
    assert bool((uc[1:X + 1, Y, 1:Z + 1] == 0).all())
    assert bool((uc[1:X + 1, 1:Y, Z] == 1).all())  # k=Z face not in the mask
    assert bool((uc[1:X + 1, 2:Y, 2:Z] == 1).all())
    # ghost planes get their face rows zeroed too (redundant ring evaluations read them)
    assert bool((uc[0, 1:Y + 1, 1] == 0).all()) and bool((uc[0, 2:Y, 2:Z] == 1).all())


def test_error_keys_order(C):
    from wave3d.ops import kernels  # noqa: F401

    vals = torch.tensor([-100.0, -1.5, -0.0, 0.0, 1e-300, 3.0, math.inf], dtype=torch.float64, device=DEV)
    keys = torch.empty(vals.numel(), dtype=torch.int64, device=DEV)
    C.k_encode_keys(vals.data_ptr(), keys.data_ptr(), vals.numel(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    u = [int(k) & ((1 << 64) - 1) for k in keys.cpu().tolist()]
    assert u == sorted(u)
    assert [C.decode_max_key(k) for k in u] == vals.cpu().tolist()
    assert u == [C.encode_max_key(v) for v in vals.cpu().tolist()]


def test_shape_checks_refuse_bad_boxes(C):
    from wave3d.ops import kernels

    shape = (6, 6, 6)
    u1 = torch.zeros(shape, dtype=torch.float64, device=DEV)
    tx, ty, tz = _tables(shape, torch.float64, 1)
    err = kernels.new_err(1)
    with pytest.raises(ValueError):
        kernels.step(u1, u1, u1, (0, 4, 1, 4, 1, 4), first=False, err_i=(1, 4), tx=tx, ty=ty,
                     tz=tz, coefs=(1, 1, 1, 1, 1), err=err)
    with pytest.raises(ValueError):
        kernels.step(u1, u1, u1, (1, 5, 1, 4, 1, 4), first=False, err_i=(1, 4), tx=tx, ty=ty,
                     tz=tz, coefs=(1, 1, 1, 1, 1), err=err)
