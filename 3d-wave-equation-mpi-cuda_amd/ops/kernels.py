"""Tensor-level access to the hand-written HIP kernels (for numerics tests and tools).

Tensors are dense ``[nx][ny][nz]`` (k contiguous, one ghost layer) on the current HIP
device; they are passed to the native kernels as raw pointers on torch's current stream.
Shapes are validated here *before* any launch (the kernels index with the boxes given).
The solver itself uses an aligned, padded layout (``csrc/hip_kernels.hpp``); these entry
points use pitch = nz, which the kernels accept as well.
"""
from __future__ import annotations

import torch

from .._native import load

_U64 = (1 << 64) - 1


def _C():
    return load()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _sfx(t: torch.Tensor) -> str:
    if t.dtype == torch.float64:
        return "f64"
    if t.dtype == torch.float32:
        return "f32"
    raise TypeError(f"unsupported dtype {t.dtype}")


def _check_grid(*ts: torch.Tensor) -> list[int]:
    u = ts[0]
    for t in ts:
        if not t.is_cuda:
            raise ValueError("wave3d kernels need HIP device tensors")
        if t.dim() != 3 or not t.is_contiguous():
            raise ValueError("grids must be contiguous 3-D [nx][ny][nz] tensors")
        if t.shape != u.shape or t.dtype != u.dtype:
            raise ValueError("grid shapes/dtypes differ")
    nx, ny, nz = u.shape
    if min(nx, ny, nz) < 3:
        raise ValueError("grid needs at least one owned node plus ghosts per axis")
    return [nx, ny, nz, nz, ny * nz]


def _check_box(box, gv) -> list[int]:
    i0, i1, j0, j1, k0, k1 = (int(v) for v in box)
    nx, ny, nz = gv[0], gv[1], gv[2]
    if not (1 <= i0 and i1 <= nx - 2 and 1 <= j0 and j1 <= ny - 2 and 1 <= k0 and k1 <= nz - 2):
        raise ValueError(f"box {box} outside the owned region of a {nx}x{ny}x{nz} grid")
    return [i0, i1, j0, j1, k0, k1]


def _check_tables(u, tx, ty, tz):
    nx, ny, nz = u.shape
    for t, n, name in ((tx, nx, "tx"), (ty, ny, "ty"), (tz, nz, "tz")):
        if not t.is_cuda or t.dtype != u.dtype or t.numel() < n or not t.is_contiguous():
            raise ValueError(f"table {name} must be a contiguous {u.dtype} device tensor of >= {n}")


def new_err(layers: int = 1, device=None) -> torch.Tensor:
    """Per-layer error slots (abs key, rel key, non-finite flag), initialised on device."""
    e = torch.empty(layers * 3, dtype=torch.int64, device=device or "cuda")
    _C().k_init_err(e.data_ptr(), layers, _stream())
    return e


def decode_err(err: torch.Tensor) -> list[tuple[float, float, bool]]:
    C = _C()
    v = [int(x) & _U64 for x in err.cpu().tolist()]
    return [(C.decode_max_key(v[q]), C.decode_max_key(v[q + 1]), v[q + 2] != 0)
            for q in range(0, len(v), 3)]


def step(u1, u2, u, boxes, *, first: bool, err_i, tx, ty, tz, coefs, err,
         kernel: str = "march", wrap=None, chunk: int = 0, pack=None) -> None:
    """One leapfrog layer over ``boxes`` (list of (i0,i1,j0,j1,k0,k1), local indices).

    coefs = (hx2, hy2, hz2, coef, ct); err_i = (ei0, ei1) rows entering the error;
    wrap = (src0, dst0, src1, dst1) periodic self-wrap planes; pack = ([zbuf0, zbuf1,
    ybuf0, ybuf1] tensors or None, [zk0, zk1, yj0, yj1]).
    """
    gv = _check_grid(u1, u2, u)
    if isinstance(boxes[0], int):
        boxes = [boxes]
    if not 1 <= len(boxes) <= 7:
        raise ValueError("1..7 boxes per launch")
    bl = [_check_box(b, gv) for b in boxes]
    _check_tables(u, tx, ty, tz)
    if err.dtype != torch.int64 or err.numel() < 3 or not err.is_cuda:
        raise ValueError("err must be >= 3 int64 device slots (new_err())")
    if wrap is not None:
        w = [int(v) for v in wrap]
        for q in range(0, 4, 2):
            if w[q] >= 0 and not (0 <= w[q + 1] < gv[0] and 1 <= w[q] <= gv[0] - 2):
                raise ValueError("bad wrap planes")
    else:
        w = []
    pb, pi = [], []
    if pack is not None:
        bufs, idx = pack
        pb = [b.data_ptr() if b is not None else 0 for b in bufs]
        pi = [int(v) for v in idx]
        nx, ny, nz = u.shape
        for q, b in enumerate(bufs):
            if b is None:
                continue
            need = (nx - 2) * (ny if q < 2 else nz)
            if b.numel() < need or b.dtype != u.dtype:
                raise ValueError("pack buffer too small")
    fn = getattr(_C(), "k_step_" + _sfx(u))
    fn(kernel, bool(first), u1.data_ptr(), u2.data_ptr(), u.data_ptr(), gv, bl, int(err_i[0]),
       int(err_i[1]), w, tx.data_ptr(), ty.data_ptr(), tz.data_ptr(), [float(c) for c in coefs],
       err.data_ptr(), int(chunk), _stream(), pb, pi)


def init(u, box, *, tx, ty, tz, ct0: float, err, wrap=None) -> None:
    gv = _check_grid(u)
    b = _check_box(box, gv)
    _check_tables(u, tx, ty, tz)
    getattr(_C(), "k_init_" + _sfx(u))(u.data_ptr(), gv, b, list(wrap or []), tx.data_ptr(),
                                      ty.data_ptr(), tz.data_ptr(), float(ct0), err.data_ptr(),
                                      _stream())


def zero_faces(u, mask: int) -> None:
    gv = _check_grid(u)
    getattr(_C(), "k_zero_faces_" + _sfx(u))(u.data_ptr(), gv, int(mask), _stream())


def faces(u, ops, to_buf: bool) -> None:
    """ops: list of (buffer, axis in {1,2}, plane index). Pack (to_buf) or unpack."""
    gv = _check_grid(u)
    nx, ny, nz = u.shape
    lst = []
    for buf, axis, index in ops:
        if axis not in (1, 2):
            raise ValueError("faces: axis must be 1 (y) or 2 (z)")
        lim = ny if axis == 1 else nz
        if not 0 <= index < lim:
            raise ValueError("faces: plane index out of range")
        need = (nx - 2) * (nz if axis == 1 else ny)
        if buf.numel() < need or buf.dtype != u.dtype or not buf.is_cuda:
            raise ValueError("faces: buffer too small")
        lst.append((buf.data_ptr(), int(axis), int(index)))
    if len(lst) > 4:
        raise ValueError("at most 4 faces per launch")
    getattr(_C(), "k_faces_" + _sfx(u))(u.data_ptr(), gv, lst, bool(to_buf), _stream())


def _check_grid_g(G: int, *ts: torch.Tensor) -> list[int]:
    """Dense [nx][ny][nz] grids with G ghost layers per side (logical 1..X owned)."""
    u = ts[0]
    for t in ts:
        if not t.is_cuda or t.dim() != 3 or not t.is_contiguous():
            raise ValueError("grids must be contiguous 3-D HIP device tensors")
        if t.shape != u.shape or t.dtype != u.dtype:
            raise ValueError("grid shapes/dtypes differ")
    nx, ny, nz = u.shape
    if min(nx, ny, nz) < 2 * G + 1:
        raise ValueError(f"grid needs at least one owned node plus {G} ghosts per side")
    return [nx, ny, nz, G]


def _check_box_g(box, gv) -> list[int]:
    i0, i1, j0, j1, k0, k1 = (int(v) for v in box)
    X, Y, Z = (gv[a] - 2 * gv[3] for a in range(3))
    if not (1 <= i0 <= i1 <= X and 1 <= j0 <= j1 <= Y and 1 <= k0 <= k1 <= Z):
        raise ValueError(f"box {box} outside the owned region 1..{X} x 1..{Y} x 1..{Z}")
    return [i0, i1, j0, j1, k0, k1]


def tb_sweep(A, B, C, D, boxes, *, first: bool, cdom, err_i, tx, ty, tz, coefs_c, coefs_d,
             err_c, err_d, rows: int = 2, waves: int = 4, chunk: int = 0, wrap_c=None,
             wrap_d=None, ghost: int = 2, delta: bool = False, kwaves: int = 1) -> None:
    """One temporal-blocking sweep (k_tb2): C = u^m and D = u^{m+1} on ``boxes`` from
    A = u^{m-1}, B = u^{m-2} (dense grids with ``ghost`` >= 2 layers; logical indices).
    ``cdom`` = (i0, i1, j0, j1, k0, k1): C is a stencil value inside it in j/k, 0 outside
    (Dirichlet faces); coefs = (hx2, hy2, hz2, coef, ct) per layer. ``delta``: increment form,
    B holds d^{m-1}, C receives d^{m+1} and D u^{m+1} (u^m only enters the errors).
    Tile = (waves / kwaves) * rows rows x 64 * kwaves columns."""
    gv = _check_grid_g(ghost, A, B, C, D)
    if ghost < 2:
        raise ValueError("k_tb2 needs ghost depth >= 2")
    if isinstance(boxes[0], int):
        boxes = [boxes]
    bl = [_check_box_g(b, gv) for b in boxes]
    if not _C().tb_supported(2, rows, waves, kwaves):
        raise ValueError(f"unsupported tile rows={rows} waves={waves} kwaves={kwaves}")
    for t in (tx, ty, tz):
        if not t.is_cuda or t.dtype != A.dtype or t.numel() < max(gv[:3]):
            raise ValueError("analytic tables must be device tensors covering the grid")
    for e in (err_c, err_d):
        if e.dtype != torch.int64 or e.numel() < 3 or not e.is_cuda:
            raise ValueError("error slots must be >= 3 int64 device values (new_err())")
    fn = getattr(_C(), "k_tb2_" + _sfx(A))
    fn(int(rows), int(waves), int(kwaves), bool(delta), bool(first), A.data_ptr(), B.data_ptr(), C.data_ptr(),
       D.data_ptr(), gv, bl, [int(v) for v in cdom], int(err_i[0]), int(err_i[1]), list(wrap_c or []),
       list(wrap_d or []), tx.data_ptr(), ty.data_ptr(), tz.data_ptr(),
       [float(c) for c in coefs_c], [float(c) for c in coefs_d], err_c.data_ptr(),
       err_d.data_ptr(), int(chunk), _stream())


def tbn_sweep(A, B, O0, O1, boxes, *, depth: int, first: bool, cdom, err_i, tx, ty, tz, coefs, errs,
              rows: int = 2, waves: int = 8, chunk: int = 0, ghost: int | None = None, fma: bool = False,
              delta: bool = False) -> None:
    """One deep sweep (k_tbn, ``depth`` layers u^m .. u^{m+depth-1}): the first depth-2 layers
    errors only, O0 = u^{m+depth-2}, O1 = u^{m+depth-1}. ``coefs[l]`` = (hx2, hy2, hz2, coef, ct)
    and ``errs[l]`` the error slot of layer m+l. ``delta``: the increment form (fp32, depth 4):
    B = d^{m-1}, O0 = d^{m+depth-1}, O1 = u^{m+depth-1}."""
    ghost = depth if ghost is None else ghost
    gv = _check_grid_g(ghost, A, B, O0, O1)
    if ghost < depth:
        raise ValueError("k_tbn needs ghost depth >= depth")
    if isinstance(boxes[0], int):
        boxes = [boxes]
    bl = [_check_box_g(b, gv) for b in boxes]
    ok = (_C().tbn_delta_supported(int(depth), int(rows), int(waves), bool(fma), A.dtype == torch.float32)
          if delta else _C().tbn_supported(int(depth), int(rows), int(waves), bool(fma), A.dtype == torch.float32))
    if not ok:
        raise ValueError(f"unsupported depth={depth} tile rows={rows} waves={waves} fma={fma} delta={delta}")
    if len(coefs) != depth or len(errs) != depth:
        raise ValueError("one coefficient set and one error slot per layer")
    for t in (tx, ty, tz):
        if not t.is_cuda or t.dtype != A.dtype or t.numel() < max(gv[:3]):
            raise ValueError("analytic tables must be device tensors covering the grid")
    fn = getattr(_C(), "k_tbn_" + _sfx(A))
    fn(int(depth), int(rows), int(waves), bool(fma), bool(first), A.data_ptr(), B.data_ptr(), O0.data_ptr(),
       O1.data_ptr(), gv, bl, [int(v) for v in cdom], int(err_i[0]), int(err_i[1]), tx.data_ptr(), ty.data_ptr(),
       tz.data_ptr(), [[float(c) for c in co] for co in coefs], [e.data_ptr() for e in errs], int(chunk), _stream(),
       bool(delta))


def tb3_sweep(A, B, D, E, boxes, *, first: bool, cdom, err_i, tx, ty, tz, coefs_c, coefs_d,
              coefs_e, err_c, err_d, err_e, rows: int = 2, waves: int = 8, chunk: int = 0,
              ghost: int = 3, fma: bool = False) -> None:
    """One three-layer sweep (k_tb3): C = u^m (errors only), D = u^{m+1}, E = u^{m+2}.
    ``fma``: the --math fma instantiation (coef/h^2 folded; not bitwise with the exact form)."""
    gv = _check_grid_g(ghost, A, B, D, E)
    if ghost < 3:
        raise ValueError("k_tb3 needs ghost depth >= 3")
    if isinstance(boxes[0], int):
        boxes = [boxes]
    bl = [_check_box_g(b, gv) for b in boxes]
    if not _C().tb_supported(3, rows, waves, fm=bool(fma)):
        raise ValueError(f"unsupported tile rows={rows} waves={waves} fma={fma}")
    for t in (tx, ty, tz):
        if not t.is_cuda or t.dtype != A.dtype or t.numel() < max(gv[:3]):
            raise ValueError("analytic tables must be device tensors covering the grid")
    fn = getattr(_C(), "k_tb3_" + _sfx(A))
    fn(int(rows), int(waves), bool(fma), bool(first), A.data_ptr(), B.data_ptr(), D.data_ptr(), E.data_ptr(),
       gv, bl, [int(v) for v in cdom], int(err_i[0]), int(err_i[1]), tx.data_ptr(),
       ty.data_ptr(), tz.data_ptr(), [float(c) for c in coefs_c], [float(c) for c in coefs_d],
       [float(c) for c in coefs_e], err_c.data_ptr(), err_d.data_ptr(), err_e.data_ptr(),
       int(chunk), _stream())
