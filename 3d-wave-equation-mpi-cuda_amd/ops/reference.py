"""Plain-PyTorch reference implementations (the oracle for the HIP kernels).

Every operation is a separate, individually rounded elementwise op in the reference's
order, so in fp64 on the CPU the results are bitwise those of mpi_new (no contraction).
"""
from __future__ import annotations

import math

import torch


def laplace7(u: torch.Tensor, hx2, hy2, hz2) -> torch.Tensor:
    """7-point Laplacian on all interior nodes u[1:-1,1:-1,1:-1] (mpi_new.cpp:104-111)."""
    c = u[1:-1, 1:-1, 1:-1]
    two_c = 2 * c
    ans = torch.zeros_like(c)
    ans = ans + (u[:-2, 1:-1, 1:-1] - two_c + u[2:, 1:-1, 1:-1]) / hx2
    ans = ans + (u[1:-1, :-2, 1:-1] - two_c + u[1:-1, 2:, 1:-1]) / hy2
    ans = ans + (u[1:-1, 1:-1, :-2] - two_c + u[1:-1, 1:-1, 2:]) / hz2
    return ans


def step(u1, u2, box, *, first: bool, hx2, hy2, hz2, coef) -> torch.Tensor:
    """Layer update on ``box`` (local inclusive indices); returns the updated box values."""
    i0, i1, j0, j1, k0, k1 = box
    lap = laplace7(u1, hx2, hy2, hz2)[i0 - 1:i1, j0 - 1:j1, k0 - 1:k1]
    c = u1[i0:i1 + 1, j0:j1 + 1, k0:k1 + 1]
    if first:
        return c + coef * lap
    return (2 * c - u2[i0:i1 + 1, j0:j1 + 1, k0:k1 + 1]) + coef * lap


def analytic(tx, ty, tz, ct) -> torch.Tensor:
    """f = ((sx*sy)*sz)*ct on the tensor product of the 1-D tables."""
    return ((tx[:, None, None] * ty[None, :, None]) * tz[None, None, :]) * ct


def max_errors(u: torch.Tensor, f: torch.Tensor, init: float = -100.0) -> tuple[float, float]:
    """max |u-f| and max |u-f|/|f| with the reference's NaN-ignoring `if (e > m)` rule."""
    d = (u - f).abs()
    r = d / f.abs()
    neg = torch.tensor(-math.inf, dtype=u.dtype, device=u.device)
    a = torch.where(torch.isnan(d), neg, d).max().item() if d.numel() else -math.inf
    b = torch.where(torch.isnan(r), neg, r).max().item() if r.numel() else -math.inf
    return max(a, init), max(b, init)


def tables(N: int, K: int, L=("pi", "pi", "pi"), T: float = 1.0, pi: str = "ref",
           phase: float = 0.0, dtype=torch.float64):
    """1-D analytic tables, evaluated with the reference's expressions (mpi_new.cpp:151)."""
    PI = 3.1415926535 if pi == "ref" else math.pi
    Lx, Ly, Lz = (PI if v == "pi" else float(v) for v in L)
    a_t = 0.5 * math.sqrt(4 / (Lx * Lx) + 1 / (Ly * Ly) + 1 / (Lz * Lz))
    tau = T / K
    hx, hy, hz = Lx / N, Ly / N, Lz / N
    if phase == 0.0:
        sx = [math.sin(2 * PI * (hx * g) / Lx) for g in range(N + 1)]
    else:
        sx = [math.sin(2 * PI * (hx * g) / Lx + phase) for g in range(N + 1)]
    sy = [math.sin(PI * (hy * g) / Ly) for g in range(N + 1)]
    sz = [math.sin(PI * (hz * g) / Lz) for g in range(N + 1)]
    ct = [math.cos(a_t * (tau * n) + 2 * PI) for n in range(K + 1)]
    a2 = 1 / (4 * PI * PI)
    consts = dict(a2=a2, a_t=a_t, tau=tau, hx=hx, hy=hy, hz=hz, hx2=hx * hx, hy2=hy * hy,
                  hz2=hz * hz, coef=a2 * tau * tau, coef_first=a2 * tau * tau * 0.5)
    t = lambda v: torch.tensor(v, dtype=dtype)  # noqa: E731
    return t(sx), t(sy), t(sz), ct, consts


def solve(N: int, K: int, L=("pi", "pi", "pi"), T: float = 1.0, pi: str = "ref",
          phase: float = 0.0, dtype=torch.float64, device="cpu", scheme: str = "leapfrog"):
    """Whole single-domain solve in PyTorch; returns (max_abs[0..K], max_rel[0..K], u_K).

    Storage: x has ghost planes (local = global + 1), y/z none (faces are Dirichlet).
    scheme "delta": increment form, d^n = d^{n-1} + coef*lap u^{n-1}, u^n = u^{n-1} + d^n.
    """
    sx, sy, sz, ct, c = tables(N, K, L, T, pi, phase, dtype)
    sx, sy, sz = sx.to(device), sy.to(device), sz.to(device)
    g = [torch.zeros(N + 3, N + 1, N + 1, dtype=dtype, device=device) for _ in range(3)]

    def wrap(u):
        u[0] = u[N]       # ghost x=-1  <- global N-1
        u[N + 2] = u[2]   # ghost x=N+1 <- global 1

    f0 = analytic(sx, sy, sz, ct[0])
    g[0][1:N + 2] = f0
    wrap(g[0])
    ma, mr = max_errors(f0, f0)
    abs_e, rel_e = [ma], [mr]
    d = None
    for n in range(1, K + 1):
        u1, u2, u = g[(n + 2) % 3], g[(n + 1) % 3], g[n % 3]
        u.zero_()
        # stencil points: all x (incl. the periodic planes), y/z global 1..N-1
        box = (1, N + 1, 1, N - 1, 1, N - 1)
        coef = c["coef_first"] if n == 1 else c["coef"]
        if scheme == "delta":
            lap = laplace7(u1, c["hx2"], c["hy2"], c["hz2"])[0:N + 1, 0:N - 1, 0:N - 1]
            d = coef * lap if n == 1 else d + coef * lap
            vals = u1[1:N + 2, 1:N, 1:N] + d
        else:
            vals = step(u1, u2, box, first=n == 1, hx2=c["hx2"], hy2=c["hy2"], hz2=c["hz2"],
                        coef=coef)
        u[1:N + 2, 1:N, 1:N] = vals
        wrap(u)
        f = analytic(sx[1:N], sy[1:N], sz[1:N], ct[n])
        ma, mr = max_errors(u[2:N + 1, 1:N, 1:N], f)
        abs_e.append(ma)
        rel_e.append(mr)
    return abs_e, rel_e, g[K % 3]


def stencil_field(u1, u2, *, first: bool, hx2, hy2, hz2, coef) -> torch.Tensor:
    """One layer on every node with a full 7-point neighbourhood: values for u1[1:-1, 1:-1, 1:-1]
    (u2 unused when ``first``). The temporal-blocking oracle chains this per layer."""
    lap = laplace7(u1, hx2, hy2, hz2)
    c = u1[1:-1, 1:-1, 1:-1]
    if first:
        return c + coef * lap
    return (2 * c - u2[1:-1, 1:-1, 1:-1]) + coef * lap


def chained_delta(A, Dm1, *, first: bool, mask, hx2, hy2, hz2, coefs):
    """Increment-form sweep oracle (k_tb2 delta): d^m = d^{m-1} + c0*lap A (c0*lap A when
    ``first``), C = A + d^m, d^{m+1} = d^m + c1*lap C, D = C + d^{m+1}; C and d are 0 where
    ``mask`` is False. Returns (C, D, d^{m+1}) on the full grid."""
    zero = torch.zeros((), dtype=A.dtype)
    inner = (slice(1, -1),) * 3

    def lap_of(u):
        v = torch.zeros_like(u)
        v[inner] = laplace7(u, hx2, hy2, hz2)
        return v
    m = mask.clone()
    m[0], m[-1], m[:, 0], m[:, -1], m[:, :, 0], m[:, :, -1] = (False,) * 6
    la = lap_of(A)
    dm = coefs[0] * la if first else Dm1 + coefs[0] * la
    dm = torch.where(m, dm, zero)
    Cf = torch.where(m, A + dm, zero)
    dn = dm + coefs[1] * lap_of(Cf)
    return Cf, Cf + dn, dn


def chained_delta_layers(A, Dm1, nlayers: int, *, first: bool, mask, hx2, hy2, hz2, coefs):
    """Increment-form deep-sweep oracle (k_tbn DELTA): d_l = d_{l-1} + c_l lap U_{l-1} (layer 0 of
    the first sweep: c_0 lap A alone), U_l = U_{l-1} + d_l with U_{-1} = A, d_{-1} = Dm1; U and d are
    0 where ``mask`` is False and on the outermost ring. Returns ([U_0 .. U_{n-1}], d_{n-1})."""
    zero = torch.zeros((), dtype=A.dtype)
    inner = (slice(1, -1),) * 3
    m = mask.clone()
    m[0], m[-1], m[:, 0], m[:, -1], m[:, :, 0], m[:, :, -1] = (False,) * 6
    out, u, d = [], A, Dm1
    for q in range(nlayers):
        la = torch.zeros_like(u)
        la[inner] = laplace7(u, hx2, hy2, hz2)
        d = coefs[q] * la if (first and q == 0) else d + coefs[q] * la
        d = torch.where(m, d, zero)
        u = torch.where(m, u + d, zero)
        out.append(u)
    return out, d


def chained_layers(A, B, nlayers: int, *, first: bool, mask, hx2, hy2, hz2, coefs):
    """Layers m, m+1, ... of a temporal-blocking sweep on full grids: C from (A, B), D from
    (C, A), E from (D, C); each layer is 0 where ``mask`` is False (Dirichlet faces) and on the
    outermost node ring of the grid (no stencil there)."""
    out, prev2, prev1 = [], B, A
    zero = torch.zeros((), dtype=A.dtype)
    for q in range(nlayers):
        v = torch.zeros_like(A)
        val = stencil_field(prev1, prev2, first=first and q == 0, hx2=hx2, hy2=hy2, hz2=hz2,
                            coef=coefs[q])
        v[1:-1, 1:-1, 1:-1] = torch.where(mask[1:-1, 1:-1, 1:-1], val, zero)
        out.append(v)
        prev2, prev1 = prev1, v
    return out
