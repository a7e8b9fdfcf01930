// Point-update arithmetic shared by the OpenMP oracle and the HIP kernels.
//
// The operation order is the reference's, term for term, so that with FP contraction off
// both backends reproduce the reference output bit for bit:
//   laplace  = 0 + (u[i-1] - 2u + u[i+1])/(hx*hx) + (..y..)/(hy*hy) + (..z..)/(hz*hz)
//                                                             (mpi_new.cpp:104-111)
//   layer 1  = u0 + (a2*tau*tau*0.5) * laplace                (mpi_new.cpp:303)
//   layer n  = (2*u1 - u2) + (a2*tau*tau) * laplace            (mpi_new.cpp:338)
//   f        = sin(..x..)*sin(..y..)*sin(..z..)*cos(..t..)    (mpi_new.cpp:151)
//   abs      = |u - f|, rel = |u - f| / |f|                   (mpi_new.cpp:341-342)
//   max      : if (e > m) m = e   (NaN never wins)            (mpi_new.cpp:343-344)
#pragma once

#include <type_traits>
#include <cmath>

#ifdef __HIPCC__
#define W3D_HD __host__ __device__ __forceinline__
#else
#define W3D_HD inline
#endif

namespace wave3d {

template <class T>
W3D_HD T laplace7(T c, T xm, T xp, T ym, T yp, T zm, T zp, T hx2, T hy2, T hz2) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    T two_c = T(2) * c;
    T ans = T(0);
    ans += (xm - two_c + xp) / hx2;
    ans += (ym - two_c + yp) / hy2;
    ans += (zm - two_c + zp) / hz2;
    return ans;
}

template <class T>
W3D_HD T leapfrog(T c, T u2, T lap, T coef) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    return (T(2) * c - u2) + coef * lap;
}

// Increment form: d^n = d^{n-1} + coef*lap, u^n = u^{n-1} + d^n (the same scheme as
// leapfrog in exact arithmetic, without the 2u - u cancellation). Returns d^n; u^n = c + d^n.
template <class T>
W3D_HD T delta_incr(T d, T lap, T coef) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    return d + coef * lap;
}

template <class T>
W3D_HD T taylor_first(T c, T lap, T coef_first) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    return c + coef_first * lap;
}

template <class T>
W3D_HD T analytic(T sx, T sy, T sz, T ct) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    return ((sx * sy) * sz) * ct;
}

W3D_HD double absval(double x) { return __builtin_fabs(x); }
W3D_HD float absval(float x) { return __builtin_fabsf(x); }

// Updates the running maxima with the reference's NaN-ignoring comparison.
template <class T>
W3D_HD void accumulate_error(T u, T f, T& mabs, T& mrel) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    T d = u - f;
    T ea = absval(d);
    T er = ea / absval(f);
    if (ea > mabs) mabs = ea;
    if (er > mrel) mrel = er;
}

// ---- correctly rounded division by a constant ----------------------------------------
// q = a*y, r = a - q*b (exact by FMA), q' = q + r*y with y = RN(1/b) is RN(a/b) absent
// under/overflow (Markstein's theorem). Three FP ops instead of the ~10-instruction IEEE
// division sequence, bitwise identical to a/b (checked against the reference's true
// divisions by the CPU/GPU parity tests).
W3D_HD double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }
W3D_HD float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
#ifdef __HIPCC__
// Two fp32 lanes of one work item (two grid rows) as one packed value: v_pk_add_f32 /
// v_pk_mul_f32 / v_pk_fma_f32 on CDNA4 — IEEE per element, so bitwise equal to two scalar
// evaluations of the same expression.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 fma_t(f32x2 a, f32x2 b, f32x2 c) {
    return __builtin_elementwise_fma(a, b, c);
}
#endif

template <class T>
W3D_HD T div_const(T a, T b, T y) {
    T q = a * y;
    T r = fma_t(-q, b, a);
    return fma_t(r, y, q);
}

template <class T>
W3D_HD T laplace7_cr(T c, T xm, T xp, T ym, T yp, T zm, T zp, T hx2, T hy2, T hz2, T rx2, T ry2,
                     T rz2) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    T two_c = T(2) * c;
    T ans = T(0);
    ans += div_const(xm - two_c + xp, hx2, rx2);
    ans += div_const(ym - two_c + yp, hy2, ry2);
    ans += div_const(zm - two_c + zp, hz2, rz2);
    return ans;
}

// ---- FMA form (--math fma): the same scheme with coef/h^2 folded into three constants ------
// coef*lap = cx*((xm + xp) - 2c) + cy*(...) + cz*(...), cd = coef/hd^2: every second difference
// is still formed before it is scaled (no loss of the small h^2 u'' term, so fp32 keeps its
// accuracy), 8 FP operations instead of the exact form's ~19 (three correctly rounded
// divisions), rounded differently from the reference CPU programs — as nvcc's default FMA
// contraction rounds the reference's own CUDA kernel (cuda_sol_kernels.cu:36-38) differently.
// fp64: s = fma(-2, c, xm + xp) (2 ops; its rounding, ~eps*|u|, is far below the scheme's
// error). fp32, whose error the rounding sets: s = (xm - c) + (xp - c) — each difference of
// neighbouring values is exact (Sterbenz), so s carries one rounding of a quantity of size h*u'
// instead of one of size u: more accurate than the reference's (xm - 2c) + xp too.
W3D_HD double second_diff(double m, double c, double p) { return fma_t(-2.0, c, m + p); }
W3D_HD float second_diff(float m, float c, float p) { return (m - c) + (p - c); }
#ifdef __HIPCC__
__device__ __forceinline__ f32x2 second_diff(f32x2 m, f32x2 c, f32x2 p) { return (m - c) + (p - c); }
#endif
template <class T>
W3D_HD T coef_lap_fma(T c, T xm, T xp, T ym, T yp, T zm, T zp, T cx, T cy, T cz) {
    const T sx = second_diff(xm, c, xp);
    const T sy = second_diff(ym, c, yp);
    const T sz = second_diff(zm, c, zp);
    return fma_t(cx, sx, fma_t(cy, sy, cz * sz));
}
// leapfrog with a pre-scaled Laplacian l = coef*lap: (2c - u2) + l
template <class T>
W3D_HD T leapfrog_fma(T c, T u2, T l) {
    return fma_t(T(2), c, -u2) + l;
}
// The --math fma leapfrog step (every layer after the Taylor start) in fewer operations. fp64:
//   l = cx (xm + xp) + cy (ym + yp) + cz (zm + zp) + kc c,  kc = -2 (cx + cy + cz);  u = (2c - u2) + l
// 9 operations instead of coef_lap_fma + leapfrog_fma's 11 (three pair sums, a product, three
// FMAs, then the leapfrog's FMA and add). coef*lap comes out of the scaled pairs minus the scaled
// centre: its rounding, ~eps (cx + cy + cz) |u|, is the size of second_diff's rounding scaled by
// c, and the leapfrog keeps its own form, so the error tables keep the reference's 6 digits
// (N=512 K=100 L-inf 6.03381294e-07 vs 6.03381293e-07). Folding 2c into kc as well (one chain,
// 8 operations) biases the rounding of the O(|u|) sum and grows quadratically under the leapfrog:
// 6.03381562e-07, which breaks the printed golden. fp32 keeps the composition above: its accuracy
// rests on the exact (Sterbenz) differences. kc = fm_kc(cx, cy, cz), loop-invariant.
template <class T>
W3D_HD T fm_kc(T cx, T cy, T cz) {
    return T(-2) * ((cx + cy) + cz);
}
template <class T>
W3D_HD T leap_fm(T c, T u2, T xm, T xp, T ym, T yp, T zm, T zp, T cx, T cy, T cz, T kc) {
    if constexpr (std::is_same_v<T, double>) {
        T t = cz * (zm + zp);
        t = fma_t(cy, ym + yp, t);
        t = fma_t(cx, xm + xp, t);
        t = fma_t(kc, c, t);
        return fma_t(T(2), c, -u2) + t;
    } else {
        (void)kc;
        return leapfrog_fma(c, u2, coef_lap_fma(c, xm, xp, ym, yp, zm, zp, cx, cy, cz));
    }
}
// leap_fm with the Dirichlet mask m (1 computed node, 0 face / outside) in the last operation:
// (2c - u2) + l*m, one rounding like the add for m = 1; on masked nodes c = u2 = 0 (the faces are
// never stored), so the result is 0 without a product per node
template <class T>
W3D_HD T leap_fm_masked(T c, T u2, T xm, T xp, T ym, T yp, T zm, T zp, T cx, T cy, T cz, T kc, T m) {
    if constexpr (std::is_same_v<T, double>) {
        T t = cz * (zm + zp);
        t = fma_t(cy, ym + yp, t);
        t = fma_t(cx, xm + xp, t);
        t = fma_t(kc, c, t);
        return fma_t(t, m, fma_t(T(2), c, -u2));
    } else {
        (void)kc;
        return fma_t(coef_lap_fma(c, xm, xp, ym, yp, zm, zp, cx, cy, cz), m, fma_t(T(2), c, -u2));
    }
}
// A deferred --math fma stencil evaluation for the temporal-blocking kernels' lap() / leap()
// lambdas: the leapfrog consumes the inputs whole (leap_fm), every other update (Taylor start,
// increment form) takes coef*lap = value() — the same operations as before for those.
template <class T>
struct FmLap {
    T c, xm, xp, ym, yp, zm, zp, cx, cy, cz;
    W3D_HD T value() const { return coef_lap_fma(c, xm, xp, ym, yp, zm, zp, cx, cy, cz); }
    W3D_HD T leap(T u2, T kc) const { return leap_fm(c, u2, xm, xp, ym, yp, zm, zp, cx, cy, cz, kc); }
    W3D_HD T leap_masked(T u2, T kc, T m) const {
        return leap_fm_masked(c, u2, xm, xp, ym, yp, zm, zp, cx, cy, cz, kc, m);
    }
};
template <class T>
W3D_HD T lap_value(const FmLap<T>& l) {
    return l.value();
}
template <class T>
W3D_HD T lap_value(T l) {
    return l;
}

// True for NaN and +-Inf (x - x is NaN exactly for those).
template <class T>
W3D_HD bool nonfinite(T x) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    T z = x - x;
    return z != z;
}

}  // namespace wave3d
