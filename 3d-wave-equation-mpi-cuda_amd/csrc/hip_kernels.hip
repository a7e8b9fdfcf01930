// Hand-written CDNA4 (gfx950) kernels of the wave3d solver.
//
// Replaces the reference's CUDA kernels (cuda_sol_kernels.cu): calculate_layer (:24-47),
// layer0 (:179-190), layer1 (:192-213), prepare_layer (:230-268), calculate_max_errors
// (:50-89), copy_to_matrices / copy_to_grid (:91-177) — with a different design:
//
//  * k_march: 2.5-D blocked leapfrog. A 256-thread workgroup (4 wave64s) owns a
//    16(j) x 64(k) tile of the (j,k) plane and marches along i. Each lane keeps its
//    4-row column strip for planes i-1, i, i+1 (and i+2 in flight) in registers, the
//    current plane is staged in a double-buffered LDS tile (one barrier per plane) for the
//    j±1 / k±1 neighbours, so u^{n-1} is read from HBM once and u^{n-2} once per point.
//    The analytic error is fused (separable tables, no transcendentals), reduced per
//    workgroup with wave shuffles and committed with one 64-bit atomicMax per slot —
//    no per-point error arrays, no memsets, no host syncs (cuda_sol.cpp:395-418).
//  * The periodic x wrap (dims[0] == 1) and the y/z halo packing can be fused into the
//    stores, so a single-GPU step is exactly one launch.
//  * 64-bit plane offsets (the reference's int indexing overflows, Appendix B7).
//
// FP contraction is off in this file (-ffp-contract=off + pragmas in stencil_math.hpp):
// every value is rounded exactly like the reference CPU programs, so the reported errors
// are bitwise those of mpi_new.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>

#include "device_common.hpp"


namespace wave3d {
namespace {

template <class T>
struct StepParams {
    int xcd;  // XCD-aware tile order (xcd_swizzle)
    int delta;  // increment form (k_naive / k_flat): u2 holds d^{n-1}, u = u1 + (u2 + coef lap)
    const T* u1;
    const T* u2;
    T* u;
    i64 si;
    int sj;
    int poff;        // see GridView::poff
    int jmax, kmax;  // largest valid j / k index in storage (ny-1, nz-1)
    int nbox;
    BoxLaunch box[kMaxBoxes];
    int ei0, ei1;
    int wsrc[kMaxWrap], wdst[kMaxWrap];  // k_naive
    int w_lo[2], w_hi[2], w_sh[2];       // k_march (wrap_ranges)
    T* zbuf0;
    T* zbuf1;
    int zk0, zk1;
    T* ybuf0;
    T* ybuf1;
    int yj0, yj1;
    int zrow, yrow;  // packed row lengths (Y+2, Z+2)
    const T* tx;
    const T* ty;
    const T* tz;
    T hx2, hy2, hz2, coef, ct;
    int fm;           // --math fma (k_naive / k_flat; k_march: the FAST instantiation)
    T fc[3];          // --math fma: coef/h^2 per axis
    T yx2, yy2, yz2;  // RN(1/h^2) in T for the correctly rounded constant division
    u64* err;
};

// One node of the one-point-per-lane kernels: exact (the reference's operation order) or the
// --math fma form; leapfrog, Taylor start, or increment form (u2 holds d^{n-1})
template <class T, bool FIRST>
__device__ __forceinline__ T point_update(const StepParams<T>& p, T c, T xm, T xp, T ym, T yp, T zm, T zp, i64 o) {
    if (p.fm) {
        if (!FIRST && !p.delta)
            return leap_fm(c, p.u2[o], xm, xp, ym, yp, zm, zp, p.fc[0], p.fc[1], p.fc[2],
                           fm_kc(p.fc[0], p.fc[1], p.fc[2]));
        const T l = coef_lap_fma(c, xm, xp, ym, yp, zm, zp, p.fc[0], p.fc[1], p.fc[2]);
        return FIRST ? c + l : c + (p.u2[o] + l);
    }
    const T lap = laplace7_cr(c, xm, xp, ym, yp, zm, zp, p.hx2, p.hy2, p.hz2, p.yx2, p.yy2, p.yz2);
    return FIRST ? taylor_first(c, lap, p.coef)
                 : (p.delta ? c + delta_incr(p.u2[o], lap, p.coef) : leapfrog(c, p.u2[o], lap, p.coef));
}

template <class T>
__device__ __forceinline__ void store_point(const StepParams<T>& p, int i, int j, int k, i64 o,
                                            int rowoff, T v) {
    p.u[o] = v;
#pragma unroll
    for (int q = 0; q < kMaxWrap; ++q)
        if (i == p.wsrc[q]) p.u[i64(p.wdst[q]) * p.si + rowoff] = v;
    if (k == p.zk0) p.zbuf0[i64(i - 1) * p.zrow + j] = v;
    if (k == p.zk1) p.zbuf1[i64(i - 1) * p.zrow + j] = v;
    if (j == p.yj0) p.ybuf0[i64(i - 1) * p.yrow + k] = v;
    if (j == p.yj1) p.ybuf1[i64(i - 1) * p.yrow + k] = v;
}

// ---------------------------------------------------------------------------------------
// 2.5-D marching kernel (LDS tile + register-rolling i column).
// R = rows (j) per lane; the workgroup tile is (4R) x 64. NT = non-temporal loads of the
// read-once level u^{n-2}. L = 2 (fp32 only): the lane's rows are processed in pairs as
// packed fp32 (v_pk_*), halving the VALU cost of the stencil arithmetic.
// Rolling state sits in fixed slots (plane number mod 4 / mod 2) and the i loop is unrolled
// by 4 with the phase as a constant, so a prefetched plane is consumed from the register it
// was loaded into (no copies of in-flight loads, no s_waitcnt vmcnt(0) per plane).
template <class T, bool FIRST, int R, bool NT, bool FAST, int L>
__global__ void __launch_bounds__(kThreads) k_march(const StepParams<T> p) {
    using V = typename RowVec<T, L>::type;
    constexpr int NV = R / L;
    constexpr int kTJ = kWaves * R;
    constexpr unsigned ES = sizeof(T);
    static_assert(R % L == 0, "rows per lane must be a multiple of the vector width");
    __shared__ T lds[2][kTJ + 2][kLW];

    const int bid = xcd_swizzle(blockIdx.x, gridDim.x, p.xcd);
    const int b = find_box(p, bid);
    const BoxLaunch B = p.box[b];
    int local = bid - B.block_begin;
    const int tk = local % B.tiles_k;
    local /= B.tiles_k;
    const int tj = local % B.tiles_j;
    const int ci = local / B.tiles_j;

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int kb = B.kbase + tk * kTK;
    const int k = kb + lane;
    const int jt = B.j0 + tj * kTJ;
    const int ib = B.i0 + ci * B.chunk;
    const int ie = min(B.i1, ib + B.chunk - 1);

    const bool kload = k <= p.kmax;
    const bool kin = k >= B.k0 && k <= B.k1;
    const i64 si = p.si;
    const unsigned pbytes = unsigned(si) * ES;
    // byte offset of (j,k) in a plane block (kOOB = masked: loads give 0, stores dropped)
    auto boff = [&](int j, int kk, bool ok) { return ok ? unsigned(j * p.sj + kk + p.poff) * ES : kOOB; };
    auto prs = [&](const T* base, int i) { return plane_rsrc(base + (i64(i) * si - p.poff), pbytes); };

    unsigned oa[R], ou2[R], os[R];
    bool valid[R];
    V ty[NV];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = jt + w * R + r;
        valid[r] = kin && j <= B.j1;
        oa[r] = boff(j, k, kload && j <= p.jmax);
        ou2[r] = boff(j, k, !FIRST && valid[r]);
        os[r] = boff(j, k, valid[r]);
        vset<L>(ty[r / L], r % L, valid[r] ? p.ty[j] : T(0));
    }
    const V tz = vsplat<L, V>(kin ? p.tz[k] : T(0));

    // halo role of this lane: one LDS cell per plane
    int hrow = 0, hcol = 0;
    unsigned hoff = kOOB;
    bool hon = false;
    if (w == 0) {  // row jt-1
        hon = true;
        hoff = boff(jt - 1, k, kload);
        hrow = 0;
        hcol = 1 + lane;
    } else if (w == kWaves - 1) {  // row jt+TJ
        const int j = jt + kTJ;
        hon = true;
        hoff = boff(j, k, kload && j <= p.jmax);
        hrow = kTJ + 1;
        hcol = 1 + lane;
    } else if (w == 1) {  // columns kb-1 (lanes 0..TJ-1) and kb+64 (lanes 32..32+TJ-1)
        const int side = lane >> 5, rr = lane & 31;
        const int j = jt + rr;
        const int kk = side ? kb + kTK : kb - 1;
        hon = rr < kTJ;
        hoff = boff(j, kk, hon && j <= p.jmax && kk <= p.kmax);
        hrow = 1 + rr;
        hcol = side ? kTK + 1 : 0;
    }
    constexpr int kU2Aux = NT ? 2 : 0;  // non-temporal u^{n-2} (read once)
    constexpr int kStAux = 2;           // non-temporal stores (write-once stream)

    // slots: u1(x) -> (x - ib + 1) & 3, u2(x), halo(x), LDS buffer -> (x - ib) & 1
    V u1[4][NV], u2[2][NV];
    T hv[2];
    {
        const auto r0 = prs(p.u1, ib - 1), r1 = prs(p.u1, ib), r2 = prs(p.u1, ib + 1);
        const auto q0 = prs(p.u2, ib);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            vset<L>(u1[0][r / L], r % L, bld<T>(r0, oa[r]));
            vset<L>(u1[1][r / L], r % L, bld<T>(r1, oa[r]));
            vset<L>(u1[2][r / L], r % L, bld<T>(r2, oa[r]));
            vset<L>(u1[3][r / L], r % L, T(0));
            vset<L>(u2[0][r / L], r % L, FIRST ? T(0) : bld<T, kU2Aux>(q0, ou2[r]));
            vset<L>(u2[1][r / L], r % L, T(0));
        }
        hv[0] = bld<T>(r1, hoff);
        hv[1] = T(0);
    }
    const V hx2 = vsplat<L, V>(p.hx2), hy2 = vsplat<L, V>(p.hy2), hz2 = vsplat<L, V>(p.hz2);
    const V yx2 = vsplat<L, V>(p.yx2), yy2 = vsplat<L, V>(p.yy2), yz2 = vsplat<L, V>(p.yz2);
    const V coef = vsplat<L, V>(p.coef), ctv = vsplat<L, V>(p.ct);

    T ma = T(kErrInit);
    RelArg<T> mr;
    T chk = T(0);  // sum of the values (commit_errors: nonfinite flag)

    auto plane = [&](auto phase, const int i) {
        constexpr int P = decltype(phase)::value;
        constexpr int S0 = P & 3, S1 = (P + 1) & 3, S2 = (P + 2) & 3, S3 = (P + 3) & 3;
        constexpr int H0 = P & 1, H1 = (P + 1) & 1;
        // prefetch u1(i+2) (own rows), u1(i+1) (halo), u2(i+1); 0-record descriptors on the
        // last plane (loads return 0 without touching memory)
        {
            const bool more = i < ie;
            const unsigned nb = more ? pbytes : 0u;
            const int d2 = more ? 2 : 0, d1 = more ? 1 : 0;
            const auto rN = plane_rsrc(p.u1 + (i64(i + d2) * si - p.poff), nb);
            const auto rH = plane_rsrc(p.u1 + (i64(i + d1) * si - p.poff), nb);
            const auto rU = plane_rsrc(p.u2 + (i64(i + d1) * si - p.poff), nb);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                vset<L>(u1[S3][r / L], r % L, bld<T>(rN, oa[r]));
                if (!FIRST) vset<L>(u2[H1][r / L], r % L, bld<T, kU2Aux>(rU, ou2[r]));
            }
            hv[H1] = bld<T>(rH, hoff);
        }

        // stage plane i
#pragma unroll
        for (int r = 0; r < R; ++r) lds[H0][1 + w * R + r][1 + lane] = vget<L>(u1[S1][r / L], r % L);
        if (hon) lds[H0][hrow][hcol] = hv[H0];
        __syncthreads();

        const T sx = ldconst(p.tx, i);
        const bool erow = i >= p.ei0 && i <= p.ei1;
        V vv[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int r0 = v * L, lr = 1 + w * R + r0;
            const V c = u1[S1][v];
            V jm, jp, km, kp;
            if constexpr (L == 1) {
                jm = v == 0 ? lds[H0][lr - 1][1 + lane] : u1[S1][v - 1];
                jp = v == NV - 1 ? lds[H0][lr + 1][1 + lane] : u1[S1][v + 1];
                km = lds[H0][lr][lane];
                kp = lds[H0][lr][lane + 2];
            } else {
                jm = V{v == 0 ? lds[H0][lr - 1][1 + lane] : u1[S1][v - 1][1], c[0]};
                jp = V{c[1], v == NV - 1 ? lds[H0][lr + 2][1 + lane] : u1[S1][v + 1][0]};
                km = V{lds[H0][lr][lane], lds[H0][lr + 1][lane]};
                kp = V{lds[H0][lr][lane + 2], lds[H0][lr + 1][lane + 2]};
            }
            if constexpr (FAST) {  // --math fma (stencil_math coef_lap_fma / leap_fm)
                const V fx = vsplat<L, V>(p.fc[0]), fy = vsplat<L, V>(p.fc[1]), fz = vsplat<L, V>(p.fc[2]);
                if constexpr (FIRST)
                    vv[v] = c + coef_lap_fma(c, u1[S0][v], u1[S2][v], jm, jp, km, kp, fx, fy, fz);
                else
                    vv[v] = leap_fm(c, u2[H0][v], u1[S0][v], u1[S2][v], jm, jp, km, kp, fx, fy, fz,
                                    vsplat<L, V>(fm_kc(p.fc[0], p.fc[1], p.fc[2])));
            } else {
                const V lap = laplace7_cr(c, u1[S0][v], u1[S2][v], jm, jp, km, kp, hx2, hy2, hz2,
                                          yx2, yy2, yz2);
                vv[v] = FIRST ? taylor_first(c, lap, coef) : leapfrog(c, u2[H0][v], lap, coef);
            }
        }
        // stores: own plane + fused periodic wrap (buffer stores, masked lanes dropped)
        {
            const auto rs = prs(p.u, i);
#pragma unroll
            for (int r = 0; r < R; ++r) bst<kStAux>(vget<L>(vv[r / L], r % L), rs, os[r]);
#pragma unroll
            for (int g = 0; g < 2; ++g)
                if (i >= p.w_lo[g] && i <= p.w_hi[g]) {
                    const auto rw = prs(p.u, i + p.w_sh[g]);
#pragma unroll
                    for (int r = 0; r < R; ++r) bst<kStAux>(vget<L>(vv[r / L], r % L), rw, os[r]);
                }
        }
        const V f0 = vsplat<L, V>(sx);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const V f = analytic(f0, ty[v], tz, ctv);
#pragma unroll
            for (int e = 0; e < L; ++e) {
                const int r = v * L + e;
                if (!valid[r]) continue;
                const int j = jt + w * R + r;
                const T x = vget<L>(vv[v], e);
                if (k == p.zk0) p.zbuf0[i64(i - 1) * p.zrow + j] = x;
                if (k == p.zk1) p.zbuf1[i64(i - 1) * p.zrow + j] = x;
                if (j == p.yj0) p.ybuf0[i64(i - 1) * p.yrow + k] = x;
                if (j == p.yj1) p.ybuf1[i64(i - 1) * p.yrow + k] = x;
                chk += x;
                if (erow) {
                    if constexpr (FAST) accumulate_error_dev(x, vget<L>(f, e), ma, mr);
                    else accumulate_error_dev(x, vget<L>(f, e), ma, mr);
                }
            }
        }
    };

    for (int i = ib;;) {
        plane(Ph<0>{}, i);
        if (++i > ie) break;
        plane(Ph<1>{}, i);
        if (++i > ie) break;
        plane(Ph<2>{}, i);
        if (++i > ie) break;
        plane(Ph<3>{}, i);
        if (++i > ie) break;
    }
    commit_errors(ma, mr.value(), chk, p.err);
}

// ---------------------------------------------------------------------------------------
// One-point-per-lane reference kernel (7 neighbour loads through L1/L2). Kept for
// ablation (profiles/) and as a second, independent device implementation.
template <class T, bool FIRST>
__global__ void __launch_bounds__(kThreads) k_naive(const StepParams<T> p) {
    const int bid = xcd_swizzle(blockIdx.x, gridDim.x, p.xcd);
    const int b = find_box(p, bid);
    const BoxLaunch B = p.box[b];
    int local = bid - B.block_begin;
    const int tk = local % B.tiles_k;
    local /= B.tiles_k;
    const int tj = local % B.tiles_j;
    const int ib = B.i0 + (local / B.tiles_j) * B.chunk;
    const int ie = min(B.i1, ib + B.chunk - 1);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int k = B.kbase + tk * kTK + lane;
    const int j = B.j0 + tj * kNaiveTJ + w;
    T ma = T(kErrInit);
    RelArg<T> mr;
    T chk = T(0);  // sum of the values (commit_errors: nonfinite flag)
    if (k >= B.k0 && k <= B.k1 && j <= B.j1) {
        const i64 si = p.si;
        const int rowoff = j * p.sj + k;
        const T tyj = p.ty[j], tzk = p.tz[k];
        for (int i = ib; i <= ie; ++i) {
            const i64 o = i64(i) * si + rowoff;
            const T c = p.u1[o];
            const T v = point_update<T, FIRST>(p, c, p.u1[o - si], p.u1[o + si], p.u1[o - p.sj], p.u1[o + p.sj],
                                               p.u1[o - 1], p.u1[o + 1], o);
            store_point(p, i, j, k, o, rowoff, v);
            chk += v;
            if (i >= p.ei0 && i <= p.ei1)
                accumulate_error_dev(v, analytic(p.tx[i], tyj, tzk, p.ct), ma, mr);
        }
    }
    commit_errors(ma, mr.value(), chk, p.err);
}

// ---------------------------------------------------------------------------------------
// Flattened kernel for the thin shells of the interior/shell overlap (one plane, row or
// column wide): one point per thread over each box with k fastest, so a one-column z shell
// still fills whole waves (a tiled kernel would run 1 of 64 lanes there).
template <class T, bool FIRST>
__global__ void __launch_bounds__(kThreads) k_flat(const StepParams<T> p) {
    const int bid = blockIdx.x;
    const int b = find_box(p, bid);
    const BoxLaunch B = p.box[b];
    const int nk = B.k1 - B.k0 + 1, nj = B.j1 - B.j0 + 1;
    const i64 total = i64(B.i1 - B.i0 + 1) * nj * nk;
    const i64 e = i64(bid - B.block_begin) * kThreads + threadIdx.x;
    T ma = T(kErrInit);
    RelArg<T> mr;
    T chk = T(0);  // sum of the values (commit_errors: nonfinite flag)
    if (e < total) {
        const int k = B.k0 + int(e % nk);
        const i64 r = e / nk;
        const int j = B.j0 + int(r % nj);
        const int i = B.i0 + int(r / nj);
        const i64 si = p.si;
        const int rowoff = j * p.sj + k;
        const i64 o = i64(i) * si + rowoff;
        const T c = p.u1[o];
        const T v = point_update<T, FIRST>(p, c, p.u1[o - si], p.u1[o + si], p.u1[o - p.sj], p.u1[o + p.sj],
                                           p.u1[o - 1], p.u1[o + 1], o);
        store_point(p, i, j, k, o, rowoff, v);
        chk += v;
        if (i >= p.ei0 && i <= p.ei1) accumulate_error_dev(v, analytic(p.tx[i], p.ty[j], p.tz[k], p.ct), ma, mr);
    }
    commit_errors(ma, mr.value(), chk, p.err);
}

// ---------------------------------------------------------------------------------------
// Layer 0 (initial condition): one workgroup per 4 rows (a wave each, its lanes along the whole
// k range) and `chunk` planes, so consecutive workgroups write consecutive rows of a plane in
// long runs (4 x 64 tiles wrote 512-B pieces one plane apart): 258-272 vs 278-301 us at N=512,
// non-temporal stores no better (profiles/deep_sweeps_r5.txt step 17).
template <class T>
__global__ void __launch_bounds__(kThreads) k_init(T* u, i64 si, int sj, Box bx, int chunk,
                                                   Wrap wrap, const T* tx, const T* ty,
                                                   const T* tz, T ct, u64* err) {
    const int lane = threadIdx.x & 63;
    const int j = bx.j0 + blockIdx.x * kWaves + (threadIdx.x >> 6);
    const int ib = bx.i0 + blockIdx.y * chunk;
    const int ie = min(bx.i1, ib + chunk - 1);
    // layer 0 is the analytic solution itself: every error is exactly 0 (the reference's
    // |f - f| and |f - f| / |f|); the relative one only where f != 0 (0/0 is NaN, which its `>`
    // ignores) — the same maxima as accumulate_error_dev without its per-node work
    T ma = T(kErrInit), mr = T(kErrInit);
    T chk = T(0);  // sum of the values (commit_errors: nonfinite flag)
    if (j <= bx.j1) {
        const T tyj = ty[j];
        bool nz = false, any = false;
        for (int i = ib; i <= ie; ++i) {
            const T txi = tx[i];
            const i64 row = i64(j) * sj;
            for (int k = bx.k0 + lane; k <= bx.k1; k += 64) {
                const T f = analytic(txi, tyj, tz[k], ct);
                u[i64(i) * si + row + k] = f;
#pragma unroll
                for (int q = 0; q < kMaxWrap; ++q)  // wrap copies of this plane (uniform tests)
                    if (i == wrap.src[q]) u[i64(wrap.dst[q]) * si + row + k] = f;
                chk += f;
                nz |= f != T(0);
                any = true;
            }
        }
        if (any) ma = T(0);
        if (nz) mr = T(0);
    }
    commit_errors(ma, mr, chk, err);
}

template <class T>
__global__ void k_zero_faces(T* u, i64 si, int sj, int X, int Y, int Z, int G, int mask) {
    const int i = 1 - G + blockIdx.y;  // ghost planes too: redundant ring computations read them
    const int t = 1 + blockIdx.x * blockDim.x + threadIdx.x;
    T* pl = u + i64(i) * si;
    if (t <= Y) {
        if (mask & 1) pl[t * sj + 1] = T(0);
        if (mask & 2) pl[t * sj + Z] = T(0);
    }
    if (t <= Z) {
        if (mask & 4) pl[1 * sj + t] = T(0);
        if (mask & 8) pl[Y * sj + t] = T(0);
    }
}

template <class T>
struct FaceOps {
    FaceOp<T> op[4];
};

template <class T>
__global__ void k_faces(T* u, i64 si, int sj, int ny, int nz, FaceOps<T> ops, bool to_buf) {
    const FaceOp<T> f = ops.op[blockIdx.z];
    const int i = 1 + blockIdx.y;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int len = f.axis == 1 ? nz : ny;
    // ghost corners/edges are never read by the 7-point stencil: skipping them keeps the
    // y and z faces of one launch from writing the same cells
    if (t < 1 || t > len - 2) return;
    T* g = f.axis == 1 ? u + i64(i) * si + i64(f.index) * sj + t
                       : u + i64(i) * si + i64(t) * sj + f.index;
    T* q = f.buf + i64(i - 1) * len + t;
    if (to_buf) *q = *g;
    else *g = *q;
}

__global__ void k_init_err(u64* err, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) err[t] = (t % 3 == 2) ? 0ull : enc_key(kErrInit);
}

// Timer mark: the device's constant-rate wall clock when the stream reaches this point
// (after every earlier kernel of the stream). One lane writes one slot.
__global__ void k_stamp(u64* ts, int slot) {
    if (threadIdx.x == 0) ts[slot] = wall_clock64();
}

// Link-time model (--model-link): one wave waits `ticks` of the constant-rate wall clock, then
// exits — a bounded wait that holds one CU's slot, as the sender/receiver kernels of a remote
// transfer would, while the data itself moves by the loopback copies after it.
__global__ void k_spin(u64 ticks) {
    const u64 t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

__global__ void k_encode(const double* v, u64* k, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) k[t] = enc_key(v[t]);
}

template <class T>
struct BoxCopyOps {
    BoxCopy<T> op[kMaxBoxCopy];
    unsigned first[kMaxBoxCopy + 1];  // first block of box q (blocks sized to each box)
    int n;
};

template <class T>
__global__ void __launch_bounds__(kThreads) k_box_copy(const BoxCopyOps<T> ops, i64 si, int sj,
                                                       bool to_buf) {
    // one 1-D grid over every box, each box getting the blocks its size needs (a launch carries
    // a peer's faces, edges and corners: blocks sized to the largest box left most idle)
    int q = 0;
    for (int t = 1; t < ops.n; ++t)
        if (blockIdx.x >= ops.first[t]) q = t;
    const BoxCopy<T> o = ops.op[q];
    const unsigned b0 = ops.first[q], nb = ops.first[q + 1] - b0;
    // 32-bit element indices (the host checks the box size): unsigned 32-bit div/mod by the
    // wave-uniform extents are a few VALU each, the 64-bit ones a long subroutine per element
    const unsigned nk = unsigned(o.b.k1 - o.b.k0 + 1), nj = unsigned(o.b.j1 - o.b.j0 + 1);
    const unsigned total = unsigned(o.b.i1 - o.b.i0 + 1) * nj * nk;
    for (unsigned e = (blockIdx.x - b0) * blockDim.x + threadIdx.x; e < total; e += nb * blockDim.x) {
        const unsigned r = e / nk, k = e - r * nk;
        const unsigned ii = r / nj, j = r - ii * nj;
        T* g = o.grid + i64(o.b.i0 + int(ii)) * si + i64(o.b.j0 + int(j)) * sj + (o.b.k0 + int(k));
        if (to_buf) o.buf[e] = *g;
        else *g = o.buf[e];
    }
}

}  // namespace

int march_rows_per_thread() { return 4; }

int march_tile_rows(const KernelVariant& v) {
    return v.march && !v.flat ? kWaves * v.rows : kNaiveTJ;
}

int tile_order() {
    static const int order = [] {
        const char* e = std::getenv("WAVE3D_TILE_ORDER");
        const std::string v = e ? e : "";
        if (v == "k") return 0;
        if (v == "j") return 1;
        if (v == "blocks") return 3;  // XCD blocks (k_tbn; the other sweeps treat it as j-fastest)
        W3D_REQUIRE(v.empty() || v == "band", "WAVE3D_TILE_ORDER must be band, blocks, j or k, not " + v);
        return 2;
    }();
    return order;
}

bool xcd_swizzle_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("WAVE3D_XCD_SWIZZLE");
        return e && e[0] == '1';
    }();
    return on;
}

KernelVariant parse_kernel_variant(const std::string& name) {
    // naive | auto | march[R][nt|f|p], R in {2,4,8} (default 4); nt = non-temporal u^{n-2},
    // f = the --math fma form, p = packed fp32 pairs of rows (fp32 runs only)
    KernelVariant v;
    if (name == "naive") {
        v.march = false;
        return v;
    }
    if (name == "flat") {
        v.march = false, v.flat = true;
        return v;
    }
    if (name == "auto") {  // best measured single-step variant on MI355X (profiles/)
        v.rows = 4;  // march4nt: 231 Gpts/s fp64 at N=512 (profiles/sweep_store_policy_r1.txt)
        v.nt = true;
        return v;
    }
    W3D_REQUIRE(name.rfind("march", 0) == 0, "wave3d: unknown kernel variant " + name);
    std::string s = name.substr(5);
    if (!s.empty() && (s[0] == '2' || s[0] == '4' || s[0] == '8')) v.rows = s[0] - '0', s = s.substr(1);
    if (s == "nt") v.nt = true;
    else if (s == "f") v.fast = true;
    else if (s == "p") v.pk = true;
    else W3D_REQUIRE(s.empty(), "wave3d: unknown kernel variant " + name);
    W3D_REQUIRE(!v.fast || v.rows != 8, "wave3d: no fast-math variant with 8 rows");
    W3D_REQUIRE(!v.pk || v.rows != 8, "wave3d: packed variants have 2 or 4 rows");
    return v;
}

std::string kernel_variant_name(const KernelVariant& v) {
    if (v.flat) return "flat";
    if (!v.march) return "naive";
    return "march" + std::to_string(v.rows) + (v.nt ? "nt" : "") + (v.fast ? "f" : "") +
           (v.pk ? "p" : "");
}

template <class T, bool FIRST>
static void (*march_kernel(const KernelVariant& v))(const StepParams<T>) {
    if (v.pk) {
        if constexpr (std::is_same_v<T, float>)
            return v.rows == 2 ? k_march<T, FIRST, 2, false, false, 2> : k_march<T, FIRST, 4, false, false, 2>;
        else throw Error("wave3d: packed march variants are fp32 only");
    }
    if (v.fast)
        return v.rows == 2 ? k_march<T, FIRST, 2, false, true, 1> : k_march<T, FIRST, 4, false, true, 1>;
    switch (v.rows * 2 + (v.nt ? 1 : 0)) {
        case 4: return k_march<T, FIRST, 2, false, false, 1>;
        case 5: return k_march<T, FIRST, 2, true, false, 1>;
        case 9: return k_march<T, FIRST, 4, true, false, 1>;
        case 16: return k_march<T, FIRST, 8, false, false, 1>;
        case 17: return k_march<T, FIRST, 8, true, false, 1>;
        default: return k_march<T, FIRST, 4, false, false, 1>;
    }
}

template <class T>
void launch_step(const KernelVariant& kind, bool first, const T* u1, const T* u2, T* u, const GridView& gv,
                 const Box* boxes, int nbox, int ei0, int ei1, const Wrap& wrap,
                 const FusedPack<T>& pack, const T* tx, const T* ty, const T* tz,
                 const StepCoefs& c, u64* err, int chunk, hipStream_t s) {
    W3D_REQUIRE(nbox >= 1 && nbox <= kMaxBoxes, "bad box count");
    StepParams<T> p{};
    p.xcd = xcd_swizzle_enabled();
    p.delta = kind.delta ? 1 : 0;
    W3D_REQUIRE(!kind.delta || !kind.march || kind.flat, "increment form: naive or flat kernel only");
    p.u1 = u1;
    p.u2 = u2;
    p.u = u;
    p.si = gv.si;
    p.sj = gv.sj;
    p.poff = gv.poff;
    p.jmax = gv.jmax();
    p.kmax = gv.kmax();
    p.ei0 = ei0;
    p.ei1 = ei1;
    for (int q = 0; q < kMaxWrap; ++q) p.wsrc[q] = wrap.src[q], p.wdst[q] = wrap.dst[q];
    wrap_ranges(wrap, p.w_lo, p.w_hi, p.w_sh);
    p.zbuf0 = pack.zbuf[0];
    p.zbuf1 = pack.zbuf[1];
    p.zk0 = pack.zbuf[0] ? pack.zk[0] : -7;
    p.zk1 = pack.zbuf[1] ? pack.zk[1] : -7;
    p.ybuf0 = pack.ybuf[0];
    p.ybuf1 = pack.ybuf[1];
    p.yj0 = pack.ybuf[0] ? pack.yj[0] : -7;
    p.yj1 = pack.ybuf[1] ? pack.yj[1] : -7;
    p.zrow = gv.Y + 2;
    p.yrow = gv.Z + 2;
    p.tx = tx;
    p.ty = ty;
    p.tz = tz;
    p.hx2 = T(c.hx2);
    p.hy2 = T(c.hy2);
    p.hz2 = T(c.hz2);
    p.coef = T(c.coef);
    p.ct = T(c.ct);
    p.yx2 = T(1) / T(c.hx2);
    p.yy2 = T(1) / T(c.hy2);
    p.yz2 = T(1) / T(c.hz2);
    p.fm = kind.fast ? 1 : 0;
    p.fc[0] = T(c.coef / c.hx2), p.fc[1] = T(c.coef / c.hy2), p.fc[2] = T(c.coef / c.hz2);
    p.err = err;
    const bool march = kind.march && !kind.flat;
    const int tj_rows = march ? kWaves * kind.rows : kNaiveTJ;
    int nb = 0, total = 0;
    if (kind.flat) {
        for (int q = 0; q < nbox; ++q) {
            const Box& bx = boxes[q];
            if (bx.empty()) continue;
            W3D_REQUIRE(bx.i0 >= 1 && bx.i1 <= gv.X && bx.j0 >= 1 && bx.j1 <= gv.Y && bx.k0 >= 1 &&
                            bx.k1 <= gv.Z,
                        "step box outside the owned region");
            BoxLaunch& L = p.box[nb++];
            L.i0 = bx.i0, L.i1 = bx.i1, L.j0 = bx.j0, L.j1 = bx.j1, L.k0 = bx.k0, L.k1 = bx.k1;
            L.kbase = L.tiles_k = L.tiles_j = L.chunk = 1;
            L.block_begin = total;
            const i64 pts = i64(bx.i1 - bx.i0 + 1) * (bx.j1 - bx.j0 + 1) * (bx.k1 - bx.k0 + 1);
            W3D_REQUIRE(pts / kThreads < (1ll << 30), "shell box too large for the flat kernel");
            total += int((pts + kThreads - 1) / kThreads);
        }
        p.nbox = nb;
        if (nb == 0) return;
        void (*kern)(const StepParams<T>) = first ? k_flat<T, true> : k_flat<T, false>;
        hipLaunchKernelGGL(kern, dim3(total), dim3(kThreads), 0, s, p);
        HIP_OK(hipGetLastError());
        return;
    }
    int btiles[kMaxBoxes], bplanes[kMaxBoxes], nbt = 0;
    for (int q = 0; q < nbox; ++q) {
        const Box& bx = boxes[q];
        if (bx.empty()) continue;
        btiles[nbt] = ((bx.k1 - 1) / kTK - (bx.k0 - 1) / kTK + 1) * cdiv(bx.j1 - bx.j0 + 1, tj_rows);
        bplanes[nbt++] = bx.i1 - bx.i0 + 1;
    }
    // 32-plane work items (chunk sweep on MI355X, profiles/), shorter on small grids so that
    // there are enough workgroups to fill the 256 CUs
    const int achunk = auto_chunk_boxes(32, btiles, bplanes, nbt);
    for (int q = 0; q < nbox; ++q) {
        const Box& bx = boxes[q];
        if (bx.empty()) continue;
        W3D_REQUIRE(bx.i0 >= 1 && bx.i1 <= gv.X && bx.j0 >= 1 && bx.j1 <= gv.Y && bx.k0 >= 1 &&
                        bx.k1 <= gv.Z,
                    "step box outside the owned region");
        BoxLaunch& L = p.box[nb];
        L.i0 = bx.i0, L.i1 = bx.i1, L.j0 = bx.j0, L.j1 = bx.j1, L.k0 = bx.k0, L.k1 = bx.k1;
        const int t0 = (bx.k0 - 1) / kTK, t1 = (bx.k1 - 1) / kTK;
        L.kbase = 1 + t0 * kTK;
        L.tiles_k = t1 - t0 + 1;
        L.tiles_j = cdiv(bx.j1 - bx.j0 + 1, tj_rows);
        const int planes = bx.i1 - bx.i0 + 1;
        int ch = std::min(chunk > 0 ? chunk : achunk, planes);
        ch = cdiv(planes, cdiv(planes, ch));  // equal work items (no short tail chunk)
        L.chunk = ch;
        L.block_begin = total;
        total += L.tiles_k * L.tiles_j * cdiv(planes, ch);
        ++nb;
    }
    p.nbox = nb;
    if (nb == 0) return;
    void (*kern)(const StepParams<T>);
    if (march) kern = first ? march_kernel<T, true>(kind) : march_kernel<T, false>(kind);
    else kern = first ? k_naive<T, true> : k_naive<T, false>;
    hipLaunchKernelGGL(kern, dim3(total), dim3(kThreads), 0, s, p);
    HIP_OK(hipGetLastError());
}

template <class T>
void launch_init(T* u, const GridView& gv, const Box& bx, const Wrap& wrap, const T* tx,
                 const T* ty, const T* tz, double ct0, u64* err, hipStream_t s) {
    if (bx.empty()) return;
    W3D_REQUIRE(bx.i0 >= 1 && bx.i1 <= gv.X && bx.j1 <= gv.Y && bx.k1 <= gv.Z,
                "init box outside the owned region");
    const int planes = bx.i1 - bx.i0 + 1;
    const int rowblocks = cdiv(bx.j1 - bx.j0 + 1, kWaves);
    const int chunk = std::min(planes, std::max(1, cdiv(planes * rowblocks, 4096)));
    dim3 grid(rowblocks, cdiv(planes, chunk));
    hipLaunchKernelGGL(k_init<T>, grid, dim3(kThreads), 0, s, u, gv.si, gv.sj, bx, chunk, wrap, tx,
                       ty, tz, T(ct0), err);
    HIP_OK(hipGetLastError());
}

template <class T>
void launch_zero_faces(T* u, const GridView& gv, int mask, hipStream_t s) {
    if (!mask) return;
    dim3 grid(cdiv(std::max(gv.Y, gv.Z), 256), gv.X + 2 * gv.G);
    hipLaunchKernelGGL(k_zero_faces<T>, grid, dim3(256), 0, s, u, gv.si, gv.sj, gv.X, gv.Y, gv.Z,
                       gv.G, mask);
    HIP_OK(hipGetLastError());
}

template <class T>
void launch_faces(T* u, const GridView& gv, const FaceOp<T>* ops, int nops, bool to_buf,
                  hipStream_t s) {
    W3D_REQUIRE(nops <= 4, "too many faces");
    if (nops <= 0) return;
    FaceOps<T> f{};
    for (int q = 0; q < nops; ++q) f.op[q] = ops[q];
    const int len = std::max(gv.Y, gv.Z) + 2;
    dim3 grid(cdiv(len, 256), gv.X, nops);
    hipLaunchKernelGGL(k_faces<T>, grid, dim3(256), 0, s, u, gv.si, gv.sj, gv.Y + 2, gv.Z + 2, f,
                       to_buf);
    HIP_OK(hipGetLastError());
}

namespace {
template <class T>
__global__ void k_txy(T* out, const T* tx, const T* ty, int X, int Y, size_t n) {
    const size_t q = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const size_t pj = size_t(Y + 2), used = size_t(X + 2) * pj;
    // the analytic product's first factor, rounded exactly as stencil_math analytic()
    out[q] = q < used ? tx[q / pj] * ty[q % pj] : T(0);
}
}  // namespace

template <class T>
void launch_txy(T* out, const T* tx, const T* ty, int X, int Y, hipStream_t s) {
    const size_t n = txy_elems(X, Y);
    hipLaunchKernelGGL(k_txy<T>, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, out, tx, ty, X, Y, n);
    HIP_OK(hipGetLastError());
}
template void launch_txy<double>(double*, const double*, const double*, int, int, hipStream_t);
template void launch_txy<float>(float*, const float*, const float*, int, int, hipStream_t);

namespace {
template <class T>
__global__ void k_recip_abs(T* out, const T* in, size_t n) {
    const size_t q = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (q < n) out[q] = T(1) / absval(in[q]);  // 1/0 = inf: |d| * inf as the reference's |d|/0
}
}  // namespace

template <class T>
void launch_recip_abs(T* out, const T* in, size_t n, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_recip_abs<T>, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, out, in, n);
    HIP_OK(hipGetLastError());
}
namespace {
template <class T>
__global__ void k_txr(T* out, const T* txy, size_t n) {
    const size_t q = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (q < n) out[2 * q] = txy[q], out[2 * q + 1] = T(1) / absval(txy[q]);
}
}  // namespace

template <class T>
void launch_txr(T* out, const T* txy, size_t n, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_txr<T>, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, out, txy, n);
    HIP_OK(hipGetLastError());
}
template void launch_txr<double>(double*, const double*, size_t, hipStream_t);
template void launch_txr<float>(float*, const float*, size_t, hipStream_t);
template void launch_recip_abs<double>(double*, const double*, size_t, hipStream_t);
template void launch_recip_abs<float>(float*, const float*, size_t, hipStream_t);

void launch_init_err(u64* err, int layers, hipStream_t s) {
    const int n = layers * 3;
    hipLaunchKernelGGL(k_init_err, dim3(cdiv(n, 256)), dim3(256), 0, s, err, n);
    HIP_OK(hipGetLastError());
}

void launch_stamp(u64* ts, int slot, hipStream_t s) {
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, s, ts, slot);
    HIP_OK(hipGetLastError());
}

void launch_spin(u64 ticks, hipStream_t s) {
    if (ticks == 0) return;
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, ticks);
    HIP_OK(hipGetLastError());
}

void launch_encode_keys(const double* v, u64* k, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_encode, dim3(cdiv(n, 256)), dim3(256), 0, s, v, k, n);
    HIP_OK(hipGetLastError());
}

#define W3D_INST(T)                                                                          \
    template void launch_step<T>(const KernelVariant&, bool, const T*, const T*, T*, const GridView&,  \
                                 const Box*, int, int, int, const Wrap&, const FusedPack<T>&, \
                                 const T*, const T*, const T*, const StepCoefs&, u64*, int,   \
                                 hipStream_t);                                               \
    template void launch_init<T>(T*, const GridView&, const Box&, const Wrap&, const T*,     \
                                 const T*, const T*, double, u64*, hipStream_t);             \
    template void launch_zero_faces<T>(T*, const GridView&, int, hipStream_t);               \
    template void launch_faces<T>(T*, const GridView&, const FaceOp<T>*, int, bool, hipStream_t);
W3D_INST(double)
W3D_INST(float)


template <class T>
void launch_box_copy(const BoxCopy<T>* ops, int nops, const GridView& gv, bool to_buf,
                     hipStream_t s) {
    W3D_REQUIRE(nops >= 0 && nops <= kMaxBoxCopy, "too many halo boxes in one launch");
    if (nops == 0) return;
    BoxCopyOps<T> p{};
    p.n = nops;
    unsigned blocks = 0;
    for (int q = 0; q < nops; ++q) {
        const Box& b = ops[q].b;
        W3D_REQUIRE(!b.empty() && b.i0 >= 1 - gv.G && b.i1 <= gv.X + gv.G && b.j0 >= 1 - gv.G &&
                        b.j1 <= gv.Y + gv.G && b.k0 >= 1 - gv.G && b.k1 <= gv.Z + gv.G,
                    "halo box outside the storage");
        p.op[q] = ops[q];
        const i64 n = i64(b.i1 - b.i0 + 1) * (b.j1 - b.j0 + 1) * (b.k1 - b.k0 + 1);
        W3D_REQUIRE(n < (i64(1) << 31), "halo box larger than 2^31 elements");
        p.first[q] = blocks;
        blocks += unsigned(std::min<i64>(2048, (n + kThreads - 1) / kThreads));
    }
    p.first[nops] = blocks;
    hipLaunchKernelGGL(k_box_copy<T>, dim3(blocks), dim3(kThreads), 0, s, p, gv.si, gv.sj, to_buf);
    HIP_OK(hipGetLastError());
}
template void launch_box_copy<double>(const BoxCopy<double>*, int, const GridView&, bool, hipStream_t);
template void launch_box_copy<float>(const BoxCopy<float>*, int, const GridView&, bool, hipStream_t);

}  // namespace wave3d
