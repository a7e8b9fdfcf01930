// Temporal blocking on CDNA4: two leapfrog layers per sweep (SURVEY §2.2 "absent in the
// reference"; the lever that moves the solver past the single-step HBM roofline).
//
// HBM traffic per node and layer: single-step reads u^{n-1}, u^{n-2} and writes u^n
// (24 B fp64). One sweep here reads A = u^{m-1}, B = u^{m-2} and writes C = u^m and
// D = u^{m+1}: 32 B per two layers = 16 B per layer.
//
// Workgroup = 4 wave64s owning a (4R rows) x 64 tile of D that marches along i. Per plane i:
//   1. the A(i) tile plus a 2-node ring goes to LDS (own values from registers, ring from
//      L2), one barrier;
//   2. C(i) is computed on the tile plus a 1-node ring (redundantly with the neighbour
//      tiles — every node is evaluated with exactly the same operations, so bitwise equal)
//      and written to a second LDS tile; own-node C values stay in registers;
//   3. D(i-1) is computed from the C(i-1) tile written one iteration earlier (no second
//      barrier: both tiles are double-buffered) and the register-resident C(i-2), C(i).
// The i-prologue of every work item recomputes C on one extra plane (ib-1) and the last
// iteration evaluates C(ie+1); the chunk length amortises that.
//
// Ghost depth 2 for A (C on the ring needs A two nodes out), 1 for B. On a periodic seam the
// ghost copy of global plane N-1 must see plane x=N (not x=0) as its x+ neighbour, because
// the reference keeps both planes (mpi_new.cpp:170-176): SeamAlias supplies that plane.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "device_common.hpp"

namespace wave3d {
namespace {

template <class T>
struct TbParams {
    const T* A;
    const T* B;
    T* C;
    T* D;
    i64 si;
    int sj;
    int poff;                    // see GridView::poff
    int jmin, jmax, kmin, kmax;  // storage bounds (logical)
    int cj0, cj1, ck0, ck1;      // C is a stencil value inside, 0 (Dirichlet face) outside
    int nbox;
    BoxLaunch box[kMaxBoxes];
    int ei0, ei1;
    int wc_src[kMaxWrap], wc_dst[kMaxWrap];
    int wd_src[kMaxWrap], wd_dst[kMaxWrap];
    int an_i, ap_i;
    const T* an;
    const T* ap;
    const T* tx;
    const T* ty;
    const T* tz;
    T hx2, hy2, hz2, coefC, coefD, ctC, ctD;
    T yx2, yy2, yz2;  // RN(1/h^2): correctly rounded constant division
    u64* errC;
    u64* errD;
};

template <class T, bool FIRST, int R>
__global__ void __launch_bounds__(kThreads) k_tb2(const TbParams<T> p) {
    constexpr int TJ = kWaves * R;
    constexpr int AH = TJ + 4, AW = kTK + 4;  // A tile: rows jt-2..jt+TJ+1, cols kb-2..kb+65
    constexpr int CH = TJ + 2, CW = kTK + 2;  // C tile: rows jt-1..jt+TJ,   cols kb-1..kb+64
    constexpr unsigned ES = sizeof(T);
    __shared__ T ldsA[2][AH][AW];
    __shared__ T ldsC[2][CH][CW];

    const int bid = blockIdx.x;
    const int b = find_box(p, bid);
    const BoxLaunch Bx = p.box[b];
    int local = bid - Bx.block_begin;
    const int tk = local % Bx.tiles_k;
    local /= Bx.tiles_k;
    const int tj = local % Bx.tiles_j;
    const int ci = local / Bx.tiles_j;
    const int kb = Bx.kbase + tk * kTK;
    const int jt = Bx.j0 + tj * TJ;
    const int ib = Bx.i0 + ci * Bx.chunk;
    const int ie = min(Bx.i1, ib + Bx.chunk - 1);
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const i64 si = p.si;
    const int sj = p.sj;
    const unsigned pbytes = unsigned(si) * ES;

    auto inb = [&](int j, int k) { return j >= p.jmin && j <= p.jmax && k >= p.kmin && k <= p.kmax; };
    auto incd = [&](int j, int k) { return j >= p.cj0 && j <= p.cj1 && k >= p.ck0 && k <= p.ck1; };
    // byte offset of (j,k) inside a plane block, or kOOB
    auto boff = [&](int j, int k, bool ok) { return ok ? unsigned(j * sj + k + p.poff) * ES : kOOB; };
    // descriptor of logical plane i of an array (wave-uniform)
    auto prs = [&](const T* base, int i) { return plane_rsrc(base + (i64(i) * si - p.poff), pbytes); };

    // ---- own nodes (D and C) ----------------------------------------------------------
    const int k = kb + lane;
    unsigned oa[R], ob[R], os[R];  // A-load, B-load, store offsets (kOOB when masked)
    bool ovalid[R], ocd[R];
    T oty[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = jt + w * R + r;
        ocd[r] = incd(j, k);
        ovalid[r] = k >= Bx.k0 && k <= Bx.k1 && j <= Bx.j1;
        oa[r] = boff(j, k, inb(j, k));
        ob[r] = boff(j, k, !FIRST && inb(j, k) && ocd[r]);
        os[r] = boff(j, k, ovalid[r]);
        oty[r] = ovalid[r] ? p.ty[j] : T(0);
    }
    const T otz = (k >= Bx.k0 && k <= Bx.k1) ? p.tz[k] : T(0);

    // ---- C-ring node of this thread (rolling A, C into the LDS tile only) --------------
    // rows jt-1 / jt+TJ over cols kb..kb+63, then cols kb-1 / kb+64 over rows jt-1..jt+TJ
    int rj = 0, rk = 0;
    bool ron = false;
    {
        const int q = threadIdx.x;
        if (q < 64) rj = jt - 1, rk = kb + q, ron = true;
        else if (q < 128) rj = jt + TJ, rk = kb + q - 64, ron = true;
        else if (q < 128 + CH) rj = jt - 1 + (q - 128), rk = kb - 1, ron = true;
        else if (q < 128 + 2 * CH) rj = jt - 1 + (q - 128 - CH), rk = kb + kTK, ron = true;
    }
    const bool rcd = ron && incd(rj, rk);
    const unsigned ra_off = boff(rj, rk, ron && inb(rj, rk));
    const unsigned rb_off = boff(rj, rk, !FIRST && ron && inb(rj, rk) && rcd);

    // ---- outer A-ring node (LDS only) ---------------------------------------------------
    int uj = 0, uk = 0;
    bool uon = false;
    {
        const int q = threadIdx.x;
        if (q < 66) uj = jt - 2, uk = kb - 1 + q, uon = true;
        else if (q < 132) uj = jt + TJ + 1, uk = kb - 1 + (q - 66), uon = true;
        else if (q < 132 + CH) uj = jt - 1 + (q - 132), uk = kb - 2, uon = true;
        else if (q < 132 + 2 * CH) uj = jt - 1 + (q - 132 - CH), uk = kb + kTK + 1, uon = true;
    }
    const unsigned ua_off = boff(uj, uk, uon && inb(uj, uk));

    // rolling registers: own A at i-1, i, i+1 (+ i+2 in flight), C at i-2..i; B per plane
    T aP[R], aC[R], aN[R], c2[R], c1[R], c0[R];
    {
        const auto r0 = prs(p.A, ib - 2), r1 = prs(p.A, ib - 1), r2 = prs(p.A, ib);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            aP[r] = bld<T>(r0, oa[r]);
            aC[r] = bld<T>(r1, oa[r]);
            aN[r] = bld<T>(r2, oa[r]);
            c2[r] = c1[r] = c0[r] = T(0);
        }
    }
    T raP = bld<T>(prs(p.A, ib - 2), ra_off);
    T raC = bld<T>(prs(p.A, ib - 1), ra_off);
    T raN = bld<T>(prs(p.A, ib), ra_off);
    T ua = bld<T>(prs(p.A, ib - 1), ua_off);

    T ma1 = T(kErrInit), mr1 = T(kErrInit), ma2 = T(kErrInit), mr2 = T(kErrInit);
    bool bad1 = false, bad2 = false;
    int buf = 0;

    for (int i = ib - 1; i <= ie + 1; ++i) {
        // prefetch A(i+2) (own, ring) and A(i+1) (outer); B(i) now, used after the barrier
        const bool more = i <= ie;
        const auto rA2 = prs(p.A, more ? i + 2 : i);
        const auto rA1 = prs(p.A, more ? i + 1 : i);
        const auto rB = prs(p.B, i);
        T aNN[R], bC[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            aNN[r] = bld<T>(rA2, more ? oa[r] : kOOB);
            bC[r] = bld<T>(rB, ob[r]);
        }
        const T raNN = bld<T>(rA2, more ? ra_off : kOOB);
        const T rbC = bld<T>(rB, rb_off);
        const T uaN = bld<T>(rA1, more ? ua_off : kOOB);

        // 1. stage A(i)
#pragma unroll
        for (int r = 0; r < R; ++r) ldsA[buf][2 + w * R + r][2 + lane] = aC[r];
        if (ron) ldsA[buf][rj - jt + 2][rk - kb + 2] = raC;
        if (uon) ldsA[buf][uj - jt + 2][uk - kb + 2] = ua;
        __syncthreads();

        // seam aliases (uniform): x+ / x- neighbour of C(i) from another plane
        const bool use_an = i == p.an_i, use_ap = i == p.ap_i;
        T xnA[R], xpA[R], rxn = raN, rxp = raP;
#pragma unroll
        for (int r = 0; r < R; ++r) xnA[r] = aN[r], xpA[r] = aP[r];
        if (use_an) {
            const auto ra = plane_rsrc(p.an - p.poff, pbytes);
#pragma unroll
            for (int r = 0; r < R; ++r) xnA[r] = bld<T>(ra, oa[r]);
            rxn = bld<T>(ra, ra_off);
        }
        if (use_ap) {
            const auto ra = plane_rsrc(p.ap - p.poff, pbytes);
#pragma unroll
            for (int r = 0; r < R; ++r) xpA[r] = bld<T>(ra, oa[r]);
            rxp = bld<T>(ra, ra_off);
        }

        // 2. C(i) on own nodes and the ring (0 on Dirichlet faces)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int ra = 2 + w * R + r, ca = 2 + lane;
            const T lap = laplace7_cr(aC[r], xpA[r], xnA[r], ldsA[buf][ra - 1][ca], ldsA[buf][ra + 1][ca],
                                      ldsA[buf][ra][ca - 1], ldsA[buf][ra][ca + 1], p.hx2, p.hy2,
                                      p.hz2, p.yx2, p.yy2, p.yz2);
            const T cv = FIRST ? taylor_first(aC[r], lap, p.coefC) : leapfrog(aC[r], bC[r], lap, p.coefC);
            c0[r] = ocd[r] ? cv : T(0);
            ldsC[buf][1 + w * R + r][1 + lane] = c0[r];
        }
        if (ron) {
            const int ra = rj - jt + 2, ca = rk - kb + 2;
            const T lap = laplace7_cr(raC, rxp, rxn, ldsA[buf][ra - 1][ca], ldsA[buf][ra + 1][ca],
                                      ldsA[buf][ra][ca - 1], ldsA[buf][ra][ca + 1], p.hx2, p.hy2,
                                      p.hz2, p.yx2, p.yy2, p.yz2);
            const T cv = FIRST ? taylor_first(raC, lap, p.coefC) : leapfrog(raC, rbC, lap, p.coefC);
            ldsC[buf][ra - 1][ca - 1] = rcd ? cv : T(0);
        }

        // own C(i): store, wrap, error (only the work item's own planes)
        if (i >= ib && i <= ie) {
            const bool erow = i >= p.ei0 && i <= p.ei1;
            const T sx = p.tx[i];
            const auto rc = prs(p.C, i);
#pragma unroll
            for (int r = 0; r < R; ++r) bst(c0[r], rc, os[r]);
#pragma unroll
            for (int q = 0; q < kMaxWrap; ++q)
                if (i == p.wc_src[q]) {
                    const auto rw = prs(p.C, p.wc_dst[q]);
#pragma unroll
                    for (int r = 0; r < R; ++r) bst(c0[r], rw, os[r]);
                }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (!ovalid[r]) continue;
                bad1 |= nonfinite(c0[r]);
                if (erow) accumulate_error(c0[r], analytic(sx, oty[r], otz, p.ctC), ma1, mr1);
            }
        }

        // 3. D(i-1) from the C(i-1) tile (written last iteration, other buffer)
        const int id = i - 1;
        if (id >= ib && id <= ie) {
            const bool erow = id >= p.ei0 && id <= p.ei1;
            const T sx = p.tx[id];
            const int pb = buf ^ 1;
            T dv[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int rc = 1 + w * R + r, cc = 1 + lane;
                const T lap = laplace7_cr(c1[r], c2[r], c0[r], ldsC[pb][rc - 1][cc], ldsC[pb][rc + 1][cc],
                                          ldsC[pb][rc][cc - 1], ldsC[pb][rc][cc + 1], p.hx2, p.hy2,
                                          p.hz2, p.yx2, p.yy2, p.yz2);
                dv[r] = leapfrog(c1[r], aP[r], lap, p.coefD);
            }
            const auto rd = prs(p.D, id);
#pragma unroll
            for (int r = 0; r < R; ++r) bst(dv[r], rd, os[r]);
#pragma unroll
            for (int q = 0; q < kMaxWrap; ++q)
                if (id == p.wd_src[q]) {
                    const auto rw = prs(p.D, p.wd_dst[q]);
#pragma unroll
                    for (int r = 0; r < R; ++r) bst(dv[r], rw, os[r]);
                }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (!ovalid[r]) continue;
                bad2 |= nonfinite(dv[r]);
                if (erow) accumulate_error(dv[r], analytic(sx, oty[r], otz, p.ctD), ma2, mr2);
            }
        }

        // roll
#pragma unroll
        for (int r = 0; r < R; ++r) {
            aP[r] = aC[r];
            aC[r] = aN[r];
            aN[r] = aNN[r];
            c2[r] = c1[r];
            c1[r] = c0[r];
        }
        raP = raC;
        raC = raN;
        raN = raNN;
        ua = uaN;
        buf ^= 1;
    }
    commit_errors(ma1, mr1, bad1, p.errC);
    __syncthreads();
    commit_errors(ma2, mr2, bad2, p.errD);
}

}  // namespace

template <class T>
void launch_tb2(int rows, bool first, const T* A, const T* B, T* C, T* D, const GridView& gv,
                const Box* boxes, int nbox, const Box& cdom, int ei0, int ei1, const Wrap& wrapC,
                const Wrap& wrapD, const SeamAlias<T>& alias, const T* tx, const T* ty,
                const T* tz, const StepCoefs& cC, const StepCoefs& cD, u64* errC, u64* errD,
                int chunk, hipStream_t s) {
    W3D_REQUIRE(gv.G >= 2, "temporal blocking needs ghost depth >= 2");
    W3D_REQUIRE(rows == 2 || rows == 4 || rows == 8, "tb2 rows per lane must be 2, 4 or 8");
    W3D_REQUIRE(nbox >= 1 && nbox <= kMaxBoxes, "bad box count");
    TbParams<T> p{};
    p.A = A;
    p.B = B;
    p.C = C;
    p.D = D;
    p.si = gv.si;
    p.sj = gv.sj;
    p.poff = gv.poff;
    p.jmin = 1 - gv.G;
    p.jmax = gv.jmax();
    p.kmin = 1 - gv.G;
    p.kmax = gv.kmax();
    p.cj0 = cdom.j0;
    p.cj1 = cdom.j1;
    p.ck0 = cdom.k0;
    p.ck1 = cdom.k1;
    p.ei0 = ei0;
    p.ei1 = ei1;
    for (int q = 0; q < kMaxWrap; ++q) {
        p.wc_src[q] = wrapC.src[q], p.wc_dst[q] = wrapC.dst[q];
        p.wd_src[q] = wrapD.src[q], p.wd_dst[q] = wrapD.dst[q];
    }
    p.an_i = alias.next ? alias.next_i : INT_MIN;
    p.ap_i = alias.prev ? alias.prev_i : INT_MIN;
    p.an = alias.next;
    p.ap = alias.prev;
    p.tx = tx;
    p.ty = ty;
    p.tz = tz;
    p.hx2 = T(cC.hx2);
    p.hy2 = T(cC.hy2);
    p.hz2 = T(cC.hz2);
    p.yx2 = T(1) / T(cC.hx2);
    p.yy2 = T(1) / T(cC.hy2);
    p.yz2 = T(1) / T(cC.hz2);
    p.coefC = T(cC.coef);
    p.coefD = T(cD.coef);
    p.ctC = T(cC.ct);
    p.ctD = T(cD.ct);
    p.errC = errC;
    p.errD = errD;
    const int TJ = kWaves * rows;
    int nb = 0, total = 0;
    for (int q = 0; q < nbox; ++q) {
        const Box& bx = boxes[q];
        if (bx.empty()) continue;
        W3D_REQUIRE(bx.i0 >= 1 && bx.i1 <= gv.X && bx.j0 >= 1 && bx.j1 <= gv.Y && bx.k0 >= 1 &&
                        bx.k1 <= gv.Z,
                    "sweep box outside the owned region");
        BoxLaunch& L = p.box[nb];
        L.i0 = bx.i0, L.i1 = bx.i1, L.j0 = bx.j0, L.j1 = bx.j1, L.k0 = bx.k0, L.k1 = bx.k1;
        const int t0 = (bx.k0 - 1) / kTK, t1 = (bx.k1 - 1) / kTK;
        L.kbase = 1 + t0 * kTK;
        L.tiles_k = t1 - t0 + 1;
        L.tiles_j = cdiv(bx.j1 - bx.j0 + 1, TJ);
        const int planes = bx.i1 - bx.i0 + 1;
        L.chunk = std::min(chunk > 0 ? chunk : 32, planes);
        L.block_begin = total;
        total += L.tiles_k * L.tiles_j * cdiv(planes, L.chunk);
        ++nb;
    }
    p.nbox = nb;
    if (nb == 0) return;
    void (*kern)(const TbParams<T>);
    if (rows == 2) kern = first ? k_tb2<T, true, 2> : k_tb2<T, false, 2>;
    else if (rows == 8) kern = first ? k_tb2<T, true, 8> : k_tb2<T, false, 8>;
    else kern = first ? k_tb2<T, true, 4> : k_tb2<T, false, 4>;
    hipLaunchKernelGGL(kern, dim3(total), dim3(kThreads), 0, s, p);
    HIP_OK(hipGetLastError());
}

#define W3D_TB_INST(T)                                                                       \
    template void launch_tb2<T>(int, bool, const T*, const T*, T*, T*, const GridView&,      \
                                const Box*, int, const Box&, int, int, const Wrap&,          \
                                const Wrap&, const SeamAlias<T>&, const T*, const T*,        \
                                const T*, const StepCoefs&, const StepCoefs&, u64*, u64*,    \
                                int, hipStream_t);
W3D_TB_INST(double)
W3D_TB_INST(float)

}  // namespace wave3d
