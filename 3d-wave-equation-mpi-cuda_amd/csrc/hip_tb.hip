// Temporal blocking on CDNA4: two leapfrog layers per sweep (SURVEY §2.2 "absent in the
// reference"; the lever that moves the solver past the single-step HBM roofline).
//
// HBM traffic per node and layer: single-step reads u^{n-1}, u^{n-2} and writes u^n
// (24 B fp64). One sweep here reads A = u^{m-1}, B = u^{m-2} and writes C = u^m and
// D = u^{m+1}: 32 B per two layers = 16 B per layer.
//
// Workgroup = NW wave64s owning a (NW*R rows) x 64 tile of D that marches along i. Per plane i:
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
#include <cstdlib>
#include <climits>
#include <cmath>
#include <type_traits>

#include "device_common.hpp"

namespace wave3d {
namespace {

template <class T>
struct TbParams {
    int xcd;     // XCD-aware tile order (xcd_swizzle)
    int order;   // tile order (tile_order(): 0 k-fastest, 1 j-fastest, 2 XCD bands)
    // Level bases pre-biased on the host so that plane i's block starts at
    // base + (i + pbias) * pbytes with i + pbias >= 0: one 32x32->64-bit product per descriptor
    // instead of a signed 64-bit plane-index multiply (~half the scalar instructions per plane).
    const char* A;
    const char* B;
    char* C;
    char* D;
    unsigned pbytes;  // plane bytes (< 4 GiB: one buffer descriptor per plane)
    int pbias;
    int sj;
    int poff;                    // see GridView::poff
    int jmin, jmax, kmin, kmax;  // storage bounds (logical)
    int cj0, cj1, ck0, ck1;      // C is a stencil value inside, 0 (Dirichlet face) outside
    int nbox;
    BoxLaunch box[kMaxBoxes];
    int ei0, ei1;
    // periodic self-wrap as <= 2 plane ranges with a constant shift: plane i in [lo, hi] is
    // also stored to plane i + sh (fewer live scalars than a per-plane table)
    int wc_lo[2], wc_hi[2], wc_sh[2];
    int wd_lo[2], wd_hi[2], wd_sh[2];
    int an_i, ap_i;
    const T* an;  // seam alias planes, block starts (logical (i,0,0) - poff)
    const T* ap;
    // txy[i * tpj + j] = RN(tx[i] * ty[j]) (launch_txy): the analytic value
    // ((sx*sy)*sz)*ct is then two multiplies per node with the reference's rounding
    const T* txy;
    int tpj;
    const T* tz;
    const T* txr;   // --math fma: (sx sy, 1/|sx sy|) pairs (launch_txr) and 1/|tz|
    const T* rtz;
    T ict[2];       // --math fma: 1/|ct| of layers C, D
    T hx2, hy2, hz2, coefC, coefD, ctC, ctD;
    T yx2, yy2, yz2;  // RN(1/h^2): correctly rounded constant division
    T fc[2][3];       // --math fma: coef/h^2 of layers C, D per axis
    u64* errC;
    u64* errD;
};

// Rolling state lives in fixed slots indexed by plane number mod 4 (A, C) or mod 2 (B, outer
// ring, LDS buffers) and the i loop is unrolled by 4 with the phase as a compile-time
// constant, so no value ever moves between registers: a prefetch load lands in the slot it
// is consumed from two planes later, and the compiler needs no s_waitcnt vmcnt(0) to copy
// an in-flight register (the rotate-by-copy form serialised every plane on load latency).
// C and D are written with the non-temporal policy (+3-5 % at N=512,
// profiles/sweep_store_policy_r1.txt; the error-reduction ablations of round 1 are in
// profiles/sweep_n512_tb_variants_r1.txt). (Prefetch distances: own A and both A rings 2
// planes, B 1 plane; B at distance 2 measured no faster, the outer ring at distance 2 +2.6 %.)
// DELTA: increment form (csrc/hip_kernels.hpp launch_tb2): B = d^{m-1}; d^m = B + coefC*lap A,
// C = A + d^m (registers: errors, D's stencil); d^{m+1} = d^m + coefD*lap C, D = C + d^{m+1};
// the C level receives d^{m+1} at D's planes, so the store count is unchanged.
// NWK: waves side by side along k — the tile is (NW/NWK)*R rows x 64*NWK columns. Wider tiles
// halve the k-side halo lines per own line (each row's halo columns kb-2..kb-1 and
// kb+TK..kb+TK+1 sit in two 128-B lines owned by the k-neighbour tile, which runs on another
// XCD, so they are fetched again from beyond L2 — the bulk of tb2's read surplus,
// profiles/dram_bytes_r2.txt).
// FM: --math fma (stencil_math coef_lap_fma), as k_tb3.
template <class T, bool FIRST, int R, int NW, int WPE = 1, bool DELTA = false,
          int NWK = 1, bool FM = false>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(WPE, 8))) k_tb2(const TbParams<T> p) {
    static_assert(NW % NWK == 0, "waves along k must divide the workgroup");
    constexpr int NWJ = NW / NWK;
    constexpr int TK = kTK * NWK;             // tile columns
    constexpr int TJ = NWJ * R;               // tile rows
    constexpr int AH = TJ + 4, AW = TK + 4;   // A tile: rows jt-2..jt+TJ+1, cols kb-2..kb+TK+1
    constexpr int CH = TJ + 2, CW = TK + 2;   // C tile: rows jt-1..jt+TJ,   cols kb-1..kb+TK
    constexpr unsigned ES = sizeof(T);
    constexpr int kStAux = 2;  // store cache policy: non-temporal
    static_assert(2 * TK + 2 * CH <= NW * 64 && 2 * (TK + 2) + 2 * CH <= NW * 64, "ring needs more lanes");
    __shared__ T ldsA[2][AH][AW];
    __shared__ T ldsC[2][CH][CW];

    const int bid = xcd_swizzle(blockIdx.x, gridDim.x, p.xcd);
    const int b = find_box(p, bid);
    const BoxLaunch Bx = p.box[b];
    int local = bid - Bx.block_begin;
    int tk, tj;
    if (p.order == 2 && Bx.tiles_j % kXcds == 0) {
        // block ids dealt round-robin over the XCDs: x = id mod 8 runs tile rows
        // [x*hb, x*hb + hb) of every k-tile and chunk, j-fastest inside its band
        const int hb = Bx.tiles_j / kXcds, x = local % kXcds;
        local /= kXcds;
        tj = x * hb + local % hb;
        local /= hb;
        tk = local % Bx.tiles_k;
        local /= Bx.tiles_k;
    } else if (p.order) {
        tj = local % Bx.tiles_j;
        local /= Bx.tiles_j;
        tk = local % Bx.tiles_k;
        local /= Bx.tiles_k;
    } else {
        tk = local % Bx.tiles_k;
        local /= Bx.tiles_k;
        tj = local % Bx.tiles_j;
        local /= Bx.tiles_j;
    }
    const int ci = local;
    const int kb = Bx.kbase + tk * TK;
    const int jt = Bx.j0 + tj * TJ;
    const int ib = Bx.i0 + ci * Bx.chunk;
    const int ie = min(Bx.i1, ib + Bx.chunk - 1);
    const int lane = threadIdx.x & 63;
    const int w8 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int w = w8 % NWJ;                 // wave's row band
    const int kl = (w8 / NWJ) * kTK + lane;  // column within the tile
    const int sj = p.sj;
    const unsigned pbytes = p.pbytes;

    auto inb = [&](int j, int k) { return j >= p.jmin && j <= p.jmax && k >= p.kmin && k <= p.kmax; };
    auto incd = [&](int j, int k) { return j >= p.cj0 && j <= p.cj1 && k >= p.ck0 && k <= p.ck1; };
    // byte offset of (j,k) inside a plane block, or kOOB
    auto boff = [&](int j, int k, bool ok) { return ok ? unsigned(j * sj + k + p.poff) * ES : kOOB; };
    // descriptor of logical plane i of a level (wave-uniform; `nb` bytes: 0 = loads return 0)
    auto prs = [&](const char* base, int i, unsigned nb) {
        return plane_rsrc(base + u64(unsigned(i + p.pbias)) * pbytes, nb);
    };

    // ---- own nodes (D and C) ----------------------------------------------------------
    const int k = kb + kl;
    const int jrow = jt + w * R;  // first row of this wave (wave-uniform)
    unsigned oa[R], ob[R], os[R];  // A-load, B-load, store offsets (kOOB when masked)
    bool ovalid[R], ocd[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = jrow + r;
        ocd[r] = incd(j, k);
        ovalid[r] = k >= Bx.k0 && k <= Bx.k1 && j <= Bx.j1;
        oa[r] = boff(j, k, inb(j, k));
        ob[r] = boff(j, k, !FIRST && inb(j, k) && ocd[r]);
        os[r] = boff(j, k, ovalid[r]);
    }
    const T otz = (k >= Bx.k0 && k <= Bx.k1) ? p.tz[k] : T(0);
    const T ortz = FM && k >= Bx.k0 && k <= Bx.k1 ? p.rtz[k] : T(0);
    // rows of this wave in the sx*sy table (launch_txy pads past the last row, so rows beyond
    // the box — never used, their lanes are masked — are in-bounds reads)
    const T* const txw = p.txy + jrow;
    T om[R];  // --math fma: 1 on valid own nodes, 0 on masked lanes (branch-free errors)
#pragma unroll
    for (int r = 0; r < R; ++r) om[r] = ovalid[r] ? T(1) : T(0);

    // Rare per-plane events of this work item as wave-uniform bits, so the common plane pays
    // one scalar test for all of them: C / D self-wrap ranges met (1, 2 / 4, 8), seam alias
    // plane met (16). Own planes [ib, ie]: C stored at i, D at i - 1.
    int rare = 0;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        if (p.wc_lo[g] <= ie && p.wc_hi[g] >= ib) rare |= 1 << g;
        if (p.wd_lo[g] <= ie && p.wd_hi[g] >= ib) rare |= 4 << g;
    }
    if ((p.an_i >= ib - 1 && p.an_i <= ie + 1) || (p.ap_i >= ib - 1 && p.ap_i <= ie + 1)) rare |= 16;
    rare = __builtin_amdgcn_readfirstlane(rare);
    // error planes of this work item: [e0, e0 + espan] (none: e0 far below every plane)
    const int e0r = max(ib, p.ei0), e1r = min(ie, p.ei1);
    const int e0 = e1r >= e0r ? e0r : INT_MIN / 2;
    const unsigned espan = e1r >= e0r ? unsigned(e1r - e0r) : 0u;
    const unsigned ospan = unsigned(ie - ib);
    auto own = [&](int i) { return unsigned(i - ib) <= ospan; };
    auto eplane = [&](int i) { return unsigned(i - e0) <= espan; };

    // ---- C-ring node of this thread (rolling A, C into the LDS tile only) --------------
    // rows jt-1 / jt+TJ over cols kb..kb+TK-1, then cols kb-1 / kb+TK over rows jt-1..jt+TJ
    int rj = 0, rk = 0;
    bool ron = false;
    {
        const int q = threadIdx.x;
        if (q < TK) rj = jt - 1, rk = kb + q, ron = true;
        else if (q < 2 * TK) rj = jt + TJ, rk = kb + q - TK, ron = true;
        else if (q < 2 * TK + CH) rj = jt - 1 + (q - 2 * TK), rk = kb - 1, ron = true;
        else if (q < 2 * TK + 2 * CH) rj = jt - 1 + (q - 2 * TK - CH), rk = kb + TK, ron = true;
    }
    const bool rcd = ron && incd(rj, rk);
    const unsigned ra_off = boff(rj, rk, ron && inb(rj, rk));
    const unsigned rb_off = boff(rj, rk, !FIRST && ron && inb(rj, rk) && rcd);

    // ---- outer A-ring node (LDS only) ---------------------------------------------------
    int uj = 0, uk = 0;
    bool uon = false;
    {
        const int q = threadIdx.x;
        constexpr int RW = TK + 2;  // outer ring rows jt-2 / jt+TJ+1: cols kb-1..kb+TK
        if (q < RW) uj = jt - 2, uk = kb - 1 + q, uon = true;
        else if (q < 2 * RW) uj = jt + TJ + 1, uk = kb - 1 + (q - RW), uon = true;
        else if (q < 2 * RW + CH) uj = jt - 1 + (q - 2 * RW), uk = kb - 2, uon = true;
        else if (q < 2 * RW + 2 * CH) uj = jt - 1 + (q - 2 * RW - CH), uk = kb + TK + 1, uon = true;
    }
    const unsigned ua_off = boff(uj, uk, uon && inb(uj, uk));

    // Slots (iteration i = ib - 1 + q, phase P = q & 3):
    //   A(x), ring A(x), outer A(x): slot (x - ib + 2) & 3 -> A(i-1) = P, A(i) = P+1,
    //                                 A(i+1) = P+2, A(i+2) = P+3
    //   C(x):            slot (x - ib + 1) & 3 -> C(i) = P, C(i-1) = P+3, C(i-2) = P+2
    //   B(x), ring B(x), LDS buffer: (x - ib + 1) & 1
    T a[4][R], c[4][R], bb[2][R];
    T dl[DELTA ? 2 : 1][R];  // increment form: d^m of planes i (H0) and i-1 (H1)
    T ra[4], rb[2], ua[4];
    {
        const auto r0 = prs(p.A, ib - 2, pbytes), r1 = prs(p.A, ib - 1, pbytes), r2 = prs(p.A, ib, pbytes);
        const auto rB = prs(p.B, ib - 1, pbytes);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            a[0][r] = bld<T>(r0, oa[r]);
            a[1][r] = bld<T>(r1, oa[r]);
            a[2][r] = bld<T>(r2, oa[r]);
            a[3][r] = T(0);
            bb[0][r] = bld<T>(rB, ob[r]);
            bb[1][r] = T(0);
#pragma unroll
            for (int q = 0; q < 4; ++q) c[q][r] = T(0);
        }
        ra[0] = bld<T>(r0, ra_off);
        ra[1] = bld<T>(r1, ra_off);
        ra[2] = bld<T>(r2, ra_off);
        ra[3] = T(0);
        rb[0] = bld<T>(rB, rb_off);
        rb[1] = T(0);
        ua[0] = ua[3] = T(0);
        ua[1] = bld<T>(r1, ua_off);
        ua[2] = bld<T>(r2, ua_off);
    }

    T ma1 = T(kErrInit), ma2 = T(kErrInit);
    using Rel = std::conditional_t<FM, RelMax<T>, RelArg<T>>;  // fma: |d| * 1/|f| max
    Rel mr1, mr2;
    T chk1 = T(0), chk2 = T(0);

    // layer L (0 = C, 1 = D) arithmetic: exact Laplacian or (FM) coef*Laplacian, and the updates
    // FM: lap() defers the stencil (FmLap): the leapfrog takes it whole (stencil_math leap_fm),
    // the Taylor start and the increment form take coef*lap
    const T kc1 = FM ? fm_kc(p.fc[1][0], p.fc[1][1], p.fc[1][2]) : T(0);
    auto lap = [&](int L, T ctr, T xm, T xp, T ym, T yp, T zm, T zp) {
        if constexpr (FM) {  // fc[0] == fc[1] unless C is the Taylor first layer
            const int f = FIRST && L == 0 ? 0 : 1;
            return FmLap<T>{ctr, xm, xp, ym, yp, zm, zp, p.fc[f][0], p.fc[f][1], p.fc[f][2]};
        }
        else
            return laplace7_cr(ctr, xm, xp, ym, yp, zm, zp, p.hx2, p.hy2, p.hz2, p.yx2, p.yy2, p.yz2);
    };
    auto leap = [&](int L, T ctr, T u2, const auto& l) {
        if constexpr (FM) return l.leap(u2, kc1);
        else return leapfrog(ctr, u2, l, L == 0 ? p.coefC : p.coefD);
    };
    auto first1 = [&](T ctr, const auto& l) {
        if constexpr (FM) return ctr + lap_value(l);
        else return taylor_first(ctr, l, p.coefC);
    };
    auto incr = [&](int L, T dprev, const auto& l) {
        if constexpr (FM) return dprev + lap_value(l);
        else return delta_incr(dprev, l, L == 0 ? p.coefC : p.coefD);
    };
    auto scaled = [&](const auto& l) {
        if constexpr (FM) return lap_value(l);
        else return p.coefC * l;
    };

    // errors and finiteness sum of one own plane i of a layer (values v[r]); the uniform plane
    // test outside the per-lane row masks keeps it a scalar branch
    auto errors_exact = [&](const T(&v)[R], const int i, const T ct, T& ma, auto& mr, T& chk) {
        if (eplane(i)) {
            const T* const trow = txw + i * p.tpj;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (!ovalid[r]) continue;
                chk += v[r];
                const T f = (ldconst(trow, r) * otz) * ct;  // = ((sx*sy)*sz)*ct, stencil_math analytic
                accumulate_error_dev(v[r], f, ma, mr);
            }
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (ovalid[r]) chk += v[r];
        }
    };

    // --math fma: branch-free — every own plane, masked lanes and planes outside the error range
    // contribute d = 0 (the multiplier om * em), so no exec-mask branches and no phi copies of the
    // running maxima; one scalar load of the (sx sy, 1/|sx sy|) pair per row (txr table)
    auto errors_fm = [&](const T(&v)[R], const int i, const T ct, T& ma, RelMax<T>& mr, T& chk) {
        const T em = (i >= p.ei0 && i <= p.ei1) ? T(1) : T(0);
        const T* const tr = p.txr + 2 * (i * p.tpj + jrow);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            chk += ovalid[r] ? v[r] : T(0);
            const T f = (ldconst(tr, 2 * r) * otz) * ct;  // = ((sx*sy)*sz)*ct
            const T dv = (v[r] - f) * (om[r] * em);
            ma = max_abs(ma, dv);
            mr.add(dv, ldconst(tr, 2 * r + 1) * ortz);
        }
    };
    auto errors = [&](const T(&v)[R], const int i, const T ct, T& ma, Rel& mr, T& chk) {
        if constexpr (FM) errors_fm(v, i, ct, ma, mr, chk);
        else errors_exact(v, i, ct, ma, mr, chk);
    };
    // prefetch A(i+2) (own, both rings), B(i+1); on the last plane the
    // descriptors get 0 records, so the loads return 0 without touching memory (uniform,
    // no per-lane masking)
    auto prefetch = [&](auto phase, const int i) {
        constexpr int P = decltype(phase)::value;
        constexpr int S3 = (P + 3) & 3, H1 = (P + 1) & 1;
        const bool more = i <= ie;
        const unsigned nb = more ? pbytes : 0u;
        const int d2 = more ? 2 : 0, d1 = more ? 1 : 0;
        const auto rA2 = prs(p.A, i + d2, nb);
        const auto rB1 = prs(p.B, i + d1, nb);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            a[S3][r] = bld<T>(rA2, oa[r]);
            bb[H1][r] = bld<T>(rB1, ob[r]);
        }
        ra[S3] = bld<T>(rA2, ra_off);
        rb[H1] = bld<T>(rB1, rb_off);
        ua[S3] = bld<T>(rA2, ua_off);
    };

    // stage A(i) (own from registers, rings from the prefetch) into LDS buffer (i - ib + 1) & 1
    auto stage = [&](auto phase) {
        constexpr int P = decltype(phase)::value;
        constexpr int S1 = (P + 1) & 3, H0 = P & 1;
#pragma unroll
        for (int r = 0; r < R; ++r) ldsA[H0][2 + w * R + r][2 + kl] = a[S1][r];
        if (ron) ldsA[H0][rj - jt + 2][rk - kb + 2] = ra[S1];
        if (uon) ldsA[H0][uj - jt + 2][uk - kb + 2] = ua[S1];
    };

    // C(i) and D(i-1). ALIAS: this plane is a periodic seam, where C(i)'s x+ / x- neighbour
    // comes from another plane (SeamAlias). A separate instantiation, so the common path
    // never merges a conditionally loaded register (that would force s_waitcnt vmcnt(0)).
    auto compute = [&](auto phase, auto alias, const int i) {
        constexpr int P = decltype(phase)::value;
        constexpr bool ALIAS = decltype(alias)::value;
        constexpr int S0 = P & 3, S1 = (P + 1) & 3, S2 = (P + 2) & 3, S3 = (P + 3) & 3;
        constexpr int H0 = P & 1, H1 = (P + 1) & 1;
        T xnA[R], xpA[R], rxn = ra[S2], rxp = ra[S0];
#pragma unroll
        for (int r = 0; r < R; ++r) xnA[r] = a[S2][r], xpA[r] = a[S0][r];
        if (ALIAS && i == p.an_i) {
            const auto rs = plane_rsrc(p.an, pbytes);
#pragma unroll
            for (int r = 0; r < R; ++r) xnA[r] = bld<T>(rs, oa[r]);
            rxn = bld<T>(rs, ra_off);
        }
        if (ALIAS && i == p.ap_i) {
            const auto rs = plane_rsrc(p.ap, pbytes);
#pragma unroll
            for (int r = 0; r < R; ++r) xpA[r] = bld<T>(rs, oa[r]);
            rxp = bld<T>(rs, ra_off);
        }

        // C(i) on own nodes and the ring (0 on Dirichlet faces)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int ya = 2 + w * R + r, xa = 2 + kl;
            const auto l = lap(0, a[S1][r], xpA[r], xnA[r], ldsA[H0][ya - 1][xa], ldsA[H0][ya + 1][xa],
                            ldsA[H0][ya][xa - 1], ldsA[H0][ya][xa + 1]);
            T cv;
            if constexpr (DELTA) {
                const T dm = FIRST ? scaled(l) : incr(0, bb[H0][r], l);
                dl[H0][r] = ocd[r] ? dm : T(0);
                cv = a[S1][r] + dm;  // FIRST: = taylor_first (u0 + coef_first*lap)
            } else {
                cv = FIRST ? first1(a[S1][r], l) : leap(0, a[S1][r], bb[H0][r], l);
            }
            c[S0][r] = ocd[r] ? cv : T(0);
            ldsC[H0][1 + w * R + r][1 + kl] = c[S0][r];
        }
        if (ron) {
            const int ya = rj - jt + 2, xa = rk - kb + 2;
            const auto l = lap(0, ra[S1], rxp, rxn, ldsA[H0][ya - 1][xa], ldsA[H0][ya + 1][xa],
                            ldsA[H0][ya][xa - 1], ldsA[H0][ya][xa + 1]);
            const T cv = FIRST ? first1(ra[S1], l)
                               : (DELTA ? ra[S1] + incr(0, rb[H0], l) : leap(0, ra[S1], rb[H0], l));
            ldsC[H0][ya - 1][xa - 1] = rcd ? cv : T(0);
        }

        // own C(i): store, wrap, error (only the work item's own planes)
        if (own(i)) {
            if constexpr (!DELTA) {
                const auto rc = prs(p.C, i, pbytes);
#pragma unroll
                for (int r = 0; r < R; ++r) bst<kStAux>(c[S0][r], rc, os[r]);
                if (rare & 3) {
#pragma unroll
                    for (int g = 0; g < 2; ++g)
                        if (i >= p.wc_lo[g] && i <= p.wc_hi[g]) {
                            const auto rw = prs(p.C, i + p.wc_sh[g], pbytes);
#pragma unroll
                            for (int r = 0; r < R; ++r) bst<kStAux>(c[S0][r], rw, os[r]);
                        }
                }
            }
            errors(c[S0], i, p.ctC, ma1, mr1, chk1);
        }

        // D(i-1) from the C(i-1) tile (written last iteration, other buffer)
        const int id = i - 1;
        if (own(id)) {
            T dv[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int yc = 1 + w * R + r, xc = 1 + kl;
                const auto l = lap(1, c[S3][r], c[S2][r], c[S0][r], ldsC[H1][yc - 1][xc], ldsC[H1][yc + 1][xc],
                                ldsC[H1][yc][xc - 1], ldsC[H1][yc][xc + 1]);
                if constexpr (DELTA) {
                    dl[H1][r] = incr(1, dl[H1][r], l);  // d^{m+1}
                    dv[r] = c[S3][r] + dl[H1][r];
                } else {
                    dv[r] = leap(1, c[S3][r], a[S0][r], l);
                }
            }
            const auto rd = prs(p.D, id, pbytes);
#pragma unroll
            for (int r = 0; r < R; ++r) bst<kStAux>(dv[r], rd, os[r]);
            if constexpr (DELTA) {
                const auto rdc = prs(p.C, id, pbytes);
#pragma unroll
                for (int r = 0; r < R; ++r) bst<kStAux>(dl[H1][r], rdc, os[r]);
                if (rare & 3) {
#pragma unroll
                    for (int g = 0; g < 2; ++g)
                        if (id >= p.wc_lo[g] && id <= p.wc_hi[g]) {
                            const auto rw = prs(p.C, id + p.wc_sh[g], pbytes);
#pragma unroll
                            for (int r = 0; r < R; ++r) bst<kStAux>(dl[H1][r], rw, os[r]);
                        }
                }
            }
            if (rare & 12) {
#pragma unroll
                for (int g = 0; g < 2; ++g)
                    if (id >= p.wd_lo[g] && id <= p.wd_hi[g]) {
                        const auto rw = prs(p.D, id + p.wd_sh[g], pbytes);
#pragma unroll
                        for (int r = 0; r < R; ++r) bst<kStAux>(dv[r], rw, os[r]);
                    }
            }
            errors(dv, id, p.ctD, ma2, mr2, chk2);
        }
    };

    auto plane = [&](auto phase, const int i) {
        prefetch(phase, i);
        stage(phase);
        __syncthreads();
        if ((rare & 16) && (i == p.an_i || i == p.ap_i)) compute(phase, std::true_type{}, i);
        else compute(phase, std::false_type{}, i);
    };

    // i = ib-1 .. ie+1 (>= 3 planes), unrolled by 4 so every slot index is a constant
    for (int i = ib - 1;;) {
        plane(Ph<0>{}, i);
        if (++i > ie + 1) break;
        plane(Ph<1>{}, i);
        if (++i > ie + 1) break;
        plane(Ph<2>{}, i);
        if (++i > ie + 1) break;
        plane(Ph<3>{}, i);
        if (++i > ie + 1) break;
    }
    auto rel = [&](const Rel& m, int L) {
        if constexpr (FM) return m.value(p.ict[L]);
        else return m.value();
    };
    commit_errors<T, NW>(ma1, rel(mr1, 0), chk1, p.errC);
    __syncthreads();
    commit_errors<T, NW>(ma2, rel(mr2, 1), chk2, p.errD);
}

}  // namespace

// increment form: the main tile shapes only
template <class T, bool F>
static void (*tb_fma_kernel(int rows, int waves, int nwk, bool delta))(const TbParams<T>) {
    switch (rows * 100 + waves * 10 + nwk + (delta ? 10000 : 0)) {
        case 281: return k_tb2<T, F, 2, 8, 1, false, 1, true>;
        case 241: return k_tb2<T, F, 2, 4, 1, false, 1, true>;
        case 10281: return k_tb2<T, F, 2, 8, 1, true, 1, true>;
        default: return nullptr;
    }
}

bool tb2_fma_supported(int rows, int waves, int nwk, bool delta) {
    return tb_fma_kernel<double, false>(rows, waves, nwk, delta) != nullptr;
}

template <class T, bool F>
static void (*tb_delta_kernel(int rows, int waves, int nwk))(const TbParams<T>) {
    switch (rows * 100 + waves * 10 + nwk) {
        case 241: return k_tb2<T, F, 2, 4, 1, true>;
        case 281: return k_tb2<T, F, 2, 8, 1, true>;
        case 441: return k_tb2<T, F, 4, 4, 1, true>;
        case 282: return k_tb2<T, F, 2, 8, 1, true, 2>;
        default: return nullptr;
    }
}

bool tb2_delta_supported(int rows, int waves, int nwk) {
    return tb_delta_kernel<double, false>(rows, waves, nwk) != nullptr;
}

// rows x waves (x minimum waves per SIMD: register cap for the compiler, 0 = none)
template <class T, bool F>
static void (*tb_kernel(int rows, int waves, int occ, int nwk))(const TbParams<T>) {
    switch (rows * 1000 + waves * 10 + occ + (nwk - 1) * 100000) {
        // 128-column tiles (two waves side by side along k)
        case 102080: return k_tb2<T, F, 2, 8, 1, false, 2>;
        case 102084: return k_tb2<T, F, 2, 8, 4, false, 2>;
        case 104080: return k_tb2<T, F, 4, 8, 1, false, 2>;
        case 102160: return k_tb2<T, F, 2, 16, 1, false, 2>;
        case 2040: return k_tb2<T, F, 2, 4>;
        case 2044: return k_tb2<T, F, 2, 4, 4>;
        case 2045: return k_tb2<T, F, 2, 4, 5>;
        case 4040: return k_tb2<T, F, 4, 4>;
        case 4043: return k_tb2<T, F, 4, 4, 3>;
        case 8040: return k_tb2<T, F, 8, 4>;
        case 2080: return k_tb2<T, F, 2, 8>;
        case 4080: return k_tb2<T, F, 4, 8>;
        case 2160: return k_tb2<T, F, 2, 16>;
        default: return nullptr;
    }
}

bool tb2_supported(int rows, int waves, int occ, int nwk) {
    return tb_kernel<double, false>(rows, waves, occ, nwk) != nullptr;
}

template <class T>
void launch_tb2(int rows, int waves, int occ, int nwk, bool delta, bool fm, bool first, const T* A, const T* B, T* C, T* D, const GridView& gv,
                const Box* boxes, int nbox, const Box& cdom, int ei0, int ei1, const Wrap& wrapC,
                const Wrap& wrapD, const SeamAlias<T>& alias, const T* txy, const T* tz,
                const T* txr, const T* rtz, const StepCoefs& cC, const StepCoefs& cD, u64* errC, u64* errD,
                int chunk, hipStream_t s) {
    W3D_REQUIRE(!fm || (txr && rtz), "tb2 --math fma needs the reciprocal analytic tables");
    W3D_REQUIRE(!fm || first || cC.coef == cD.coef, "tb2 --math fma: the non-first layers must share one coefficient");
    W3D_REQUIRE(gv.G >= 2, "temporal blocking needs ghost depth >= 2");
    W3D_REQUIRE(tb2_supported(rows, waves, occ, nwk), "tb2: unsupported rows x waves x occupancy x k-waves");
    W3D_REQUIRE(!delta || (occ == 0 && tb2_delta_supported(rows, waves, nwk)),
                "tb2 increment form: tiles r2w4, r2w8, r4w4, r2w8k2 only");
    W3D_REQUIRE(!fm || (occ == 0 && tb2_fma_supported(rows, waves, nwk, delta)),
                "tb2 --math fma: tiles r2w8, r2w4 (leapfrog), r2w8 (increment form) only");
    W3D_REQUIRE(nbox >= 1 && nbox <= kMaxBoxes, "bad box count");
    W3D_REQUIRE(gv.si * i64(sizeof(T)) < (i64(1) << 31), "tb2: plane larger than 2 GiB");
    TbParams<T> p{};
    p.xcd = xcd_swizzle_enabled();
    p.order = tile_order();
    // plane indices reach 1 - G (wrap targets) and ib - 2 >= -1
    p.pbytes = unsigned(gv.si * i64(sizeof(T)));
    p.pbias = gv.G + 1;
    auto biased = [&](const T* base) {
        return reinterpret_cast<char*>(reinterpret_cast<uintptr_t>(base - gv.poff) -
                                       uintptr_t(p.pbias) * p.pbytes);
    };
    p.A = biased(A);
    p.B = biased(B);
    p.C = biased(C);
    p.D = biased(D);
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
    wrap_ranges(wrapC, p.wc_lo, p.wc_hi, p.wc_sh);
    wrap_ranges(wrapD, p.wd_lo, p.wd_hi, p.wd_sh);
    p.an_i = alias.next ? alias.next_i : INT_MIN;
    p.ap_i = alias.prev ? alias.prev_i : INT_MIN;
    p.an = alias.next ? alias.next - gv.poff : nullptr;
    p.ap = alias.prev ? alias.prev - gv.poff : nullptr;
    p.txy = txy;
    p.tpj = gv.Y + 2;
    p.tz = tz;
    p.txr = txr, p.rtz = rtz;
    p.ict[0] = T(1 / std::fabs(cC.ct)), p.ict[1] = T(1 / std::fabs(cD.ct));
    p.hx2 = T(cC.hx2);
    p.hy2 = T(cC.hy2);
    p.hz2 = T(cC.hz2);
    p.yx2 = T(1) / T(cC.hx2);
    p.yy2 = T(1) / T(cC.hy2);
    p.yz2 = T(1) / T(cC.hz2);
    p.coefC = T(cC.coef);
    p.coefD = T(cD.coef);
    for (int L = 0; L < 2; ++L) {
        const StepCoefs& c = L ? cD : cC;
        p.fc[L][0] = T(c.coef / c.hx2), p.fc[L][1] = T(c.coef / c.hy2), p.fc[L][2] = T(c.coef / c.hz2);
    }
    p.ctC = T(cC.ct);
    p.ctD = T(cD.ct);
    p.errC = errC;
    p.errD = errD;
    const int TJ = waves / nwk * rows, TK = kTK * nwk;
    int btiles[kMaxBoxes], bplanes[kMaxBoxes], nbt = 0;
    for (int q = 0; q < nbox; ++q) {
        const Box& bx = boxes[q];
        if (bx.empty()) continue;
        btiles[nbt] = ((bx.k1 - 1) / TK - (bx.k0 - 1) / TK + 1) * cdiv(bx.j1 - bx.j0 + 1, TJ) * nwk;
        bplanes[nbt++] = bx.i1 - bx.i0 + 1;
    }
    auto kern = fm ? (first ? tb_fma_kernel<T, true>(rows, waves, nwk, delta) : tb_fma_kernel<T, false>(rows, waves, nwk, delta))
              : delta ? (first ? tb_delta_kernel<T, true>(rows, waves, nwk) : tb_delta_kernel<T, false>(rows, waves, nwk))
                      : (first ? tb_kernel<T, true>(rows, waves, occ, nwk) : tb_kernel<T, false>(rows, waves, occ, nwk));
    // one box: work items by resident-workgroup rounds (as launch_tb3); several: auto_chunk_boxes
    const int achunk = nbt == 1 ? rounds_chunk(bplanes[0], btiles[0] / nwk, 2,
                                               resident_slots(reinterpret_cast<const void*>(kern), waves * 64))
                                : auto_chunk_boxes(96, btiles, bplanes, nbt);
    int nb = 0, total = 0;
    for (int q = 0; q < nbox; ++q) {
        const Box& bx = boxes[q];
        if (bx.empty()) continue;
        W3D_REQUIRE(bx.i0 >= 1 && bx.i1 <= gv.X && bx.j0 >= 1 && bx.j1 <= gv.Y && bx.k0 >= 1 &&
                        bx.k1 <= gv.Z,
                    "sweep box outside the owned region");
        BoxLaunch& L = p.box[nb];
        L.i0 = bx.i0, L.i1 = bx.i1, L.j0 = bx.j0, L.j1 = bx.j1, L.k0 = bx.k0, L.k1 = bx.k1;
        const int t0 = (bx.k0 - 1) / TK, t1 = (bx.k1 - 1) / TK;
        L.kbase = 1 + t0 * TK;
        L.tiles_k = t1 - t0 + 1;
        L.tiles_j = cdiv(bx.j1 - bx.j0 + 1, TJ);
        const int planes = bx.i1 - bx.i0 + 1;
        const int want = std::min(chunk > 0 ? chunk : achunk, planes);
        L.chunk = cdiv(planes, cdiv(planes, want));  // equal work items (no short tail chunk)
        L.block_begin = total;
        total += L.tiles_k * L.tiles_j * cdiv(planes, L.chunk);
        ++nb;
    }
    p.nbox = nb;
    if (nb == 0) return;
    hipLaunchKernelGGL(kern, dim3(total), dim3(waves * 64), 0, s, p);
    HIP_OK(hipGetLastError());
}

#define W3D_TB_INST(T)                                                                       \
    template void launch_tb2<T>(int, int, int, int, bool, bool, bool, const T*, const T*, T*, T*, const GridView&, \
                                const Box*, int, const Box&, int, int, const Wrap&,          \
                                const Wrap&, const SeamAlias<T>&, const T*, const T*,        \
                                const T*, const T*, const StepCoefs&, const StepCoefs&, u64*, u64*, \
                                int, hipStream_t);
W3D_TB_INST(double)
W3D_TB_INST(float)

}  // namespace wave3d
