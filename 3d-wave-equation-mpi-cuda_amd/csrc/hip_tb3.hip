// Temporal blocking, three leapfrog layers per sweep (TB3) on CDNA4.
//
// One sweep reads A = u^{m-1}, B = u^{m-2} and writes only D = u^{m+1} and E = u^{m+2}: the
// middle layer C = u^m lives in registers and LDS (its errors are still reduced). HBM traffic
// is 32 B per node per three layers = 10.7 B per layer, against 16 for two-layer blocking and
// 24 for a single-step kernel.
//
// Workgroup = NW wave64s owning a (NW*R rows) x 64 tile of E that marches along i. Layer l is
// evaluated one plane behind layer l-1, on a (3-l)-node ring around the tile (redundantly with
// the neighbour tiles; identical operations, so bitwise equal):
//   iteration i:  stage A(i) (+ 3-node ring) -> barrier
//                 C(i)   on tile + 2-ring  -> LDS C tile
//                 D(i-1) on tile + 1-ring  from the C tile written last iteration
//                 E(i-2) on tile           from the D tile written last iteration
// Every tile is double-buffered, so one barrier per plane. Register state sits in slots indexed
// by plane number mod 4 / mod 2 with the i loop unrolled by 4 (no copies of in-flight loads).
//
// Periodic seam (the reference keeps both x = 0 and x = N, mpi_new.cpp:170-176): the ghost copy
// of global N-1 sees x = N as its x+ neighbour and the ghost copy of global 1 sees x = 0 as its
// x- neighbour. For C that is an A plane in memory (or an alias buffer received from the
// other end of the x ring); for D it is C at that plane, which the sweep never stores: a
// small kernel (k_seam_c) evaluates C on the two partner planes into a scratch pair before
// the sweep, and the seam planes load it like the A partner (separate, rarely taken
// instantiation of the plane body, so the common path carries no extra registers).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <type_traits>

#include "device_common.hpp"

// The measured winners of round 3-4's A/B switches are built in (profiles/deep_sweeps_r4.txt,
// tb3_mem_ablation_r4.txt): the plane loop split into checked / steady bodies, fp64 face masks
// as products, one __shared__ object per staged tile and buffer, register j-neighbours, odd LDS
// pitches only where they came for free, B one plane ahead, no wave-priority bumps.
namespace wave3d {
namespace {

template <class T>
struct Tb3Params {
    // level bases pre-biased on the host (as in k_tb2): plane i's block starts at
    // base + (i + pbias) * pbytes, one 32x32->64-bit product per descriptor
    const char* A;
    const char* B;
    char* D;
    char* E;
    unsigned pbytes;
    int pbias;
    int order;  // tile order (tile_order(): 0 k-fastest, 1 j-fastest, 2 XCD bands; as k_tb2)
    int sj;
    int poff;
    int jmin, jmax, kmin, kmax;  // storage bounds (logical)
    int cj0, cj1, ck0, ck1;      // stencil-valued region of C/D/E (0 outside: Dirichlet)
    int nbox;
    BoxLaunch box[kMaxBoxes];
    int ei0, ei1;
    int wd_lo[2], wd_hi[2], wd_sh[2];  // self-wrap of D (depth 2) and E (depth 3)
    int we_lo[2], we_hi[2], we_sh[2];
    // seam partners (logical plane pointers): at plane an_i the x+ neighbour of C is nA and
    // the x+ neighbour of D is nC (C at the partner plane); mirrored for ap_i / x-.
    int an_i, ap_i;
    const T *nA, *nC, *pA, *pC;
    // txy[i * tpj + j] = RN(tx[i] * ty[j]) (launch_txy): f = (txy * sz) * ct, two multiplies
    const T* txy;
    int tpj;
    const T* tz;
    const T* txr;   // --math fma: (sx sy, 1/|sx sy|) pairs (launch_txr) and 1/|tz|
    const T* rtz;
    T hx2, hy2, hz2, yx2, yy2, yz2;
    T coefC, coefD, coefE, ctC, ctD, ctE;
    T fc[2][3];  // --math fma: coef/h^2 per axis of layer C (fc[0]) and of layers D, E (fc[1]);
                 // equal unless C is the Taylor first layer (FIRST), so the non-FIRST sweep
                 // keeps one triple in SGPRs
    T ict[3];    // --math fma: 1/|ct| per layer
    u64* errC;
    u64* errD;
    u64* errE;
};

// Ring ownership: each ring node belongs to ONE thread (threads [0, N1) the 1-ring, then the
// 2-ring, then the 3-ring without its corners, which no in-plane 5-point stencil reads), RP
// positions per thread when the rings outnumber the threads. A thread keeps four A slots, two B
// slots and (1-ring) four C slots per position — 10 values instead of the 18 a thread held when
// every thread owned one node of each ring (round 1), which put the fp64 kernel at 191-256 VGPRs.
// WPE: minimum waves per SIMD the register allocation must allow (1-row tiles: 4, i.e. two
// 8-wave or one 16-wave workgroup per CU).
// DELTA: increment form (as k_tb2): B = d^{m-1}; d^m = B + coefC lap A, C = A + d^m;
// d^{m+1} = d^m + coefD lap C, D = C + d^{m+1}; d^{m+2} = d^{m+1} + coefE lap D, E = D + d^{m+2}.
// The D level receives d^{m+2} (the next sweep's B), so the bytes moved are unchanged.
// FM: --math fma (stencil_math coef_lap_fma): the update with coef/h^2 folded, not bitwise with
// the reference CPU programs; fewer VALU operations per node (the fp64 sweep is issue-bound).
template <class T, bool FIRST, int R, int NW, bool DELTA = false, bool FM = false,
          int WPE = (R == 1 || (DELTA && sizeof(T) == 4) ? 4 : 1)>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(WPE, 8))) k_tb3(const Tb3Params<T> p) {
    constexpr int TJ = NW * R;
    constexpr int AH = TJ + 6, AW = kTK + 6;  // A tile origin (jt-3, kb-3)
    constexpr int CH = TJ + 4, CW = kTK + 4;  // C tile origin (jt-2, kb-2)
    constexpr int DH = TJ + 2, DW = kTK + 2;  // D tile origin (jt-1, kb-1)
    constexpr int N1 = 2 * kTK + 2 * (TJ + 2);        // 1-ring positions
    constexpr int N2 = 2 * (kTK + 2) + 2 * (TJ + 4);  // 2-ring positions
    constexpr int N3 = 2 * (kTK + 4) + 2 * (TJ + 4);  // 3-ring positions (A only, no corners)
    constexpr int NT = NW * 64;
    constexpr int RP = (N1 + N2 + N3 + NT - 1) / NT;  // ring positions per thread
    constexpr unsigned ES = sizeof(T);
    // one __shared__ object per staged tile and buffer: distinct objects cannot alias, so the
    // compiler may move a tile's LDS reads past another tile's writes
    __shared__ T ldsA0[AH][AW], ldsA1[AH][AW];
    __shared__ T ldsC0[CH][CW], ldsC1[CH][CW];
    __shared__ T ldsD0[DH][DW], ldsD1[DH][DW];
    auto LA = [&](int h) -> T(*)[AW] { return h ? ldsA1 : ldsA0; };
    auto LC = [&](int h) -> T(*)[CW] { return h ? ldsC1 : ldsC0; };
    auto LD = [&](int h) -> T(*)[DW] { return h ? ldsD1 : ldsD0; };

    const int bid = blockIdx.x;
    const int b = find_box(p, bid);
    const BoxLaunch Bx = p.box[b];
    int local = bid - Bx.block_begin;
    int tk, tj;
    if (p.order == 2 && Bx.tiles_j % kXcds == 0) {
        // XCD x = id mod 8 runs tile rows [x*hb, x*hb + hb) of every k-tile and chunk
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
    const int kb = Bx.kbase + tk * kTK;
    const int jt = Bx.j0 + tj * TJ;
    const int ib = Bx.i0 + ci * Bx.chunk;
    const int ie = min(Bx.i1, ib + Bx.chunk - 1);
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sj = p.sj;
    const unsigned pbytes = p.pbytes;

    auto inb = [&](int j, int k) { return j >= p.jmin && j <= p.jmax && k >= p.kmin && k <= p.kmax; };
    auto incd = [&](int j, int k) { return j >= p.cj0 && j <= p.cj1 && k >= p.ck0 && k <= p.ck1; };
    auto boff = [&](int j, int k, bool ok) { return ok ? unsigned(j * sj + k + p.poff) * ES : kOOB; };
    // descriptor of logical plane i of a level (`nb` bytes: 0 = loads return 0)
    auto prs = [&](const char* base, int i, unsigned nb) {
        return plane_rsrc(base + u64(unsigned(i + p.pbias)) * pbytes, nb);
    };
    // timing ablations 4-6: loads (A, B) / stores (D, E) pinned to one plane (wrong results)
    auto prl = [&](const char* base, int i, unsigned nb) {
        return prs(base, i, nb);
    };
    auto pst = [&](char* base, int i, unsigned nb) {
        return prs(base, i, nb);
    };
    auto lrs = [&](const T* plane) { return plane_rsrc(plane - p.poff, pbytes); };

    // ---- own nodes ------------------------------------------------------------------------
    const int k = kb + lane;
    unsigned oa[R], ob[R], os[R];
    bool ovalid[R], ocd[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = jt + w * R + r;
        ocd[r] = incd(j, k);
        ovalid[r] = k >= Bx.k0 && k <= Bx.k1 && j <= Bx.j1;
        oa[r] = boff(j, k, inb(j, k));
        ob[r] = boff(j, k, !FIRST && inb(j, k) && ocd[r]);
        os[r] = boff(j, k, ovalid[r]);
    }
    const T otz = (k >= Bx.k0 && k <= Bx.k1) ? p.tz[k] : T(0);
    const T ortz = FM && k >= Bx.k0 && k <= Bx.k1 ? p.rtz[k] : T(0);
    // rows of this wave in the sx*sy table (padded past the last row: masked rows read in bounds)
    const T* const txw = p.txy + (jt + w * R);
    T om[R];  // --math fma: 1 on valid own nodes, 0 on masked lanes (branch-free errors)
#pragma unroll
    for (int r = 0; r < R; ++r) om[r] = ovalid[r] ? T(1) : T(0);
    // Dirichlet-face masks of computed values: a select (fp32) or a product (fp64)
    // with a 0/1 register — one op instead of two v_cndmask, and no lane masks held in SGPRs
    constexpr bool MM = sizeof(T) == 8;
    T ocm[R];
#pragma unroll
    for (int r = 0; r < R; ++r) ocm[r] = ocd[r] ? T(1) : T(0);
    auto cmask = [&](bool keep, T m, T v) {
        if constexpr (MM) return v * m;
        else return keep ? v : T(0);
    };
    // self-wrap ranges of D / E met by this work item (wave-uniform bits, one test per plane)
    int rare = 0;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        if (p.wd_lo[g] <= ie && p.wd_hi[g] >= ib) rare |= 1;
        if (p.we_lo[g] <= ie && p.we_hi[g] >= ib) rare |= 2;
    }
    rare = __builtin_amdgcn_readfirstlane(rare);
    // steady-state window [flo, fhi] of plane bodies: C(i), D(i-1), E(i-2) all own planes, off
    // the periodic seam and the self-wrap planes. Those sit at the ends of the x range, so each
    // one trims the window from its nearer end (a plane inside would only cost speed).
    int flo = ib + 2, fhi = ie;
    auto cut = [&](int lo, int hi) {
        if (lo > hi || hi < flo || lo > fhi) return;
        if (lo - flo <= fhi - hi) flo = hi + 1;
        else fhi = lo - 1;
    };
    cut(p.an_i, p.an_i + 1);
    cut(p.ap_i, p.ap_i + 1);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        cut(p.wd_lo[g] + 1, p.wd_hi[g] + 1);
        cut(p.we_lo[g] + 2, p.we_hi[g] + 2);
    }
    flo = __builtin_amdgcn_readfirstlane(flo);
    fhi = __builtin_amdgcn_readfirstlane(fhi);

    // ---- ring positions of this thread ------------------------------------------------------
    // d-ring = rows jt-d / jt+TJ-1+d over cols kb-d+1 .. kb+64+d-2, then cols kb-d / kb+63+d over
    // rows jt-d+c .. jt+TJ-1+d-c (c = 1 drops the corners)
    auto ring = [&](int d, int c, int idx, int& rj, int& rk) {
        const int wd = kTK + 2 * (d - 1), hd = TJ + 2 * (d - c);
        if (idx < wd) rj = jt - d, rk = kb - (d - 1) + idx;
        else if (idx < 2 * wd) rj = jt + TJ - 1 + d, rk = kb - (d - 1) + idx - wd;
        else if (idx < 2 * wd + hd) rj = jt - d + c + (idx - 2 * wd), rk = kb - d;
        else rj = jt - d + c + (idx - 2 * wd - hd), rk = kb + kTK - 1 + d;
    };
    int rg[RP], ry[RP], rx[RP];      // ring (0: none) and A-tile coordinates
    unsigned ra_off[RP], rb_off[RP];  // A / B load offsets (kOOB when masked)
    bool rcd[RP];                     // stencil-valued node (else 0: Dirichlet face)
#pragma unroll
    for (int s = 0; s < RP; ++s) {
        const int q = threadIdx.x + s * NT;
        int g = 0, rj = jt, rk = kb;
        if (q < N1) g = 1, ring(1, 0, q, rj, rk);
        else if (q < N1 + N2) g = 2, ring(2, 0, q - N1, rj, rk);
        else if (q < N1 + N2 + N3) g = 3, ring(3, 1, q - N1 - N2, rj, rk);
        rg[s] = g;
        ry[s] = rj - jt + 3, rx[s] = rk - kb + 3;
        rcd[s] = g != 0 && g != 3 && incd(rj, rk);
        ra_off[s] = boff(rj, rk, g != 0 && inb(rj, rk));
        rb_off[s] = boff(rj, rk, !FIRST && rcd[s] && inb(rj, rk));
    }
    T rcm[RP];
#pragma unroll
    for (int s = 0; s < RP; ++s) rcm[s] = rcd[s] ? T(1) : T(0);

    // slots (iteration i = ib - 2 + q, phase P = q & 3):
    //   A(x), ring A(x): (x - ib + 3) & 3  -> A(i-1) = P, A(i) = P+1, A(i+1) = P+2, A(i+2) = P+3
    //   C(x), ring C(x): (x - ib + 2) & 3  -> C(i) = P, C(i-1) = P+3, C(i-2) = P+2
    //   D(x): (x - ib + 3) & 3             -> D(i-1) = P, D(i-2) = P+3, D(i-3) = P+2
    //   B(x), ring B(x), LDS buffers: (x - ib + 2) & 1
    constexpr int NB = 2, BD = 1;  // B slots, B prefetch distance (planes)
    T a[4][R], c[4][R], d[4][R], bb[NB][R];
    T ra[RP][4], rb[RP][NB], rc[RP][4];
    // increment form: d^m of own planes i (H0) / i-1 (H1) and of the ring, d^{m+1} of own
    // planes i-1 (H0) / i-2 (H1)
    constexpr int ND = DELTA ? 2 : 1;
    T dm[ND][R], dm1[ND][R], rdm[RP][ND];
    {
        const auto r0 = prl(p.A, ib - 3, pbytes), rA1 = prl(p.A, ib - 2, pbytes), rA2 = prl(p.A, ib - 1, pbytes);
        const auto rB = prl(p.B, ib - 2, pbytes), rBn = prl(p.B, ib - 1, NB == 4 ? pbytes : 0u);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            a[0][r] = bld<T>(r0, oa[r]);
            a[1][r] = bld<T>(rA1, oa[r]);
            a[2][r] = bld<T>(rA2, oa[r]);
            a[3][r] = T(0);
            bb[0][r] = bld<T>(rB, ob[r]);
#pragma unroll
            for (int t = 1; t < NB; ++t) bb[t][r] = t == 1 && NB == 4 ? bld<T>(rBn, ob[r]) : T(0);
#pragma unroll
            for (int s = 0; s < 4; ++s) c[s][r] = d[s][r] = T(0);
        }
#pragma unroll
        for (int s = 0; s < RP; ++s) {
            ra[s][0] = bld<T>(r0, ra_off[s]);
            ra[s][1] = bld<T>(rA1, ra_off[s]);
            ra[s][2] = bld<T>(rA2, ra_off[s]);
            ra[s][3] = T(0);
            rb[s][0] = bld<T>(rB, rb_off[s]);
#pragma unroll
            for (int t = 1; t < NB; ++t) rb[s][t] = t == 1 && NB == 4 ? bld<T>(rBn, rb_off[s]) : T(0);
#pragma unroll
            for (int t = 0; t < 4; ++t) rc[s][t] = T(0);
        }
    }

    T ma1 = T(kErrInit), ma2 = T(kErrInit);
    using Rel = std::conditional_t<FM, RelMax<T>, RelArg<T>>;  // fma: |d| * 1/|f| max
    Rel mr1, mr2;
    T ma3 = T(kErrInit);
    Rel mr3;
    T chk1 = T(0), chk2 = T(0), chk3 = T(0);

    // Layer L (0 = C, 1 = D, 2 = E) arithmetic. lap(): the Laplacian (exact) or, FM, the deferred
    // stencil (FmLap: the leapfrog takes it whole, stencil_math leap_fm; the Taylor start and the
    // increment form take coef*lap); leap / first / incr: the updates from it.
    const T kc1 = FM ? fm_kc(p.fc[1][0], p.fc[1][1], p.fc[1][2]) : T(0);
    auto lap = [&](int L, T ctr, T xm, T xp, T ym, T yp, T zm, T zp) {
        if constexpr (FM) {
            const int f = FIRST && L == 0 ? 0 : 1;
            return FmLap<T>{ctr, xm, xp, ym, yp, zm, zp, p.fc[f][0], p.fc[f][1], p.fc[f][2]};
        } else {
            return laplace7_cr(ctr, xm, xp, ym, yp, zm, zp, p.hx2, p.hy2, p.hz2, p.yx2, p.yy2, p.yz2);
        }
    };
    auto coefL = [&](int L) { return L == 0 ? p.coefC : (L == 1 ? p.coefD : p.coefE); };
    auto leap = [&](int L, T ctr, T u2, const auto& l) {
        if constexpr (FM) return l.leap(u2, kc1);
        else return leapfrog(ctr, u2, l, coefL(L));
    };
    auto incr = [&](int L, T dprev, const auto& l) {  // increment form: d_new = d_prev + coef*lap
        if constexpr (FM) return dprev + lap_value(l);
        else return delta_incr(dprev, l, coefL(L));
    };
    auto scaled = [&](int L, const auto& l) {  // coef*lap (FIRST increment: d = coef*lap)
        if constexpr (FM) return lap_value(l);
        else return coefL(L) * l;
    };
    auto lapA = [&](int H, int y, int x, T ctr, T xm, T xp) {
        return lap(0, ctr, xm, xp, LA(H)[y - 1][x], LA(H)[y + 1][x], LA(H)[y][x - 1], LA(H)[y][x + 1]);
    };
    // own row r's j neighbours: rows r-1 / r+1 of the same wave are centre values in registers
    // (v[], as staged to LDS at (y -/+ 1, x)); the wave's edge rows read the tile
    auto jm = [&](const T(&v)[R], int r, const auto& tile, int y, int x) {
        return (r > 0) ? v[r > 0 ? r - 1 : 0] : tile[y - 1][x];
    };
    auto jp = [&](const T(&v)[R], int r, const auto& tile, int y, int x) {
        return (r < R - 1) ? v[r < R - 1 ? r + 1 : 0] : tile[y + 1][x];
    };
    auto cval = [&](T ctr, T bv, const auto& l) {
        if constexpr (FM) return FIRST ? ctr + lap_value(l) : l.leap(bv, kc1);
        else return FIRST ? taylor_first(ctr, l, p.coefC) : leapfrog(ctr, bv, l, p.coefC);
    };
    // Errors are taken two planes late: at iteration i those of C(i-2), D(i-2) and E(i-2), all
    // still in registers, so one analytic-table row per plane serves the three layers (f =
    // ((sx sy) sz) ct per layer, as stencil_math analytic()). The row of plane i-1 is loaded at
    // iteration i into the plane-parity slot (a scalar load a whole iteration ahead of its use).
    // --math fma: the (sx sy, 1/|sx sy|) pair (txr); exact: sx sy (txy).
    constexpr int NQ = FM ? 2 : 1;
    T tq[2][R][NQ];
    auto load_row = [&](int slot, int q) {
        q = min(max(q, ib), ie);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if constexpr (FM) {
                const T* const tr = p.txr + 2 * (q * p.tpj + (jt + w * R));
                tq[slot][r][0] = ldconst(tr, 2 * r);
                tq[slot][r][1] = ldconst(tr, 2 * r + 1);
            } else {
                tq[slot][r][0] = ldconst(txw + q * p.tpj, r);
            }
        }
    };
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int n = 0; n < NQ; ++n) tq[0][r][n] = tq[1][r][n] = T(0);
    // exact: the reference's per-node error update (RelArg: bitwise relative error); the uniform
    // error-plane test sits outside the per-lane row masks (a scalar branch)
    auto errors_exact = [&](const T(&v)[R], const T(&fb)[R], const bool eplane, const T ct, T& ma, auto& mr,
                            T& chk) {
        if (eplane) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (!ovalid[r]) continue;
                chk += v[r];
                accumulate_error_dev(v[r], fb[r] * ct, ma, mr);
            }
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (ovalid[r]) chk += v[r];
        }
    };
    // --math fma: branch-free — masked lanes and planes outside the error range contribute
    // d = 0 (the multiplier m = om * em), so no exec-mask branches and no phi copies of the
    // running maxima; the relative weight wq = 1/|sx sy| * 1/|sz| is shared by the three layers
    auto errors_fm = [&](const T(&v)[R], const T(&fb)[R], const T(&m)[R], const T(&wq)[R], const T ct, T& ma,
                         RelMax<T>& mr, T& chk) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if constexpr (MM) chk = fma_t(v[r], om[r], chk);
            else chk += ovalid[r] ? v[r] : T(0);
            const T dv = (v[r] - fb[r] * ct) * m[r];
            ma = max_abs(ma, dv);
            mr.add(dv, wq[r]);
        }
    };
    // the three layers of own plane q (table row in slot H)
    auto errors3 = [&](const int H, const int q, const T(&vc)[R], const T(&vd)[R], const T(&ve)[R]) {
        const bool eplane = q >= p.ei0 && q <= p.ei1;
        T fb[R];
#pragma unroll
        for (int r = 0; r < R; ++r) fb[r] = tq[H][r][0] * otz;  // (sx sy) sz
        if constexpr (FM) {
            const T em = eplane ? T(1) : T(0);
            T m[R], wq[R];
#pragma unroll
            for (int r = 0; r < R; ++r) m[r] = om[r] * em, wq[r] = tq[H][r][1] * ortz;
            errors_fm(vc, fb, m, wq, p.ctC, ma1, mr1, chk1);
            errors_fm(vd, fb, m, wq, p.ctD, ma2, mr2, chk2);
            errors_fm(ve, fb, m, wq, p.ctE, ma3, mr3, chk3);
        } else {
            errors_exact(vc, fb, eplane, p.ctC, ma1, mr1, chk1);
            errors_exact(vd, fb, eplane, p.ctD, ma2, mr2, chk2);
            errors_exact(ve, fb, eplane, p.ctE, ma3, mr3, chk3);
        }
    };
    // SLOW (ALIAS): the prologue / epilogue planes of the work item and the periodic seam
    // planes — every range check and the seam partners. FAST: the steady state (planes
    // ib+2 .. ie off the seam), where C(i), D(i-1) and E(i-2) are all own planes and the
    // prefetch is live, so the body has no range tests (fewer scalar branches per plane).
    auto plane = [&](auto phase, auto alias, const int i) {
        constexpr int P = decltype(phase)::value;
        constexpr bool ALIAS = decltype(alias)::value;
        constexpr bool FAST = !ALIAS;
        constexpr int S0 = P & 3, S1 = (P + 1) & 3, S2 = (P + 2) & 3, S3 = (P + 3) & 3;
        constexpr int H0 = P & 1, H1 = (P + 1) & 1;
        constexpr int BC = P & (NB - 1), BP = (P + BD) & (NB - 1);  // B(i), B(i+BD) slots

        // ---- prefetch A(i+2), B(i+BD) (own and ring; 0-record descriptors when done) -------
        {
            const bool more = FAST || i <= ie + 1, moreB = FAST || i + BD <= ie + 2;
            const unsigned nb = more ? pbytes : 0u;
            const int d2 = more ? 2 : 0, d1 = moreB ? BD : 0;
            const auto rA2 = prl(p.A, i + d2, nb);
            const auto rB1 = prl(p.B, i + d1, moreB ? pbytes : 0u);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                a[S3][r] = bld<T>(rA2, oa[r]);
                bb[BP][r] = bld<T>(rB1, ob[r]);
            }
#pragma unroll
            for (int s = 0; s < RP; ++s) {
                ra[s][S3] = bld<T>(rA2, ra_off[s]);
                rb[s][BP] = bld<T>(rB1, rb_off[s]);
            }
        }
        // ---- stage A(i) --------------------------------------------------------------------
#pragma unroll
        for (int r = 0; r < R; ++r) LA(H0)[3 + w * R + r][3 + lane] = a[S1][r];
#pragma unroll
        for (int s = 0; s < RP; ++s)
            if (rg[s]) LA(H0)[ry[s]][rx[s]] = ra[s][S1];
        __syncthreads();

        // ---- seam partners (uniform branch, rare) -------------------------------------------
        T xnA[R], xpA[R], cnx[R], cpx[R];
        T rxn[RP], rxp[RP], rcn[RP], rcp[RP];
#pragma unroll
        for (int r = 0; r < R; ++r) xnA[r] = a[S2][r], xpA[r] = a[S0][r], cnx[r] = c[S0][r], cpx[r] = c[S2][r];
#pragma unroll
        for (int s = 0; s < RP; ++s) rxn[s] = ra[s][S2], rxp[s] = ra[s][S0], rcn[s] = rc[s][S0], rcp[s] = rc[s][S2];
        if constexpr (ALIAS) {
            // C(i): A partner as x+ (i == an_i) or x- (i == ap_i) neighbour
            if (i == p.an_i) {
                const auto rs = lrs(p.nA);
#pragma unroll
                for (int r = 0; r < R; ++r) xnA[r] = bld<T>(rs, oa[r]);
#pragma unroll
                for (int s = 0; s < RP; ++s) rxn[s] = bld<T>(rs, ra_off[s]);
            }
            if (i == p.ap_i) {
                const auto rs = lrs(p.pA);
#pragma unroll
                for (int r = 0; r < R; ++r) xpA[r] = bld<T>(rs, oa[r]);
#pragma unroll
                for (int s = 0; s < RP; ++s) rxp[s] = bld<T>(rs, ra_off[s]);
            }
            // D(i-1): C at the partner plane (k_seam_c, before the sweep)
            if (i - 1 == p.an_i) {
                const auto rs = lrs(p.nC);
#pragma unroll
                for (int r = 0; r < R; ++r) cnx[r] = bld<T>(rs, oa[r]);
#pragma unroll
                for (int s = 0; s < RP; ++s) rcn[s] = bld<T>(rs, ra_off[s]);
            }
            if (i - 1 == p.ap_i) {
                const auto rs = lrs(p.pC);
#pragma unroll
                for (int r = 0; r < R; ++r) cpx[r] = bld<T>(rs, oa[r]);
#pragma unroll
                for (int s = 0; s < RP; ++s) rcp[s] = bld<T>(rs, ra_off[s]);
            }
        }

        // ---- C(i) on tile + 2-ring ----------------------------------------------------------
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int y = 3 + w * R + r, x = 3 + lane;
            const auto l = lap(0, a[S1][r], xpA[r], xnA[r], jm(a[S1], r, LA(H0), y, x), jp(a[S1], r, LA(H0), y, x),
                               LA(H0)[y][x - 1], LA(H0)[y][x + 1]);
            if constexpr (DELTA) {
                const T dv = FIRST ? scaled(0, l) : incr(0, bb[BC][r], l);
                dm[H0][r] = cmask(ocd[r], ocm[r], dv);
                c[S0][r] = cmask(ocd[r], ocm[r], a[S1][r] + dv);  // FIRST: = taylor_first
            } else {
                c[S0][r] = cmask(ocd[r], ocm[r], cval(a[S1][r], bb[BC][r], l));
            }
            LC(H0)[y - 1][x - 1] = c[S0][r];
        }
#pragma unroll
        for (int s = 0; s < RP; ++s) {
            if (rg[s] == 1 || rg[s] == 2) {
                const auto lap = lapA(H0, ry[s], rx[s], ra[s][S1], rxp[s], rxn[s]);
                T cv;
                if constexpr (DELTA) {
                    const T dv = FIRST ? scaled(0, lap) : incr(0, rb[s][BC], lap);
                    rdm[s][H0] = cmask(rcd[s], rcm[s], dv);
                    cv = cmask(rcd[s], rcm[s], ra[s][S1] + dv);
                } else {
                    cv = cmask(rcd[s], rcm[s], cval(ra[s][S1], rb[s][BC], lap));
                }
                rc[s][S0] = cv;
                LC(H0)[ry[s] - 1][rx[s] - 1] = cv;
            }
        }
        if constexpr (!ALIAS) {
            // the x neighbours of D(i-1) are C(i) (computed just now) and C(i-2)
#pragma unroll
            for (int r = 0; r < R; ++r) cnx[r] = c[S0][r];
#pragma unroll
            for (int s = 0; s < RP; ++s) rcn[s] = rc[s][S0];
        } else {
            if (i - 1 != p.an_i) {
#pragma unroll
                for (int r = 0; r < R; ++r) cnx[r] = c[S0][r];
#pragma unroll
                for (int s = 0; s < RP; ++s) rcn[s] = rc[s][S0];
            }
        }

        // ---- D(i-1) on tile + 1-ring, from the C(i-1) tile --------------------------------
        const int id = i - 1;
        if (FAST || (id >= ib - 1 && id <= ie + 1)) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int y = 2 + w * R + r, x = 2 + lane;  // C tile coordinates
                const auto l = lap(1, c[S3][r], cpx[r], cnx[r], jm(c[S3], r, LC(H1), y, x), jp(c[S3], r, LC(H1), y, x),
                                LC(H1)[y][x - 1], LC(H1)[y][x + 1]);
                if constexpr (DELTA) {
                    const T d1 = incr(1, dm[H1][r], l);  // d^{m+1}
                    dm1[H0][r] = cmask(ocd[r], ocm[r], d1);
                    d[S0][r] = cmask(ocd[r], ocm[r], c[S3][r] + d1);
                } else {
                    d[S0][r] = cmask(ocd[r], ocm[r], leap(1, c[S3][r], a[S0][r], l));
                }
                LD(H0)[y - 1][x - 1] = d[S0][r];
            }
#pragma unroll
            for (int s = 0; s < RP; ++s) {
                if (rg[s] == 1) {
                    const int y = ry[s] - 1, x = rx[s] - 1;
                    const auto l = lap(1, rc[s][S3], rcp[s], rcn[s], LC(H1)[y - 1][x], LC(H1)[y + 1][x],
                                    LC(H1)[y][x - 1], LC(H1)[y][x + 1]);
                    if constexpr (DELTA)
                        LD(H0)[y - 1][x - 1] = cmask(rcd[s], rcm[s], rc[s][S3] + incr(1, rdm[s][H1], l));
                    else
                        LD(H0)[y - 1][x - 1] = cmask(rcd[s], rcm[s], leap(1, rc[s][S3], ra[s][S0], l));
                }
            }
            if (FAST || (id >= ib && id <= ie)) {
                if constexpr (!DELTA) {
                    const auto rd = pst(p.D, id, pbytes);
#pragma unroll
                    for (int r = 0; r < R; ++r) bst<2>(d[S0][r], rd, os[r]);
                    if (!FAST && (rare & 1)) {
#pragma unroll
                        for (int g = 0; g < 2; ++g)
                            if (id >= p.wd_lo[g] && id <= p.wd_hi[g]) {
                                const auto rw = pst(p.D, id + p.wd_sh[g], pbytes);
#pragma unroll
                                for (int r = 0; r < R; ++r) bst<2>(d[S0][r], rw, os[r]);
                            }
                    }
                }
            }
        }

        // ---- E(i-2) on the tile, from the D(i-2) tile -----------------------------------------
        const int ie2 = i - 2;
        if (FAST || (ie2 >= ib && ie2 <= ie)) {
            T ev[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int y = 1 + w * R + r, x = 1 + lane;  // D tile coordinates
                const auto l = lap(2, d[S3][r], d[S2][r], d[S0][r], jm(d[S3], r, LD(H1), y, x),
                                jp(d[S3], r, LD(H1), y, x), LD(H1)[y][x - 1], LD(H1)[y][x + 1]);
                if constexpr (DELTA) {
                    dm1[H1][r] = incr(2, dm1[H1][r], l);  // d^{m+2}
                    ev[r] = d[S3][r] + dm1[H1][r];
                } else {
                    ev[r] = leap(2, d[S3][r], c[S2][r], l);
                }
            }
            if constexpr (DELTA) {
                // d^{m+2} into the D level (+ its periodic self-wrap), the next sweep's B
                const auto rd = pst(p.D, ie2, pbytes);
#pragma unroll
                for (int r = 0; r < R; ++r) bst<2>(dm1[H1][r], rd, os[r]);
                if (!FAST && (rare & 2)) {
#pragma unroll
                    for (int g = 0; g < 2; ++g)
                        if (ie2 >= p.we_lo[g] && ie2 <= p.we_hi[g]) {
                            const auto rw = pst(p.D, ie2 + p.we_sh[g], pbytes);
#pragma unroll
                            for (int r = 0; r < R; ++r) bst<2>(dm1[H1][r], rw, os[r]);
                        }
                }
            }
            const auto re = pst(p.E, ie2, pbytes);
#pragma unroll
            for (int r = 0; r < R; ++r) bst<2>(ev[r], re, os[r]);
            if (!FAST && (rare & 2)) {
#pragma unroll
                for (int g = 0; g < 2; ++g)
                    if (ie2 >= p.we_lo[g] && ie2 <= p.we_hi[g]) {
                        const auto rw = pst(p.E, ie2 + p.we_sh[g], pbytes);
#pragma unroll
                        for (int r = 0; r < R; ++r) bst<2>(ev[r], rw, os[r]);
                    }
            }
            // errors of plane i-2: C(i-2) and D(i-2) from their register slots, E(i-2) just now
            errors3(H0, ie2, c[S2], d[S3], ev);
        }
        load_row(H1, i - 1);
    };

    // i = ib-2 .. ie+2 (>= 5 planes) in three loops, each unrolled by 4 from phase 0 so every
    // slot index is a constant: the checked body (ALIAS: seam / wrap / work-item ends) up to the
    // first phase-0 plane of the steady window [flo, fhi], the steady body over whole groups of 4
    // inside it, the checked body for the rest. Choosing the body per plane in one loop keeps the
    // checked body's values live through the steady one (SGPR spills: hip_tbn.hip, same split).
    const int i0 = ib - 2, iend = ie + 2;
    const int fstart = __builtin_amdgcn_readfirstlane(i0 + ((max(flo, i0) - i0 + 3) & ~3));
    const int fend = __builtin_amdgcn_readfirstlane(fstart + (fhi >= fstart ? (fhi - fstart + 1) & ~3 : 0));
    auto checked = [&](int& i, const int stop) {  // i = i0 mod 4 on entry; runs while i < stop
        if (i >= stop) return;
        for (;;) {
            plane(Ph<0>{}, std::true_type{}, i);
            if (++i >= stop) break;
            plane(Ph<1>{}, std::true_type{}, i);
            if (++i >= stop) break;
            plane(Ph<2>{}, std::true_type{}, i);
            if (++i >= stop) break;
            plane(Ph<3>{}, std::true_type{}, i);
            if (++i >= stop) break;
        }
    };
    int i = i0;
#pragma nounroll
    for (int pass = 0; pass < 2; ++pass) {
        checked(i, pass == 0 ? min(fstart, iend + 1) : iend + 1);
        if (pass == 0 && i == fstart)
            for (; i < fend; i += 4) {
                plane(Ph<0>{}, std::false_type{}, i);
                plane(Ph<1>{}, std::false_type{}, i + 1);
                plane(Ph<2>{}, std::false_type{}, i + 2);
                plane(Ph<3>{}, std::false_type{}, i + 3);
            }
    }
    auto rel = [&](const Rel& m, int L) {
        if constexpr (FM) return m.value(p.ict[L]);
        else return m.value();
    };
    commit_errors<T, NW>(ma1, rel(mr1, 0), chk1, p.errC);
    __syncthreads();
    commit_errors<T, NW>(ma2, rel(mr2, 1), chk2, p.errD);
    __syncthreads();
    commit_errors<T, NW>(ma3, rel(mr3, 2), chk3, p.errE);
}

// C (layer m) on one partner plane of the periodic seam, every (j, k) of the storage except
// its outermost row/column: out = leapfrog(A_c, B_c, lap) with x neighbours A_m / A_p and
// j/k neighbours from A_c itself; 0 outside the stencil region. Logical plane pointers.
template <class T>
struct SeamCOp {
    T* out;
    const T *Ac, *Am, *Ap, *Bc;
    T* dout;  // increment form: d of the evaluated layer too (nullptr: not kept)
};
template <class T>
struct SeamCParams {
    SeamCOp<T> op[kMaxSeamOps];
    int sj, jmin, jmax, kmin, kmax;
    int cj0, cj1, ck0, ck1;
    T hx2, hy2, hz2, yx2, yy2, yz2, coef;
    T fc[3];  // --math fma: coef/h^2 per axis
};

template <class T, bool FIRST, bool DELTA, bool FM>
__global__ void __launch_bounds__(kThreads) k_seam_c(const SeamCParams<T> p) {
    const SeamCOp<T> o = p.op[blockIdx.y];
    const int ktiles = (p.kmax - p.kmin - 1 + kTK - 1) / kTK;
    const int j = p.jmin + 1 + (int(blockIdx.x) / ktiles) * kWaves + int(threadIdx.x >> 6);
    const int k = p.kmin + 1 + (int(blockIdx.x) % ktiles) * kTK + int(threadIdx.x & 63);
    if (j > p.jmax - 1 || k > p.kmax - 1) return;
    const i64 c = i64(j) * p.sj + k;
    T v = T(0), d = T(0);
    if (j >= p.cj0 && j <= p.cj1 && k >= p.ck0 && k <= p.ck1) {
        const T a = o.Ac[c];
        if constexpr (FM) {  // as the sweep's FM instantiation, so the seam C is the sweep's C
            const T l = coef_lap_fma(a, o.Am[c], o.Ap[c], o.Ac[c - p.sj], o.Ac[c + p.sj], o.Ac[c - 1], o.Ac[c + 1],
                                     p.fc[0], p.fc[1], p.fc[2]);
            if constexpr (DELTA)
                d = FIRST ? l : o.Bc[c] + l, v = a + d;
            else if constexpr (FIRST)
                v = a + l;
            else  // the sweeps' leapfrog (stencil_math leap_fm)
                v = leap_fm(a, o.Bc[c], o.Am[c], o.Ap[c], o.Ac[c - p.sj], o.Ac[c + p.sj], o.Ac[c - 1], o.Ac[c + 1],
                            p.fc[0], p.fc[1], p.fc[2], fm_kc(p.fc[0], p.fc[1], p.fc[2]));
        } else {
            const T lap = laplace7_cr(a, o.Am[c], o.Ap[c], o.Ac[c - p.sj], o.Ac[c + p.sj], o.Ac[c - 1],
                                      o.Ac[c + 1], p.hx2, p.hy2, p.hz2, p.yx2, p.yy2, p.yz2);
            if constexpr (DELTA)  // Bc = d^{m-1}
                d = FIRST ? p.coef * lap : delta_incr(o.Bc[c], lap, p.coef), v = a + d;
            else
                v = FIRST ? taylor_first(a, lap, p.coef) : leapfrog(a, o.Bc[c], lap, p.coef);
        }
    }
    o.out[c] = v;
    if (DELTA && o.dout) o.dout[c] = d;
}

template <class T, bool F>
static void (*tb3_kernel(int rows, int waves, bool fm = false))(const Tb3Params<T>) {
    if (fm) {  // --math fma: the main tile shapes
        switch (rows * 100 + waves) {
            case 208: return k_tb3<T, F, 2, 8, false, true>;
            case 108: return k_tb3<T, F, 1, 8, false, true>;
            case 116: return k_tb3<T, F, 1, 16, false, true>;
            default: return nullptr;
        }
    }
    switch (rows * 100 + waves) {
        case 404: return k_tb3<T, F, 4, 4>;
        case 208: return k_tb3<T, F, 2, 8>;
        case 204: return k_tb3<T, F, 2, 4>;
        case 116: return k_tb3<T, F, 1, 16>;
        case 108: return k_tb3<T, F, 1, 8>;
        default: return nullptr;
    }
}

}  // namespace

// increment form: the 16-row and 1-row tiles (fp32 delta auto = r2w8: 537k vs tb2r2w8 520k Mpts/s
// at N=512, profiles/tb3_diet_r2.txt)
template <class T, bool F>
static void (*tb3_delta_kernel(int rows, int waves, bool fm = false))(const Tb3Params<T>) {
    switch (rows * 100 + waves + (fm ? 10000 : 0)) {
        case 208: return k_tb3<T, F, 2, 8, true>;
        case 108: return k_tb3<T, F, 1, 8, true>;
        case 10208: return k_tb3<T, F, 2, 8, true, true>;
        case 10108: return k_tb3<T, F, 1, 8, true, true>;
        default: return nullptr;
    }
}

bool tb3_supported(int rows, int waves, bool fm) { return tb3_kernel<double, false>(rows, waves, fm) != nullptr; }
bool tb3_delta_supported(int rows, int waves, bool fm) {
    return tb3_delta_kernel<double, false>(rows, waves, fm) != nullptr;
}

// coef/h^2 of one layer for the FMA form
template <class T>
static void fma_coefs(const StepCoefs& c, T out[3]) {
    out[0] = T(c.coef / c.hx2), out[1] = T(c.coef / c.hy2), out[2] = T(c.coef / c.hz2);
}

template <class T>
void launch_tb3(int rows, int waves, bool delta, bool fm, bool first, const T* A, const T* B, T* D, T* E,
                const GridView& gv, const Box* boxes, int nbox, const Box& cdom, int ei0, int ei1,
                const Wrap& wrapD, const Wrap& wrapE, const SeamPartners<T>& seam, const T* txy,
                const T* tz, const T* txr, const T* rtz, const StepCoefs& cC, const StepCoefs& cD,
                const StepCoefs& cE, u64* errC, u64* errD, u64* errE, int chunk, hipStream_t s) {
    W3D_REQUIRE(!fm || (txr && rtz), "tb3 --math fma needs the reciprocal analytic tables");
    W3D_REQUIRE(gv.G >= 3, "three-layer temporal blocking needs ghost depth >= 3");
    W3D_REQUIRE(tb3_supported(rows, waves, fm && !delta), "tb3: unsupported rows x waves (x --math fma)");
    W3D_REQUIRE(!delta || tb3_delta_supported(rows, waves, fm), "tb3 increment form: tiles r2w8, r1w8 only");
    W3D_REQUIRE(nbox >= 1 && nbox <= kMaxBoxes, "bad box count");
    W3D_REQUIRE(gv.si * i64(sizeof(T)) < (i64(1) << 31), "tb3: plane larger than 2 GiB");
    Tb3Params<T> p{};
    // plane indices reach 1 - G (wrap targets) and ib - 3 >= -2
    p.pbytes = unsigned(gv.si * i64(sizeof(T)));
    p.pbias = gv.G + 1;
    p.order = tile_order();
    auto biased = [&](const T* base) {
        return reinterpret_cast<char*>(reinterpret_cast<uintptr_t>(base - gv.poff) -
                                       uintptr_t(p.pbias) * p.pbytes);
    };
    p.A = biased(A), p.B = biased(B), p.D = biased(D), p.E = biased(E);
    p.sj = gv.sj;
    p.poff = gv.poff;
    p.jmin = 1 - gv.G, p.jmax = gv.jmax(), p.kmin = 1 - gv.G, p.kmax = gv.kmax();
    p.cj0 = cdom.j0, p.cj1 = cdom.j1, p.ck0 = cdom.k0, p.ck1 = cdom.k1;
    p.ei0 = ei0, p.ei1 = ei1;
    wrap_ranges(wrapD, p.wd_lo, p.wd_hi, p.wd_sh);
    wrap_ranges(wrapE, p.we_lo, p.we_hi, p.we_sh);
    p.an_i = seam.nA ? seam.next_i : INT_MIN / 2;
    p.ap_i = seam.pA ? seam.prev_i : INT_MIN / 2;
    W3D_REQUIRE((!seam.nA || seam.nC) && (!seam.pA || seam.pC), "tb3: seam partner without its C plane");
    p.nA = seam.nA, p.nC = seam.nC, p.pA = seam.pA, p.pC = seam.pC;
    p.txy = txy, p.tpj = gv.Y + 2, p.tz = tz;
    p.hx2 = T(cC.hx2), p.hy2 = T(cC.hy2), p.hz2 = T(cC.hz2);
    p.yx2 = T(1) / T(cC.hx2), p.yy2 = T(1) / T(cC.hy2), p.yz2 = T(1) / T(cC.hz2);
    p.coefC = T(cC.coef), p.coefD = T(cD.coef), p.coefE = T(cE.coef);
    p.ctC = T(cC.ct), p.ctD = T(cD.ct), p.ctE = T(cE.ct);
    W3D_REQUIRE(!fm || (cD.coef == cE.coef && (first || cC.coef == cD.coef)),
                "tb3 --math fma: the non-first layers must share one coefficient");
    fma_coefs(cC, p.fc[0]), fma_coefs(cD, p.fc[1]);
    p.txr = txr, p.rtz = rtz;
    p.ict[0] = T(1 / std::fabs(cC.ct)), p.ict[1] = T(1 / std::fabs(cD.ct)), p.ict[2] = T(1 / std::fabs(cE.ct));
    p.errC = errC, p.errD = errD, p.errE = errE;
    const int TJ = waves * rows;
    auto kern = delta ? (first ? tb3_delta_kernel<T, true>(rows, waves, fm) : tb3_delta_kernel<T, false>(rows, waves, fm))
                      : (first ? tb3_kernel<T, true>(rows, waves, fm) : tb3_kernel<T, false>(rows, waves, fm));
    int live = 0;
    for (int q = 0; q < nbox; ++q) live += !boxes[q].empty();
    // several boxes (overlap shells): one work-item length for the launch as a whole
    int multi_chunk = 0;
    if (chunk <= 0 && live > 1) {
        int bt[kMaxBoxes], bp[kMaxBoxes], m = 0;
        for (int q = 0; q < nbox; ++q) {
            const Box& bx = boxes[q];
            if (bx.empty()) continue;
            bt[m] = ((bx.k1 - 1) / kTK - (bx.k0 - 1) / kTK + 1) * cdiv(bx.j1 - bx.j0 + 1, TJ);
            bp[m++] = bx.i1 - bx.i0 + 1;
        }
        multi_chunk = rounds_chunk_boxes(bt, bp, m, 4, resident_slots(reinterpret_cast<const void*>(kern), waves * 64));
    }
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
        const int want = chunk > 0 ? std::min(chunk, planes)
                         : live == 1 ? rounds_chunk(planes, L.tiles_k * L.tiles_j, 4,
                                                    resident_slots(reinterpret_cast<const void*>(kern), waves * 64))
                                     : std::min(multi_chunk, planes);
        L.chunk = cdiv(planes, cdiv(planes, want));
        L.block_begin = total;
        total += L.tiles_k * L.tiles_j * cdiv(planes, L.chunk);
        ++nb;
    }
    p.nbox = nb;
    if (nb == 0) return;
    hipLaunchKernelGGL(kern, dim3(total), dim3(waves * 64), 0, s, p);
    HIP_OK(hipGetLastError());
}

template <class T>
void launch_seam_c(bool first, bool delta, bool fm, const SeamCPlane<T>* ops, int nops, const GridView& gv,
                   const Box& cdom, const StepCoefs& cC, hipStream_t s) {
    W3D_REQUIRE(nops >= 0 && nops <= kMaxSeamOps, "seam C: too many planes");
    if (nops == 0) return;
    SeamCParams<T> p{};
    for (int q = 0; q < nops; ++q)
        p.op[q] = SeamCOp<T>{ops[q].out, ops[q].Ac, ops[q].Am, ops[q].Ap, ops[q].Bc ? ops[q].Bc : ops[q].Ac, ops[q].dout};
    p.sj = gv.sj;
    p.jmin = 1 - gv.G, p.jmax = gv.jmax(), p.kmin = 1 - gv.G, p.kmax = gv.kmax();
    p.cj0 = cdom.j0, p.cj1 = cdom.j1, p.ck0 = cdom.k0, p.ck1 = cdom.k1;
    p.hx2 = T(cC.hx2), p.hy2 = T(cC.hy2), p.hz2 = T(cC.hz2);
    p.yx2 = T(1) / T(cC.hx2), p.yy2 = T(1) / T(cC.hy2), p.yz2 = T(1) / T(cC.hz2);
    p.coef = T(cC.coef);
    fma_coefs(cC, p.fc);
    const int rows = p.jmax - p.jmin - 1, ktiles = cdiv(p.kmax - p.kmin - 1, kTK);
    const dim3 grid(cdiv(rows, kWaves) * ktiles, nops);
    void (*kern)(const SeamCParams<T>) =
        fm ? (delta ? (first ? k_seam_c<T, true, true, true> : k_seam_c<T, false, true, true>)
                    : (first ? k_seam_c<T, true, false, true> : k_seam_c<T, false, false, true>))
           : (delta ? (first ? k_seam_c<T, true, true, false> : k_seam_c<T, false, true, false>)
                    : (first ? k_seam_c<T, true, false, false> : k_seam_c<T, false, false, false>));
    hipLaunchKernelGGL(kern, grid, dim3(kThreads), 0, s, p);
    HIP_OK(hipGetLastError());
}
template void launch_seam_c<double>(bool, bool, bool, const SeamCPlane<double>*, int, const GridView&, const Box&,
                                    const StepCoefs&, hipStream_t);
template void launch_seam_c<float>(bool, bool, bool, const SeamCPlane<float>*, int, const GridView&, const Box&,
                                   const StepCoefs&, hipStream_t);

#define W3D_TB3_INST(T)                                                                       \
    template void launch_tb3<T>(int, int, bool, bool, bool, const T*, const T*, T*, T*, const GridView&, \
                                const Box*, int, const Box&, int, int, const Wrap&,           \
                                const Wrap&, const SeamPartners<T>&, const T*,                \
                                const T*, const T*, const T*, const StepCoefs&, const StepCoefs&, \
                                const StepCoefs&, u64*, u64*, u64*, int, hipStream_t);
W3D_TB3_INST(double)
W3D_TB3_INST(float)

}  // namespace wave3d
