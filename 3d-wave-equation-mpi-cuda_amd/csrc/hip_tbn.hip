// Deep temporal blocking: D leapfrog layers per sweep (TBN, D = 3 or 4) on CDNA4.
//
// One sweep reads A = u^{m-1} and B = u^{m-2} and writes only the last two layers
// U_{D-2} = u^{m+D-2} and U_{D-1} = u^{m+D-1} (the next sweep's B and A); the layers before them
// live in registers and LDS (their errors are still reduced). HBM traffic is 32 B per node per
// D layers: 10.7 B per layer at D = 3 (hip_tb3.hip), 8 B at D = 4 — against 24 for one layer
// per pass (the reference's loop, mpi_new.cpp:335-347 / cuda_sol_kernels.cu:24-47).
//
// Workgroup = NW wave64s owning a (NW*R rows) x 64 tile of U_{D-1} that marches along i. Layer
// l is evaluated l planes behind layer 0, on a (D-1-l)-node ring around the tile (redundantly
// with the neighbour tiles; identical operations, so bitwise equal):
//   iteration i:  wait for A(i+1), B(i) -> barrier -> LDS-DMA of B(i+1), A(i+2)
//                 U_0(i)       on tile + (D-1)-ring  from A(i-1..i+1), B(i)
//                 U_l(i - l)   on tile + (D-1-l)-ring from U_{l-1} (staged last iteration) and
//                              U_{l-2} (A for l = 1) of the same plane
//
// Staging (gfx950 LDS-DMA, buffer_load_dword ... lds): A and B never pass through VGPRs. Every
// A plane (tile + D-ring: (TJ+2D) x (64+2D) values) lands in a 4-slot LDS ring, every B plane
// (tile + (D-1)-ring) in a 2-slot ring, each row as 256-B pieces (64 lanes x 4 B, lane-linear
// into the odd-pitch frame row); all of a plane's A/B reads — centre, x+-1 planes, y/z
// neighbours — are LDS reads. The loads are invisible to the compiler (inline asm), so its own
// s_waitcnt never drains them; each iteration waits with a counted vmcnt for the pieces issued
// one iteration earlier (the stores issued after them stay in flight) and crosses one barrier.
// Compared with register staging (round 4: 248 VGPRs, A/B prefetch slots + ds_write of A) this
// frees the prefetch registers and the staging writes, and the ring's column halos are read as
// rows (256-B pieces) instead of one 8-B lane per row.
//
// The U frames are double-buffered (layer l reads U_{l-1} of the last iteration while writing
// its own), so one barrier per plane. Register state sits in slots indexed by plane number mod
// 4 with the i loop unrolled by 4 (no copies): U_l(x) lives in slot (x + l - i0) & 3.
//
// Ring ownership (as k_tb3): every computed ring node belongs to ONE thread, RP positions per
// thread, in the order rings 1..D-2 whole, ring D-1 without its corners (no later layer reads
// layer 0 there). With 16-row tiles the positions of D = 4 are exactly 512 (one per thread of
// 8 waves). A slot whose first possible ring is r only carries the history of the layers
// evaluated on ring r (compile-time).
//
// Periodic seam (the reference keeps both x = 0 and x = N, mpi_new.cpp:170-176): at plane an_i
// (the ghost copy of global N-1) the x+ neighbour of layer l is the partner plane nP[l] — A at
// x = N for layer 0, U_{l-1} evaluated there (launch_seam_c, before the sweep) for l >= 1 —
// and mirrored at ap_i; separate, rarely taken instantiation of the plane body.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <type_traits>
#include <utility>

#include "device_common.hpp"

// Timing ablation (wrong error tables): no error reduction in the planes (what the fused errors
// cost: profiles/deep_sweeps_r5.txt)
#ifndef W3D_TBN_ABL_ERR
#define W3D_TBN_ABL_ERR 0
#endif

// W3D_TBN_PART 2 (hip_tbn_exact.hip): only the --math exact instantiations, in an object of
// their own under LLVM's max-memory-clause scheduler; the fma ones keep max-ilp (Makefile,
// profiles/deep_sweeps_r5.txt step 16)
#ifndef W3D_TBN_PART
#define W3D_TBN_PART 1
#endif

namespace wave3d {
// the --math exact kernel of a depth / first-sweep / scheme (hip_tbn_exact.hip), a kernel stub
template <class T>
const void* tbn_exact_kernel(int depth, bool first, bool delta);

namespace {

template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
// f(integral_constant<0>) .. f(integral_constant<N-1>), unrolled at compile time
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}
template <int V>
using Ic = std::integral_constant<int, V>;

template <class T>
struct TbnParams {
    // level bases pre-biased on the host: plane i's block starts at base + (i + pbias) * pbytes
    const char* A;
    const char* B;
    char* O[2];  // U_{D-2}, U_{D-1}
    unsigned pbytes;
    int pbias;
    int order;  // tile order (tile_order(), as k_tb3)
    int sj;
    int poff;
    int jmin, jmax, kmin, kmax;  // storage bounds (logical)
    int cj0, cj1, ck0, ck1;      // stencil-valued region (0 outside: Dirichlet)
    int nbox;
    BoxLaunch box[kMaxBoxes];
    int ei0, ei1;
    int w_lo[2][2], w_hi[2][2], w_sh[2][2];  // self-wrap of O[0] (depth D-1) and O[1] (depth D)
    int an_i, ap_i;
    const T* nP[kTbnMaxDepth - 1];  // x+ partners at an_i: A, then U_0 .. U_{D-3} (logical planes)
    const T* pP[kTbnMaxDepth - 1];  // x- partners at ap_i
    const T* txy;  // sx*sy rows (launch_txy)
    int tpj;
    const T* tz;
    const T* txr;  // --math fma: (sx sy, 1/|sx sy|) pairs and 1/|tz|
    const T* rtz;
    T hx2, hy2, hz2, yx2, yy2, yz2;
    T coef[kTbnMaxDepth], ct[kTbnMaxDepth];
    T fc[2][3];  // --math fma: coef/h^2 per axis of layer 0 (fc[0]) and of every later layer
    T ict[kTbnMaxDepth];
    u64* err[kTbnMaxDepth];
};

// Tile geometry of a D-layer sweep over TJ x 64 tiles of ES-byte values on NW waves
// (coordinates in the "A frame": row y = j - jt + D, column x = k - kb + D).
template <int D, int TJ, int ES, int NW>
struct TbnGeom {
    // staged layer s: 0 = A (ring D), s >= 1 = U_{s-1} (ring D - s); frame origin (s, s)
    static constexpr int H(int s) { return TJ + 2 * (D - s); }
    // row pitch: the staged width rounded up to odd, so the lanes of a ring column (one k,
    // consecutive rows) hit 32 distinct ds_read_b64 bank pairs (an even pitch of 72 doubles put
    // 8 rows on one pair: 4.6x the bank-conflict cycles of k_tb3 in the first tb4 PMC; 74 still
    // 2-way: twice the conflict cycles of 73 in the LDS-DMA build). The fp64 A/B slots' rows are
    // filled by 16-B DMA pieces from an 8-B-aligned LDS row start every other row: the gfx950
    // LDS-DMA writes them in place (tools/microbench/lds_dma_probe.hip, case E).
    static constexpr int W(int s) { return (kTK + 2 * (D - s)) | 1; }
    static constexpr int cells(int s) { return H(s) * W(s); }
    static constexpr int at(int s, int y, int x) { return (y - s) * W(s) + (x - s); }
    // A slots: the A frame rounded up to RPW rows per wave (rows past the frame are loaded and
    // never read). B (= u^{m-2}, read by layer 0 on the tile + (D-1)-ring only): the same rows,
    // columns 1 .. 64+2D-2 of the A frame at the U_0 frame's pitch W(1): B(y, x) at y W(1) + x - 1
    static constexpr int RPW = (H(0) + NW - 1) / NW;
    static constexpr int scells = RPW * NW * W(0);
    static constexpr int bcells = RPW * NW * W(1);
    static constexpr int rowb = (kTK + 2 * D) * ES;         // bytes an A row's DMA moves
    static constexpr int browb = (kTK + 2 * D - 2) * ES;    // ... a B row's
    static constexpr int bat(int y, int x) { return y * W(1) + x - 1; }
    // one-array layout (fp32): A slots 0..3, B slots 0..2, then U_{s-1} frames x 2 buffers
    static constexpr int a_off(int q) { return q * scells; }
    static constexpr int b_off(int q) { return 4 * scells + q * bcells; }
    static constexpr int u_off(int s, int h) {
        return s == 1 ? b_off(2) + h * cells(1) : u_off(s - 1, 1) + cells(s - 1) + h * cells(s);
    }
    static constexpr int total = u_off(D - 1, 1) + cells(D - 1);
    // computed positions of ring r: rings 1..D-2 whole, D-1 without corners
    static constexpr int npos(int r) {
        return 2 * (kTK + 2 * (r - 1)) + 2 * (TJ + 2 * (r - (r == D - 1 ? 1 : 0)));
    }
    static constexpr int first(int r) { return r <= 1 ? 0 : first(r - 1) + npos(r - 1); }
    static constexpr int ncomp = first(D);
    // ring of position q (D: none)
    static constexpr int ring_of(int q) {
        int r = 1;
        while (r < D && q >= first(r + 1)) ++r;
        return r;
    }
};

// LDS byte address of a __shared__ object (the DMA destination base in M0)
template <class T>
__device__ __forceinline__ unsigned lds_addr(T* ptr) {
    return static_cast<unsigned>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) T*)ptr));
}
// LDS-DMA fill of a wave's three consecutive slot rows (probed on gfx950, tools/microbench/
// lds_dma_probe.hip: the destination is M0 + instruction offset + size * lane, the source moves
// by the instruction offset too, out-of-range lanes write 0, masked lanes nothing). Row q: source
// src0 + q sjb (+ lane piece), LDS slot + lds0 + q ROWB.
//   fp64: one buffer_load_dwordx4 per row (rowb / 16 lanes, 16 B each);
//   fp32: two buffer_load_dword per row (256 B, then the rowb - 256 B tail; odd pitch).
// One asm statement per fill, so hipcc neither counts nor drains the pieces (vmcnt is ours:
// vm_wait) and nothing per row is hoisted into SGPRs. M0 is written in the statement that reads
// it (hipcc keeps nothing in M0 in these kernels: no M0 use outside these statements); the
// s_add's write SCC, declared clobbered (or hipcc may split a 64-bit s_add_u32 / s_addc_u32 pair,
// a plane descriptor's base, around the statement).
template <int ES, int ROWB, int RB>
__device__ __forceinline__ void dma_fill3(__amdgpu_buffer_rsrc_t r, unsigned src0, unsigned sjb, unsigned slot,
                                          unsigned lds0) {
    unsigned v0, v1, v2;
    u64 keep;
    const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    if constexpr (ES == 8) {
        static_assert(RB % 16 == 0 && RB <= 1024, "fp64 rows: one dwordx4 piece per lane");
        asm volatile(
            "s_add_u32 m0, %[slot], %[lds0]\n\t"
            "v_add_u32 %[v0], %[src0], %[l16]\n\t"
            "v_add_u32 %[v1], %[sjb], %[v0]\n\t"
            "v_add_u32 %[v2], %[sjb], %[v1]\n\t"
            "s_mov_b64 %[keep], exec\n\t"
            "s_mov_b64 exec, %[mask]\n\t"
            "buffer_load_dwordx4 %[v0], %[rs], 0 offen lds\n\t"
            "s_add_u32 m0, m0, %[rowb]\n\t"
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %[v1], %[rs], 0 offen lds\n\t"
            "s_add_u32 m0, m0, %[rowb]\n\t"
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %[v2], %[rs], 0 offen lds\n\t"
            "s_mov_b64 exec, %[keep]"
            : [v0] "=&v"(v0), [v1] "=&v"(v1), [v2] "=&v"(v2), [keep] "=&s"(keep)
            : [slot] "s"(slot), [lds0] "s"(lds0), [src0] "s"(src0), [sjb] "s"(sjb), [l16] "v"(16u * lane),
              [rs] "s"(r), [rowb] "i"(ROWB), [mask] "s"(u64(RB / 16 >= 64 ? ~0ull : (1ull << (RB / 16)) - 1))
            : "memory", "scc");
    } else {
        static_assert(RB > 256 && RB <= 512 && RB % 4 == 0, "fp32 rows: 256 B + a tail");
        asm volatile(
            "s_add_u32 m0, %[slot], %[lds0]\n\t"
            "v_add_u32 %[v0], %[src0], %[l4]\n\t"
            "v_add_u32 %[v1], %[sjb], %[v0]\n\t"
            "v_add_u32 %[v2], %[sjb], %[v1]\n\t"
            "buffer_load_dword %[v0], %[rs], 0 offen lds\n\t"
            "s_add_u32 m0, m0, %[rowb]\n\t"
            "s_nop 0\n\t"
            "buffer_load_dword %[v1], %[rs], 0 offen lds\n\t"
            "s_add_u32 m0, m0, %[rowb]\n\t"
            "s_nop 0\n\t"
            "buffer_load_dword %[v2], %[rs], 0 offen lds\n\t"
            "s_mov_b64 %[keep], exec\n\t"
            "s_mov_b64 exec, %[mask]\n\t"
            "buffer_load_dword %[v2], %[rs], 0 offen offset:256 lds\n\t"
            "s_sub_u32 m0, m0, %[rowb]\n\t"
            "s_nop 0\n\t"
            "buffer_load_dword %[v1], %[rs], 0 offen offset:256 lds\n\t"
            "s_sub_u32 m0, m0, %[rowb]\n\t"
            "s_nop 0\n\t"
            "buffer_load_dword %[v0], %[rs], 0 offen offset:256 lds\n\t"
            "s_mov_b64 exec, %[keep]"
            : [v0] "=&v"(v0), [v1] "=&v"(v1), [v2] "=&v"(v2), [keep] "=&s"(keep)
            : [slot] "s"(slot), [lds0] "s"(lds0), [src0] "s"(src0), [sjb] "s"(sjb), [l4] "v"(4u * lane),
              [rs] "s"(r), [rowb] "i"(ROWB), [mask] "s"(u64((1ull << ((RB - 256) / 4)) - 1))
            : "memory", "scc");
    }
}
// LDS read of t[o] for the layer gathers: volatile, so LLVM neither sinks it into the branch
// that consumes it (the ring nodes': behind the own nodes' LDS writes, a second LDS round trip
// per layer) nor pairs two of them into a ds_read2_b64, which moves 16 B per lane in 8 LDS
// cycles where two ds_read_b64 take 4 (MI355X LDS rates; 13 pairs per plane before: +3-4 %,
// profiles/deep_sweeps_r5.txt). Through an LDS-address-space pointer: a volatile generic access
// would be a flat load.
template <class T>
__device__ __forceinline__ T ldsr(const T* t, int o) {
    using LP = const volatile __attribute__((address_space(3))) T*;
    return ((LP)(t))[o];
}
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// DELTA: the increment form (as k_tb3's): B = d^{m-1}; layer l keeps d_l = d_{l-1} + coef lap U_{l-1}
// (d_{-1} = B, U_{-1} = A) and U_l = U_{l-1} + d_l; d is pointwise, so it rides in registers from
// one layer to the next (same plane, next iteration) and never in LDS. The sweep stores d and U of
// its last layer (O[0] = the next sweep's B, O[1] its A), with the last layer's self-wrap ranges.
template <class T, int D, bool FIRST, int R, int NW, bool FM, bool DELTA = false>
// fp32: at least 4 waves per SIMD, i.e. two workgroups per CU (LDS 75 KB each): the increment
// form's 132 VGPRs had dropped it to one (634k vs 872-878k Mpts/s at N=512, deep_sweeps_r5.txt)
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 4 ? 4 : 1, 8)))
k_tbn(const TbnParams<T> p) {
    constexpr int TJ = NW * R;
    constexpr int ES = sizeof(T);
    using Gm = TbnGeom<D, TJ, ES, NW>;
    constexpr int NT = NW * 64;
    constexpr int RP = (Gm::ncomp + NT - 1) / NT;  // computed ring positions per thread
    constexpr int NU = D - 1;                      // own history: U_0 .. U_{D-2}
    constexpr int NRU = D >= 3 ? D - 2 : 1;        // ring history: U_0 .. U_{D-3}
    constexpr int W0 = Gm::W(0);
    // Staged tiles: fp64 one __shared__ object per (layer, buffer) / DMA slot — distinct objects
    // cannot alias, so the compiler may hoist a layer's LDS reads above the previous layer's
    // writes; fp32 one array (measured faster there, profiles/deep_sweeps_r4.txt batches 21/30)
    constexpr bool ONE = sizeof(T) == 4;
    __shared__ T lds[ONE ? Gm::total : 1];
    constexpr int ZA = ONE ? 1 : Gm::scells, ZB = ONE ? 1 : 2 * Gm::bcells, Z1 = ONE ? 1 : Gm::cells(1);
    constexpr int Z2 = ONE || D <= 2 ? 1 : Gm::cells(2), Z3 = ONE || D <= 3 ? 1 : Gm::cells(3);
    __shared__ T tA0[ZA], tA1[ZA], tA2[ZA], tA3[ZA], tB[ZB];
    __shared__ T t10[Z1], t11[Z1], t20[Z2], t21[Z2], t30[Z3], t31[Z3];
    // A slot q / B slot q (A-frame offsets) / U_{s-1} frame s, buffer h
    auto Ap = [&](auto qc) -> T* {
        constexpr int q = decltype(qc)::value;
        if constexpr (ONE) return lds + Gm::a_off(q);
        else if constexpr (q == 0) return tA0;
        else if constexpr (q == 1) return tA1;
        else if constexpr (q == 2) return tA2;
        else return tA3;
    };
    // B slot q (B(x) in slot (x - i0) & 1)
    auto Bp = [&](int q) -> T* {
        if constexpr (ONE) return lds + Gm::b_off(0) + q * Gm::bcells;
        else return tB + q * Gm::bcells;
    };
    auto Up = [&](auto sc, auto hc) -> T* {
        constexpr int s = decltype(sc)::value, h = decltype(hc)::value;
        if constexpr (ONE) return lds + Gm::u_off(s, h);
        else if constexpr (s == 1) return h ? t11 : t10;
        else if constexpr (s == 2) return h ? t21 : t20;
        else return h ? t31 : t30;
    };

    const int bid = blockIdx.x;
    const int b = find_box(p, bid);
    const BoxLaunch Bx = p.box[b];
    int local = bid - Bx.block_begin;
    int tk, tj;
    if (p.order == 3 && Bx.tiles_j % 4 == 0 && Bx.tiles_k % 2 == 0) {
        // XCD blocks: the 8 XCDs tile the (j, k) tile grid 4 x 2, XCD x running a block of
        // tiles_j/4 rows x tiles_k/2 k-tiles for every chunk (fewer tile edges between XCDs,
        // whose halo lines each XCD's L2 fetches separately, than the full-width bands)
        const int x = local % kXcds, bh = Bx.tiles_j / 4, bw = Bx.tiles_k / 2;
        local /= kXcds;
        tj = (x >> 1) * bh + local % bh;
        local /= bh;
        tk = (x & 1) * bw + local % bw;
        local /= bw;
    } else if (p.order == 2 && Bx.tiles_j % kXcds == 0) {
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
    const int i0 = ib - (D - 1);  // first iteration (layer 0 of plane i0)
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sj = p.sj;
    const unsigned pbytes = p.pbytes;

    auto inb = [&](int j, int k) { return j >= p.jmin && j <= p.jmax && k >= p.kmin && k <= p.kmax; };
    auto incd = [&](int j, int k) { return j >= p.cj0 && j <= p.cj1 && k >= p.ck0 && k <= p.ck1; };
    auto boff = [&](int j, int k, bool ok) { return ok ? unsigned(j * sj + k + p.poff) * ES : kOOB; };
    auto prs = [&](const char* base, int i, unsigned nb) {
        return plane_rsrc(base + u64(unsigned(i + p.pbias)) * pbytes, nb);
    };
    auto lrs = [&](const T* plane) { return plane_rsrc(plane - p.poff, pbytes); };

    // ---- own nodes ------------------------------------------------------------------------
    const int k = kb + lane;
    unsigned oa[R], os[R];  // seam-partner loads (ALIAS body), stores
    bool ovalid[R], ocd[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int j = jt + w * R + r;
        ocd[r] = incd(j, k);
        ovalid[r] = k >= Bx.k0 && k <= Bx.k1 && j <= Bx.j1;
        oa[r] = boff(j, k, inb(j, k));
        os[r] = boff(j, k, ovalid[r]);
    }
    const T ortz = FM && k >= Bx.k0 && k <= Bx.k1 ? p.rtz[k] : T(0);
    const T* const txw = p.txy + (jt + w * R);
    // om: 1 on valid own nodes, 0 on masked lanes (the non-finite detector); otzr: sz, a quiet
    // NaN on masked lanes — their analytic values and so their errors are NaN, which max_abs,
    // RelMax and RelArg ignore (no product or branch per node: profiles/deep_sweeps_r5.txt)
    T om[R], otzr[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        om[r] = ovalid[r] ? T(1) : T(0);
        otzr[r] = nan_unless(ovalid[r], k >= Bx.k0 && k <= Bx.k1 ? p.tz[k] : T(0));
    }
    // self-wrap ranges of O[0] / O[1] met by this work item (wave-uniform bits)
    int rare = 0;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        if (p.w_lo[0][g] <= ie && p.w_hi[0][g] >= ib) rare |= 1;
        if (p.w_lo[1][g] <= ie && p.w_hi[1][g] >= ib) rare |= 2;
    }
    rare = __builtin_amdgcn_readfirstlane(rare);
    // steady-state window [flo, fhi]: every layer on an own-range plane, A(i+3) / B(i+1) still
    // inside the work item, off the periodic seam and the self-wrap planes (those sit at the
    // ends of the x range, so each one trims the window from its nearer end)
    int flo = ib + D - 1, fhi = ie + D - 3;
    auto cut = [&](int lo, int hi) {
        if (lo > hi || hi < flo || lo > fhi) return;
        if (lo - flo <= fhi - hi) flo = hi + 1;
        else fhi = lo - 1;
    };
    // ... and inside the error planes [ei0, ei1] (the periodic x planes 0 and N are outside), so
    // the steady-state body takes the errors of every plane without a range test
    flo = max(flo, p.ei0 + D - 1), fhi = min(fhi, p.ei1 + D - 1);
    cut(p.an_i, p.an_i + D - 2);
    cut(p.ap_i, p.ap_i + D - 2);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        // O[0]'s stores run at iteration x + D - 2 (leapfrog: U_{D-2}) or x + D - 1 (DELTA: d_{D-1})
        cut(p.w_lo[0][g] + (DELTA ? D - 1 : D - 2), p.w_hi[0][g] + (DELTA ? D - 1 : D - 2));
        cut(p.w_lo[1][g] + D - 1, p.w_hi[1][g] + D - 1);
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
    int rg[RP], ro0[RP], rb0[RP];  // ring (0: none), A-frame and B-slot offsets
    unsigned ra_off[RP];  // seam-partner load offsets (kOOB when masked)
    bool rcd[RP];         // stencil-valued node (else 0: Dirichlet face)
    int ry[RP], rx[RP];
#pragma unroll
    for (int s = 0; s < RP; ++s) {
        const int q = threadIdx.x + s * NT;
        int g = 0, rj = jt, rk = kb;
#pragma unroll
        for (int d = 1; d < D; ++d)
            if (g == 0 && q < Gm::first(d + 1)) {
                g = d;
                ring(d, d == D - 1 ? 1 : 0, q - Gm::first(d), rj, rk);
            }
        rg[s] = g;
        ry[s] = rj - jt + D, rx[s] = rk - kb + D;
        ro0[s] = Gm::at(0, ry[s], rx[s]);
        rb0[s] = Gm::bat(ry[s], rx[s]);
        rcd[s] = g != 0 && incd(rj, rk);
        ra_off[s] = boff(rj, rk, g != 0 && inb(rj, rk));
    }

    // ---- LDS-DMA staging of A and B -------------------------------------------------------
    // wave w fills slot rows w*RPW .. w*RPW + RPW-1 of A and B alike (rows past the frame are
    // loaded and never read). Frame rows past the storage read 0 (past the plane's num_records)
    // and frame columns past it the finite row padding / next row: both only ever feed nodes
    // outside the stencil-valued region (masked to 0).
    static_assert(Gm::RPW == 3, "dma_fill3: three slot rows per wave");
    const unsigned sjb = unsigned(sj) * ES;
    const unsigned src0 = unsigned((jt - D + w * Gm::RPW) * sj + kb - D + p.poff) * ES;
    const unsigned lds0 = unsigned(w * Gm::RPW * W0 * ES), bds0 = unsigned(w * Gm::RPW * Gm::W(1) * ES);
    auto fillA = [&](auto qc, int plane, bool live) {
        dma_fill3<ES, W0 * ES, Gm::rowb>(prs(p.A, plane, live ? pbytes : 0u), src0, sjb, lds_addr(Ap(qc)), lds0);
    };
    auto fillB = [&](int q, int plane, bool live) {
        dma_fill3<ES, Gm::W(1) * ES, Gm::browb>(prs(p.B, plane, live ? pbytes : 0u), src0 + ES, sjb,
                                                __builtin_amdgcn_readfirstlane(lds_addr(Bp(q))), bds0);
    };
    // Two planes of lookahead for A, one for B: A(x) in A slot (x - i0) & 3 — A(i), A(i+1) read
    // at iteration i, A(i+2) in flight, A(i+3) issued into the slot of A(i-1), whose own-node and
    // ring values ride in registers from the last iteration (aw / raw: its x- neighbour for layer
    // 0, U_{-1} for layer 1); B(x) in B slot (x - i0) & 1 — B(i) read, B(i+1) issued into the slot
    // of B(i-1). Each iteration issues its B piece first, then its A pieces, then its stores; a
    // steady iteration waits for B(i) and what came before it, i.e. for all but the A pieces and
    // stores of iteration i-1: NA + NST (the first sweep, with no B: NDMA + 2 NST).
    constexpr int NST = 2 * R;                                  // stores of the last two layers
    // pieces per iteration: A, and B unless this is the first sweep (which reads no B)
    constexpr int NDMA = (ES == 8 ? 1 : 2) * Gm::RPW * (FIRST ? 1 : 2);
    // prologue: A(i0-1) .. A(i0+2) into slots 3, 0, 1, 2; B(i0) into slot 0; then
    // A(i0-1)'s register copies
    fillA(Ic<3>{}, i0 - 1, true);
    fillA(Ic<0>{}, i0, true);
    fillA(Ic<1>{}, i0 + 1, true);
    fillA(Ic<2>{}, i0 + 2, true);
    if constexpr (!FIRST) fillB(0, i0, true);
    vm_wait<0>();
    __syncthreads();
    T aw[2][R], raw[2][RP];  // A of the own rows / ring slots in a plane-parity slot (iteration i: A(i) in i - i0 & 1)
#pragma unroll
    for (int r = 0; r < R; ++r) aw[0][r] = T(0), aw[1][r] = ldsr(Ap(Ic<3>{}), Gm::at(0, D + w * R + r, D + lane));
#pragma unroll
    for (int s = 0; s < RP; ++s) raw[0][s] = T(0), raw[1][s] = ldsr(Ap(Ic<3>{}), ro0[s]);

    // slots (iteration i = i0 + q, phase P = q & 3): U_l(x) (x + l - i0) & 3 -> U_l of this
    // iteration in P, of the last in P+3, of the one before in P+2
    T u[NU][4][R];
    T ru[RP][NRU][4];
#pragma unroll
    for (int l = 0; l < NU; ++l)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < R; ++r) u[l][t][r] = T(0);
#pragma unroll
    for (int s = 0; s < RP; ++s)
#pragma unroll
        for (int l = 0; l < NRU; ++l)
#pragma unroll
            for (int t = 0; t < 4; ++t) ru[s][l][t] = T(0);

    // Dirichlet-face masks of the computed values: a product with a 0/1 register (one op; a
    // face value may become -0)
    T ocm[R], rcm[RP];
#pragma unroll
    for (int r = 0; r < R; ++r) ocm[r] = ocd[r] ? T(1) : T(0);
#pragma unroll
    for (int s = 0; s < RP; ++s) rcm[s] = rcd[s] ? T(1) : T(0);
    // increment form: d_l of the own rows / ring slots in a plane-parity slot (written at
    // iteration i for plane i - l, read by layer l+1 at iteration i+1: the same plane)
    constexpr int ND = DELTA ? D - 1 : 1, NRD = DELTA && D >= 3 ? D - 2 : 1;
    T dq[ND][2][R], rdq[RP][NRD][2];
#pragma unroll
    for (int l = 0; l < ND; ++l)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
            for (int r = 0; r < R; ++r) dq[l][h][r] = T(0);
#pragma unroll
            for (int s = 0; s < RP; ++s) rdq[s][l < NRD ? l : 0][h] = T(0);
        }
    using Rel = std::conditional_t<FM, RelMax<T>, RelArg<T>>;  // fma: |d| * 1/|f| max
    T ma[D], chk[D];
    Rel mr[D];
#pragma unroll
    for (int l = 0; l < D; ++l) ma[l] = T(kErrInit), chk[l] = T(0);

    // layer-l arithmetic: lap() = Laplacian (exact) or the deferred coef*Laplacian (FM, FmLap:
    // the leapfrog takes it whole, stencil_math leap_fm); upd() = the Taylor start (layer 0 of
    // the first sweep) or the leapfrog from it
    const T kc1 = FM ? fm_kc(p.fc[1][0], p.fc[1][1], p.fc[1][2]) : T(0);
    auto lap = [&](auto lc, T ctr, T xm, T xp, T ym, T yp, T zm, T zp) {
        constexpr int l = decltype(lc)::value;
        if constexpr (FM) {
            constexpr int f = FIRST && l == 0 ? 0 : 1;
            return FmLap<T>{ctr, xm, xp, ym, yp, zm, zp, p.fc[f][0], p.fc[f][1], p.fc[f][2]};
        } else {
            return laplace7_cr(ctr, xm, xp, ym, yp, zm, zp, p.hx2, p.hy2, p.hz2, p.yx2, p.yy2, p.yz2);
        }
    };
    // increment form: d_l from d_{l-1} (FIRST layer 0: coef*lap alone)
    auto dnew = [&](auto lc, T dprev, const auto& l_) {
        constexpr int l = decltype(lc)::value;
        if constexpr (FM) {
            if constexpr (FIRST && l == 0) return lap_value(l_);
            else return dprev + lap_value(l_);
        } else {
            if constexpr (FIRST && l == 0) return p.coef[0] * l_;
            else return delta_incr(dprev, l_, p.coef[l]);
        }
    };
    // The Dirichlet mask (m = 1 computed, 0 face / outside): layers 0 and 1 take c or u2 from
    // memory, whose faces may hold the initial condition's analytic values (~1e-16, as in the
    // reference), so they multiply the result by m. From layer 2 on both come from masked
    // layers (exactly 0 there), and m rides in the last operation instead: fma(l, m, 2c - u2)
    // (fma) or the masked coefficient coef*m (exact: bitwise the same products for m = 1)
    // — no product per node (profiles/deep_sweeps_r5.txt)
    auto upd = [&](auto lc, T ctr, T pw, const auto& l_, T m) {
        constexpr int l = decltype(lc)::value;
        if constexpr (FM) {
            if constexpr (FIRST && l == 0) return (ctr + lap_value(l_)) * m;
            else if constexpr (l <= 1) return l_.leap(pw, kc1) * m;
            else return l_.leap_masked(pw, kc1, m);
        } else {
            if constexpr (FIRST && l == 0) return taylor_first(ctr, l_, p.coef[0]) * m;
            else if constexpr (l <= 1) return leapfrog(ctr, pw, l_, p.coef[l]) * m;
            else return leapfrog(ctr, pw, l_, p.coef[l] * m);  // loop-invariant product
        }
    };

    // Errors of every layer are taken at plane i - (D-1), when all D values of that plane are
    // in registers: one analytic-table row per plane (f = ((sx sy) sz) ct per layer, stencil_math
    // analytic()), loaded an iteration ahead into a plane-parity slot (a scalar load). --math fma:
    // the (sx sy, 1/|sx sy|) pair (txr); exact: sx sy (txy).
    constexpr int NQ = FM ? 2 : 1;
    T tq[2][R][NQ];
    auto load_row = [&](auto slotc, int q) {  // slot as a constant: tq stays in registers
        constexpr int slot = decltype(slotc)::value;
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

    auto plane = [&](auto phase, auto alias, const int i) {
        constexpr int P = decltype(phase)::value;
        constexpr bool ALIAS = decltype(alias)::value;
        constexpr bool FAST = !ALIAS;
        constexpr int S0 = P & 3, S1 = (P + 1) & 3, S2 = (P + 2) & 3, S3 = (P + 3) & 3;
        constexpr int H0 = P & 1, H1 = (P + 1) & 1;
        // A(i) .. A(i+3) in A slots S0 .. S3; B(i) in B slot H0, B(i+1) into H1 (two B slots, B
        // issued first: +0.6 % fma, +1.2 % exact against three slots with two planes of
        // lookahead, profiles/deep_sweeps_r5.txt)

        // ---- what iteration i-2 issued has landed (A(i+1); the checked body waits for
        // everything), and B(i), which iteration i-1 issued first (wait for it and what came
        // before, leaving its A pieces and stores in flight) -> barrier -> DMA B(i+1), A(i+3)
        // into the slots of B(i-1), A(i-1), whose last readers passed the barrier
        constexpr int NA = (ES == 8 ? 1 : 2) * Gm::RPW;
        if constexpr (FAST && !FIRST) vm_wait<NA + NST>();
        else if constexpr (FAST) vm_wait<NDMA + 2 * NST>();
        else vm_wait<0>();
        __syncthreads();
        // (issued right here: later in the plane measured 7-16 % slower)
        if constexpr (!FIRST) fillB(H1, i + 1, FAST || i + 1 <= ie + D - 1);
        fillA(Ic<S3>{}, i + 3, FAST || i + 3 <= ie + D);

        T ev[R];  // U_{D-1}(i - D + 1): stored and its errors taken below
#pragma unroll
        for (int r = 0; r < R; ++r) ev[r] = T(0);
        // staged layer l at frame offset o: A(i) for layer 0, U_{l-1} of the last iteration else
        auto St = [&](auto lc, int o) -> T {
            constexpr int l = decltype(lc)::value;
            if constexpr (l == 0) return ldsr(Ap(Ic<S0>{}), o);
            else return ldsr(Up(lc, Ic<H1>{}), o);
        };
        // ---- a layer's LDS reads, own nodes and ring together (one LDS round trip per layer);
        // issuing the next layer's ahead of this layer's arithmetic measured no faster, even
        // with the registers for it (profiles/deep_sweeps_r5.txt)
        struct Gath {
            T gy[R][2], gz[R][2], gc[R], gxp[R], gpw[R];
            T grn[RP][4], grc[RP], grxp[RP], grpw[RP];
        };
        Gath gt[2];
        auto gather = [&](auto lc) {
            constexpr int l = decltype(lc)::value;
            constexpr int Wl = Gm::W(l);
            Gath& g = gt[l & 1];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int y = D + w * R + r, xx = D + lane;
                const int o = Gm::at(l, y, xx), oA = Gm::at(0, y, xx);
                if (r == 0) g.gy[r][0] = St(lc, o - Wl);
                if (r == R - 1) g.gy[r][1] = St(lc, o + Wl);
                g.gz[r][0] = St(lc, o - 1), g.gz[r][1] = St(lc, o + 1);
                if constexpr (l == 0) {
                    g.gc[r] = ldsr(Ap(Ic<S0>{}), oA), g.gxp[r] = ldsr(Ap(Ic<S1>{}), oA);
                    if constexpr (!FIRST) g.gpw[r] = ldsr(Bp(H0), Gm::bat(y, xx));
                }
            }
            if constexpr (l <= D - 2)
                sfor<RP>([&](auto sc) {
                    constexpr int s = decltype(sc)::value;
                    if constexpr (Gm::ring_of(s * NT) <= D - 1 - l) {
                        const int ro = Gm::at(l, ry[s], rx[s]);
                        g.grn[s][0] = St(lc, ro - Wl), g.grn[s][1] = St(lc, ro + Wl);
                        g.grn[s][2] = St(lc, ro - 1), g.grn[s][3] = St(lc, ro + 1);
                        if constexpr (l == 0) {
                            g.grc[s] = ldsr(Ap(Ic<S0>{}), ro0[s]), g.grxp[s] = ldsr(Ap(Ic<S1>{}), ro0[s]);
                            if constexpr (!FIRST) g.grpw[s] = ldsr(Bp(H0), rb0[s]);
                        }
                    }
                });
        };
        sfor<D>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            const int x = i - l;
            gather(lc);
            Gath& g = gt[l & 1];
            auto& gy = g.gy;
            auto& gz = g.gz;
            auto& gc = g.gc;
            auto& gxp = g.gxp;
            auto& gpw = g.gpw;
            auto& grn = g.grn;
            auto& grc = g.grc;
            auto& grxp = g.grxp;
            auto& grpw = g.grpw;
            // A(i) of the own rows and ring slot: next iteration's A(i-1) (register window)
            if constexpr (l == 0) {
#pragma unroll
                for (int r = 0; r < R; ++r) aw[H0][r] = gc[r];
#pragma unroll
                for (int s = 0; s < RP; ++s) raw[H0][s] = grc[s];
            }
            if (!(FAST || (x >= ib - (D - 1 - l) && x <= ie + (D - 1 - l)))) return;
            // ---- own nodes ----
            T v[R], dl[R];  // dl: the increment form's d of the last layer (stored to O[0])
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int y = D + w * R + r, xx = D + lane;
                T ctr, xm, xp, pw = T(0);
                if constexpr (l == 0) {
                    ctr = gc[r], xm = aw[H1][r], xp = gxp[r];
                    if constexpr (!FIRST) pw = gpw[r];
                } else {
                    ctr = u[l - 1][S3][r], xp = u[l - 1][S0][r], xm = u[l - 1][S2][r];
                    if constexpr (l == 1 && !DELTA) pw = aw[H1][r];  // U_{-1} = A(i-1)
                    else if constexpr (l >= 2) pw = u[l - 2][S2][r];
                }
                if constexpr (ALIAS && l <= D - 2) {
                    if (x == p.an_i) xp = bld<T>(lrs(p.nP[l]), oa[r]);
                    if (x == p.ap_i) xm = bld<T>(lrs(p.pP[l]), oa[r]);
                }
                // j neighbours inside the wave's R rows come from registers (the same values
                // as the staged tile), only the outer two from LDS
                auto ctr_of = [&](int q) { return l == 0 ? gc[q] : u[l > 0 ? l - 1 : 0][S3][q]; };
                const T ym = r > 0 ? ctr_of(r - 1) : gy[r][0];
                const T yp = r < R - 1 ? ctr_of(r + 1) : gy[r][1];
                const auto lp = lap(lc, ctr, xm, xp, ym, yp, gz[r][0], gz[r][1]);
                if constexpr (DELTA) {
                    const T dprev = l == 0 ? pw : dq[l > 0 ? l - 1 : 0][H1][r];
                    const T dv = dnew(lc, dprev, lp) * ocm[r];
                    v[r] = (ctr + dv) * ocm[r];
                    if constexpr (l <= D - 2) dq[l][H0][r] = dv;
                    else dl[r] = dv;
                } else {
                    v[r] = upd(lc, ctr, pw, lp, ocm[r]);
                }
                if constexpr (l <= D - 2) {
                    u[l][S0][r] = v[r];
                    Up(Ic<l + 1>{}, Ic<H0>{})[Gm::at(l + 1, y, xx)] = v[r];
                }
            }
            // ---- ring nodes (rings 1 .. D-1-l) ----
            if constexpr (l <= D - 2) {
                sfor<RP>([&](auto sc) {
                    constexpr int s = decltype(sc)::value;
                    if constexpr (Gm::ring_of(s * NT) <= D - 1 - l) {
                        if (rg[s] >= 1 && rg[s] <= D - 1 - l) {
                            T ctr, xm, xp, pw = T(0);
                            if constexpr (l == 0) {
                                ctr = grc[s], xm = raw[H1][s], xp = grxp[s];
                                if constexpr (!FIRST) pw = grpw[s];
                            } else {
                                ctr = ru[s][l - 1][S3], xp = ru[s][l - 1][S0], xm = ru[s][l - 1][S2];
                                if constexpr (l == 1 && !DELTA) pw = raw[H1][s];
                                else if constexpr (l >= 2) pw = ru[s][l - 2][S2];
                            }
                            if constexpr (ALIAS) {
                                if (x == p.an_i) xp = bld<T>(lrs(p.nP[l]), ra_off[s]);
                                if (x == p.ap_i) xm = bld<T>(lrs(p.pP[l]), ra_off[s]);
                            }
                            const auto lp = lap(lc, ctr, xm, xp, grn[s][0], grn[s][1], grn[s][2], grn[s][3]);
                            T cv;
                            if constexpr (DELTA) {
                                const T dprev = l == 0 ? pw : rdq[s][l > 0 ? l - 1 : 0][H1];
                                const T dv = dnew(lc, dprev, lp) * rcm[s];
                                cv = (ctr + dv) * rcm[s];
                                if constexpr (l <= D - 3) rdq[s][l][H0] = dv;
                            } else {
                                cv = upd(lc, ctr, pw, lp, rcm[s]);
                            }
                            if constexpr (l <= D - 3) ru[s][l][S0] = cv;
                            Up(Ic<l + 1>{}, Ic<H0>{})[Gm::at(l + 1, ry[s], rx[s])] = cv;
                        }
                    }
                });
            }
            // ---- stores of the last two layers (own planes, + periodic self-wrap); the increment
            // form stores d and U of the last layer (O[0] then has the last layer's wrap ranges) --
            auto put = [&](const int o, const T(&val)[R]) {
                const auto rd = prs(p.O[o], x, pbytes);
#pragma unroll
                for (int r = 0; r < R; ++r) bst<2>(val[r], rd, os[r]);
                if (!FAST && (rare & (1 << o))) {
#pragma unroll
                    for (int g = 0; g < 2; ++g)
                        if (x >= p.w_lo[o][g] && x <= p.w_hi[o][g]) {
                            const auto rw = prs(p.O[o], x + p.w_sh[o][g], pbytes);
#pragma unroll
                            for (int r = 0; r < R; ++r) bst<2>(val[r], rw, os[r]);
                        }
                }
            };
            if constexpr (DELTA ? l == D - 1 : l >= D - 2) {
                if (FAST || (x >= ib && x <= ie)) {
                    if constexpr (DELTA) put(0, dl);
                    put(DELTA ? 1 : l - (D - 2), v);
                }
            }
            if constexpr (l == D - 1) {
#pragma unroll
                for (int r = 0; r < R; ++r) ev[r] = v[r];
            }
        });

        // ---- errors of plane e = i - (D-1), every layer ----------------------------------------
        const int e = i - (D - 1);
        if ((FAST || (e >= ib && e <= ie)) && !W3D_TBN_ABL_ERR) {
            constexpr int HE = (P + 4 - (D - 1)) & 1;  // table row slot of plane e
            const bool eplane = FAST || (e >= p.ei0 && e <= p.ei1);
            // (sx sy) sz: NaN on masked lanes (otzr) and outside the error planes
            T fb[R], wq[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                fb[r] = tq[HE][r][0] * otzr[r];
                if (!FAST && !eplane) fb[r] = nan_unless(false, fb[r]);
                if constexpr (FM) wq[r] = tq[HE][r][NQ - 1] * ortz;
            }
            sfor<D>([&](auto lc) {
                constexpr int l = decltype(lc)::value;
                constexpr int SE = (P + 4 - (D - 1) + l) & 3;  // slot of U_l(e)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    T val;
                    if constexpr (l == D - 1) val = ev[r];
                    else val = u[l][SE][r];
                    // chk (the non-finite detector) on the last layer only: a NaN / Inf in layer
                    // l reaches U_{D-1} at the same node within the sweep (through the centre
                    // term, masked nodes included), so the sweep's last layer carries the flag
                    if constexpr (l == D - 1) chk[l] = fma_t(val, om[r], chk[l]);
                    if constexpr (FM) {
                        const T dv = val - fb[r] * p.ct[l];
                        ma[l] = max_abs(ma[l], dv);
                        mr[l].add(dv, wq[r]);
                    } else {
                        const T f = fb[r] * p.ct[l];
                        const T d = val - f;
                        ma[l] = max_abs(ma[l], d);
                        mr[l].add(d, f);
                    }
                }
            });
        }
        load_row(Ic<(P + 4 - (D - 1) + 1) & 1>{}, e + 1);
    };

    // i = i0 .. ie + D - 1 in three loops, each unrolled by 4 from phase 0 so every slot index
    // is a constant: the checked body (ALIAS: seam / wrap / work-item ends) up to the first
    // phase-0 plane of the steady window, the steady body over whole groups of 4 inside it, the
    // checked body for the rest. One loop choosing the body per plane kept every value of the
    // checked body live through the steady one: 337 SGPR spills and 249 VGPRs at D = 4, against
    // none and 196 for the steady body alone (round 4, register staging).
    const int iend = ie + D - 1;
    const int fstart = __builtin_amdgcn_readfirstlane(i0 + ((max(flo, i0) - i0 + 3) & ~3));
    // whole groups of 4 steady planes from fstart (none when the window is shorter)
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
    // one instance of the checked body: pass 0 runs it up to the steady window, then the steady
    // loop; pass 1 runs it to the end
#pragma nounroll
    for (int pass = 0; pass < 2; ++pass) {
        checked(i, pass == 0 ? min(fstart, iend + 1) : iend + 1);
        if (pass == 0 && i == fstart) {  // (a work item shorter than the window start ran through)
            // the steady body's counted wait assumes its two predecessors issued exactly their
            // pieces and NST stores; the checked body's stores may differ: drain them here
            vm_wait<0>();
            for (; i < fend; i += 4) {
                plane(Ph<0>{}, std::false_type{}, i);
                plane(Ph<1>{}, std::false_type{}, i + 1);
                plane(Ph<2>{}, std::false_type{}, i + 2);
                plane(Ph<3>{}, std::false_type{}, i + 3);
            }
        }
    }
    // no DMA may still be writing this workgroup's LDS when it exits
    vm_wait<0>();
    sfor<D>([&](auto lc) {
        constexpr int l = decltype(lc)::value;
        T rel;
        if constexpr (FM) rel = mr[l].value(p.ict[l]);
        else rel = mr[l].value();
        if constexpr (l > 0) __syncthreads();
        commit_errors<T, NW>(ma[l], rel, chk[l], p.err[l]);
    });
}

// the kernel of one math mode; the increment form: fp32 at depth 4 (config 5's scheme; fp64 uses
// the leapfrog)
template <class T, int D, bool F, bool FM>
static const void* tbn_kernel_m(bool delta) {
    if (delta) {
        if constexpr (std::is_same_v<T, float> && D == 4)
            return reinterpret_cast<const void*>(k_tbn<T, D, F, 2, 8, FM, true>);
        return nullptr;
    }
    return reinterpret_cast<const void*>(k_tbn<T, D, F, 2, 8, FM>);
}

#if W3D_TBN_PART == 1
template <class T, int D, bool F>
static void (*tbn_kernel(int rows, int waves, bool fm, bool delta))(const TbnParams<T>) {
    if (rows != 2 || waves != 8) return nullptr;
    const void* k = fm ? tbn_kernel_m<T, D, F, true>(delta) : tbn_exact_kernel<T>(D, F, delta);
    return reinterpret_cast<void (*)(const TbnParams<T>)>(const_cast<void*>(k));
}

template <class T, bool F>
static void (*tbn_kernel_d(int depth, int rows, int waves, bool fm, bool delta = false))(const TbnParams<T>) {
    if (depth == 4) return tbn_kernel<T, 4, F>(rows, waves, fm, delta);
    if constexpr (std::is_same_v<T, double>)  // depth 3: fp64 (the cross-check of k_tb3, A/B)
        if (depth == 3) return tbn_kernel<T, 3, F>(rows, waves, fm, delta);
    return nullptr;
}
#endif

}  // namespace

#if W3D_TBN_PART == 2
template <class T>
const void* tbn_exact_kernel(int depth, bool first, bool delta) {
    if (depth == 4) return first ? tbn_kernel_m<T, 4, true, false>(delta) : tbn_kernel_m<T, 4, false, false>(delta);
    if constexpr (std::is_same_v<T, double>)  // depth 3: fp64 (the cross-check of k_tb3, A/B)
        if (depth == 3) return first ? tbn_kernel_m<T, 3, true, false>(delta) : tbn_kernel_m<T, 3, false, false>(delta);
    return nullptr;
}
template const void* tbn_exact_kernel<double>(int, bool, bool);
template const void* tbn_exact_kernel<float>(int, bool, bool);
#else
bool tbn_supported(int depth, int rows, int waves, bool fm, bool fp32) {
    return fp32 ? tbn_kernel_d<float, false>(depth, rows, waves, fm) != nullptr
                : tbn_kernel_d<double, false>(depth, rows, waves, fm) != nullptr;
}
bool tbn_delta_supported(int depth, int rows, int waves, bool fm, bool fp32) {
    return fp32 ? tbn_kernel_d<float, false>(depth, rows, waves, fm, true) != nullptr
                : tbn_kernel_d<double, false>(depth, rows, waves, fm, true) != nullptr;
}

template <class T>
void launch_tbn(int depth, int rows, int waves, bool fm, bool first, const T* A, const T* B, T* O0, T* O1,
                const GridView& gv, const Box* boxes, int nbox, const Box& cdom, int ei0, int ei1,
                const Wrap& wrap0, const Wrap& wrap1, const TbnSeam<T>& seam, const T* txy, const T* tz,
                const T* txr, const T* rtz, const StepCoefs* c, u64* const* err, int chunk, hipStream_t s,
                bool delta) {
    W3D_REQUIRE(depth >= 3 && depth <= kTbnMaxDepth, "tbn: depth 3..4");
    W3D_REQUIRE(!fm || (txr && rtz), "tbn --math fma needs the reciprocal analytic tables");
    W3D_REQUIRE(gv.G >= depth, "deep temporal blocking needs ghost depth >= layers per sweep");
    W3D_REQUIRE(nbox >= 1 && nbox <= kMaxBoxes, "bad box count");
    W3D_REQUIRE(gv.si * i64(sizeof(T)) < (i64(1) << 30), "tbn: plane larger than 1 GiB (LDS-DMA range marker)");
    auto kern = first ? tbn_kernel_d<T, true>(depth, rows, waves, fm, delta)
                      : tbn_kernel_d<T, false>(depth, rows, waves, fm, delta);
    W3D_REQUIRE(kern, "tbn: no instantiation of this depth x tile x dtype x math x scheme");
    TbnParams<T> p{};
    p.pbytes = unsigned(gv.si * i64(sizeof(T)));
    p.pbias = gv.G + 1;  // plane indices reach ib - depth >= 1 - G and the wrap targets
    p.order = tile_order();
    auto biased = [&](const T* base) {
        return reinterpret_cast<char*>(reinterpret_cast<uintptr_t>(base - gv.poff) - uintptr_t(p.pbias) * p.pbytes);
    };
    p.A = biased(A), p.B = biased(B), p.O[0] = biased(O0), p.O[1] = biased(O1);
    p.sj = gv.sj;
    p.poff = gv.poff;
    p.jmin = 1 - gv.G, p.jmax = gv.jmax(), p.kmin = 1 - gv.G, p.kmax = gv.kmax();
    p.cj0 = cdom.j0, p.cj1 = cdom.j1, p.ck0 = cdom.k0, p.ck1 = cdom.k1;
    p.ei0 = ei0, p.ei1 = ei1;
    wrap_ranges(wrap0, p.w_lo[0], p.w_hi[0], p.w_sh[0]);
    wrap_ranges(wrap1, p.w_lo[1], p.w_hi[1], p.w_sh[1]);
    p.an_i = seam.nP[0] ? seam.next_i : INT_MIN / 2;
    p.ap_i = seam.pP[0] ? seam.prev_i : INT_MIN / 2;
    for (int l = 0; l + 1 < depth; ++l) {
        W3D_REQUIRE((!seam.nP[0] || seam.nP[l]) && (!seam.pP[0] || seam.pP[l]), "tbn: seam partner plane missing");
        p.nP[l] = seam.nP[l], p.pP[l] = seam.pP[l];
    }
    p.txy = txy, p.tpj = gv.Y + 2, p.tz = tz;
    p.txr = txr, p.rtz = rtz;
    p.hx2 = T(c[0].hx2), p.hy2 = T(c[0].hy2), p.hz2 = T(c[0].hz2);
    p.yx2 = T(1) / T(c[0].hx2), p.yy2 = T(1) / T(c[0].hy2), p.yz2 = T(1) / T(c[0].hz2);
    for (int l = 0; l < depth; ++l) {
        p.coef[l] = T(c[l].coef), p.ct[l] = T(c[l].ct), p.ict[l] = T(1 / std::fabs(c[l].ct));
        p.err[l] = err[l];
        W3D_REQUIRE(!fm || l == 0 || c[l].coef == c[1].coef, "tbn --math fma: the later layers share one coefficient");
    }
    W3D_REQUIRE(!fm || first || c[0].coef == c[1].coef, "tbn --math fma: one coefficient after the first sweep");
    auto fcoefs = [](const StepCoefs& q, T out[3]) {
        out[0] = T(q.coef / q.hx2), out[1] = T(q.coef / q.hy2), out[2] = T(q.coef / q.hz2);
    };
    fcoefs(c[0], p.fc[0]), fcoefs(c[1], p.fc[1]);
    const int TJ = waves * rows;
    int live = 0;
    for (int q = 0; q < nbox; ++q) live += !boxes[q].empty();
    const int extra = 2 * (depth - 1);  // prologue + epilogue planes of a work item
    int multi_chunk = 0;
    if (chunk <= 0 && live > 1) {
        int bt[kMaxBoxes], bp[kMaxBoxes], m = 0;
        for (int q = 0; q < nbox; ++q) {
            const Box& bx = boxes[q];
            if (bx.empty()) continue;
            bt[m] = ((bx.k1 - 1) / kTK - (bx.k0 - 1) / kTK + 1) * cdiv(bx.j1 - bx.j0 + 1, TJ);
            bp[m++] = bx.i1 - bx.i0 + 1;
        }
        multi_chunk = rounds_chunk_boxes(bt, bp, m, extra, resident_slots(reinterpret_cast<const void*>(kern), waves * 64));
    }
    int nb = 0, total = 0;
    for (int q = 0; q < nbox; ++q) {
        const Box& bx = boxes[q];
        if (bx.empty()) continue;
        W3D_REQUIRE(bx.i0 >= 1 && bx.i1 <= gv.X && bx.j0 >= 1 && bx.j1 <= gv.Y && bx.k0 >= 1 && bx.k1 <= gv.Z,
                    "sweep box outside the owned region");
        BoxLaunch& Lb = p.box[nb];
        Lb.i0 = bx.i0, Lb.i1 = bx.i1, Lb.j0 = bx.j0, Lb.j1 = bx.j1, Lb.k0 = bx.k0, Lb.k1 = bx.k1;
        const int t0 = (bx.k0 - 1) / kTK, t1 = (bx.k1 - 1) / kTK;
        Lb.kbase = 1 + t0 * kTK;
        Lb.tiles_k = t1 - t0 + 1;
        Lb.tiles_j = cdiv(bx.j1 - bx.j0 + 1, TJ);
        const int planes = bx.i1 - bx.i0 + 1;
        const int want = chunk > 0 ? std::min(chunk, planes)
                         : live == 1 ? rounds_chunk(planes, Lb.tiles_k * Lb.tiles_j, extra,
                                                    resident_slots(reinterpret_cast<const void*>(kern), waves * 64))
                                     : std::min(multi_chunk, planes);
        Lb.chunk = cdiv(planes, cdiv(planes, want));
        Lb.block_begin = total;
        total += Lb.tiles_k * Lb.tiles_j * cdiv(planes, Lb.chunk);
        ++nb;
    }
    p.nbox = nb;
    if (nb == 0) return;
    hipLaunchKernelGGL(kern, dim3(total), dim3(waves * 64), 0, s, p);
    HIP_OK(hipGetLastError());
}

#define W3D_TBN_INST(T)                                                                                          \
    template void launch_tbn<T>(int, int, int, bool, bool, const T*, const T*, T*, T*, const GridView&,         \
                                const Box*, int, const Box&, int, int, const Wrap&, const Wrap&,                \
                                const TbnSeam<T>&, const T*, const T*, const T*, const T*, const StepCoefs*,   \
                                u64* const*, int, hipStream_t, bool);
W3D_TBN_INST(double)
W3D_TBN_INST(float)
#endif

}  // namespace wave3d
