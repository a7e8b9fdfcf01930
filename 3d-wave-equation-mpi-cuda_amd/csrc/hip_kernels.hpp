// Host-side interface of the hand-written CDNA4 kernels (hip_kernels.hip).
//
// Storage of one time level (per rank): [i][j][k], k contiguous, G ghost layers per side.
//   ptr(i,j,k) = g + i*si + j*sj + k  for logical i in [1-G, X+G] (owned 1..X), same in j,k;
//   sj = row pitch (elements), si = (Y+2G)*sj. `g` points at logical (0,0,0) and is placed
// so that (i,j,k=1) is 128-B aligned: 64-lane k-tiles start at k = 1 + 64t and every wave
// row load is whole cache lines.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "common.hpp"

namespace wave3d {

struct GridView {
    int X = 0, Y = 0, Z = 0;  // owned nodes per axis (logical indices 1..X etc.)
    int G = 1;                // ghost depth: logical indices 1-G .. X+G exist in storage
    int sj = 0;               // row pitch (elements)
    i64 si = 0;               // plane stride (elements)
    int poff = 0;             // logical (i,0,0) - physical start of plane i: j*sj+k+poff >= 0
    int jmax() const { return Y + G; }
    int kmax() const { return Z + G; }
};

// Up to this many boxes per launch (interior + 6 shell slabs).
constexpr int kMaxBoxes = 7;
constexpr int kTileK = 64;  // k columns per tile of the marching kernels (one wave64), tiles
                            // start at k = 1 + 64 t

struct StepCoefs {
    double hx2 = 1, hy2 = 1, hz2 = 1;  // h*h divisors
    double coef = 0;                   // a2*tau*tau (or a2*tau*tau*0.5 on layer 1)
    double ct = 0;                     // cos(a_t*t_n + 2π) of this layer
};

// Optional fused halo packing: values at k == zk[s] / j == yj[s] are also written to the
// packed z / y face buffers (index layout of halo.hpp). nullptr = off.
template <class T>
struct FusedPack {
    T* zbuf[2] = {nullptr, nullptr};
    int zk[2] = {-1, -1};
    T* ybuf[2] = {nullptr, nullptr};
    int yj[2] = {-1, -1};
};

// Periodic self-wrap fused into the stores (dims[0] == 1): plane `src[q]` is also written
// to ghost plane `dst[q]` (depth-2 ghosts need 4 pairs). -1 = unused.
constexpr int kMaxWrap = 8;  // depth-4 ghosts: 4 pairs per side
struct Wrap {
    int src[kMaxWrap] = {-1, -1, -1, -1, -1, -1, -1, -1};
    int dst[kMaxWrap] = {-1, -1, -1, -1, -1, -1, -1, -1};
};

// Stencil kernel variant: 2.5-D marching (rows per lane, non-temporal u^{n-2} loads) or
// the one-point-per-lane kernel.
struct KernelVariant {
    bool march = true;
    int rows = 4;
    bool nt = false;
    bool fast = false;  // --math fma form (stencil_math coef_lap_fma): not bitwise with the reference
    bool pk = false;    // packed fp32: two rows per v_pk_* instruction (fp32 only)
    bool flat = false;  // one point per thread over the flattened boxes (thin overlap shells)
    bool delta = false; // increment form: u2 holds d^{n-1} (naive / flat kernels only)
};
KernelVariant parse_kernel_variant(const std::string& name);
std::string kernel_variant_name(const KernelVariant& v);

// One time layer n >= 1 over `nbox` boxes. Errors are accumulated for i in [ei0, ei1]
// into err[0..2] = {abs key, rel key, nonfinite flag}.
template <class T>
void launch_step(const KernelVariant& kind, bool first, const T* u1, const T* u2, T* u, const GridView& gv,
                 const Box* boxes, int nbox, int ei0, int ei1, const Wrap& wrap,
                 const FusedPack<T>& pack, const T* tx, const T* ty, const T* tz,
                 const StepCoefs& c, u64* err, int chunk, hipStream_t s);

// Layer 0: u = analytic over `box` (owned nodes), errors over the same box.
template <class T>
void launch_init(T* u, const GridView& gv, const Box& box, const Wrap& wrap, const T* tx,
                 const T* ty, const T* tz, double ct0, u64* err, hipStream_t s);

// Dirichlet faces (prepare_layer, mpi_new.cpp:157-169): mask bit 0/1 = z minus/plus face
// (k = 1 / k = Z), bit 2/3 = y minus/plus face (j = 1 / j = Y); over i in 1..X.
template <class T>
void launch_zero_faces(T* u, const GridView& gv, int mask, hipStream_t s);

// y face (axis 1): buf[(i-1)*(Z+2) + k] <-> u(i, j, k), i = 1..X, k = 0..Z+1
// z face (axis 2): buf[(i-1)*(Y+2) + j] <-> u(i, j, k), i = 1..X, j = 0..Y+1
// Several faces per launch; `to_buf` = pack, else unpack.
template <class T>
struct FaceOp {
    T* buf = nullptr;
    int axis = 1;
    int index = 0;  // j (axis 1) or k (axis 2) of the grid plane
};
template <class T>
void launch_faces(T* u, const GridView& gv, const FaceOp<T>* ops, int nops, bool to_buf,
                  hipStream_t s);

// Three-layer temporal blocking (hip_tb3.hip): one sweep computes C = u^m (errors only, never
// stored), D = u^{m+1} and E = u^{m+2} from A = u^{m-1}, B = u^{m-2}. Needs ghost depth >= 3
// of A and >= 2 of B. Periodic seam: at plane next_i the x+ neighbour of C is the plane nA and
// the x+ neighbour of D is nC, C evaluated at that partner plane before the sweep
// (launch_seam_c); mirrored for prev_i. Pointers address logical (0, 0) of a plane.
template <class T>
struct SeamPartners {
    int next_i = -(1 << 30), prev_i = -(1 << 30);
    const T *nA = nullptr, *nC = nullptr;  // partner A plane, C evaluated there (launch_seam_c)
    const T *pA = nullptr, *pC = nullptr;
};
// C on a seam partner plane: out = C(Ac; x neighbours Am, Ap; u^{m-2} = Bc), 0 outside cdom
// (logical plane pointers, full storage extent minus the outermost row/column).
template <class T>
struct SeamCPlane {
    T* out = nullptr;
    const T *Ac = nullptr, *Am = nullptr, *Ap = nullptr, *Bc = nullptr;
    T* dout = nullptr;  // increment form: also the new d there (the next stage's Bc)
};
// fm: --math fma instantiations (stencil_math coef_lap_fma), not bitwise with the reference.
// The same operator evaluates any later layer on a partner plane (Ac = layer l-1 there, Am / Ap
// its x neighbours, Bc = layer l-2): up to kMaxSeamOps planes per launch.
constexpr int kMaxSeamOps = 6;
template <class T>
void launch_seam_c(bool first, bool delta, bool fm, const SeamCPlane<T>* ops, int nops, const GridView& gv,
                   const Box& cdom, const StepCoefs& cC, hipStream_t s);
bool tb3_supported(int rows, int waves, bool fm = false);
bool tb3_delta_supported(int rows, int waves, bool fm = false);
template <class T>
void launch_tb3(int rows, int waves, bool delta, bool fm, bool first, const T* A, const T* B, T* D, T* E,
                const GridView& gv, const Box* boxes, int nbox, const Box& cdom, int ei0, int ei1,
                const Wrap& wrapD, const Wrap& wrapE, const SeamPartners<T>& seam, const T* txy,
                const T* tz, const T* txr, const T* rtz, const StepCoefs& cC, const StepCoefs& cD,
                const StepCoefs& cE, u64* errC, u64* errD, u64* errE, int chunk, hipStream_t s);

// Deep temporal blocking (hip_tbn.hip): one sweep computes D = depth layers u^m .. u^{m+D-1}
// from A = u^{m-1}, B = u^{m-2} and stores only the last two (O0 = u^{m+D-2}, O1 = u^{m+D-1}, the
// next sweep's B and A). Needs ghost depth >= D of A and >= D-1 of B; O0 / O1 get the periodic
// self-wrap of depth D-1 / D. Periodic seam: at plane next_i the x+ neighbour of layer l is
// nP[l] (A at the partner plane for l = 0, layer l-1 evaluated there by launch_seam_c for
// l >= 1); mirrored for prev_i / pP. c[l] / err[l]: coefficients and error slots of layer m+l.
constexpr int kTbnMaxDepth = 4;
template <class T>
struct TbnSeam {
    int next_i = -(1 << 30), prev_i = -(1 << 30);
    const T* nP[kTbnMaxDepth - 1] = {};
    const T* pP[kTbnMaxDepth - 1] = {};
};
bool tbn_supported(int depth, int rows, int waves, bool fm, bool fp32);
// the increment form (DELTA): fp32 at depth 4 only
bool tbn_delta_supported(int depth, int rows, int waves, bool fm, bool fp32);
template <class T>
void launch_tbn(int depth, int rows, int waves, bool fm, bool first, const T* A, const T* B, T* O0, T* O1,
                const GridView& gv, const Box* boxes, int nbox, const Box& cdom, int ei0, int ei1,
                const Wrap& wrap0, const Wrap& wrap1, const TbnSeam<T>& seam, const T* txy, const T* tz,
                const T* txr, const T* rtz, const StepCoefs* c, u64* const* err, int chunk, hipStream_t s,
                bool delta = false);

// Box halo staging for the temporal-blocking exchange on y/z splits: copy the logical box
// `b` of a level (origin `grid` = logical (0,0,0), strides of `gv`) to / from a contiguous
// buffer (k fastest). Up to kMaxBoxCopy boxes per launch.
constexpr int kMaxBoxCopy = 32;
template <class T>
struct BoxCopy {
    T* grid = nullptr;
    T* buf = nullptr;
    Box b;
};
template <class T>
void launch_box_copy(const BoxCopy<T>* ops, int nops, const GridView& gv, bool to_buf,
                     hipStream_t s);

// Initialise per-layer error slots: abs/rel keys = encode(-100), flag = 0.
void launch_init_err(u64* err, int layers, hipStream_t s);
// ts[slot] = device wall clock (hipDeviceAttributeWallClockRate kHz) in stream order
void launch_stamp(u64* ts, int slot, hipStream_t s);
// one wave spins `ticks` of the device wall clock (hipDeviceAttributeWallClockRate kHz), bounded
void launch_spin(u64 ticks, hipStream_t s);

// Device encode of a double into the order-preserving key (exposed for tests).
void launch_encode_keys(const double* v, u64* k, int n, hipStream_t s);

int march_rows_per_thread();
// j rows of one tile of a single-step kernel variant (march: waves x rows per lane)
int march_tile_rows(const KernelVariant& v);

// XCD-aware workgroup order for the stencil kernels (device_common.hpp xcd_swizzle);
// opt-in via env WAVE3D_XCD_SWIZZLE=1 (ablation, not faster on MI355X).
bool xcd_swizzle_enabled();
// Temporal-blocking tile order (env WAVE3D_TILE_ORDER): 2 = "band" (default): XCD x (block id
// mod 8) owns a band of tiles_j/8 adjacent tile rows for every k-tile, so k-neighbours and the
// j-neighbours inside a band share its L2 (-12 % memory-side reads vs "j", -30 % vs "k";
// profiles/tile_order_r2.txt; needs tiles_j % 8 == 0, else "j"); 1 = "j": j-neighbour tiles at
// consecutive block ids (k-neighbours a multiple of 8 ids apart, same XCD); 0 = "k": k-fastest.
int tile_order();

// Temporal blocking: one sweep computes layers m (C) and m+1 (D) from A = u^{m-1} and
// B = u^{m-2} (unused when m == 1), D-boxes as for launch_step. C is evaluated on a one-node
// ring around every tile (redundantly, bitwise identical), inside `cdom` in j/k and as 0 on
// the Dirichlet faces outside it. Needs ghost depth >= 2 of A and >= 1 of B.
// Periodic seam: C at plane `alias.next_i` takes its x+ neighbour from `alias.next`
// (a plane base pointer) and C at `alias.prev_i` its x- neighbour from `alias.prev` —
// the reference keeps both x=0 and x=N planes, so the ghost copy of global N-1 must see
// x=N, not x=0, as its neighbour (csrc/hip_tb.hip).
template <class T>
struct SeamAlias {
    int next_i = -(1 << 30), prev_i = -(1 << 30);
    const T* next = nullptr;
    const T* prev = nullptr;
};

// Tile = (waves / nwk) * rows rows x 64 * nwk columns (nwk waves side by side along k);
// tb2_supported() lists the instantiated shapes. `occ` > 0 caps registers so that many waves
// fit per SIMD (may spill a little).
bool tb2_supported(int rows, int waves, int occ = 0, int nwk = 1);
// delta: increment form — B holds d^{m-1}; C receives d^{m+1} (planes of D, with C's wrap
// planes), D receives u^{m+1}; u^m is formed in registers for its errors only.
bool tb2_delta_supported(int rows, int waves, int nwk = 1);
// `txy` = the sx*sy product table of launch_txy (X, Y of gv).
// fm: the --math fma instantiations (r2w8, r2w4; increment form r2w8)
bool tb2_fma_supported(int rows, int waves, int nwk, bool delta);
template <class T>
void launch_tb2(int rows, int waves, int occ, int nwk, bool delta, bool fm, bool first, const T* A, const T* B, T* C, T* D, const GridView& gv,
                const Box* boxes, int nbox, const Box& cdom, int ei0, int ei1, const Wrap& wrapC,
                const Wrap& wrapD, const SeamAlias<T>& alias, const T* txy, const T* tz,
                const T* txr, const T* rtz, const StepCoefs& cC, const StepCoefs& cD, u64* errC, u64* errD,
                int chunk, hipStream_t s);

// Analytic-product table of the temporal-blocking kernels: out[i*(Y+2) + j] = RN(tx[i]*ty[j])
// for i in 0..X+1, j in 0..Y+1 (tables of X+2 / Y+2 entries), then txy_pad zero elements (rows
// past the last are read, unused, by masked waves). Holds txy_elems(X, Y) elements.
constexpr int kTxyPad = 256;
inline size_t txy_elems(int X, int Y) { return size_t(X + 2) * size_t(Y + 2) + kTxyPad; }
template <class T>
void launch_txy(T* out, const T* tx, const T* ty, int X, int Y, hipStream_t s);
// out[q] = 1 / |in[q]| for q < n (the --math fma relative error: |d| * (1/|sx sy|) * (1/|sz|),
// then / |ct| once per layer, instead of a division or an exact argmax per node)
template <class T>
void launch_recip_abs(T* out, const T* in, size_t n, hipStream_t s);
// --math fma pair table: out[2q] = txy[q], out[2q+1] = 1/|txy[q]| for q < txy_elems(X, Y): one
// scalar load of both per row in the sweeps
template <class T>
void launch_txr(T* out, const T* txy, size_t n, hipStream_t s);

}  // namespace wave3d
