// Host-side interface of the hand-written CDNA4 kernels (hip_kernels.hip).
//
// Storage of one time level (per rank): [i][j][k], k contiguous, one ghost layer.
//   ptr(i,j,k) = g + i*si + j*sj + k,   sj = pitch (row pitch, elements), si = ny*pitch.
// The solver offsets `g` so that (i,j,k=1) is 128-B aligned: k-tiles of 64 lanes start at
// k = 1 + 64t and every wave row load is whole cache lines.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "common.hpp"

namespace wave3d {

struct GridView {
    int nx = 0, ny = 0, nz = 0;  // padded extents (X+2, Y+2, Z+2)
    int sj = 0;                  // row pitch (elements)
    i64 si = 0;                  // plane stride (elements)
};

// Up to this many boxes per launch (interior + 6 shell slabs).
constexpr int kMaxBoxes = 7;

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

// Periodic self-wrap fused into the stores (dims[0] == 1): the plane `src[s]` is also
// written to ghost plane `dst[s]`. -1 = off.
struct Wrap {
    int src[2] = {-1, -1};
    int dst[2] = {-1, -1};
};

// Stencil kernel variant: 2.5-D marching (rows per lane, non-temporal u^{n-2} loads) or
// the one-point-per-lane kernel.
struct KernelVariant {
    bool march = true;
    int rows = 4;
    bool nt = false;
    bool fast = false;  // reciprocal/FMA math: not bitwise-reproducible (benchmark ablation)
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

// Initialise per-layer error slots: abs/rel keys = encode(-100), flag = 0.
void launch_init_err(u64* err, int layers, hipStream_t s);

// Device encode of a double into the order-preserving key (exposed for tests).
void launch_encode_keys(const double* v, u64* k, int n, hipStream_t s);

int march_rows_per_thread();

}  // namespace wave3d
