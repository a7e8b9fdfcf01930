// Device-side helpers shared by the stencil kernels (hip_kernels.hip, hip_tb.hip).
// Internal to the HIP translation units (anonymous namespace per includer).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "hip_kernels.hpp"
#include "stencil_math.hpp"

#define HIP_OK(x)                                                                      \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess)                                                          \
            throw ::wave3d::Error(std::string("HIP error ") + hipGetErrorString(e_) + \
                                  " at " __FILE__ ":" + std::to_string(__LINE__));     \
    } while (0)

namespace wave3d {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kTK = kTileK;              // tile columns (k) = one wave64
constexpr int kLW = kTK + 2;             // LDS row incl. k halos
constexpr int kNaiveTJ = kWaves;         // naive kernel: one row per wave

struct BoxLaunch {
    int i0, i1, j0, j1, k0, k1;
    int kbase;     // k of lane 0 of the first tile (aligned to 1 + 64t)
    int tiles_k, tiles_j, chunk;
    int block_begin;
};

__device__ __forceinline__ u64 enc_key(double d) {
    u64 b = (u64)__double_as_longlong(d);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

template <class T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        T o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ u64 wave_sum_u64(u64 v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ u64 wave_min_u64(u64 v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const u64 o = __shfl_xor(v, off, 64);
        v = o < v ? o : v;
    }
    return v;
}

// m = max(m, |d|) as one v_max with an abs source modifier. fmax() of a loop-carried value
// costs two extra canonicalising v_max per node (plus a v_and for the |.|); the raw
// instruction in IEEE mode already returns the other operand for a quiet-NaN input, and every
// NaN here is an arithmetic result (quiet) — the reference's NaN-ignoring `if (e > m) m = e`.
__device__ __forceinline__ double max_abs(double m, double d) {
    double r;
    asm("v_max_f64 %0, %1, |%2|" : "=v"(r) : "v"(m), "v"(d));
    return r;
}
__device__ __forceinline__ float max_abs(float m, float d) {
    float r;
    asm("v_max_f32_e64 %0, %1, |%2|" : "=v"(r) : "v"(m), "v"(d));
    return r;
}

// up ? |t| : k without materialising |t|: a double select is two 32-bit v_cndmask, and the
// sign bit lives in the high word, whose select takes |.| as a free source modifier.
__device__ __forceinline__ double pick_abs(bool up, double k, double t) {
    const u64 kb = __builtin_bit_cast(u64, k), tb = __builtin_bit_cast(u64, t);
    const unsigned lo = up ? unsigned(tb) : unsigned(kb);
    unsigned hi;
    asm("v_cndmask_b32_e64 %0, %1, |%2|, %3"
        : "=v"(hi)
        : "v"(unsigned(kb >> 32)), "v"(unsigned(tb >> 32)), "s"(__builtin_amdgcn_ballot_w64(up)));
    return __builtin_bit_cast(double, (u64(hi) << 32) | lo);
}
__device__ __forceinline__ float pick_abs(bool up, float k, float t) {
    float r;
    asm("v_cndmask_b32_e64 %0, %1, |%2|, %3" : "=v"(r) : "v"(k), "v"(t), "s"(__builtin_amdgcn_ballot_w64(up)));
    return r;
}

// d, or a quiet NaN on masked lanes (max_abs and RelArg ignore NaN errors): one v_cndmask on
// the high word
__device__ __forceinline__ double nan_unless(bool v, double d) {
    const u64 b = __builtin_bit_cast(u64, d);
    const unsigned hi = v ? unsigned(b >> 32) : 0x7ff80000u;
    return __builtin_bit_cast(double, (u64(hi) << 32) | (b & 0xffffffffull));
}
__device__ __forceinline__ float nan_unless(bool v, float d) {
    return v ? d : __builtin_bit_cast(float, 0x7fc00000u);
}

// Running maximum of the relative error |u-f|/|f| without a division per node: the argmax is
// tracked exactly as the pair (num, den) by comparing num'*den vs num*den' through products
// split into RN value + exact FMA residual, and the one IEEE division happens at the end.
// RN is monotone, so value() = RN(max exact quotient) = max of the reference's RN quotients
// (mpi_new.cpp:341-344): bitwise equal, including its NaN-ignoring `>` and the x/0 = inf case
// (exact as long as the products are normal numbers, i.e. |errors| and |f| above ~1e-150).
// add() takes the signed d = u - f and f: the |.| are source modifiers of the products and of
// the selects (pick_abs), so num, den hold |d|, |f| without a v_and per node.
template <class T>
struct RelArg {
    T num = T(kErrInit), den = T(1);
    __device__ __forceinline__ void add(T d, T f) {
#pragma clang fp contract(off)
        const T p1 = absval(d) * den, p2 = num * absval(f);
        // one rarely taken branch (the wave skips it unless some lane may take a new maximum):
        // the selects and the exact tie-break on the FMA residuals where the rounded products tie
        // (mirror-symmetric nodes). Against selects on every node: 1,330 VALU per 4 planes of the
        // depth-4 sweep instead of 1,586, --math exact +6 % (profiles/deep_sweeps_r5.txt)
        if (__builtin_expect(p1 >= p2, 0)) {
            const bool up = p1 > p2 || fma_t(absval(d), den, -p1) > fma_t(num, absval(f), -p2);
            num = pick_abs(up, num, d);
            den = pick_abs(up, den, f);
        }
    }
    __device__ __forceinline__ T value() const { return num / den; }
};

// --math fma relative error: the running max of |d| * w with w = 1/|sx sy| * 1/|sz| (reciprocal
// tables), i.e. |d|/|f| * |ct|; value() divides by |ct| once. Two operations per node instead of
// RelArg's eight, within a few ulps of the reference's quotient (not bitwise).
template <class T>
struct RelMax {
    T m = T(kErrInit);
    __device__ __forceinline__ void add(T d, T w) { m = max_abs(m, d * w); }
    __device__ __forceinline__ T value(T ict) const { return m == T(kErrInit) ? m : m * ict; }
};

// Per node: |u - f| into the running maximum and the relative-error argmax, and u into `chk`.
// The maximum ignores a NaN error exactly like the reference's `if (e > m) m = e`
// (mpi_new.cpp:343-344; max_abs). `chk` is the sum of the layer's values: non-finite iff some
// value was NaN/Inf (or the values overflow a double, i.e. the run diverged anyway) — one add
// per node instead of a compare-and-or; commit_errors() turns it into the nonfinite flag.
template <class T>
__device__ __forceinline__ void accumulate_error_dev(T u, T f, T& mabs, RelArg<T>& mrel) {
#pragma clang fp contract(off)
    const T d = u - f;
    mabs = max_abs(mabs, d);
    mrel.add(d, f);
}

// Workgroup reduction of the running maxima + one atomic per slot (race-free, no
// divergent barrier: every thread reaches the __syncthreads, cf. Appendix B5).
template <class T, int NW = kWaves>
__device__ __forceinline__ void commit_errors(T ma, T mr, T chk, u64* err) {
    const bool bad = nonfinite(chk);
    __shared__ double red[2][NW];
    __shared__ int redb[NW];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    ma = wave_max(ma);
    mr = wave_max(mr);
    unsigned long long any = __ballot(bad);
    if (lane == 0) {
        red[0][w] = double(ma);
        red[1][w] = double(mr);
        redb[w] = any != 0ull;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = red[0][0], r = red[1][0];
        int b = redb[0];
#pragma unroll
        for (int q = 1; q < NW; ++q) {
            if (red[0][q] > a) a = red[0][q];
            if (red[1][q] > r) r = red[1][q];
            b |= redb[q];
        }
        atomicMax(err + 0, enc_key(a));
        atomicMax(err + 1, enc_key(r));
        if (b) atomicMax(err + 2, 1ull);
    }
}

// XCD-aware work order. Workgroups are dispatched round-robin over the 8 XCDs
// (blockIdx % 8), each with its own L2. Renumbering so that XCD x runs one contiguous range
// of logical tiles keeps k- and j-neighbour tiles — which read each other's edge rows and
// columns as halo — on the same L2 instead of always on different ones. Measured on
// MI355X (profiles/sweep_n512_tb_variants_r1.txt) it does not pay here (halo lines come
// from the memory-side Infinity Cache either way), so it is opt-in: WAVE3D_XCD_SWIZZLE=1.
constexpr int kXcds = 8;
__device__ __forceinline__ int xcd_swizzle(int bid, int total, bool on) {
    if (!on) return bid;
    const int x = bid % kXcds, q = bid / kXcds;
    const int base = total / kXcds, rem = total % kXcds;
    return x * base + min(x, rem) + q;
}

template <class P>
__device__ __forceinline__ int find_box(const P& p, int bid) {
    int b = 0;
#pragma unroll
    for (int q = 1; q < kMaxBoxes; ++q)
        if (q < p.nbox && bid >= p.box[q].block_begin) b = q;
    return b;
}

inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// Planes per marching work item: `best` (measured at N = 512) unless that leaves fewer than
// ~4 workgroups per CU; then shorter chunks (>= 8 planes) trade prologue work for occupancy.
inline int auto_chunk(int best, int planes, int tiles) {
    constexpr int kTarget = 4 * 256;
    int c = best;
    if (i64(tiles) * cdiv(planes, c) < kTarget) c = std::max(8, int(i64(planes) * tiles / kTarget));
    return std::min(std::max(1, c), planes);
}

// The same decision for one launch over several boxes (tiles[q] x planes[q] each), taken for
// the launch as a whole: decided per box, the thin overlap shells (a few tiles each) got 8-16-
// plane work items whose 2-plane prologues were 12-25 % redundant work, while the launch had
// plenty of workgroups. Returns the chunk before clamping to each box's planes.
inline int auto_chunk_boxes(int best, const int* tiles, const int* planes, int n) {
    constexpr int kTarget = 4 * 256;
    i64 items = 0, work = 0;
    for (int q = 0; q < n; ++q) {
        items += i64(tiles[q]) * cdiv(planes[q], best);
        work += i64(tiles[q]) * planes[q];
    }
    if (items >= kTarget) return best;
    return std::max(1, std::max(8, int(work / kTarget)));
}

// CUs withheld from this host thread's sweep launches: while overlap is on, the compute stream
// is CU-masked so the halo stream's kernels (RCCL, pack/unpack, shells) always find free CUs,
// and work items are sized for the CUs it keeps (hip_solver comm_cu_reserve()).
inline int& launch_cu_reserve() {
    thread_local int r = 0;
    return r;
}
struct CuReserveScope {
    int old;
    explicit CuReserveScope(int r) : old(launch_cu_reserve()) { launch_cu_reserve() = r; }
    ~CuReserveScope() { launch_cu_reserve() = old; }
};

// Resident workgroups of a sweep kernel on the device (CUs x occupancy, less the reserved CUs),
// cached per kernel and device (thread-per-GPU ranks launch concurrently).
inline int resident_slots(const void* kern, int threads) {
    static std::mutex mu;
    static std::unordered_map<const void*, int> occ;
    static int cus[64] = {};
    int dev = 0;
    HIP_OK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    if (dev >= 0 && dev < 64 && cus[dev] == 0)
        HIP_OK(hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev));
    auto it = occ.find(kern);
    if (it == occ.end()) {
        int n = 0;
        HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, threads, 0));
        it = occ.emplace(kern, std::max(1, n)).first;
    }
    const int n = dev >= 0 && dev < 64 ? cus[dev] : 256;
    return std::max(1, std::max(1, n - launch_cu_reserve()) * it->second);
}

// Work-item length of a one-box sweep: the march pays `extra` planes of prologue/epilogue per
// work item (tb3: 4, tb2: 2), and a launch runs in rounds of `slots` resident workgroups, so its
// time goes as rounds x (chunk + extra). The 1-workgroup-per-CU fp64 tb3 sweep at N=512 (256 tiles): chunk 86
// (the general auto_chunk) 430k, 171 450k, 256 453k, 512 449k Mpts/s (profiles/tb3_salu_r3.txt).
// Takes the cheapest split; among splits within 1 % of it, the one with the most work items.
inline int rounds_chunk(int planes, int tiles, int extra, int slots) {
    auto cost = [&](int n) {
        const int c = cdiv(planes, n), items = tiles * cdiv(planes, c);
        return i64(cdiv(items, slots)) * (c + extra);
    };
    const int nmax = std::max(1, std::min(64, planes / 8));
    i64 best = cost(1);
    for (int n = 2; n <= nmax; ++n) best = std::min(best, cost(n));
    int pick = 1;
    for (int n = 1; n <= nmax; ++n)
        if (cost(n) * 100 <= best * 101) pick = n;
    return cdiv(planes, pick);
}

// The same for a launch over several boxes (overlap shells: thin x slabs, one tile band in j
// and k): one chunk c for every box (each box's items cut to min(c, planes)); the launch takes
// about max(longest item, total item-planes / slots), items costing planes + `extra` each.
inline int rounds_chunk_boxes(const int* tiles, const int* planes, int n, int extra, int slots) {
    int pmax = 1;
    for (int q = 0; q < n; ++q) pmax = std::max(pmax, planes[q]);
    auto cost = [&](int c) {
        i64 work = 0;
        int longest = 0;
        for (int q = 0; q < n; ++q) {
            const int cq = cdiv(planes[q], cdiv(planes[q], std::min(c, planes[q])));
            work += i64(tiles[q]) * cdiv(planes[q], cq) * (cq + extra);
            longest = std::max(longest, cq + extra);
        }
        return std::max<i64>(longest * i64(slots), work);  // in plane-iterations x slots
    };
    int best_c = pmax;
    i64 best = cost(pmax);
    for (int c = 8; c < pmax; c += (c < 64 ? 8 : 16)) {
        const i64 v = cost(c);
        if (v < best) best = v, best_c = c;
    }
    return best_c;
}

// ---- buffer addressing (T8): wave-uniform plane descriptor + 32-bit lane byte offset -----
// An offset >= the descriptor's byte size is out of range: loads return 0, stores are
// dropped — masked lanes use kOOB instead of a branch around the access.
constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, int(bytes),
                                             0x00020000);
}
// Wave-uniform read of a small read-only table through the constant address space, so it
// is a scalar load (s_load, lgkmcnt) instead of a vector load whose vmcnt wait would also
// drain every prefetch issued before it.
template <class T>
__device__ __forceinline__ T ldconst(const T* base, int i) {
    using CP = const __attribute__((address_space(4))) T*;
    return ((CP)(base))[i];
}

// compile-time loop phase (unrolled rolling-register loops)
template <int V>
using Ph = std::integral_constant<int, V>;

// ---- row vectors: L = 1 (scalar T) or 2 (packed fp32 pair of rows) --------------------
template <class T, int L>
struct RowVec {
    using type = T;
};
template <>
struct RowVec<float, 2> {
    using type = f32x2;
};
template <int L, class V>
__device__ __forceinline__ auto vget(const V& v, int e) {
    if constexpr (L == 1) return v;
    else return v[e];
}
template <int L, class V, class T>
__device__ __forceinline__ void vset(V& v, int e, T x) {
    if constexpr (L == 1) v = x;
    else v[e] = x;
}
template <int L, class V, class T>
__device__ __forceinline__ V vsplat(T x) {
    if constexpr (L == 1) return x;
    else return V{x, x};
}

// Periodic self-wrap table -> <= 2 (lo, hi, shift) plane ranges (plane i in [lo, hi] is
// also stored to plane i + shift): fewer live scalars in the kernels than a 4-entry table.
inline void wrap_ranges(const Wrap& w, int lo[2], int hi[2], int sh[2]) {
    int n = 0;
    lo[0] = lo[1] = 1 << 30;
    hi[0] = hi[1] = -(1 << 30);
    sh[0] = sh[1] = 0;
    for (int q = 0; q < kMaxWrap; ++q) {
        if (w.src[q] < 1) continue;
        const int s = w.dst[q] - w.src[q];
        int g = 0;
        for (; g < n; ++g)
            if (sh[g] == s && (w.src[q] == hi[g] + 1 || w.src[q] == lo[g] - 1)) break;
        if (g == n) {
            W3D_REQUIRE(n < 2, "self-wrap needs more than two plane ranges");
            ++n;
            sh[g] = s;
            lo[g] = hi[g] = w.src[q];
        }
        lo[g] = lo[g] < w.src[q] ? lo[g] : w.src[q];
        hi[g] = hi[g] > w.src[q] ? hi[g] : w.src[q];
    }
}

// AUX = cache policy bits of the buffer instruction (0 default, 2 = nt: read-once streams)
template <int AUX>
__device__ __forceinline__ double bload(double*, __amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX));
}
template <int AUX>
__device__ __forceinline__ float bload(float*, __amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, AUX));
}
template <class T, int AUX = 0>
__device__ __forceinline__ T bld(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return bload<AUX>((T*)nullptr, r, off);
}
template <int AUX = 0>
__device__ __forceinline__ void bst(double v, __amdgpu_buffer_rsrc_t r, unsigned off) {
    using V2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V2, v), r, off, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void bst(float v, __amdgpu_buffer_rsrc_t r, unsigned off) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, AUX);
}

}  // namespace
}  // namespace wave3d
