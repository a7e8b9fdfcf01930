// Halo-plan self-test and RCCL mirror kernels (hip_selftest.hpp).
//
// The reference finds a wrong halo only as a wrong error table after a whole run
// (cuda_sol.cpp:245-310: nothing checks what arrived). Here every rank fills its time levels
// with a value that encodes the GLOBAL node position (and the level), runs one real exchange
// through its plan and transport, and compares every received cell with the value its global
// position must hold — ghost planes across the periodic seam included. A wrong peer, tag, size,
// level or placement shows up at setup time as a count per message.
#include "device_common.hpp"
#include "hip_selftest.hpp"

namespace wave3d {
namespace {

template <class T>
__device__ __forceinline__ T expected_at(i64 gi, i64 gj, i64 gk, int N, unsigned salt) {
    if (gi < 0) gi += N;  // periodic x: global -1 is N-1 (x = N duplicates x = 0)
    if (gi > N) gi -= N;
    if (gj < 0 || gj > N || gk < 0 || gk > N) return T(kPatternSentinel);
    return T(halo_pattern_value(gi, gj, gk, salt));
}

// Logical box of a level: owned nodes get their pattern, everything else the sentinel
// (mode 0); mode 1 writes `v` everywhere in the box (fault injection).
template <class T>
__global__ void __launch_bounds__(256) k_pattern_fill(T* g, i64 si, int sj, Box b, int X, int Y, int Z,
                                                      PatternCoords pc, int mode, T v) {
    const int nk = b.k1 - b.k0 + 1, nj = b.j1 - b.j0 + 1;
    const i64 total = i64(b.i1 - b.i0 + 1) * nj * nk;
    for (i64 e = i64(blockIdx.x) * blockDim.x + threadIdx.x; e < total; e += i64(gridDim.x) * blockDim.x) {
        const int k = b.k0 + int(e % nk);
        const i64 r = e / nk;
        const int j = b.j0 + int(r % nj);
        const int i = b.i0 + int(r / nj);
        T val = v;
        if (mode == 0) {
            const bool owned = i >= 1 && i <= X && j >= 1 && j <= Y && k >= 1 && k <= Z;
            val = owned ? T(halo_pattern_value(pc.off[0] + i - 1, pc.off[1] + j - 1, pc.off[2] + k - 1, pc.salt))
                        : T(kPatternSentinel);
        }
        g[i64(i) * si + i64(j) * sj + k] = val;
    }
}

// res[0] += mismatches, res[1] = min(linear index in the box of a mismatch)
template <class T>
__global__ void __launch_bounds__(256) k_pattern_check(const T* g, i64 si, int sj, Box b, PatternCoords pc,
                                                       u64* res) {
    const int nk = b.k1 - b.k0 + 1, nj = b.j1 - b.j0 + 1;
    const i64 total = i64(b.i1 - b.i0 + 1) * nj * nk;
    u64 bad = 0, first = ~0ull;
    for (i64 e = i64(blockIdx.x) * blockDim.x + threadIdx.x; e < total; e += i64(gridDim.x) * blockDim.x) {
        const int k = b.k0 + int(e % nk);
        const i64 r = e / nk;
        const int j = b.j0 + int(r % nj);
        const int i = b.i0 + int(r / nj);
        const i64 gi = pc.gi_fixed >= 0 ? pc.gi_fixed : pc.off[0] + i - 1;
        const T want = expected_at<T>(gi, pc.off[1] + j - 1, pc.off[2] + k - 1, pc.N, pc.salt);
        const T got = g[i64(i) * si + i64(j) * sj + k];
        if (!(got == want)) {
            ++bad;
            first = first < u64(e) ? first : u64(e);
        }
    }
    // one atomic pair per wave (vector atomics on a global address)
    bad = wave_sum_u64(bad);
    first = wave_min_u64(first);
    if ((threadIdx.x & 63) == 0 && bad) {
        atomicAdd(&res[0], bad);
        atomicMin(&res[1], first);
    }
}

// res[0] += differing 4-byte words, res[1] = min(word index of a difference)
__global__ void __launch_bounds__(256) k_compare_words(const unsigned* a, const unsigned* b, size_t n, u64* res) {
    u64 bad = 0, first = ~0ull;
    for (size_t e = size_t(blockIdx.x) * blockDim.x + threadIdx.x; e < n; e += size_t(gridDim.x) * blockDim.x)
        if (a[e] != b[e]) {
            ++bad;
            first = first < u64(e) ? first : u64(e);
        }
    bad = wave_sum_u64(bad);
    first = wave_min_u64(first);
    if ((threadIdx.x & 63) == 0 && bad) {
        atomicAdd(&res[0], bad);
        atomicMin(&res[1], first);
    }
}

int grid_for(i64 total) { return int(std::max<i64>(1, std::min<i64>(4096, (total + 255) / 256))); }

}  // namespace

template <class T>
void launch_pattern_fill(T* g, const GridView& gv, const Box& b, const PatternCoords& pc, int mode, double v,
                         hipStream_t s) {
    if (b.empty()) return;
    W3D_REQUIRE(b.i0 >= 1 - gv.G && b.i1 <= gv.X + gv.G && b.j0 >= 1 - gv.G && b.j1 <= gv.Y + gv.G &&
                    b.k0 >= 1 - gv.G && b.k1 <= gv.Z + gv.G,
                "pattern box outside the storage");
    hipLaunchKernelGGL(k_pattern_fill<T>, dim3(grid_for(b.count())), dim3(256), 0, s, g, gv.si, gv.sj, b, gv.X,
                       gv.Y, gv.Z, pc, mode, T(v));
    HIP_OK(hipGetLastError());
}

template <class T>
void launch_pattern_check(const T* g, const GridView& gv, const Box& b, const PatternCoords& pc, u64* res,
                          hipStream_t s) {
    if (b.empty()) return;
    W3D_REQUIRE(b.i0 >= 1 - gv.G && b.i1 <= gv.X + gv.G && b.j0 >= 1 - gv.G && b.j1 <= gv.Y + gv.G &&
                    b.k0 >= 1 - gv.G && b.k1 <= gv.Z + gv.G,
                "check box outside the storage");
    hipLaunchKernelGGL(k_pattern_check<T>, dim3(grid_for(b.count())), dim3(256), 0, s, g, gv.si, gv.sj, b, pc,
                       res);
    HIP_OK(hipGetLastError());
}

void launch_compare_bytes(const void* a, const void* b, size_t bytes, u64* res, hipStream_t s) {
    W3D_REQUIRE(bytes % 4 == 0, "mirror compare needs whole 4-byte words");
    const size_t n = bytes / 4;
    if (n == 0) return;
    hipLaunchKernelGGL(k_compare_words, dim3(grid_for(i64(n))), dim3(256), 0, s, static_cast<const unsigned*>(a),
                       static_cast<const unsigned*>(b), n, res);
    HIP_OK(hipGetLastError());
}

template void launch_pattern_fill<double>(double*, const GridView&, const Box&, const PatternCoords&, int, double,
                                          hipStream_t);
template void launch_pattern_fill<float>(float*, const GridView&, const Box&, const PatternCoords&, int, double,
                                         hipStream_t);
template void launch_pattern_check<double>(const double*, const GridView&, const Box&, const PatternCoords&, u64*,
                                           hipStream_t);
template void launch_pattern_check<float>(const float*, const GridView&, const Box&, const PatternCoords&, u64*,
                                          hipStream_t);

}  // namespace wave3d
