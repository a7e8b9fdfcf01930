// Halo-plan self-test and RCCL mirror checks (hip_selftest.hip), host interface.
//
// Pattern: every node of the global grid has a value that depends on its global position
// (x wrapped on the periodic axis) and a per-level salt; nodes outside the global domain
// (ghosts beyond a Dirichlet face) and unreceived ghosts hold the sentinel. The values are
// integers below 2^23, exact in fp32 and fp64, never 0 and never the sentinel.
#pragma once

#include <hip/hip_runtime.h>

#include "hip_kernels.hpp"

namespace wave3d {

constexpr double kPatternSentinel = -1.0;

#ifdef __HIPCC__
#define W3D_SHD __host__ __device__ __forceinline__
#else
#define W3D_SHD inline
#endif

W3D_SHD double halo_pattern_value(i64 gi, i64 gj, i64 gk, unsigned salt) {
    u64 h = u64(gi) * 0x9E3779B97F4A7C15ull ^ u64(gj) * 0xC2B2AE3D27D4EB4Full ^ u64(gk) * 0x165667B19E3779F9ull ^
            u64(salt) * 0xD6E8FEB86659FD93ull;
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    return double(1 + (h & 0x3FFFFFull));
}

struct PatternCoords {
    int off[3] = {0, 0, 0};  // global index of local index 1 per axis
    int N = 0;
    unsigned salt = 0;
    i64 gi_fixed = -1;       // >= 0: every cell is global plane gi_fixed (seam alias planes)
};

template <class T>
void launch_pattern_fill(T* g, const GridView& gv, const Box& b, const PatternCoords& pc, int mode, double v,
                         hipStream_t s);
// res[0] += mismatches in the box, res[1] = min linear (k fastest) index of one (u64 max: none)
template <class T>
void launch_pattern_check(const T* g, const GridView& gv, const Box& b, const PatternCoords& pc, u64* res,
                          hipStream_t s);
// res[0] += differing 4-byte words of a and b, res[1] = min index of one
void launch_compare_bytes(const void* a, const void* b, size_t bytes, u64* res, hipStream_t s);

}  // namespace wave3d
