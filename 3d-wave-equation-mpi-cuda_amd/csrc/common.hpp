// wave3d — MI355X-native 3-D acoustic wave-equation solver.
// Shared plain-C++ definitions (no HIP): boxes, error-slot encoding, checks.
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace wave3d {

using i64 = long long;
using u64 = unsigned long long;

enum class DType { F64, F32 };

inline const char* dtype_name(DType d) { return d == DType::F64 ? "fp64" : "fp32"; }

// Inclusive index box in *local padded* coordinates (ghost layer at 0 and X+1).
struct Box {
    int i0 = 0, i1 = -1, j0 = 0, j1 = -1, k0 = 0, k1 = -1;
    bool empty() const { return i1 < i0 || j1 < j0 || k1 < k0; }
    i64 count() const {
        return empty() ? 0 : i64(i1 - i0 + 1) * i64(j1 - j0 + 1) * i64(k1 - k0 + 1);
    }
};

// Order-preserving map double -> u64 so that an unsigned integer max (atomicMax on the
// device, std::max on the host, ncclMax over ranks) equals the IEEE max of the doubles.
// NaNs never reach this encoding: the fused error loops skip them with the reference's
// `if (e > m) m = e` rule (mpi_new.cpp:343-344).
inline u64 encode_max_key(double d) {
    u64 b;
    std::memcpy(&b, &d, 8);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
inline double decode_max_key(u64 k) {
    u64 b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    double d;
    std::memcpy(&d, &b, 8);
    return d;
}

// Initial value of every per-layer maximum, as in the reference (mpi_new.cpp:25-26).
constexpr double kErrInit = -100.0;

struct Error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define W3D_REQUIRE(cond, msg)                                                   \
    do {                                                                         \
        if (!(cond)) throw ::wave3d::Error(std::string("wave3d: ") + (msg));     \
    } while (0)

}  // namespace wave3d
