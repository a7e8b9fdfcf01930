// Device-memory layout of the HIP solver and HBM sizing (SURVEY §5.7, §7.3 step 7:
// "288-GB sizing helper (--fill-hbm)"). Host-only, shared by the solver, the programs and
// the Python layer, so a planned N is exactly what the solver will allocate.
#pragma once

#include <cstddef>

#include "config.hpp"

namespace wave3d {

// Kernel family and storage shape the HIP solver picks for a configuration.
struct Layout {
    bool tb = false;          // temporal blocking
    int depth = 1;            // layers per sweep: 1 (single step), 2 (tb2), 3 (tb3) or 4 (tb4)
    bool generic = false;     // deep sweeps through the depth-generic kernel (k_tbn; "tbn3")
    int rows = 2, waves = 4;  // TB tile shape
    int occ = 0;              // TB register cap (min waves per SIMD, 0 = compiler's choice)
    int kwaves = 1;           // TB waves side by side along k (tile width 64 * kwaves)
    int G = 1;                // ghost depth
    int L = 3;                // time levels
    int dims[3] = {0, 0, 0};  // decomposition override (0 = Dims_create)
};
Layout plan_layout(const Config& c, int world);

// Elements of one padded time level of a rank with X x Y x Z owned nodes.
size_t level_elems(int X, int Y, int Z, int G, int elem_size);

// Largest device allocation of any rank (levels + tables + error slots), bytes.
size_t device_bytes_per_rank(const Config& c, int world);

// Largest N whose per-rank footprint fits `budget_bytes` (>= 8).
int fill_hbm_N(const Config& c, int world, double budget_bytes);

}  // namespace wave3d
