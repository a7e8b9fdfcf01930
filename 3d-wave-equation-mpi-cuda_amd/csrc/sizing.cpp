#include "sizing.hpp"

#include <algorithm>

#include "common.hpp"
#include "topology.hpp"

namespace wave3d {

// "tb2[r<R>][w<W>][k<NWK>][o<OCC>]" / "tb3[r<R>w<W>]" / "tb4[r<R>w<W>]"
static void parse_tb(const std::string& name, int& rows, int& waves, int& occ, int& kwaves) {
    if (name.rfind("tb3", 0) != 0 && name.rfind("tb4", 0) != 0) rows = 2, waves = 4;
    occ = 0;
    kwaves = 1;
    std::string s = name.substr(3);
    auto num = [&](char tag, int& out) {
        if (!s.empty() && s[0] == tag) {
            size_t n = 0;
            out = std::stoi(s.substr(1), &n);
            s = s.substr(1 + n);
        }
    };
    num('r', rows);
    num('w', waves);
    num('k', kwaves);
    num('o', occ);
    W3D_REQUIRE(s.empty(), "wave3d: unknown kernel variant " + name);
}

Layout plan_layout(const Config& c, int world) {
    Layout l;
    // "auto": temporal blocking (the measured fastest sweep per dtype / scheme / math, below). The process
    // grid is MPI_Dims_create's as in the reference (2x2x2 at 8 ranks; y/z splits get 2-deep
    // row/column halos); `--dims P,1,1` selects x slabs (contiguous planes, 2 peers)
    const bool auto_tb = c.kernel == "auto";
    // fp32: three-layer blocking (tb3r2w8, 4 waves per SIMD after the register diet) moves
    // 10.7 instead of 16 B per node-layer and beats tb2r2w8 by 12-14 % (leapfrog) / 3-4 %
    // (increment form), N=512 / 2048 (profiles/tb3_diet_r2.txt)
    // fp64 with --math fma: three-layer blocking too — the FMA form cuts the issue-bound fp64
    // sweep's VALU work (profiles/math_fma_r3.txt). After the scalar diet (steady-state body,
    // errors of three layers per table row) the 16-row r2w8 tile (2 waves/SIMD) beats the
    // 1-row r1w8 (4 waves/SIMD): 425-431k vs 402k Mpts/s at N=512 (profiles/tb3_salu_r3.txt)
    // fp64 exact leapfrog: tb3 too since the scalar diet — 373-374k vs tb2r2w8 317k Mpts/s at
    // N=512, bitwise equal (profiles/tb3_salu_r3.txt)
    // Since round 4 the leapfrog (fp64 and fp32, exact and FMA) runs four layers per sweep (tb4,
    // k_tbn r2w8: 8 B per node-layer instead of 10.7): fp64 fma 521-528k vs tb3 428-435k, exact
    // 433k vs 374k, fp32 fma 794k vs 791k, fp32 exact 825k vs 717k Mpts/s at N=512 K=100
    // (profiles/deep_sweeps_r4.txt). The increment form runs on tb3 (k_tbn's fp32 one is slower),
    // since round 4 the fp64 exact one too: 378-379k vs tb2r2w4 298k Mpts/s at N=512 after tb3's
    // register j-neighbours and the max-ilp build (deep_sweeps_r4.txt batch 33).
    // Round 5: the fp32 increment form with --math fma runs on tb4 too, two workgroups per CU:
    // 872-878k vs tb3 787-790k Mpts/s at N=512 (exact stays on tb3: 766k vs 675k;
    // profiles/deep_sweeps_r5.txt)
    const bool auto_tb4 = auto_tb && (!c.delta || (c.dtype == DType::F32 && c.fma));
    const bool auto_tb3 = auto_tb && !auto_tb4;
    const bool tbn3 = c.kernel.rfind("tbn3", 0) == 0;  // k_tbn at depth 3 (A/B of k_tb3)
    const bool tb4 = auto_tb4 || c.kernel.rfind("tb4", 0) == 0;
    const bool tb3 = !tb4 && (auto_tb3 || tbn3 || c.kernel.rfind("tb3", 0) == 0);
    l.generic = tb4 || tbn3;
    l.tb = auto_tb || tb3 || tb4 || c.kernel.rfind("tb2", 0) == 0;
    l.depth = tb4 ? 4 : (tb3 ? 3 : (l.tb ? 2 : 1));
    if (tb3 || tb4) l.rows = 2, l.waves = 8;  // measured best deep-sweep tile (profiles/)
    // 16-row tiles of 8 waves (tb2r2w8, 2 workgroups per CU): fp64 +2-3 % over r2w4 (128
    // VGPRs, 4 waves/SIMD), fp32 +3.5 % (N=512) / +5 % (N=2048) over tb2r4 (profiles/
    // ab_tiles_r2.txt, fp32_accuracy_r2.txt). The fp64 increment form needs a few more
    // registers: r2w8 drops to 3 waves/SIMD there, so it keeps the 8-row r2w4 tiles.
    if (auto_tb && !(c.delta && c.dtype == DType::F64)) l.waves = 8;
    if (l.tb && !auto_tb) parse_tb(tbn3 ? "tb3" + c.kernel.substr(4) : c.kernel, l.rows, l.waves, l.occ, l.kwaves);
    l.G = l.depth;      // ghost depth = layers per sweep
    // time levels: one stored layer per single step -> 3; a sweep stores two layers (tb2: u^m and
    // u^{m+1}; tb3: D and E, C never stored) and reads two -> 4 (hip_solver plan_slots)
    l.L = l.depth == 1 ? 3 : 4;
    for (int a = 0; a < 3; ++a) l.dims[a] = c.dims[a];
    (void)world;
    return l;
}

size_t level_elems(int X, int Y, int Z, int G, int elem_size) {
    const int A = 128 / elem_size;  // rows start on a 128-B boundary
    const size_t sj = size_t((A + Z + G + A - 1) / A) * A;
    return size_t(X + 2 * G) * size_t(Y + 2 * G) * sj;
}

size_t device_bytes_per_rank(const Config& c, int world) {
    const Layout l = plan_layout(c, world);
    const int es = c.dtype == DType::F64 ? 8 : 4;
    const bool have = l.dims[0] || l.dims[1] || l.dims[2];
    size_t best = 0;
    // extents differ only for the last coordinate on an axis: the last rank is the largest
    const Topology t = Topology::make(c.N, world, world - 1, have ? l.dims : nullptr);
    const int X = t.X(), Y = t.Y(), Z = t.Z();
    best = size_t(l.L) * level_elems(X, Y, Z, l.G, es) * es;
    best += size_t(X + Y + Z + 6) * es;                   // analytic tables
    best += size_t(c.timesteps + 1) * 3 * 8;              // error slots
    best += 2 * size_t(std::max(X, 1)) * (std::max(Y, Z) + 2) * es * 4;  // y/z face buffers
    if (l.tb && world > 1) best += size_t(Y + 2 * l.G) * (Z + 2 * l.G + 32) * es;  // seam plane
    return best;
}

int fill_hbm_N(const Config& c, int world, double budget_bytes) {
    Config q = c;
    int lo = 8, hi = 8;
    auto fits = [&](int N) {
        q.N = N;
        return double(device_bytes_per_rank(q, world)) <= budget_bytes;
    };
    W3D_REQUIRE(fits(lo), "fill-hbm: not even N=8 fits the budget");
    while (fits(hi * 2)) hi *= 2;
    lo = hi, hi = hi * 2;  // fits(lo), !fits(hi)
    while (hi - lo > 1) {
        const int mid = lo + (hi - lo) / 2;
        (fits(mid) ? lo : hi) = mid;
    }
    return lo;
}

}  // namespace wave3d
