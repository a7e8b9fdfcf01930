#include "topology.hpp"

#include <algorithm>
#include <sstream>
#include <vector>

namespace wave3d {

namespace {

// Most balanced non-increasing factorisation of p into n factors (n <= 3).
std::vector<int> balanced(int p, int n) {
    std::vector<int> best;
    if (n == 1) return {p};
    long best_spread = -1;
    if (n == 2) {
        for (int a = p; a >= 1; --a) {
            if (p % a) continue;
            int b = p / a;
            if (b > a) break;
            long s = a - b;
            if (best_spread < 0 || s < best_spread) best_spread = s, best = {a, b};
        }
        return best;
    }
    for (int a = p; a >= 1; --a) {
        if (p % a) continue;
        int q = p / a;
        for (int b = std::min(a, q); b >= 1; --b) {
            if (q % b) continue;
            int c = q / b;
            if (c > b) break;
            long s = a - c;
            if (best_spread < 0 || s < best_spread ||
                (s == best_spread && a < best[0])) {
                best_spread = s;
                best = {a, b, c};
            }
        }
    }
    return best;
}

}  // namespace

void Topology::dims_create(int nprocs, int dims[3]) {
    W3D_REQUIRE(nprocs >= 1, "nprocs must be >= 1");
    int fixed = 1, nfree = 0;
    for (int d = 0; d < 3; ++d) {
        W3D_REQUIRE(dims[d] >= 0, "negative dims");
        if (dims[d] > 0) fixed *= dims[d];
        else ++nfree;
    }
    W3D_REQUIRE(nprocs % fixed == 0, "nprocs not divisible by the preset dims");
    int rest = nprocs / fixed;
    if (nfree == 0) {
        W3D_REQUIRE(rest == 1, "dims product != nprocs");
        return;
    }
    std::vector<int> f = balanced(rest, nfree);
    int k = 0;
    for (int d = 0; d < 3; ++d)
        if (dims[d] == 0) dims[d] = f[k++];
}

Topology Topology::make(int N, int nprocs, int rank, const int* dims_override) {
    Topology t;
    t.N = N;
    t.nprocs = nprocs;
    t.rank = rank;
    W3D_REQUIRE(rank >= 0 && rank < nprocs, "rank out of range");
    int d[3] = {0, 0, 0};
    if (dims_override)
        for (int a = 0; a < 3; ++a) d[a] = dims_override[a];
    dims_create(nprocs, d);
    for (int a = 0; a < 3; ++a) t.dims[a] = d[a];
    t.coords[2] = rank % d[2];
    t.coords[1] = (rank / d[2]) % d[1];
    t.coords[0] = rank / (d[1] * d[2]);
    for (int a = 0; a < 3; ++a) {
        int base = (N + 1) / d[a];
        W3D_REQUIRE(base >= 1, "more ranks than nodes along an axis");
        t.off[a] = t.coords[a] * base;
        t.ext[a] = base + (t.last(a) ? (N + 1) % d[a] : 0);
    }
    for (int a = 0; a < 3; ++a) {
        for (int s = 0; s < 2; ++s) {
            int c[3] = {t.coords[0], t.coords[1], t.coords[2]};
            c[a] += s == 0 ? -1 : 1;
            if (c[a] < 0 || c[a] >= d[a]) {
                if (a != 0) {  // non-periodic: MPI_PROC_NULL
                    t.nbr[a][s] = -1;
                    continue;
                }
                c[a] = (c[a] + d[a]) % d[a];
            }
            t.nbr[a][s] = t.rank_of(c[0], c[1], c[2]);
        }
    }
    return t;
}

Box Topology::compute_box() const {
    Box b;
    b.i0 = 1;
    b.i1 = ext[0];
    b.j0 = first(1) ? 2 : 1;
    b.j1 = last(1) ? ext[1] - 1 : ext[1];
    b.k0 = first(2) ? 2 : 1;
    b.k1 = last(2) ? ext[2] - 1 : ext[2];
    return b;
}

Box Topology::error_box() const {
    Box b = compute_box();
    b.i0 = first(0) ? 2 : 1;
    b.i1 = last(0) ? ext[0] - 1 : ext[0];
    return b;
}

Box Topology::owned_box() const {
    Box b;
    b.i0 = b.j0 = b.k0 = 1;
    b.i1 = ext[0];
    b.j1 = ext[1];
    b.k1 = ext[2];
    return b;
}

std::string Topology::describe() const {
    std::ostringstream s;
    s << "rank " << rank << "/" << nprocs << " dims " << dims[0] << "x" << dims[1] << "x"
      << dims[2] << " coords (" << coords[0] << "," << coords[1] << "," << coords[2]
      << ") ext " << ext[0] << "x" << ext[1] << "x" << ext[2] << " off (" << off[0] << ","
      << off[1] << "," << off[2] << ")";
    return s.str();
}

}  // namespace wave3d
