// Built with -ffp-contract=off: every expression below must round exactly like the
// reference's (mpi_new.cpp:150-152, 396-400) so the tables are bitwise identical.
#include "problem.hpp"

#include <algorithm>
#include <cmath>

namespace wave3d {

Problem Problem::from_config(const Config& c) {
    Problem p;
    p.pi = c.pi == PiMode::Ref ? kPiRef : kPiExact;
    const double PI = p.pi;
    p.N = c.N;
    p.K = c.timesteps;
    p.T = c.T;
    p.Lx = c.Lx_is_pi ? PI : c.Lx;
    p.Ly = c.Ly_is_pi ? PI : c.Ly;
    p.Lz = c.Lz_is_pi ? PI : c.Lz;
    p.phase = c.ic == ICMode::Shifted ? 0.7 : 0.0;
    p.a2 = 1 / (4 * PI * PI);
    p.a_t = 0.5 * std::sqrt(4 / (p.Lx * p.Lx) + 1 / (p.Ly * p.Ly) + 1 / (p.Lz * p.Lz));
    p.tau = p.T / p.K;
    p.hx = p.Lx / p.N;
    p.hy = p.Ly / p.N;
    p.hz = p.Lz / p.N;
    p.hx2 = p.hx * p.hx;
    p.hy2 = p.hy * p.hy;
    p.hz2 = p.hz * p.hz;
    p.coef = p.a2 * p.tau * p.tau;
    p.coef_first = p.a2 * p.tau * p.tau * 0.5;
    p.courant = std::sqrt(p.a2) * p.tau / std::min(p.hx, std::min(p.hy, p.hz));
    return p;
}

double Problem::an_sol(double t, double x, double y, double z) const {
    const double PI = pi;
    double sx = phase == 0.0 ? std::sin(2 * PI * x / Lx) : std::sin(2 * PI * x / Lx + phase);
    return sx * std::sin(PI * y / Ly) * std::sin(PI * z / Lz) * std::cos(a_t * t + 2 * PI);
}

std::vector<double> Problem::table_x() const {
    const double PI = pi;
    std::vector<double> v(N + 1);
    for (int g = 0; g <= N; ++g) {
        double x = hx * g;
        v[g] = phase == 0.0 ? std::sin(2 * PI * x / Lx) : std::sin(2 * PI * x / Lx + phase);
    }
    return v;
}

std::vector<double> Problem::table_y() const {
    const double PI = pi;
    std::vector<double> v(N + 1);
    for (int g = 0; g <= N; ++g) v[g] = std::sin(PI * (hy * g) / Ly);
    return v;
}

std::vector<double> Problem::table_z() const {
    const double PI = pi;
    std::vector<double> v(N + 1);
    for (int g = 0; g <= N; ++g) v[g] = std::sin(PI * (hz * g) / Lz);
    return v;
}

std::vector<double> Problem::table_t() const {
    const double PI = pi;
    std::vector<double> v(K + 1);
    for (int n = 0; n <= K; ++n) v[n] = std::cos(a_t * (tau * n) + 2 * PI);
    return v;
}

}  // namespace wave3d
