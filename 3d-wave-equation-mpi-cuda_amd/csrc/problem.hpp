// Physics of the test problem:
//   u_tt = a^2 Δu on [0,Lx]x[0,Ly]x[0,Lz], periodic in x, u = 0 on the y/z faces,
//   a^2 = 1/(4π^2), analytic u = sin(2πx/Lx) sin(πy/Ly) sin(πz/Lz) cos(a_t t + 2π),
//   a_t = ½ sqrt(4/Lx² + 1/Ly² + 1/Lz²)       (mpi_new.cpp:150-152, 396-400).
//
// The analytic factor is separable, so instead of 4 transcendentals per node and step
// (mpi_new.cpp:340) we keep 1-D tables sx[gx], sy[gy], sz[gz], ct[n] and evaluate
// f = ((sx*sy)*sz)*ct — each table entry is computed with *exactly* the reference's
// expression, so f is bitwise equal to the reference's an_sol() value.
#pragma once

#include <vector>

#include "config.hpp"

namespace wave3d {

struct Problem {
    int N = 0, K = 0;
    double Lx = 0, Ly = 0, Lz = 0, T = 0;
    double pi = 0;
    double phase = 0;  // IC phase shift in x (0 = reference IC)
    double a2 = 0, a_t = 0, tau = 0, hx = 0, hy = 0, hz = 0;
    double hx2 = 0, hy2 = 0, hz2 = 0;  // h*h, used as divisors exactly like laplace()
    double coef = 0;                   // a2*tau*tau          (mpi_new.cpp:338)
    double coef_first = 0;             // a2*tau*tau*0.5      (mpi_new.cpp:303)
    double courant = 0;                // sqrt(a2)*tau/min(h) (mpi_new.cpp:404)

    static Problem from_config(const Config& c);

    // Reference analytic solution, evaluated the reference way (4 transcendentals).
    double an_sol(double t, double x, double y, double z) const;

    // Separable tables over global node indices 0..N and layers 0..K.
    std::vector<double> table_x() const;
    std::vector<double> table_y() const;
    std::vector<double> table_z() const;
    std::vector<double> table_t() const;

    static constexpr double kPiRef = 3.1415926535;  // mpi_new.cpp:23
    static constexpr double kPiExact = 3.14159265358979323846;
    static constexpr double kCflLimit = 0.57735026918962576451;  // 1/sqrt(3), 3-D leapfrog
};

}  // namespace wave3d
