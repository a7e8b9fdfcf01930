// Negative control for the TSan + Archer test (tests/test_sanitizers.py): the update pattern
// of the reference's hybrid_new (hybrid_new.cpp:281-291) — threads of an
// OpenMP loop raise a shared running maximum without a reduction or atomic. The sanitizer
// build must report this program, so a clean report on the solver means something.
#include <cmath>
#include <cstdio>
#include <vector>

static double g_max_err = -100.0;  // shared, unsynchronised: the defect under test

int main() {
    const int n = 1 << 14;
    std::vector<double> u(n), f(n);
    for (int i = 0; i < n; ++i) u[i] = std::sin(0.001 * i), f[i] = std::sin(0.001 * i + 1e-7);
#pragma omp parallel for num_threads(4)
    for (int i = 0; i < n; ++i) {
        const double e = std::fabs(u[i] - f[i]);
        if (e > g_max_err) g_max_err = e;
    }
    std::printf("max %g\n", g_max_err);
    return 0;
}
