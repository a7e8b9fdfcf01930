// wave3d_cpu — OpenMP backend program. Replaces the reference's omp / mpi_sol / mpi_new /
// hyb_sol / hyb_new programs (one algorithm): `Np` = OpenMP threads
// (openmp_sol.cpp:194), `--ranks P` decomposes the domain over P in-process ranks exactly
// as mpirun -n P would (deterministic loopback transport).
#include <iostream>

#include "cli_common.hpp"
#include "solver.hpp"

int main(int argc, char** argv) {
    using namespace wave3d;
    try {
        Config c = parse_cli(argc, argv);
        if (c.format == ReportFormat::New && c.ranks == 0) c.format = ReportFormat::Omp;
        Problem p = Problem::from_config(c);
        if (!courant_check(c, p, true)) return 2;
        if (!c.quiet) {
            int P = std::max(1, c.ranks);
            for (int r = 0; r < P; ++r)
                std::cout << "Process " << r << " local rank = " << r << " local size = " << P
                          << " hostname = " << host_name() << std::endl;
        }
        RunResult r = run_cpu(c);
        finish(c, r, true);
        return r.aborted ? 3 : 0;
    } catch (const std::exception& e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
}
