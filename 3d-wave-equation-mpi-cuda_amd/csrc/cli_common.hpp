// Shared pieces of the wave3d / wave3d_cpu programs (reference stdout).
#pragma once

#include <unistd.h>

#include <iostream>
#include <string>

#include "config.hpp"
#include "problem.hpp"
#include "report.hpp"

namespace wave3d {

inline std::string host_name() {
    char h[256] = {0};
    gethostname(h, sizeof(h) - 1);
    return h;
}

// "C = ..." (mpi_new.cpp:402-405) plus the stability guard the reference lacks (B9).
// Returns false when --strict-cfl refuses the run.
inline bool courant_check(const Config& c, const Problem& p, bool print) {
    if (print && !c.quiet) std::cout << "C = " << p.courant << std::endl;
    if (p.courant > Problem::kCflLimit) {
        if (print)
            std::cerr << "wave3d: warning: Courant number " << p.courant
                      << " exceeds the 3-D leapfrog limit 1/sqrt(3); the scheme will diverge"
                      << (c.strict_cfl ? " (refused: --strict-cfl)" : "") << std::endl;
        if (c.strict_cfl) return false;
    }
    return true;
}

inline void finish(const Config& c, const RunResult& r, bool root) {
    if (!root) return;
    write_report(c, r);
    if (c.json) std::cout << json_summary(c, r) << std::endl;
    if (r.aborted)
        std::cerr << "wave3d: aborted on layer " << r.abort_layer << " (" << r.abort_reason << ")"
                  << std::endl;
}

}  // namespace wave3d
