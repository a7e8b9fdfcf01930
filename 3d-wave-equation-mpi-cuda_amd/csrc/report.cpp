#include "report.hpp"

#include <algorithm>
#include <cmath>
#include <fstream>
#include <sstream>

namespace wave3d {

double RunResult::mpts_per_s() const {
    if (t.total_ms <= 0) return 0.0;
    return points() * double(K) / (t.total_ms * 1e-3) / 1e6;
}

double RunResult::mpts_per_s_best() const {
    double best = 0.0;
    for (double ms : solve_ms) {
        if (ms > 0) best = std::max(best, points() * double(K) / (ms * 1e-3) / 1e6);
    }
    return best > 0 ? best : mpts_per_s();
}

std::string fmt_double(double v) {
    std::ostringstream s;
    s << v;
    return s.str();
}

std::string output_filename(const Config& c, const RunResult& r) {
    if (!c.out_name.empty()) return c.out_name;
    return "output_N" + std::to_string(r.N) + "_Np" + std::to_string(r.Np) + ".txt";
}

std::string format_report(const Config& c, const RunResult& r) {
    std::ostringstream out;
    auto ums = [](double ms) { return (unsigned)(ms); };
    auto errors = [&]() {
        for (size_t n = 0; n < r.max_abs.size(); ++n)
            out << "max abs and rel errors on layer " << n << ": " << r.max_abs[n] << " "
                << r.max_rel[n] << "\n";
    };
    switch (c.format) {
        case ReportFormat::Omp:  // openmp_sol.cpp:166,188
            out << "numerical solution calculated in " << ums(r.t.total_ms) << "ms\n";
            errors();
            break;
        case ReportFormat::Cuda:  // cuda_sol.cpp:572,427,435,438-441
            out << "initialization done in " << ums(r.t.init_ms) << "ms\n";
            out << "numerical solution calculated in " << float(r.t.total_ms) << "ms\n";
            errors();
            // cuda_sol's D2H/H2D staging time; here the pack/unpack (and box staging) kernels
            // around the transport: the exchange interval minus the transport itself
            out << "total host-device exchange time: " << float(std::max(0.0, r.t.exchange_ms - r.t.comm_ms))
                << " ms\n";
            out << "total loop time: " << float(r.t.loop_ms) << " ms\n";
            out << "total MPI exchange time: " << float(r.t.comm_ms) << " ms\n";
            out << "total error calculation time: " << float(r.t.error_ms) << " ms\n";
            break;
        case ReportFormat::New:  // mpi_new.cpp:474,356,364,369-370
            out << "grids initialized in " << ums(r.t.init_ms) << "ms\n";
            out << "numerical solution calculated in " << ums(r.t.total_ms) << "ms\n";
            errors();
            out << "total MPI exchange time: " << ums(r.t.comm_ms) << "ms\n";
            out << "total loop time: " << ums(r.t.loop_ms) << "ms\n";
            break;
        case ReportFormat::None:
            break;
    }
    if (r.aborted)
        out << "aborted on layer " << r.abort_layer << ": " << r.abort_reason << "\n";
    return out.str();
}

void write_report(const Config& c, const RunResult& r) {
    if (c.format == ReportFormat::None) return;
    std::string path = c.out_dir.empty() ? output_filename(c, r)
                                         : c.out_dir + "/" + output_filename(c, r);
    std::ofstream f(path);
    W3D_REQUIRE(f.good(), "cannot open " + path);
    f << format_report(c, r);
}

namespace {
std::string jnum(double v) {
    if (!std::isfinite(v)) return "null";
    std::ostringstream s;
    s.precision(9);
    s << v;
    return s.str();
}
}  // namespace

std::string json_summary(const Config& c, const RunResult& r) {
    std::ostringstream s;
    s << "{\"N\": " << r.N << ", \"timesteps\": " << r.K << ", \"nprocs\": " << r.nprocs
      << ", \"dims\": [" << r.dims[0] << ", " << r.dims[1] << ", " << r.dims[2] << "]"
      << ", \"dtype\": \"" << dtype_name(r.dtype) << "\", \"backend\": \"" << r.backend
      << "\", \"kernel\": \"" << r.kernel << "\", \"scheme\": \"" << r.scheme << "\", \"math\": \"" << r.math
      << "\", \"transport\": \"" << r.transport << "\""
      << ", \"overlap\": " << (r.overlap ? "true" : "false") << ", \"overlap_mode\": \"" << r.overlap_mode
      << "\", \"overlap_order\": \"" << r.overlap_order << "\", \"overlap_order_run\": \"" << r.overlap_order_run
      << "\""
      << ", \"overlap_trial_ms\": [" << jnum(r.overlap_trial_ms[0]) << ", " << jnum(r.overlap_trial_ms[1]) << ", "
      << jnum(r.overlap_trial_ms[2]) << "]"
      << ", \"overlap_trials_ms\": [";
    for (int q = 0; q < kOverlapTrialSolves; ++q) s << (q ? ", " : "") << jnum(r.overlap_trials[q]);
    s << "]"
      << ", \"comm_size\": " << r.comm_size << ", \"rccl_max_ctas\": " << r.rccl_max_ctas
      << ", \"halo_checked\": " << r.halo_checked
      << ", \"rccl_mirror_msgs\": " << r.rccl_mirror_msgs
      << ", \"courant\": " << jnum(r.courant) << ", \"total_ms\": " << jnum(r.t.total_ms)
      << ", \"init_ms\": " << jnum(r.t.init_ms) << ", \"loop_ms\": " << jnum(r.t.loop_ms)
      << ", \"exchange_ms\": " << jnum(r.t.exchange_ms) << ", \"comm_ms\": " << jnum(r.t.comm_ms)
      << ", \"mpts_per_s\": " << jnum(r.mpts_per_s())
      << ", \"mpts_per_s_best\": " << jnum(r.mpts_per_s_best())
      << ", \"linf_abs\": " << jnum(r.linf_final())
      << ", \"max_rel_final\": " << jnum(r.max_rel.empty() ? 0.0 : r.max_rel.back())
      << ", \"solve_ms\": [";
    for (size_t i = 0; i < r.solve_ms.size(); ++i) s << (i ? ", " : "") << jnum(r.solve_ms[i]);
    s << "], \"aborted\": " << (r.aborted ? "true" : "false")
      << ", \"graph\": " << (r.graph ? "true" : "false") << "}";
    return s.str();
}

}  // namespace wave3d
