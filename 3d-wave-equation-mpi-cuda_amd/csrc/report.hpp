// Results, the reference-format output file and a JSON summary.
#pragma once

#include <string>
#include <vector>

#include "config.hpp"
#include "problem.hpp"
#include "topology.hpp"

namespace wave3d {

// --overlap auto: trial solves 2..7 (three arms, twice each)
constexpr int kOverlapTrialSolves = 6;

struct Timings {
    double init_ms = 0;      // allocation + table upload ("grids initialized in")
    double total_ms = 0;     // IC through last layer ("numerical solution calculated in")
    double loop_ms = 0;      // stencil / IC / boundary kernels
    double exchange_ms = 0;  // pack + transport + unpack (host-device exchange in cuda_sol)
    double comm_ms = 0;      // transport only ("total MPI exchange time")
    double error_ms = 0;     // error reduction finalisation
};

struct RunResult {
    int N = 0, K = 0, nprocs = 1, Np = 1;
    int dims[3] = {1, 1, 1};
    DType dtype = DType::F64;
    std::string backend;     // "hip" | "cpu"
    std::string kernel;      // stencil variant actually used
    std::string scheme = "leapfrog";  // time stepping: "leapfrog" | "delta" (increment form)
    std::string math = "exact";       // stencil arithmetic: "exact" (reference order) | "fma"
    std::string transport;   // "self" | "loopback" | "rccl" | "external"
    double courant = 0;
    std::vector<double> max_abs, max_rel;  // per layer, max over all ranks
    Timings t;                             // last timed solve, max over ranks
    std::vector<double> solve_ms;          // every timed solve (max over ranks)
    int layers_done = 0;
    bool aborted = false;
    int abort_layer = -1;
    std::string abort_reason;
    int resumed_from = -1;
    bool graph = false;  // time loop replayed as one hipGraph
    bool overlap = false;  // interior/shell split with the halo on a second stream (effective)
    std::string overlap_mode = "off";  // "on" | "off" | "auto" (requested; "none" = no halo)
    // --overlap auto: best trial solve time per arm (on with the shells beside the interior, off,
    // on with the shells first) and every trial in order (the three arms, twice)
    double overlap_trial_ms[3] = {0, 0, 0};
    double overlap_trials[kOverlapTrialSolves] = {};
    std::string overlap_order = "none";  // effective overlap order: beside | shells_first | none
    std::string overlap_order_run = "none";  // order of the enqueued (or replayed) layers
    int comm_size = 0;     // ranks the transport's communicator reports (ncclCommCount), 0 = none
    int rccl_max_ctas = -1;  // CTA budget of the RCCL communicator (0 = RCCL's own), -1 = none
    long rccl_mirror_msgs = 0;  // --rccl-mirror: messages sent through RCCL and compared
    long long overlap_interior = -1;  // min over ranks of nodes in the interior box that runs
                                      // concurrently with the halo (tb2/tb3: per sweep; -1: none)
    int halo_checked = 0;  // halo messages verified by the init-time self-test (0 = none ran)

    double points() const { return double(N + 1) * double(N + 1) * double(N + 1); }
    // Mpoints/s = (N+1)^3 * timesteps / t  (BASELINE.md metric definition)
    double mpts_per_s() const;
    double mpts_per_s_best() const;
    double linf_final() const { return max_abs.empty() ? 0.0 : max_abs.back(); }
};

// Default ostream formatting, identical to the reference's `out << double`.
std::string fmt_double(double v);

std::string output_filename(const Config& c, const RunResult& r);
// Text of the output file for the selected flavour (Appendix A).
std::string format_report(const Config& c, const RunResult& r);
void write_report(const Config& c, const RunResult& r);  // no-op for ReportFormat::None
std::string json_summary(const Config& c, const RunResult& r);

}  // namespace wave3d
