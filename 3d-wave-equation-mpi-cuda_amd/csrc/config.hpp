// Command-line / run configuration.
//
// Positional part is identical to every reference program (C03):
//   prog N Np Lx Ly Lz [T=1] [timesteps=20]      (mpi_new.cpp:382-393, cuda_sol.cpp:453-464)
// `Lx|Ly|Lz` accept the literal `pi`. Long flags may follow the positionals.
#pragma once

#include <string>
#include <vector>

#include "common.hpp"

namespace wave3d {

enum class PiMode { Ref, Exact };      // truncated 3.1415926535 (CPU variants) vs full precision
enum class ICMode { Ref, Shifted };    // sin(2πx/Lx) vs sin(2πx/Lx + 0.7)
enum class ReportFormat { New, Omp, Cuda, None };

struct Config {
    // positionals
    int N = 32;
    int Np = 1;
    double Lx = 0, Ly = 0, Lz = 0;
    double T = 1.0;
    int timesteps = 20;
    bool Lx_is_pi = false, Ly_is_pi = false, Lz_is_pi = false;

    // extensions
    DType dtype = DType::F64;
    bool delta = false;             // --scheme delta: increment form u^n = u^{n-1} + d^n,
                                    // d^n = d^{n-1} + a2 tau^2 lap u^{n-1} (same scheme in exact
                                    // arithmetic; no 2u - u cancellation, fp32 accuracy)
    bool fma = false;               // --math fma: stencil update with coef/h^2 folded into FMAs
                                    // (temporal-blocking kernels; not bitwise with the reference)
    PiMode pi = PiMode::Ref;
    ICMode ic = ICMode::Ref;
    int dims[3] = {0, 0, 0};        // 0 = let dims_create choose (MPI_Dims_create semantics)
    bool overlap = true;            // interior/shell split with comm on a second stream
    bool overlap_auto = true;       // --overlap auto (default): solves 2-7 with halos run overlap
                                    // on / off / on with the shells first, twice each; the arm
                                    // with the fastest best is kept
    bool json = false;              // one-line JSON summary on stdout (rank 0)
    int check_every = 0;            // >0: abort early when a layer's error is NaN/Inf/>1
    bool strict_cfl = false;        // refuse C > 1/sqrt(3)
    std::string transport = "auto"; // auto | rccl | loopback
    bool halo_direct = true;        // --halo direct|rounds: deep halos of the temporal-blocking
                                    // kernels in one round (faces, edges, corners from their owners)
                                    // or in three dependent rounds (x planes, then y, then z boxes)
    bool x_self_transport = false;  // dims[0] == 1 with an external transport: the periodic
                                    // x wrap travels as messages to this rank (RCCL self
                                    // send/recv) instead of the fused local wrap (testing)
    int ranks = 0;                  // >0: number of logical ranks simulated in-process
    bool rccl_mirror = false;       // --ranks P: every loopback halo message also through a
                                    // 1-rank RCCL communicator, compared bitwise (testing)
    ReportFormat format = ReportFormat::New;
    std::string out_dir = ".";
    std::string out_name;           // override of output_N{N}_Np{Np}.txt
    bool quiet = false;
    int checkpoint_every = 0;
    std::string checkpoint_dir;
    std::string resume_dir;
    std::string kernel = "auto";    // auto | march* | naive | flat | tb2* | tb3* | tbn3 | tb4 (usage())
    int chunk = 0;                  // i-planes per marching work item (0 = auto)
    int repeat = 1;                 // timed solves (benchmark mode)
    int warmup = 0;                 // untimed solves before the timed ones
    bool profile = false;           // per-phase hipEvent timers
    int graph = -1;                 // hipGraph replay of the time loop: 1 on, 0 off, -1 auto
    double fill_hbm = 0;            // >0: replace N by the largest N using this HBM fraction
    bool halo_check = true;         // init-time halo self-test through the real plan/transport
    double model_link_gbps = 0;     // --model-link: simulated ranks' exchanges also wait the
    double model_link_lat_us = 0;   // modelled time of their busiest peer link (overlap studies)
    std::string fault;              // fault injection spec, e.g. "drop_face:1:5" (or env WAVE_FI)
    int device = -1;                // explicit device id (default: local rank)
    int threads = 0;                // CPU backend OpenMP threads (0 = Np)
    bool print_layers = true;       // "calculating layer n" lines on stdout (rank 0), as the
                                    // reference (cuda_sol.cpp:385, hybrid_new.cpp:340); off with
                                    // --no-print-layers or --quiet
    std::string dump;               // write the final layer as .npy (print_layer analogue)
};

// Parse argv; throws wave3d::Error with a usage message on malformed input.
Config parse_cli(int argc, const char* const* argv);
Config parse_cli(const std::vector<std::string>& args);  // args without argv[0]

std::string usage();

// "on" | "off" | "auto" — the run's --overlap mode (sizes the RCCL CTA budget)
inline std::string overlap_mode(const Config& c) { return !c.overlap ? "off" : (c.overlap_auto ? "auto" : "on"); }

}  // namespace wave3d
