// Solver entry points.
//
//  run_cpu : OpenMP backend — the test oracle and the `wave3d_cpu` program. Covers the
//            reference's omp / mpi_* / hybrid_* programs: P ranks are either simulated
//            in-process (--ranks P, deterministic loopback) or are real processes that
//            exchange through an external Transport (e.g. torch.distributed/gloo).
//  run_hip : MI355X backend (hip_solver.hip). P ranks are one process per GPU over RCCL,
//            or simulated in-process on one GPU (--ranks P, loopback D2D copies).
#pragma once

#include <memory>

#include "config.hpp"
#include "halo.hpp"
#include "report.hpp"

namespace wave3d {

// Owned nodes of one rank's block of a time level, k fastest (the reference's print_layer
// debug aid, C30: mpi_new.cpp:113-124).
struct FieldBlock {
    int rank = 0;
    int off[3] = {0, 0, 0};  // global index of the block's first node
    int ext[3] = {0, 0, 0};
    std::vector<double> data;
};

// A solver instance: allocation/tables once, then any number of complete solves
// (IC through layer K + error reduction). Each solve() is one timed benchmark step.
class Session {
public:
    virtual ~Session() = default;
    virtual RunResult solve() = 0;
    virtual double init_ms() const = 0;
    // After a solve: layer K (or K-1) of every rank of this process.
    virtual std::vector<FieldBlock> field(int layer) = 0;
};

// Writes the blocks as one (N+1)^3 float64 .npy file (all ranks local) or one file per rank
// (`path` + ".r<rank>.npy", the block with its offset in the header comment).
void dump_field(const std::string& path, int N, const std::vector<FieldBlock>& blocks, int world);

std::unique_ptr<Session> make_cpu_session(const Config& c, Transport* external = nullptr);
std::unique_ptr<Session> make_hip_session(const Config& c, Transport* external = nullptr);

RunResult run_session(Session& s, const Config& c);
RunResult run_cpu(const Config& c, Transport* external = nullptr);

// Implemented in the HIP library; `external` may be an RcclTransport or any device
// transport. `world_size/world_rank` describe the process group when external is null
// and no in-process ranks are requested.
RunResult run_hip(const Config& c, Transport* external = nullptr);

// Fault-injection spec parsed from --fault / WAVE_FI.
struct FaultSpec {
    std::string kind;  // "" | "drop_face" | "nan" | "corrupt_tag" (layer = the halo tag)
    int rank = -1;
    int layer = -1;
    static FaultSpec parse(const std::string& s);
    bool hits(int r, int n) const { return !kind.empty() && r == rank && n == layer; }
    // blocked sweeps exchange / store only some layers: a fault on a layer inside (lo, hi]
    // applies at the next layer that is exchanged / stored
    bool hits_range(int r, int lo, int hi) const {
        return !kind.empty() && r == rank && layer > lo && layer <= hi;
    }
};

// Early-abort rule for --check-every: a non-finite value was produced on the
// layer, or the max error is not a finite number in [0, 1].
bool layer_diverged(double max_abs, bool nonfinite);

// Per-layer reduction slots: {abs key, rel key, non-finite flag}, all max-reduced.
constexpr int kSlotsPerLayer = 3;

}  // namespace wave3d
