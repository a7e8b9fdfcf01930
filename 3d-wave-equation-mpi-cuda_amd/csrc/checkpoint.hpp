// Checkpoint / resume (SURVEY §5.4 — absent in the reference).
//
// State needed to resume after layer n: the two newest levels u^{n-1}, u^n (owned nodes
// only, no ghosts), n itself, and the global per-layer error maxima for layers 0..n.
// One file per rank, `<dir>/ckpt_r<rank>.bin`, written to a temp name then renamed so a
// crash never leaves a torn checkpoint. The header pins N, K, the decomposition and the
// physics so a resume with a different configuration is refused.
#pragma once

#include <string>
#include <vector>

#include "config.hpp"
#include "topology.hpp"

namespace wave3d {

struct CheckpointHeader {
    char magic[8] = {'W', '3', 'D', 'C', 'K', 'P', 'T', '1'};
    int N = 0, K = 0, nprocs = 0, rank = 0;
    int dims[3] = {0, 0, 0};
    int coords[3] = {0, 0, 0};
    int ext[3] = {0, 0, 0};
    int layer = 0;
    int elem_size = 0;
    int pi_mode = 0, ic_mode = 0;
    double T = 0, Lx = 0, Ly = 0, Lz = 0;
};

CheckpointHeader make_header(const Config& c, const Topology& t, int layer, int elem_size);
std::string checkpoint_path(const std::string& dir, int rank);

// Host view of one level: element (i,j,k) of the owned block (1..X, 1..Y, 1..Z) lives at
// origin + (i*si + j*sj + k) elements. Only owned nodes are stored.
struct HostLevel {
    void* origin = nullptr;
    int X = 0, Y = 0, Z = 0;
    long long sj = 0, si = 0;
};

void write_checkpoint(const std::string& dir, const CheckpointHeader& h, const HostLevel& prev,
                      const HostLevel& cur, const std::vector<double>& max_abs,
                      const std::vector<double>& max_rel);

// Validates the header against `expect` (layer ignored), fills the owned nodes of `prev`
// (u^{n-1}) and `cur` (u^n), returns n. Call checkpoint_layer() first to learn n.
int read_checkpoint(const std::string& dir, const CheckpointHeader& expect, const HostLevel& prev,
                    const HostLevel& cur, std::vector<double>& max_abs, std::vector<double>& max_rel);
int checkpoint_layer(const std::string& dir, int rank);

}  // namespace wave3d
