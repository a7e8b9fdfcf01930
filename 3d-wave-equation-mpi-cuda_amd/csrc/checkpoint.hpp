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

// `prev`/`cur` are padded host arrays [nx][ny][pitch] (ghost layer 1); owned nodes only
// are written.
void write_checkpoint(const std::string& dir, const CheckpointHeader& h, const void* prev,
                      const void* cur, int nx, int ny, int nz, int pitch,
                      const std::vector<double>& max_abs, const std::vector<double>& max_rel);

// Validates the header against `expect` (layer ignored), fills the owned nodes of
// levels[(n+2)%3] (u^{n-1}) and levels[n%3] (u^n), returns n.
int read_checkpoint_raw(const std::string& dir, const CheckpointHeader& expect, void* levels[3],
                        int nx, int ny, int nz, int pitch, std::vector<double>& max_abs,
                        std::vector<double>& max_rel);

template <class V>
int read_checkpoint(const std::string& dir, const CheckpointHeader& expect, V (&g)[3], int nx,
                    int ny, int nz, int pitch, std::vector<double>& max_abs,
                    std::vector<double>& max_rel) {
    void* lv[3] = {g[0].data(), g[1].data(), g[2].data()};
    return read_checkpoint_raw(dir, expect, lv, nx, ny, nz, pitch, max_abs, max_rel);
}

}  // namespace wave3d
