// Checkpoint / resume (SURVEY §5.4 — absent in the reference).
//
// State needed to resume after layer n: the two newest levels u^{n-1}, u^n (increment form:
// d^n, u^n) — owned nodes only, no ghosts — n itself, and the global per-layer error maxima
// for layers 0..n.
// One file per rank and checkpoint layer, `<dir>/ckpt_r<rank>_L<n>.bin`, written to a temp
// name, fsync'ed, then renamed (and the directory fsync'ed) so a crash never leaves a torn
// file. Every rank keeps its two newest complete generations: ranks write asynchronously,
// but the halo exchanges keep them within one checkpoint of each other, so the newest layer
// that *every* rank has complete is always still on disk. Resume agrees on that layer across
// all ranks (local ones and, through the transport, every process) before reading anything,
// so processes never resume from different layers. The header pins N, K, the decomposition
// and the physics so a resume with a different configuration is refused.
#pragma once

#include <string>
#include <vector>

#include "config.hpp"
#include "halo.hpp"
#include "topology.hpp"

namespace wave3d {

struct CheckpointHeader {
    char magic[8] = {'W', '3', 'D', 'C', 'K', 'P', 'T', '3'};  // 3: + math (files of version 2 are refused)
    int N = 0, K = 0, nprocs = 0, rank = 0;
    int dims[3] = {0, 0, 0};
    int coords[3] = {0, 0, 0};
    int ext[3] = {0, 0, 0};
    int layer = 0;
    int elem_size = 0;
    int pi_mode = 0, ic_mode = 0;
    double T = 0, Lx = 0, Ly = 0, Lz = 0;
    int scheme = 0;  // 0 leapfrog: levels u^{n-1}, u^n; 1 increment form: d^n, u^n
    int math = 0;    // 0 exact (bitwise with the reference programs), 1 --math fma
};

CheckpointHeader make_header(const Config& c, const Topology& t, int layer, int elem_size);
std::string checkpoint_path(const std::string& dir, int rank, int layer);
// Same run: every header field but the layer (N, K, decomposition, physics, dtype, scheme,
// arithmetic: an fma run never resumes from — or prunes — an exact run's files, or the reverse).
bool same_run(const CheckpointHeader& a, const CheckpointHeader& b);
// Layers for which `rank` has a complete checkpoint file in `dir`, ascending; with `match`,
// only files written by the same run configuration (a directory may hold files of others).
std::vector<int> checkpoint_layers(const std::string& dir, int rank, const CheckpointHeader* match = nullptr);
// After this run wrote layer `newest`: remove the rank's files of this configuration with a
// higher layer (left by an earlier run that got further: never newer state than this run's),
// then every one older than the `keep` newest complete generations. Files of other
// configurations are left alone.
void prune_checkpoints(const std::string& dir, const CheckpointHeader& mine, int newest, int keep = 2);
// The resume layer: newest layer for which every rank (the local ones, and every process
// through `ext` when given) has a complete file matching its expected header (`expect`, one
// per local rank, layer ignored); throws if some rank lacks it.
int agree_resume_layer(const std::string& dir, const std::vector<CheckpointHeader>& expect, Transport* ext);

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

// Reads the checkpoint of expect.rank at expect.layer: validates the header against `expect`,
// fills the owned nodes of `prev` (u^{n-1}) and `cur` (u^n), returns n.
int read_checkpoint(const std::string& dir, const CheckpointHeader& expect, const HostLevel& prev,
                    const HostLevel& cur, std::vector<double>& max_abs, std::vector<double>& max_rel);

}  // namespace wave3d
