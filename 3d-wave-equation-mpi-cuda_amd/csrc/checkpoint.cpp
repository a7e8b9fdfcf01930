#include "checkpoint.hpp"

#include <cstdio>
#include <cstring>
#include <fstream>

namespace wave3d {

CheckpointHeader make_header(const Config& c, const Topology& t, int layer, int elem_size) {
    CheckpointHeader h;
    h.N = c.N;
    h.K = c.timesteps;
    h.nprocs = t.nprocs;
    h.rank = t.rank;
    for (int a = 0; a < 3; ++a) {
        h.dims[a] = t.dims[a];
        h.coords[a] = t.coords[a];
        h.ext[a] = t.ext[a];
    }
    h.layer = layer;
    h.elem_size = elem_size;
    h.pi_mode = int(c.pi);
    h.ic_mode = int(c.ic);
    h.T = c.T;
    h.Lx = c.Lx_is_pi ? -1.0 : c.Lx;
    h.Ly = c.Ly_is_pi ? -1.0 : c.Ly;
    h.Lz = c.Lz_is_pi ? -1.0 : c.Lz;
    return h;
}

std::string checkpoint_path(const std::string& dir, int rank) {
    return dir + "/ckpt_r" + std::to_string(rank) + ".bin";
}

namespace {

void io_owned(std::fstream& f, const HostLevel& L, int es, bool write) {
    const size_t row = size_t(L.Z) * es;
    char* base = static_cast<char*>(L.origin);
    for (int i = 1; i <= L.X; ++i)
        for (int j = 1; j <= L.Y; ++j) {
            char* p = base + (size_t(i) * L.si + size_t(j) * L.sj + 1) * es;
            if (write) f.write(p, row);
            else f.read(p, row);
        }
}

}  // namespace

void write_checkpoint(const std::string& dir, const CheckpointHeader& h, const HostLevel& prev,
                      const HostLevel& cur, const std::vector<double>& max_abs,
                      const std::vector<double>& max_rel) {
    std::string path = checkpoint_path(dir, h.rank);
    std::string tmp = path + ".tmp";
    {
        std::fstream f(tmp, std::ios::out | std::ios::binary | std::ios::trunc);
        W3D_REQUIRE(f.good(), "cannot write checkpoint " + tmp);
        f.write(reinterpret_cast<const char*>(&h), sizeof(h));
        int n = h.layer + 1;
        f.write(reinterpret_cast<const char*>(max_abs.data()), sizeof(double) * n);
        f.write(reinterpret_cast<const char*>(max_rel.data()), sizeof(double) * n);
        io_owned(f, prev, h.elem_size, true);
        io_owned(f, cur, h.elem_size, true);
        W3D_REQUIRE(f.good(), "checkpoint write failed " + tmp);
    }
    W3D_REQUIRE(std::rename(tmp.c_str(), path.c_str()) == 0, "cannot rename " + tmp);
}

int checkpoint_layer(const std::string& dir, int rank) {
    std::string path = checkpoint_path(dir, rank);
    std::fstream f(path, std::ios::in | std::ios::binary);
    W3D_REQUIRE(f.good(), "cannot open checkpoint " + path);
    CheckpointHeader h;
    f.read(reinterpret_cast<char*>(&h), sizeof(h));
    W3D_REQUIRE(f.good() && std::memcmp(h.magic, CheckpointHeader().magic, 8) == 0,
                "not a checkpoint: " + path);
    return h.layer;
}

int read_checkpoint(const std::string& dir, const CheckpointHeader& expect, const HostLevel& prev,
                    const HostLevel& cur, std::vector<double>& max_abs,
                    std::vector<double>& max_rel) {
    std::string path = checkpoint_path(dir, expect.rank);
    std::fstream f(path, std::ios::in | std::ios::binary);
    W3D_REQUIRE(f.good(), "cannot open checkpoint " + path);
    CheckpointHeader h;
    f.read(reinterpret_cast<char*>(&h), sizeof(h));
    W3D_REQUIRE(f.good() && std::memcmp(h.magic, expect.magic, 8) == 0, "not a checkpoint: " + path);
    bool same = h.N == expect.N && h.K == expect.K && h.nprocs == expect.nprocs &&
                h.rank == expect.rank && h.elem_size == expect.elem_size &&
                h.pi_mode == expect.pi_mode && h.ic_mode == expect.ic_mode && h.T == expect.T &&
                h.Lx == expect.Lx && h.Ly == expect.Ly && h.Lz == expect.Lz;
    for (int a = 0; a < 3; ++a)
        same = same && h.dims[a] == expect.dims[a] && h.coords[a] == expect.coords[a] &&
               h.ext[a] == expect.ext[a];
    W3D_REQUIRE(same, "checkpoint " + path + " does not match this configuration");
    const int n = h.layer;
    W3D_REQUIRE(n >= 1 && n < h.K, "checkpoint layer out of range");
    max_abs.assign(n + 1, 0.0);
    max_rel.assign(n + 1, 0.0);
    f.read(reinterpret_cast<char*>(max_abs.data()), sizeof(double) * (n + 1));
    f.read(reinterpret_cast<char*>(max_rel.data()), sizeof(double) * (n + 1));
    io_owned(f, prev, h.elem_size, false);
    io_owned(f, cur, h.elem_size, false);
    W3D_REQUIRE(f.good(), "truncated checkpoint " + path);
    return n;
}

}  // namespace wave3d
