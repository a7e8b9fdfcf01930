#include "checkpoint.hpp"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>

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
    h.scheme = c.delta ? 1 : 0;
    h.math = c.fma ? 1 : 0;
    return h;
}

std::string checkpoint_path(const std::string& dir, int rank, int layer) {
    return dir + "/ckpt_r" + std::to_string(rank) + "_L" + std::to_string(layer) + ".bin";
}

namespace {

void io_owned(const HostLevel& L, int es, const std::function<void(char*, size_t)>& op) {
    const size_t row = size_t(L.Z) * es;
    char* base = static_cast<char*>(L.origin);
    for (int i = 1; i <= L.X; ++i)
        for (int j = 1; j <= L.Y; ++j) op(base + (size_t(i) * L.si + size_t(j) * L.sj + 1) * es, row);
}

void write_all(int fd, const void* p, size_t n, const std::string& path) {
    const char* c = static_cast<const char*>(p);
    while (n > 0) {
        const ssize_t w = ::write(fd, c, n);
        if (w < 0 && errno == EINTR) continue;
        W3D_REQUIRE(w > 0, "checkpoint write failed " + path + ": " + std::strerror(errno));
        c += w, n -= size_t(w);
    }
}

void fsync_dir(const std::string& dir) {
    const int fd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY);
    if (fd >= 0) {
        (void)::fsync(fd);
        ::close(fd);
    }
}

bool read_header(const std::string& path, CheckpointHeader& h) {
    std::ifstream f(path, std::ios::binary);
    if (!f.good()) return false;
    f.read(reinterpret_cast<char*>(&h), sizeof(h));
    return f.good() && std::memcmp(h.magic, CheckpointHeader().magic, 8) == 0;
}

}  // namespace

void make_dirs(const std::string& dir) {  // mkdir -p
    for (size_t p = 1; p <= dir.size(); ++p)
        if (p == dir.size() || dir[p] == '/') {
            const std::string sub = dir.substr(0, p);
            if (::mkdir(sub.c_str(), 0755) != 0 && errno != EEXIST)
                throw Error("cannot create checkpoint directory " + sub + ": " + std::strerror(errno));
        }
}

void write_checkpoint(const std::string& dir, const CheckpointHeader& h, const HostLevel& prev,
                      const HostLevel& cur, const std::vector<double>& max_abs,
                      const std::vector<double>& max_rel) {
    make_dirs(dir);
    const std::string path = checkpoint_path(dir, h.rank, h.layer);
    const std::string tmp = path + ".tmp";
    const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    W3D_REQUIRE(fd >= 0, "cannot write checkpoint " + tmp + ": " + std::strerror(errno));
    try {
        write_all(fd, &h, sizeof(h), tmp);
        const size_t n = size_t(h.layer) + 1;
        write_all(fd, max_abs.data(), sizeof(double) * n, tmp);
        write_all(fd, max_rel.data(), sizeof(double) * n, tmp);
        auto w = [&](char* p, size_t b) { write_all(fd, p, b, tmp); };
        io_owned(prev, h.elem_size, w);
        io_owned(cur, h.elem_size, w);
        W3D_REQUIRE(::fsync(fd) == 0, "fsync failed on " + tmp);
    } catch (...) {
        ::close(fd);
        throw;
    }
    ::close(fd);
    W3D_REQUIRE(std::rename(tmp.c_str(), path.c_str()) == 0, "cannot rename " + tmp);
    fsync_dir(dir);
}

bool same_run(const CheckpointHeader& h, const CheckpointHeader& e) {
    bool same = std::memcmp(h.magic, e.magic, 8) == 0 && h.N == e.N && h.K == e.K && h.nprocs == e.nprocs &&
                h.rank == e.rank && h.elem_size == e.elem_size && h.pi_mode == e.pi_mode &&
                h.ic_mode == e.ic_mode && h.T == e.T && h.Lx == e.Lx && h.Ly == e.Ly && h.Lz == e.Lz &&
                h.scheme == e.scheme && h.math == e.math;
    for (int a = 0; a < 3; ++a)
        same = same && h.dims[a] == e.dims[a] && h.coords[a] == e.coords[a] && h.ext[a] == e.ext[a];
    return same;
}

std::vector<int> checkpoint_layers(const std::string& dir, int rank, const CheckpointHeader* match) {
    std::vector<int> out;
    DIR* d = ::opendir(dir.c_str());
    if (!d) return out;
    const std::string pre = "ckpt_r" + std::to_string(rank) + "_L";
    while (dirent* e = ::readdir(d)) {
        const std::string name = e->d_name;
        if (name.rfind(pre, 0) != 0 || name.size() < pre.size() + 5) continue;
        if (name.compare(name.size() - 4, 4, ".bin") != 0) continue;  // skips *.bin.tmp
        const std::string num = name.substr(pre.size(), name.size() - pre.size() - 4);
        // digits only, at most 9 of them (a layer is an int): anything else is not ours
        if (num.empty() || num.size() > 9 || num.find_first_not_of("0123456789") != std::string::npos) continue;
        CheckpointHeader h;
        const int layer = int(std::strtol(num.c_str(), nullptr, 10));
        if (read_header(dir + "/" + name, h) && h.layer == layer && h.rank == rank && (!match || same_run(h, *match)))
            out.push_back(layer);
    }
    ::closedir(d);
    std::sort(out.begin(), out.end());
    return out;
}

void prune_checkpoints(const std::string& dir, const CheckpointHeader& mine, int newest, int keep) {
    std::vector<int> l = checkpoint_layers(dir, mine.rank, &mine);
    for (int n : l)
        if (n > newest) (void)std::remove(checkpoint_path(dir, mine.rank, n).c_str());
    l.erase(std::remove_if(l.begin(), l.end(), [&](int n) { return n > newest; }), l.end());
    for (size_t q = 0; q + size_t(keep) < l.size(); ++q)
        (void)std::remove(checkpoint_path(dir, mine.rank, l[q]).c_str());
}

int agree_resume_layer(const std::string& dir, const std::vector<CheckpointHeader>& expect, Transport* ext) {
    // newest layer complete on every local rank (ranks keep two generations, see header)
    double neg = -1e300;  // max over ranks of -(newest common layer) = -(min)
    for (const auto& e : expect) {
        const std::vector<int> l = checkpoint_layers(dir, e.rank, &e);
        W3D_REQUIRE(!l.empty(), "no checkpoint of rank " + std::to_string(e.rank) + " for this configuration in " + dir);
        neg = std::max(neg, -double(l.back()));
    }
    if (ext) ext->allreduce_max_host(&neg, 1);
    const int n = int(-neg);
    double missing = 0;
    for (const auto& e : expect) {
        const std::vector<int> l = checkpoint_layers(dir, e.rank, &e);
        if (!std::binary_search(l.begin(), l.end(), n)) missing = 1;
    }
    if (ext) ext->allreduce_max_host(&missing, 1);
    W3D_REQUIRE(missing == 0, "checkpoints in " + dir + " have no layer common to every rank (newest common " +
                                  std::to_string(n) + ")");
    return n;
}

int read_checkpoint(const std::string& dir, const CheckpointHeader& expect, const HostLevel& prev,
                    const HostLevel& cur, std::vector<double>& max_abs,
                    std::vector<double>& max_rel) {
    const std::string path = checkpoint_path(dir, expect.rank, expect.layer);
    std::ifstream f(path, std::ios::binary);
    W3D_REQUIRE(f.good(), "cannot open checkpoint " + path);
    CheckpointHeader h;
    f.read(reinterpret_cast<char*>(&h), sizeof(h));
    W3D_REQUIRE(f.good() && std::memcmp(h.magic, expect.magic, 8) == 0, "not a checkpoint: " + path);
    W3D_REQUIRE(same_run(h, expect) && h.layer == expect.layer,
                "checkpoint " + path + " does not match this configuration");
    const int n = h.layer;
    W3D_REQUIRE(n >= 1 && n < h.K, "checkpoint layer out of range");
    max_abs.assign(n + 1, 0.0);
    max_rel.assign(n + 1, 0.0);
    f.read(reinterpret_cast<char*>(max_abs.data()), sizeof(double) * (n + 1));
    f.read(reinterpret_cast<char*>(max_rel.data()), sizeof(double) * (n + 1));
    auto r = [&](char* p, size_t b) { f.read(p, std::streamsize(b)); };
    io_owned(prev, h.elem_size, r);
    io_owned(cur, h.elem_size, r);
    W3D_REQUIRE(f.good(), "truncated checkpoint " + path);
    return n;
}

}  // namespace wave3d
