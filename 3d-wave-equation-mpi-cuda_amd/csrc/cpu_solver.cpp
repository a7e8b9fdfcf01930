// OpenMP backend: the oracle for every HIP kernel and the `wave3d_cpu` program.
//
// Same algorithm as the reference's mpi_new / hybrid_new with the
// defects of Appendix B fixed: proper (N+1) strides (B3), race-free maxima (B4),
// 64-bit indexing (B7). P ranks run either in this process (loopback, deterministic:
// all ranks pack, the hub copies, all ranks unpack) or as separate processes that use
// an external Transport.
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <memory>
#include <sstream>

#include "checkpoint.hpp"
#include "log.hpp"
#include "problem.hpp"
#include "solver.hpp"
#include "stencil_math.hpp"
#include "topology.hpp"

namespace wave3d {

FaultSpec FaultSpec::parse(const std::string& s) {
    FaultSpec f;
    if (s.empty()) return f;
    std::stringstream ss(s);
    std::string kind, r, n;
    std::getline(ss, kind, ':');
    std::getline(ss, r, ':');
    std::getline(ss, n, ':');
    W3D_REQUIRE(kind == "drop_face" || kind == "nan" || kind == "corrupt_tag", "bad fault spec " + s);
    f.kind = kind;
    f.rank = std::stoi(r);
    f.layer = std::stoi(n);
    return f;
}

bool layer_diverged(double max_abs, bool nonfinite_seen) {
    if (nonfinite_seen) return true;
    return !(max_abs >= 0.0 && max_abs <= 1.0);
}

namespace {

using clk = std::chrono::steady_clock;
double ms_since(clk::time_point t0) {
    return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

template <class T>
struct RankState {
    Topology topo;
    int nx = 0, ny = 0, nz = 0;  // padded extents
    i64 sj = 0, si = 0;          // strides of j and i (k stride 1)
    std::vector<T> g[3];
    std::vector<T> tx, ty, tz;   // analytic tables indexed by local index
    HaloPlan plan;
    std::vector<std::vector<T>> sbuf, rbuf;
    std::vector<double> mabs, mrel;
    std::vector<unsigned char> bad;  // non-finite seen, per layer

    i64 idx(int i, int j, int k) const { return i64(i) * si + i64(j) * sj + k; }
};

template <class T>
class CpuSolver {
public:
    CpuSolver(const Config& c, Transport* ext) : cfg_(c), ext_(ext) {
        prob_ = Problem::from_config(c);
        fault_ = FaultSpec::parse(c.fault);
        if (ext_) {
            world_ = ext_->size();
            local_ranks_ = {ext_->rank()};
        } else {
            world_ = std::max(1, c.ranks);
            for (int r = 0; r < world_; ++r) local_ranks_.push_back(r);
        }
        threads_ = c.threads > 0 ? c.threads : std::max(1, c.Np);
        W3D_REQUIRE(!c.x_self_transport, "--x-self-transport is a HIP/RCCL test mode");
    }

    void init() {
        auto t_init = clk::now();
        setup();
        init_ms_ = ms_since(t_init);
    }

    double init_ms() const { return init_ms_; }

    std::vector<FieldBlock> field(int layer) {
        const int K = prob_.K;
        W3D_REQUIRE(layer >= std::max(0, K - 1) && layer <= K, "field: only layers K-1 and K are kept");
        std::vector<FieldBlock> out;
        for (auto& R : ranks_) {
            FieldBlock b;
            b.rank = R.topo.rank;
            for (int a = 0; a < 3; ++a) b.off[a] = R.topo.off[a], b.ext[a] = R.topo.ext[a];
            const auto& u = R.g[layer % 3];
            b.data.reserve(size_t(b.ext[0]) * b.ext[1] * b.ext[2]);
            for (int i = 1; i <= b.ext[0]; ++i)
                for (int j = 1; j <= b.ext[1]; ++j)
                    for (int k = 1; k <= b.ext[2]; ++k) b.data.push_back(double(u[R.idx(i, j, k)]));
            out.push_back(std::move(b));
        }
        return out;
    }

    RunResult solve_one() {
        RunResult res;
        res.N = prob_.N;
        res.K = prob_.K;
        res.nprocs = world_;
        res.Np = cfg_.Np;
        res.dtype = cfg_.dtype;
        res.backend = "cpu";
        res.kernel = "openmp";
        res.transport = ext_ ? ext_->name() : (world_ > 1 ? "loopback" : "self");
        res.comm_size = ext_ ? ext_->comm_size() : 0;
        res.scheme = cfg_.delta ? "delta" : "leapfrog";
        res.math = cfg_.fma ? "fma" : "exact";
        res.courant = prob_.courant;
        for (int a = 0; a < 3; ++a) res.dims[a] = ranks_[0].topo.dims[a];
        Timings t;
        solve(res, t);
        t.init_ms = init_ms_;
        double tv[5] = {t.total_ms, t.loop_ms, t.exchange_ms, t.comm_ms, t.error_ms};
        if (ext_) ext_->allreduce_max_host(tv, 5);
        t.total_ms = tv[0], t.loop_ms = tv[1], t.exchange_ms = tv[2], t.comm_ms = tv[3];
        t.error_ms = tv[4];
        res.t = t;
        res.solve_ms.push_back(t.total_ms);
        return res;
    }

private:
    void setup() {
        auto tx = prob_.table_x(), ty = prob_.table_y(), tz = prob_.table_z();
        ranks_.resize(local_ranks_.size());
        for (size_t q = 0; q < local_ranks_.size(); ++q) {
            auto& R = ranks_[q];
            R.topo = Topology::make(prob_.N, world_, local_ranks_[q],
                                    (cfg_.dims[0] || cfg_.dims[1] || cfg_.dims[2]) ? cfg_.dims
                                                                                   : nullptr);
            R.nx = R.topo.X() + 2;
            R.ny = R.topo.Y() + 2;
            R.nz = R.topo.Z() + 2;
            R.sj = R.nz;
            R.si = i64(R.ny) * R.nz;
            for (auto& g : R.g) g.assign(size_t(R.nx) * R.si, T(0));
            auto local = [&](const std::vector<double>& tab, int n, int off) {
                std::vector<T> v(n + 2, T(0));
                for (int i = 1; i <= n; ++i) v[i] = T(tab[off + i - 1]);
                return v;
            };
            R.tx = local(tx, R.topo.X(), R.topo.off[0]);
            R.ty = local(ty, R.topo.Y(), R.topo.off[1]);
            R.tz = local(tz, R.topo.Z(), R.topo.off[2]);
            R.plan = make_halo_plan(R.topo, R.si, R.nz);
            R.sbuf.clear();
            R.rbuf.clear();
            for (auto& m : R.plan.sends) R.sbuf.emplace_back(size_t(m.count));
            for (auto& m : R.plan.recvs) R.rbuf.emplace_back(size_t(m.count));
        }
        ct_.clear();
        for (double v : prob_.table_t()) ct_.push_back(v);
        for (auto& R : ranks_)
            log_msg(LogLevel::Info, R.topo.describe(), " backend cpu threads ",
                    cfg_.threads > 0 ? cfg_.threads : omp_get_max_threads());
    }

    // ---- compute ---------------------------------------------------------------------
    void layer0(RankState<T>& R) {
        Box ob = R.topo.owned_box();
        T* u = R.g[0].data();
        const T c0 = T(ct_[0]);
        double mabs = kErrInit, mrel = kErrInit;
        bool bad = false;
#pragma omp parallel num_threads(threads_)
        {
            T la = T(kErrInit), lr = T(kErrInit);
            bool lb = false;
#pragma omp for schedule(static)
            for (int i = ob.i0; i <= ob.i1; ++i)
                for (int j = ob.j0; j <= ob.j1; ++j)
                    for (int k = ob.k0; k <= ob.k1; ++k) {
                        T f = analytic(R.tx[i], R.ty[j], R.tz[k], c0);
                        u[R.idx(i, j, k)] = f;
                        accumulate_error(f, analytic(R.tx[i], R.ty[j], R.tz[k], c0), la, lr);
                        lb |= nonfinite(f);
                    }
#pragma omp critical
            {
                if (double(la) > mabs) mabs = la;
                if (double(lr) > mrel) mrel = lr;
                bad |= lb;
            }
        }
        R.mabs[0] = mabs;
        R.mrel[0] = mrel;
        R.bad[0] = bad;
    }

    // prepare_layer's Dirichlet part (mpi_new.cpp:157-169): zero the global y/z faces
    // owned by this rank. The periodic x planes are ordinary stencil points here.
    void zero_faces(RankState<T>& R, int n) {
        T* u = R.g[n % 3].data();
        const auto& t = R.topo;
        const int X = t.X(), Y = t.Y(), Z = t.Z();
#pragma omp parallel for num_threads(threads_) schedule(static)
        for (int i = 1; i <= X; ++i) {
            for (int j = 1; j <= Y; ++j) {
                if (t.nbr[2][0] < 0) u[R.idx(i, j, 1)] = T(0);
                if (t.nbr[2][1] < 0) u[R.idx(i, j, Z)] = T(0);
            }
            for (int k = 1; k <= Z; ++k) {
                if (t.nbr[1][0] < 0) u[R.idx(i, 1, k)] = T(0);
                if (t.nbr[1][1] < 0) u[R.idx(i, Y, k)] = T(0);
            }
        }
    }

    // Leapfrog: u^n -> slot n%3 from u^{n-1} (slot (n+2)%3) and u^{n-2} (slot (n+1)%3).
    // Increment form (--scheme delta): d^{n-1} lives in slot n%3, so d^n = d^{n-1} + coef*lap
    // and u^n = u^{n-1} + d^n are formed point by point, u^n overwriting d^{n-1} in place and
    // d^n going to slot (n+1)%3 (u^{n-2}, no longer needed); halos and wraps concern u only.
    void step(RankState<T>& R, int n) {
        const T* u1 = R.g[(n + 2) % 3].data();
        const T* u2 = R.g[(n + 1) % 3].data();
        T* u = R.g[n % 3].data();
        T* dnext = cfg_.delta ? R.g[(n + 1) % 3].data() : nullptr;
        Box cb = R.topo.compute_box();
        Box eb = R.topo.error_box();
        const T hx2 = T(prob_.hx2), hy2 = T(prob_.hy2), hz2 = T(prob_.hz2);
        const T coef = T(prob_.coef), coef1 = T(prob_.coef_first);
        const T cn = T(ct_[n]);
        // --math fma: coef/h^2 folded (stencil_math coef_lap_fma), as the HIP kernels
        const double cf = n == 1 ? prob_.coef_first : prob_.coef;
        const T fx = T(cf / prob_.hx2), fy = T(cf / prob_.hy2), fz = T(cf / prob_.hz2);
        const T fk = fm_kc(fx, fy, fz);  // leap_fm's centre factor
        const bool fm = cfg_.fma;
        const i64 si = R.si, sj = R.sj;
        const bool first = n == 1;
        double mabs = kErrInit, mrel = kErrInit;
        bool bad = false;
#pragma omp parallel num_threads(threads_)
        {
            T la = T(kErrInit), lr = T(kErrInit);
            bool lb = false;
#pragma omp for schedule(static)
            for (int i = cb.i0; i <= cb.i1; ++i) {
                const bool erow = i >= eb.i0 && i <= eb.i1;
                for (int j = cb.j0; j <= cb.j1; ++j) {
                    const i64 base = R.idx(i, j, 0);
                    for (int k = cb.k0; k <= cb.k1; ++k) {
                        const i64 p = base + k;
                        const T c = u1[p];
                        T v;
                        if (fm && !dnext && !first) {
                            v = leap_fm(c, u2[p], u1[p - si], u1[p + si], u1[p - sj], u1[p + sj], u1[p - 1],
                                        u1[p + 1], fx, fy, fz, fk);
                        } else if (fm) {
                            const T l = coef_lap_fma(c, u1[p - si], u1[p + si], u1[p - sj], u1[p + sj], u1[p - 1],
                                                     u1[p + 1], fx, fy, fz);
                            if (dnext) {
                                const T d = first ? l : u[p] + l;
                                v = c + d;
                                dnext[p] = d;
                            } else {
                                v = c + l;  // the Taylor start
                            }
                        } else {
                            T lap = laplace7(c, u1[p - si], u1[p + si], u1[p - sj], u1[p + sj],
                                             u1[p - 1], u1[p + 1], hx2, hy2, hz2);
                            if (dnext) {
                                const T d = first ? coef1 * lap : delta_incr(u[p], lap, coef);
                                v = c + d;
                                dnext[p] = d;
                            } else {
                                v = first ? taylor_first(c, lap, coef1) : leapfrog(c, u2[p], lap, coef);
                            }
                        }
                        u[p] = v;
                        lb |= nonfinite(v);
                        if (erow) accumulate_error(v, analytic(R.tx[i], R.ty[j], R.tz[k], cn), la, lr);
                    }
                }
            }
#pragma omp critical
            {
                if (double(la) > mabs) mabs = la;
                if (double(lr) > mrel) mrel = lr;
                bad |= lb;
            }
        }
        // fault injection: poison one node after the layer is computed; the detector
        // must see it through the next layer (same semantics as the HIP backend)
        if (fault_.kind == "nan" && fault_.hits(R.topo.rank, n)) {
            Box b = R.topo.compute_box();
            if (!b.empty())
                u[R.idx((b.i0 + b.i1) / 2, (b.j0 + b.j1) / 2, (b.k0 + b.k1) / 2)] = T(NAN);
        }
        R.mabs[n] = mabs;
        R.mrel[n] = mrel;
        R.bad[n] = bad;
    }

    // ---- halo exchange ---------------------------------------------------------------
    // Owned plane/row that face (axis, side) sends; ghost that it receives into.
    static int send_index(const Topology& t, int axis, int side) {
        if (axis == 0) return side == 1 ? t.x_send_plus() : t.x_send_minus();
        return side == 1 ? t.ext[axis] : 1;
    }
    static int ghost_index(const Topology& t, int axis, int side) {
        return side == 1 ? t.ext[axis] + 1 : 0;
    }

    void copy_face(RankState<T>& R, T* grid, int axis, int index, T* buf, bool to_buf) {
        const int X = R.topo.X();
        if (axis == 0) {
            T* p = grid + i64(index) * R.si;
            if (to_buf) std::memcpy(buf, p, sizeof(T) * R.si);
            else std::memcpy(p, buf, sizeof(T) * R.si);
        } else if (axis == 1) {
            for (int i = 1; i <= X; ++i) {
                T* p = grid + R.idx(i, index, 0);
                T* b = buf + i64(i - 1) * R.nz;
                if (to_buf) std::memcpy(b, p, sizeof(T) * R.nz);
                else std::memcpy(p, b, sizeof(T) * R.nz);
            }
        } else {
            for (int i = 1; i <= X; ++i)
                for (int j = 0; j < R.ny; ++j) {
                    T* p = grid + R.idx(i, j, index);
                    T* b = buf + i64(i - 1) * R.ny + j;
                    if (to_buf) *b = *p;
                    else *p = *b;
                }
        }
    }

    void self_wrap(RankState<T>& R, int n) {
        T* u = R.g[n % 3].data();
        const auto& t = R.topo;
        // ghost 0 <- plane sent "plus" (global N-1), ghost X+1 <- plane sent "minus" (global 1)
        std::memcpy(u + 0 * R.si, u + i64(t.x_send_plus()) * R.si, sizeof(T) * R.si);
        std::memcpy(u + i64(t.X() + 1) * R.si, u + i64(t.x_send_minus()) * R.si, sizeof(T) * R.si);
    }

    void exchange(int n, Timings& tm) {
        auto t0 = clk::now();
        for (auto& R : ranks_) {
            T* u = R.g[n % 3].data();
            if (R.plan.self_x) self_wrap(R, n);
            for (size_t m = 0; m < R.plan.sends.size(); ++m) {
                const auto& f = R.plan.sends[m];
                copy_face(R, u, f.axis, send_index(R.topo, f.axis, f.side), R.sbuf[m].data(), true);
            }
        }
        auto t1 = clk::now();
        if (ext_) {
            auto& R = ranks_[0];
            std::vector<Message> s, r;
            for (size_t m = 0; m < R.plan.sends.size(); ++m)
                s.push_back({R.plan.sends[m].peer, R.plan.sends[m].tag, R.sbuf[m].data(),
                             R.sbuf[m].size() * sizeof(T)});
            for (size_t m = 0; m < R.plan.recvs.size(); ++m)
                r.push_back({R.plan.recvs[m].peer, R.plan.recvs[m].tag, R.rbuf[m].data(),
                             R.rbuf[m].size() * sizeof(T)});
            ext_->exchange(s, r, nullptr);
        } else {
            // loopback hub: match (src, tag) -> receiver's recv slot
            for (auto& S : ranks_)
                for (size_t m = 0; m < S.plan.sends.size(); ++m) {
                    const auto& f = S.plan.sends[m];
                    auto& D = ranks_[f.peer];
                    bool done = false;
                    for (size_t q = 0; q < D.plan.recvs.size(); ++q) {
                        const auto& g = D.plan.recvs[q];
                        if (g.peer == S.topo.rank && g.tag == f.tag) {
                            W3D_REQUIRE(g.count == f.count, "halo size mismatch");
                            std::memcpy(D.rbuf[q].data(), S.sbuf[m].data(), sizeof(T) * f.count);
                            done = true;
                            break;
                        }
                    }
                    W3D_REQUIRE(done, "unmatched halo message");
                }
        }
        auto t2 = clk::now();
        for (auto& R : ranks_) {
            T* u = R.g[n % 3].data();
            for (size_t m = 0; m < R.plan.recvs.size(); ++m) {
                const auto& f = R.plan.recvs[m];
                copy_face(R, u, f.axis, ghost_index(R.topo, f.axis, f.side), R.rbuf[m].data(), false);
            }
            // fault injection: the x-minus ghost of this layer is lost
            if (fault_.kind == "drop_face" && fault_.hits(R.topo.rank, n))
                std::fill(u, u + R.si, T(0));
        }
        tm.comm_ms += std::chrono::duration<double, std::milli>(t2 - t1).count();
        tm.exchange_ms += ms_since(t0);
    }

    // ---- driver ----------------------------------------------------------------------
    void solve(RunResult& res, Timings& tm) {
        const int K = prob_.K;
        for (auto& R : ranks_) {
            R.mabs.assign(K + 1, kErrInit);
            R.mrel.assign(K + 1, kErrInit);
            R.bad.assign(K + 1, 0);
            for (auto& g : R.g) std::fill(g.begin(), g.end(), T(0));
        }
        if (ext_) ext_->barrier();
        auto t0 = clk::now();
        int start = 1;
        res.resumed_from = -1;
        if (!cfg_.resume_dir.empty()) {
            int n = load_checkpoints();
            res.resumed_from = n;
            start = n + 1;
        } else {
            auto tl = clk::now();
            for (auto& R : ranks_) layer0(R);
            tm.loop_ms += ms_since(tl);
            if (K >= 1) exchange(0, tm);
        }
        res.aborted = false;
        int done = start - 1;
        for (int n = start; n <= K; ++n) {
            if (cfg_.print_layers && !cfg_.quiet && local_ranks_[0] == 0) std::cout << "calculating layer " << n << "\n";
            auto tl = clk::now();
            for (auto& R : ranks_) {
                zero_faces(R, n);
                step(R, n);
            }
            tm.loop_ms += ms_since(tl);
            if (n < K) exchange(n, tm);
            done = n;
            if (cfg_.checkpoint_every > 0 && n % cfg_.checkpoint_every == 0 && n < K)
                save_checkpoints(n);
            if (cfg_.check_every > 0 && (n % cfg_.check_every == 0 || n == K)) {
                double ma = kErrInit;
                bool bad = false;
                for (auto& R : ranks_) ma = std::max(ma, R.mabs[n]), bad |= R.bad[n] != 0;
                double v[2] = {ma, bad ? 1.0 : 0.0};
                if (ext_) ext_->allreduce_max_host(v, 2);
                if (layer_diverged(v[0], v[1] != 0.0)) {
                    res.aborted = true;
                    res.abort_layer = n;
                    res.abort_reason = v[1] != 0.0 ? "non-finite values" : "error out of range";
                    break;
                }
            }
        }
        res.layers_done = done;
        // global reduction (mpi_new.cpp:358-361), all ranks get the result
        std::vector<double> a(K + 1, kErrInit), r(K + 1, kErrInit);
        for (auto& R : ranks_)
            for (int n = 0; n <= K; ++n) {
                if (R.mabs[n] > a[n]) a[n] = R.mabs[n];
                if (R.mrel[n] > r[n]) r[n] = R.mrel[n];
            }
        if (ext_) {
            ext_->allreduce_max_host(a.data(), a.size());
            ext_->allreduce_max_host(r.data(), r.size());
        }
        tm.total_ms = ms_since(t0);
        if (res.resumed_from >= 0) {
            // layers before the checkpoint come from the checkpoint header
            for (int n = 0; n <= res.resumed_from && n < int(ckpt_abs_.size()); ++n) {
                a[n] = ckpt_abs_[n];
                r[n] = ckpt_rel_[n];
            }
        }
        res.max_abs = a;
        res.max_rel = r;
    }

    void save_checkpoints(int n) {
        const int K = prob_.K;
        std::vector<double> a(K + 1, kErrInit), r(K + 1, kErrInit);
        for (auto& R : ranks_)
            for (int q = 0; q <= n; ++q) a[q] = std::max(a[q], R.mabs[q]), r[q] = std::max(r[q], R.mrel[q]);
        if (ext_) {
            ext_->allreduce_max_host(a.data(), a.size());
            ext_->allreduce_max_host(r.data(), r.size());
        }
        for (auto& R : ranks_) {
            CheckpointHeader h = make_header(cfg_, R.topo, n, sizeof(T));
            // leapfrog keeps u^{n-1} (slot (n+2)%3), the increment form d^n (slot (n+1)%3)
            write_checkpoint(cfg_.checkpoint_dir, h, host_level(R, (n + (cfg_.delta ? 1 : 2)) % 3),
                             host_level(R, n % 3), a, r);
            prune_checkpoints(cfg_.checkpoint_dir, h, n, 2);
        }
    }

    static HostLevel host_level(RankState<T>& R, int level) {
        HostLevel L;
        L.origin = R.g[level].data();
        L.X = R.topo.X();
        L.Y = R.topo.Y();
        L.Z = R.topo.Z();
        L.sj = R.sj;
        L.si = R.si;
        return L;
    }

    int load_checkpoints() {
        std::vector<CheckpointHeader> ex;
        for (auto& R : ranks_) ex.push_back(make_header(cfg_, R.topo, 0, sizeof(T)));
        const int n = agree_resume_layer(cfg_.resume_dir, ex, ext_);  // same layer on every rank
        for (auto& R : ranks_) {
            CheckpointHeader h = make_header(cfg_, R.topo, n, sizeof(T));
            read_checkpoint(cfg_.resume_dir, h, host_level(R, (n + (cfg_.delta ? 1 : 2)) % 3),
                            host_level(R, n % 3),
                            ckpt_abs_, ckpt_rel_);
        }
        // refill ghosts of both levels with one exchange each
        Timings dummy;
        exchange(n - 1, dummy);
        exchange(n, dummy);
        for (auto& R : ranks_)
            for (int q = 0; q <= n; ++q) R.mabs[q] = ckpt_abs_[q], R.mrel[q] = ckpt_rel_[q];
        return n;
    }

    Config cfg_;
    Transport* ext_;
    Problem prob_;
    FaultSpec fault_;
    int world_ = 1;
    int threads_ = 1;
    std::vector<int> local_ranks_;
    std::vector<RankState<T>> ranks_;
    std::vector<double> ct_;
    std::vector<double> ckpt_abs_, ckpt_rel_;
    double init_ms_ = 0;
};

template <class T>
class CpuSession : public Session {
public:
    CpuSession(const Config& c, Transport* ext) : s_(c, ext) { s_.init(); }
    RunResult solve() override { return s_.solve_one(); }
    double init_ms() const override { return s_.init_ms(); }
    std::vector<FieldBlock> field(int layer) override { return s_.field(layer); }

private:
    CpuSolver<T> s_;
};

}  // namespace

std::unique_ptr<Session> make_cpu_session(const Config& c, Transport* external) {
    if (c.dtype == DType::F64) return std::make_unique<CpuSession<double>>(c, external);
    return std::make_unique<CpuSession<float>>(c, external);
}

// warmup + repeat solves on one session; the result of the last one, all solve times
RunResult run_session(Session& s, const Config& c) {
    RunResult last;
    std::vector<double> times;
    for (int it = 0; it < c.warmup + c.repeat; ++it) {
        last = s.solve();
        if (it >= c.warmup) times.push_back(last.t.total_ms);
        if (last.aborted) break;
    }
    last.solve_ms = times;
    if (!c.dump.empty() && !last.aborted) dump_field(c.dump, c.N, s.field(c.timesteps), last.nprocs);
    return last;
}

static void write_npy(const std::string& path, const std::vector<int>& shape, const double* data,
                      const std::string& comment) {
    std::string dict = "{'descr': '<f8', 'fortran_order': False, 'shape': (";
    for (size_t q = 0; q < shape.size(); ++q) dict += std::to_string(shape[q]) + ", ";
    dict += "), }";
    if (!comment.empty()) dict += " # " + comment;
    std::string hdr = dict;
    while ((10 + hdr.size() + 1) % 64 != 0) hdr += ' ';
    hdr += '\n';
    std::FILE* f = std::fopen(path.c_str(), "wb");
    W3D_REQUIRE(f, "cannot write " + path);
    const unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
    std::fwrite(magic, 1, 8, f);
    const unsigned short hl = (unsigned short)hdr.size();
    std::fwrite(&hl, 2, 1, f);
    std::fwrite(hdr.data(), 1, hdr.size(), f);
    size_t n = 1;
    for (int d : shape) n *= size_t(d);
    const bool ok = std::fwrite(data, sizeof(double), n, f) == n;
    std::fclose(f);
    W3D_REQUIRE(ok, "short write " + path);
}

void dump_field(const std::string& path, int N, const std::vector<FieldBlock>& blocks, int world) {
    if (int(blocks.size()) == world) {  // every rank in this process: one global array
        const size_t n1 = size_t(N) + 1;
        std::vector<double> g(n1 * n1 * n1, 0.0);
        for (const auto& b : blocks)
            for (int i = 0; i < b.ext[0]; ++i)
                for (int j = 0; j < b.ext[1]; ++j)
                    std::copy_n(b.data.begin() + (size_t(i) * b.ext[1] + j) * b.ext[2], b.ext[2],
                                g.begin() + ((b.off[0] + i) * n1 + (b.off[1] + j)) * n1 + b.off[2]);
        write_npy(path, {int(n1), int(n1), int(n1)}, g.data(), "");
        return;
    }
    for (const auto& b : blocks)
        write_npy(path + ".r" + std::to_string(b.rank) + ".npy", {b.ext[0], b.ext[1], b.ext[2]},
                  b.data.data(),
                  "offset " + std::to_string(b.off[0]) + " " + std::to_string(b.off[1]) + " " +
                      std::to_string(b.off[2]));
}

RunResult run_cpu(const Config& c, Transport* external) {
    auto s = make_cpu_session(c, external);
    return run_session(*s, c);
}

}  // namespace wave3d
