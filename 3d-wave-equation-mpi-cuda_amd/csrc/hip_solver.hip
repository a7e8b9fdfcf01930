// MI355X solver driver (replaces cuda_sol.cpp's calculate_num_sol/exchange, §3.3-3.4).
//
// Execution model per time layer n (one process per GPU, device transport):
//   compute stream : [zero Dirichlet faces, n<=3] -> interior(n) -> wait halo(n-1)
//                    -> shell(n) (+ fused y/z face packing) -> record layer(n)
//   comm stream    : wait layer(n) -> transport send/recv (x planes in place, packed y/z)
//                    -> unpack y/z ghosts -> record halo(n)
// so the RCCL exchange of layer n overlaps the interior of layer n+1. No host
// synchronisation inside the time loop (the reference syncs >= 4x per layer); errors stay
// in per-layer device slots until one max-allreduce at the end.
// Single GPU (dims 1x1x1): one launch per layer, the periodic wrap fused into the stores.
// In-process ranks (--ranks P): P subdomains on this GPU, one stream, D2D loopback copies.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <memory>
#include <thread>

#include "checkpoint.hpp"
#include "device_common.hpp"
#include "hip_kernels.hpp"
#include "hip_selftest.hpp"
#include "rccl_transport.hpp"
#include "problem.hpp"
#include "sizing.hpp"
#include "solver.hpp"
#include "log.hpp"
#include "trace.hpp"

#define HIP_CHECK(x)                                                                   \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess)                                                          \
            throw ::wave3d::Error(std::string("HIP error ") + hipGetErrorString(e_) + \
                                  " at " __FILE__ ":" + std::to_string(__LINE__));     \
    } while (0)

namespace wave3d {
namespace {

using clk = std::chrono::steady_clock;

// Temporal-blocking variant names: "tb2" (2 rows/lane, 4 waves), "tb2r<R>", "tb2r<R>w<W>".
std::string tb_name(int rows, int waves, int occ, int depth = 2, int kwaves = 1) {
    if (depth >= 3) {
        const std::string b = "tb" + std::to_string(depth);
        return rows == 2 && waves == 8 ? b : b + "r" + std::to_string(rows) + "w" + std::to_string(waves);
    }
    std::string s = rows == 2 && waves == 4 && occ == 0 && kwaves == 1 ? "tb2" : "tb2r" + std::to_string(rows);
    if (waves != 4 || occ || kwaves != 1) s += "w" + std::to_string(waves);
    if (kwaves != 1) s += "k" + std::to_string(kwaves);
    if (occ) s += "o" + std::to_string(occ);
    return s;
}

// CUs the compute stream leaves to the halo stream while overlap is on (WAVE3D_COMM_CUS,
// default kCommCus; 0 = no CU-masked stream)
constexpr int kCommCus = 0;
// Overlap order of the deep sweeps (WAVE3D_OVERLAP_SHELLS_FIRST=1): the shells first on the compute
// stream, then the exchange beside the interior; default: the shells beside the interior
bool overlap_shells_first() {
    const char* e = std::getenv("WAVE3D_OVERLAP_SHELLS_FIRST");
    return e && e[0] == '1';
}
int comm_cu_reserve() {
    const char* e = std::getenv("WAVE3D_COMM_CUS");
    return e && *e ? std::max(0, std::atoi(e)) : kCommCus;
}

constexpr int kMaxLevels = 4;  // time levels: 3 single-step, 4 with two- / three-layer sweeps
constexpr int kSeamPlanes = 10;  // seam scratch: tb3 C at 2 partners; tb4 6 C + 2 D planes (+ 2 d planes
                                 // of the increment form: layer m's d at the partners, stage 2's input)

template <class T>
struct DevRank {
    Topology topo;
    GridView gv;
    int lead = 0;
    T* alloc[kMaxLevels] = {};
    T* g[kMaxLevels] = {};  // logical (0,0,0) of each level
    i64 plane_off = 0;                                 // g - (start of logical plane 0)
    size_t elems = 0;                                  // allocation per level
    T *tx = nullptr, *ty = nullptr, *tz = nullptr;
    T* txy = nullptr;  // sx*sy table of the temporal-blocking sweep (launch_txy)
    T* rtxy = nullptr;  // --math fma: (txy, 1/|txy|) pairs and 1/|tz| (relative error without division)
    T* rtz = nullptr;
    HaloPlan plan;
    std::vector<T*> sbuf, rbuf;  // y/z messages only (x messages live in the grid)
    u64* err = nullptr;          // (K+1) * kSlotsPerLayer
    Box compute, error, owned, interior;
    std::vector<Box> shell;      // single step: x shells (flat kernel) first, then y/z shells
    int shell_x = 0;             // how many of `shell` are x shells
    int zero_mask = 0;
    Wrap wrap;                   // single-step periodic self-wrap (depth 1)
    Wrap wrap2;                  // depth-2 self-wrap (temporal blocking: IC and D layers)
    Wrap wrap3;                  // depth-3 self-wrap (three-layer blocking: IC and E layers)
    Wrap wrap4;                  // depth-4 self-wrap (four-layer blocking: IC and the last layer)
    Box cdom;                    // temporal blocking: where C is a stencil value
    FusedPack<T> pack;           // pointers into sbuf
    // temporal blocking across ranks (x slabs): plane messages, seam alias plane, boxes
    struct PlaneMsg {
        int peer, tag;
        int level;      // 0 = A level (D of the sweep), 1 = B level (C of the sweep)
        int plane;      // first logical plane; kAliasPlane = the alias buffer
        int nplanes;
    };
    std::vector<PlaneMsg> tb_sends, tb_recvs;
    // y/z splits: rows / columns of depth 2 (D) and 1 (C), staged through buffers; round 0
    // (y) and round 1 (z) run after the x planes, each over the full extent of the previous
    // axes (ghosts included), so edges arrive without diagonal messages
    struct BoxMsg {
        int peer, tag;
        int level;      // 0 = next A level, 1 = next B level, 2 = seam alias plane (A)
        Box box;
        T* buf;
    };
    std::vector<BoxMsg> tb_bsends[2], tb_brecvs[2];
    // --halo direct: one round — every face, edge and corner ghost region of the A / B levels
    // and of the seam alias planes straight from the rank that owns it (level 0 = A, 1 = B,
    // 2 = alias A, 3 = alias B; box = source region on sends, ghost region on receives)
    std::vector<BoxMsg> tb_dsends, tb_drecvs;
    // ... packed back to back per peer: one message per peer and direction of travel (2x2x2:
    // 7 peers, one xGMI link each); BoxMsg::buf points into these
    struct PeerBuf {
        int peer;
        T* buf;
        size_t count;
    };
    std::vector<PeerBuf> tb_psends, tb_precvs;
    T* alias_buf = nullptr;      // one plane: x=N (first x-rank) or x=0 (last x-rank)
    T* alias_bufB = nullptr;     // the same plane of the B level (three-layer blocking)
    T* seamc_buf = nullptr;      // earlier layers on the seam partner planes (tb3: 2 planes, tb4: 8)
    T* seamc_in = nullptr;       // the interior's copy (overlapped self-wrap runs)
    T* pinned = nullptr;         // checkpoint staging (2 levels, pinned host memory)
    Box tb_interior;
    std::vector<Box> tb_shell;
};

constexpr int kAliasPlane = -1000;

template <class T>
class HipSolver {
public:
    HipSolver(const Config& c, Transport* ext) : cfg_(c), ext_(ext) {
        prob_ = Problem::from_config(c);
        fault_ = FaultSpec::parse(c.fault);
        if (ext_) {
            W3D_REQUIRE(ext_->device(), "run_hip needs a device transport");
            world_ = ext_->size();
            local_ = {ext_->rank()};
        } else {
            world_ = std::max(1, c.ranks);
            for (int r = 0; r < world_; ++r) local_.push_back(r);
        }
        // kernel family, ghost depth, levels and decomposition (sizing.cpp: shared with the
        // --fill-hbm planner, so a planned N is exactly what gets allocated)
        const Layout lay = plan_layout(c, world_);
        tb_ = lay.tb;
        tbd_ = lay.depth;
        tbn_ = lay.generic;
        tb_rows_ = lay.rows;
        tb_waves_ = lay.waves;
        tb_occ_ = lay.occ;
        tb_nwk_ = lay.kwaves;
        G_ = lay.G;
        L_ = lay.L;
        for (int a = 0; a < 3; ++a) cfg_.dims[a] = lay.dims[a];
        W3D_REQUIRE(tbd_ < 4 || (c.delta ? tbn_delta_supported(4, tb_rows_, tb_waves_, c.fma, c.dtype == DType::F32)
                                         : tbn_supported(4, tb_rows_, tb_waves_, c.fma, c.dtype == DType::F32)),
                    "four-layer blocking: tile r2w8; the increment form in fp32 only");
        W3D_REQUIRE(!c.fma || !tb_ || tbd_ == 4 ||
                        (tbd_ == 3 ? (c.delta ? tb3_delta_supported(tb_rows_, tb_waves_, true)
                                              : tb3_supported(tb_rows_, tb_waves_, true))
                                   : tb_occ_ == 0 && tb2_fma_supported(tb_rows_, tb_waves_, tb_nwk_, c.delta)),
                    "--math fma: no fma instantiation of this temporal-blocking tile (tb3, tb3r1w8, tb3r1w16, "
                    "tb2r2w8, tb2)");
        W3D_REQUIRE(!tbn_ || tbd_ == 4 || (!c.delta && tbn_supported(3, tb_rows_, tb_waves_, c.fma, c.dtype == DType::F32)),
                    "tbn3: leapfrog, tile r2w8");
        W3D_REQUIRE(!tb_ || tbd_ == 4 || (tbd_ == 3 ? tb3_supported(tb_rows_, tb_waves_)
                                        : tb2_supported(tb_rows_, tb_waves_, tb_occ_, tb_nwk_)),
                    "wave3d: unknown kernel variant " + c.kernel);
        kind_ = parse_kernel_variant(tb_ ? std::string("auto") : c.kernel);
        naive_.march = false;
        naive_.flat = true;  // thin overlap shells: flattened one-point-per-thread kernel
        if (c.delta) {
            // increment form: temporal blocking sweeps (u and d levels in the ring: after a
            // sweep, lvl(m+1) = u^{m+1}, lvl(m) = d^{m+1}); an odd last layer is one step of
            // the naive/flat kernel reading that d level
            W3D_REQUIRE(tb_ && (tbd_ == 2 ? tb2_delta_supported(tb_rows_, tb_waves_, tb_nwk_) && tb_occ_ == 0
                                          : tbd_ == 4 || tb3_delta_supported(tb_rows_, tb_waves_)),
                        "--scheme delta needs a tb2 kernel with an increment-form instantiation (tb2, tb2r2w8, "
                        "tb2r4w4, tb2r2w8k2), tb3 / tb3r1w8 or (fp32) tb4");
            kind_ = KernelVariant{};
            kind_.march = false;
            kind_.delta = true;
            naive_.delta = true;
        }
        if (c.fma) {
            // every kernel of the run (single-step tails and shells too) uses the FMA form, so a
            // node's value does not depend on which kernel computed it
            W3D_REQUIRE(!kind_.pk, "--math fma: no packed-fp32 march variant");
            kind_.fast = true;
            naive_.fast = true;
        }
        // interior/shell split + comm stream whenever there is a remote halo to hide
        overlap_ = c.overlap && (ext_ != nullptr || world_ > 1);
        overlap_auto_ = overlap_ && c.overlap_auto;
        // test mode: the periodic x wrap of a dims[0] == 1 rank goes through the transport as
        // messages to itself (RCCL send/recv exercised on one GPU), not the fused local wrap
        xself_ = c.x_self_transport;
        direct_ = c.halo_direct;
        W3D_REQUIRE(!xself_ || ext_, "--x-self-transport needs an external (e.g. RCCL) transport");
        W3D_REQUIRE(!c.rccl_mirror || (!ext_ && world_ > 1), "--rccl-mirror needs simulated ranks (--ranks P)");
    }

    ~HipSolver() { release(); }

    void init() {
        TraceRange tr("wave3d.setup");
        auto t0 = clk::now();
        setup();
        plan_slots(1);
        if (cfg_.rccl_mirror) setup_mirror();
        bool msgs = false;
        for (auto& R : ranks_) msgs |= !R.plan.sends.empty() || !R.plan.recvs.empty() || tb_halo(R);
        if (msgs && cfg_.halo_check) halo_self_test();
        const bool halos = msgs || fault_.kind == "drop_face";
        fine_ = cfg_.profile || halos;
        // every mark of a solve: IC + per sweep (compute, exchange) + reduction
        ts_cap_ = size_t(12) * (prob_.K + 4) + 16;
        ev_marks_.resize(ts_cap_, nullptr);
        for (auto& e : ev_marks_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDefault));
        no_timers_ = std::getenv("WAVE3D_NO_TIMERS") && std::string(std::getenv("WAVE3D_NO_TIMERS")) == "1";
        void* h = nullptr;
        HIP_CHECK(hipHostMalloc(&h, ts_cap_ * sizeof(u64), hipHostMallocCoherent | hipHostMallocMapped));
        ts_host_ = static_cast<u64*>(h);
        void* d = nullptr;
        HIP_CHECK(hipHostGetDevicePointer(&d, h, 0));
        ts_dev_ = static_cast<u64*>(d);
        int dev = 0, khz = 0;
        HIP_CHECK(hipGetDevice(&dev));
        HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
        if (khz > 0) clock_khz_ = khz;
        HIP_CHECK(hipDeviceSynchronize());
        init_ms_ = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        if (log_on(LogLevel::Info)) {
            for (auto& R : ranks_) {
                log_msg(LogLevel::Info, R.topo.describe(), " kernel ",
                        tb_ ? tb_name(tb_rows_, tb_waves_, tb_occ_, tbd_, tb_nwk_) : kernel_variant_name(kind_), " levels ",
                        L_, " ghost ", G_, " bytes/level ", R.elems * sizeof(T), " overlap ",
                        overlap_ ? "on" : "off", " transport ",
                        ext_ ? ext_->name() : (world_ > 1 ? "loopback" : "self"));
                log_msg(LogLevel::Debug, "rank ", R.topo.rank, ": ", R.plan.sends.size(),
                        " face sends, ", R.tb_sends.size(), " deep-halo sends, interior ",
                        R.interior.empty() ? 0 : 1, " shell boxes ", R.shell.size(), "/",
                        R.tb_shell.size());
            }
            log_msg(LogLevel::Info, "setup ", init_ms_, " ms");
        }
    }

    double init_ms() const { return init_ms_; }

    RunResult solve_one() {
        RunResult res;
        res.N = prob_.N;
        res.K = prob_.K;
        res.nprocs = world_;
        res.Np = world_;
        res.dtype = cfg_.dtype;
        res.backend = "hip";
        res.kernel = tb_ ? tb_name(tb_rows_, tb_waves_, tb_occ_, tbd_, tb_nwk_) : kernel_variant_name(kind_);
        if (tbn_ && tbd_ == 3) res.kernel = "tbn" + res.kernel.substr(2);
        res.courant = prob_.courant;
        res.transport = ext_ ? ext_->name() : (world_ > 1 ? "loopback" : "self");
        // --overlap auto: solves 2..7 are the trials of three arms, twice each (on with the shells
        // beside the interior, off, on with the shells first; the first solve only warms up —
        // first launches, RCCL connections of every message shape); the arm with the shortest
        // best-of-two max-over-ranks solve time is kept for every later solve (one noisy sample
        // cannot lock in a slower arm) — the same decision on every rank, since the times are
        // reduced before the comparison. Which overlap order hides a real xGMI exchange better
        // is the hardware's call (profiles/overlap_model_r4.txt: beside won on one GPU).
        const int trial = overlap_auto_ && solves_ >= 1 && trials_done_ < kOverlapTrials ? trials_done_ : -1;
        ++solves_;
        if (trial >= 0) set_overlap(trial % 3 != 1, trial % 3 == 2);
        res.overlap = overlap_;  // of this solve (an --overlap auto decision applies from the next)
        res.overlap_order = !overlap_ ? "none" : shells_first_ ? "shells_first" : "beside";
        res.overlap_mode = !(ext_ || world_ > 1) ? "none"
                           : overlap_auto_       ? "auto"
                           : (overlap_ ? "on" : "off");
        res.scheme = cfg_.delta ? "delta" : "leapfrog";
        res.math = cfg_.fma ? "fma" : "exact";
        res.comm_size = ext_ ? ext_->comm_size() : 0;
        res.rccl_max_ctas = ext_ ? ext_->cta_budget() : -1;
        res.halo_checked = halo_checked_;
        if (ext_ || world_ > 1) {
            res.overlap_interior = -1;
            for (auto& R : ranks_) {
                const i64 c = (tb_ ? R.tb_interior : R.interior).count();
                res.overlap_interior = res.overlap_interior < 0 ? c : std::min<long long>(res.overlap_interior, c);
            }
        }
        for (int a = 0; a < 3; ++a) res.dims[a] = ranks_[0].topo.dims[a];
        Timings t;
        solve(res, t);
        t.init_ms = init_ms_;
        double tv[5] = {t.total_ms, t.loop_ms, t.exchange_ms, t.comm_ms, t.error_ms};
        if (ext_) ext_->allreduce_max_host(tv, 5);
        t.total_ms = tv[0], t.loop_ms = tv[1], t.exchange_ms = tv[2], t.comm_ms = tv[3];
        t.error_ms = tv[4];
        if (trial >= 0) {
            trial_ms_[trial] = t.total_ms;
            if (++trials_done_ == kOverlapTrials) {
                int arm = 0;  // ties keep the earlier arm: on (beside), then off
                for (int a = 1; a < 3; ++a)
                    if (best_trial(a) < best_trial(arm)) arm = a;
                set_overlap(arm != 1, arm == 2);
                log_msg(LogLevel::Info, "overlap auto: on ", best_trial(0), " ms, off ", best_trial(1),
                        " ms, on shells-first ", best_trial(2), " ms -> ",
                        arm == 1 ? "off" : (arm == 2 ? "on, shells first" : "on"));
            }
        }
        for (int a = 0; a < 3; ++a) res.overlap_trial_ms[a] = best_trial(a);
        for (int q = 0; q < kOverlapTrials; ++q) res.overlap_trials[q] = trial_ms_[q];
        res.overlap_order_run = order_enqueued_;
        res.t = t;
        res.solve_ms.push_back(t.total_ms);
        return res;
    }

    // owned block of layer K or K-1 of every local rank (both are always stored)
    std::vector<FieldBlock> field(int layer) {
        const int K = prob_.K;
        W3D_REQUIRE(layer >= std::max(0, K - 1) && layer <= K, "field: only layers K-1 and K are kept");
        W3D_REQUIRE(!cfg_.delta || layer == K, "field: the increment form keeps only layer K");
        HIP_CHECK(hipDeviceSynchronize());
        std::vector<FieldBlock> out;
        for (auto& R : ranks_) {
            const int l = lvl(layer);
            std::vector<T> h(R.elems);
            HIP_CHECK(hipMemcpy(h.data(), R.alloc[l], R.elems * sizeof(T), hipMemcpyDeviceToHost));
            const HostLevel L = host_level(R, h, l);
            FieldBlock b;
            b.rank = R.topo.rank;
            for (int a = 0; a < 3; ++a) b.off[a] = R.topo.off[a], b.ext[a] = R.topo.ext[a];
            b.data.reserve(size_t(L.X) * L.Y * L.Z);
            const T* o = static_cast<const T*>(L.origin);
            for (int i = 1; i <= L.X; ++i)
                for (int j = 1; j <= L.Y; ++j)
                    for (int k = 1; k <= L.Z; ++k) b.data.push_back(double(o[i * L.si + j * L.sj + k]));
            out.push_back(std::move(b));
        }
        return out;
    }

private:
    // ---- setup ------------------------------------------------------------------------
    void setup() {
        const int A = int(128 / sizeof(T));  // alignment in elements
        auto tabx = prob_.table_x(), taby = prob_.table_y(), tabz = prob_.table_z();
        ct_ = prob_.table_t();
        HIP_CHECK(hipStreamCreateWithFlags(&s_comp_, hipStreamNonBlocking));
        // the halo stream (pack/unpack, RCCL kernels) at the highest priority, so its small
        // launches are dispatched ahead of the interior sweep's queued workgroups instead of
        // waiting for CU slots behind them
        int prio_lo = 0, prio_hi = 0;
        HIP_CHECK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
        HIP_CHECK(hipStreamCreateWithPriority(&s_comm_, hipStreamNonBlocking, prio_hi));
        // While overlap is on, the sweeps run on a CU-masked twin of the compute stream: an
        // interior sweep holds one workgroup per CU for its whole march, so without a reserve the
        // halo stream's kernels (RCCL send/recv, pack/unpack, the next shells) wait for it to
        // drain and the exchange serialises behind it
        s_comp_full_ = s_comp_;
        comm_cus_ = comm_cu_reserve();
        if (comm_cus_ > 0 && (ext_ || world_ > 1) && cfg_.overlap) {
            int dev = 0, cus = 0;
            HIP_CHECK(hipGetDevice(&dev));
            HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            comm_cus_ = std::min(comm_cus_, cus / 2);
            // every (cus / reserve)-th CU index: spread over the shader engines and XCDs
            std::vector<uint32_t> mask(size_t(cus + 31) / 32, 0u);
            const int stride = cus / comm_cus_;
            for (int c = 0; c < cus; ++c)
                if (!(c % stride == stride - 1 && c / stride < comm_cus_)) mask[size_t(c) / 32] |= 1u << (c % 32);
            HIP_CHECK(hipExtStreamCreateWithCUMask(&s_comp_cu_, uint32_t(mask.size()), mask.data()));
            if (overlap_) s_comp_ = s_comp_cu_;
        } else {
            comm_cus_ = 0;
        }
        HIP_CHECK(hipEventCreateWithFlags(&ev_start_, hipEventDefault));
        HIP_CHECK(hipEventCreateWithFlags(&ev_end_, hipEventDefault));
        HIP_CHECK(hipEventCreateWithFlags(&ev_layer_, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&ev_halo_, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&ev_shell_, hipEventDisableTiming));
        ranks_.resize(local_.size());
        const bool have_dims = cfg_.dims[0] || cfg_.dims[1] || cfg_.dims[2];
        for (size_t q = 0; q < local_.size(); ++q) {
            auto& R = ranks_[q];
            R.topo = Topology::make(prob_.N, world_, local_[q], have_dims ? cfg_.dims : nullptr);
            const int X = R.topo.X(), Y = R.topo.Y(), Z = R.topo.Z();
            // row: k = 1-G .. Z+G at offset A-1+k (k = 1 on a 128-B boundary)
            R.gv.X = X;
            R.gv.Y = Y;
            R.gv.Z = Z;
            R.gv.G = G_;
            R.gv.sj = ((A + Z + G_ + A - 1) / A) * A;
            R.gv.si = i64(Y + 2 * G_) * R.gv.sj;
            R.plane_off = i64(G_ - 1) * R.gv.sj + (A - 1);
            R.gv.poff = int(R.plane_off);
            R.lead = int(R.plane_off);
            R.elems = size_t(X + 2 * G_) * size_t(R.gv.si);
            W3D_REQUIRE(L_ <= kMaxLevels, "too many time levels");
            for (int l = 0; l < L_; ++l) {
                HIP_CHECK(hipMalloc(&R.alloc[l], R.elems * sizeof(T)));
                HIP_CHECK(hipMemset(R.alloc[l], 0, R.elems * sizeof(T)));
                R.g[l] = R.alloc[l] + i64(G_ - 1) * R.gv.si + R.plane_off;
            }
            auto upload = [&](const std::vector<double>& tab, int n, int off) {
                std::vector<T> v(n + 2, T(0));
                for (int i = 1; i <= n; ++i) v[i] = T(tab[off + i - 1]);
                T* d = nullptr;
                HIP_CHECK(hipMalloc(&d, v.size() * sizeof(T)));
                HIP_CHECK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
                return d;
            };
            R.tx = upload(tabx, X, R.topo.off[0]);
            R.ty = upload(taby, Y, R.topo.off[1]);
            R.tz = upload(tabz, Z, R.topo.off[2]);
            if (tb_) {
                HIP_CHECK(hipMalloc(&R.txy, txy_elems(X, Y) * sizeof(T)));
                launch_txy<T>(R.txy, R.tx, R.ty, X, Y, nullptr);
                if (cfg_.fma) {
                    HIP_CHECK(hipMalloc(&R.rtxy, 2 * txy_elems(X, Y) * sizeof(T)));
                    HIP_CHECK(hipMalloc(&R.rtz, size_t(Z + 2) * sizeof(T)));
                    launch_txr<T>(R.rtxy, R.txy, txy_elems(X, Y), nullptr);
                    launch_recip_abs<T>(R.rtz, R.tz, size_t(Z + 2), nullptr);
                }
                HIP_CHECK(hipDeviceSynchronize());
            }
            R.plan = make_halo_plan(R.topo, R.gv.si, Z + 2, xself_);
            if (R.plan.self_x) W3D_REQUIRE(X >= 3, "periodic self-wrap needs >= 3 x planes");
            R.sbuf.assign(R.plan.sends.size(), nullptr);
            R.rbuf.assign(R.plan.recvs.size(), nullptr);
            for (size_t m = 0; m < R.plan.sends.size(); ++m)
                if (R.plan.sends[m].axis != 0)
                    HIP_CHECK(hipMalloc(&R.sbuf[m], R.plan.sends[m].count * sizeof(T)));
            for (size_t m = 0; m < R.plan.recvs.size(); ++m)
                if (R.plan.recvs[m].axis != 0)
                    HIP_CHECK(hipMalloc(&R.rbuf[m], R.plan.recvs[m].count * sizeof(T)));
            HIP_CHECK(hipMalloc(&R.err, sizeof(u64) * (prob_.K + 1) * kSlotsPerLayer));

            R.compute = R.topo.compute_box();
            R.error = R.topo.error_box();
            R.owned = R.topo.owned_box();
            const auto& t = R.topo;
            R.zero_mask = (t.nbr[2][0] < 0 ? 1 : 0) | (t.nbr[2][1] < 0 ? 2 : 0) |
                          (t.nbr[1][0] < 0 ? 4 : 0) | (t.nbr[1][1] < 0 ? 8 : 0);
            if (R.plan.self_x) {
                R.wrap.src[0] = t.x_send_plus();   // global N-1 -> ghost 0
                R.wrap.dst[0] = 0;
                R.wrap.src[1] = t.x_send_minus();  // global 1   -> ghost X+1
                R.wrap.dst[1] = X + 1;
                // depth 2: global N-2, N-1 -> ghosts -1, 0; global 1, 2 -> ghosts X+1, X+2
                R.wrap2.src[0] = X - 2, R.wrap2.dst[0] = -1;
                R.wrap2.src[1] = X - 1, R.wrap2.dst[1] = 0;
                R.wrap2.src[2] = 2, R.wrap2.dst[2] = X + 1;
                R.wrap2.src[3] = 3, R.wrap2.dst[3] = X + 2;
                for (int q = 0; q < 3; ++q) {
                    R.wrap3.src[q] = X - 3 + q, R.wrap3.dst[q] = -2 + q;
                    R.wrap3.src[3 + q] = 2 + q, R.wrap3.dst[3 + q] = X + 1 + q;
                }
                for (int q = 0; q < 4; ++q) {
                    R.wrap4.src[q] = X - 4 + q, R.wrap4.dst[q] = -3 + q;
                    R.wrap4.src[4 + q] = 2 + q, R.wrap4.dst[4 + q] = X + 1 + q;
                }
                if (tbd_ >= 3)
                    W3D_REQUIRE(X >= 2 * tbd_ + 1, "deep temporal blocking self-wrap needs >= 2 x depth + 1 x planes");
                if (tb_) W3D_REQUIRE(X >= 5, "temporal blocking self-wrap needs >= 5 x planes");
            }
            // stencil-valued region of the blocked layers: C/D/E are evaluated on rings up to
            // G-1 nodes into a neighbour's ghosts; Dirichlet faces (no neighbour) stay 0
            R.cdom = R.compute;
            if (t.nbr[1][0] >= 0) R.cdom.j0 -= G_ - 1;
            if (t.nbr[1][1] >= 0) R.cdom.j1 += G_ - 1;
            if (t.nbr[2][0] >= 0) R.cdom.k0 -= G_ - 1;
            if (t.nbr[2][1] >= 0) R.cdom.k1 += G_ - 1;
            for (size_t m = 0; m < R.plan.sends.size(); ++m) {
                const auto& f = R.plan.sends[m];
                if (f.axis == 1) {
                    R.pack.ybuf[f.side] = R.sbuf[m];
                    R.pack.yj[f.side] = f.side ? Y : 1;
                } else if (f.axis == 2) {
                    R.pack.zbuf[f.side] = R.sbuf[m];
                    R.pack.zk[f.side] = f.side ? Z : 1;
                }
            }
            // interior = compute box minus the layer next to every remote ghost. With a tiled
            // march kernel the j/k shells are widened to whole tiles (its tile rows; k on the
            // 64-column grid) and run with that kernel; the one-plane x shells (and every shell
            // of the naive/flat kernels) use the flat one-point-per-thread kernel.
            Box c = R.compute, in = c;
            const int TJm = shells_tiled() ? march_tile_rows(kind_) : 1;
            const int TKm = shells_tiled() ? kTileK : 1;
            if (!R.plan.self_x) {
                // the shells hold every plane the exchange sends: the first / last x-rank (or
                // one x rank messaging itself) sends plane 2 / X-1, skipping the duplicate plane
                const bool xs = t.dims[0] > 1;
                in.i0 = std::max(in.i0, 2 + ((t.first(0) || !xs) ? 1 : 0));
                in.i1 = std::min(in.i1, X - 1 - ((t.last(0) || !xs) ? 1 : 0));
            }
            if (t.nbr[1][0] >= 0) in.j0 = std::max(in.j0, std::max(2, c.j0 + TJm));
            if (t.nbr[1][1] >= 0) in.j1 = std::min(in.j1, std::min(Y - 1, c.j1 - TJm));
            if (t.nbr[2][0] >= 0) in.k0 = std::max(in.k0, TKm > 1 ? 1 + TKm : 2);
            if (t.nbr[2][1] >= 0) in.k1 = std::min(in.k1, TKm > 1 ? TKm * ((Z - 1) / TKm) : Z - 1);
            R.interior = in;
            build_tb_plan(R);
            if (tbd_ >= 3 && (R.plan.self_x || t.first(0) || t.last(0))) {
                // earlier layers on the seam partner planes (three- / four-layer sweeps);
                // allocated here, never inside a hipGraph capture
                const i64 np = kSeamPlanes;
                HIP_CHECK(hipMalloc(&R.seamc_buf, np * R.gv.si * sizeof(T)));
                HIP_CHECK(hipMemset(R.seamc_buf, 0, np * R.gv.si * sizeof(T)));
                if (R.plan.self_x && (t.dims[1] > 1 || t.dims[2] > 1)) {
                    HIP_CHECK(hipMalloc(&R.seamc_in, np * R.gv.si * sizeof(T)));
                    HIP_CHECK(hipMemset(R.seamc_in, 0, np * R.gv.si * sizeof(T)));
                }
            }
            R.shell.clear();
            auto add = [&](Box b) {
                if (!b.empty()) R.shell.push_back(b);
            };
            if (in.empty()) {
                add(c);
                R.shell_x = int(R.shell.size());
            } else {
                add({c.i0, in.i0 - 1, c.j0, c.j1, c.k0, c.k1});
                add({in.i1 + 1, c.i1, c.j0, c.j1, c.k0, c.k1});
                R.shell_x = int(R.shell.size());
                add({in.i0, in.i1, c.j0, in.j0 - 1, c.k0, c.k1});
                add({in.i0, in.i1, in.j1 + 1, c.j1, c.k0, c.k1});
                add({in.i0, in.i1, in.j0, in.j1, c.k0, in.k0 - 1});
                add({in.i0, in.i1, in.j0, in.j1, in.k1 + 1, c.k1});
            }
        }
        host_err_.assign(size_t(prob_.K + 1) * kSlotsPerLayer, 0);
    }

    void release() {
        if (ckpt_thread_.joinable()) ckpt_thread_.join();
        if (s_ckpt_) (void)hipStreamDestroy(s_ckpt_);
        if (ev_ckpt_) (void)hipEventDestroy(ev_ckpt_);
        s_ckpt_ = nullptr, ev_ckpt_ = nullptr;
        for (auto& R : ranks_) {
            for (int l = 0; l < kMaxLevels; ++l) (void)hipFree(R.alloc[l]);
            (void)hipFree(R.tx);
            (void)hipFree(R.ty);
            (void)hipFree(R.tz);
            (void)hipFree(R.txy);
            (void)hipFree(R.rtxy);
            (void)hipFree(R.rtz);
            for (auto* p : R.sbuf) (void)hipFree(p);
            for (auto* p : R.rbuf) (void)hipFree(p);
            (void)hipFree(R.err);
            (void)hipFree(R.alias_buf);
            (void)hipFree(R.alias_bufB);
            (void)hipFree(R.seamc_buf);
            (void)hipFree(R.seamc_in);
            if (R.pinned) (void)hipHostFree(R.pinned);
            for (int q = 0; q < 2; ++q) {
                for (auto& m : R.tb_bsends[q]) (void)hipFree(m.buf);
                for (auto& m : R.tb_brecvs[q]) (void)hipFree(m.buf);
            }
            for (auto* v : {&R.tb_psends, &R.tb_precvs}) {
                for (auto& m : *v) (void)hipFree(m.buf);
            }
        }
        ranks_.clear();
        if (mirror_buf_) (void)hipFree(mirror_buf_);
        if (mirror_res_) (void)hipFree(mirror_res_);
        mirror_buf_ = nullptr, mirror_res_ = nullptr;
        mirror_.reset();
        if (s_comp_full_) (void)hipStreamDestroy(s_comp_full_);
        if (s_comp_cu_) (void)hipStreamDestroy(s_comp_cu_);
        if (s_comm_) (void)hipStreamDestroy(s_comm_);
        for (auto e : {ev_start_, ev_end_, ev_layer_, ev_halo_, ev_shell_})
            if (e) (void)hipEventDestroy(e);
        for (auto e : ev_marks_)
            if (e) (void)hipEventDestroy(e);
        ev_marks_.clear();
        if (ts_host_) (void)hipHostFree(ts_host_);
        ts_host_ = ts_dev_ = nullptr;
        if (gexec_) (void)hipGraphExecDestroy(gexec_);
        gexec_ = nullptr;
        s_comp_ = s_comm_ = s_comp_full_ = s_comp_cu_ = nullptr;
    }

    // ---- helpers ----------------------------------------------------------------------
    // the enqueue order depends on overlap_ and shells_first_: a captured graph of another arm
    // (either field) is dropped
    void set_overlap(bool on, bool shells_first) {
        if (on == overlap_ && shells_first == shells_first_) return;
        shells_first_ = shells_first;
        if (on == overlap_) {
            if (gexec_) (void)hipGraphExecDestroy(gexec_);
            gexec_ = nullptr;
            return;
        }
        overlap_ = on;
        // between solves (both streams idle): the sweeps move to the CU-masked stream and back
        if (s_comp_cu_) s_comp_ = on ? s_comp_cu_ : s_comp_full_;
        if (gexec_) (void)hipGraphExecDestroy(gexec_);
        gexec_ = nullptr;
    }
    // start of the contiguous block of logical plane i (all rows, ghosts included)
    T* plane(DevRank<T>& R, int level, int i) {
        return R.g[level] + i64(i) * R.gv.si - R.plane_off;
    }
    // Level buffer of layer n (n = -1 .. K): slot_[n + 1], planned by plan_slots() from the
    // run's own schedule of sweeps. Each sweep reads the two newest stored layers and writes
    // its stored layers into the other slots, so L_ = 4 buffers serve every schedule with up
    // to two stored layers per operation — three-layer sweeps included (their C = u^m is never
    // stored), where a `n % L` ring needed 5 (the slot of u^m sat idle). The reference keeps 3
    // rolling levels (mpi_new.cpp:458-460) for one stored layer per step.
    int lvl(int n) const {
        W3D_REQUIRE(n >= -1 && size_t(n + 1) < slot_.size(), "level of a layer outside the planned schedule");
        return slot_[n + 1];
    }
    // layers computed by the operation that starts at layer n (3: three-layer sweep, 2: two-
    // layer sweep, 1: single step) — the schedule of enqueue_layers()
    int span_at(int n) const {
        const int left = prob_.K - n + 1;
        return tb_ ? std::max(1, std::min(tbd_, left)) : 1;
    }
    // Slot plan of a solve that starts at layer `start` (1, or the layer after a resumed
    // checkpoint): layers start-1 / start-2 in slots 0 / 1; every operation then takes the
    // lowest free slots for the layers it stores. A three-layer sweep's C layer maps to the slot
    // of its E layer (n + 2), so lookups of it (checkpoint guards) name a level the sweep writes.
    // first_write_[n + 1]: layer n is the first of this solve written into its slot.
    void plan_slots(int start) {
        const int K = prob_.K;
        slot_.assign(size_t(K) + 2, 0);
        first_write_.assign(size_t(K) + 2, 0);
        W3D_REQUIRE(start >= 1 && start <= K + 1, "bad first layer");
        slot_[start] = 0;       // layer start - 1
        slot_[start - 1] = 1;   // layer start - 2
        std::vector<char> used(size_t(L_), 0);
        for (int n = start; n <= K;) {
            const int span = span_at(n);
            const int live[2] = {slot_[n], slot_[n - 1]};  // layers n - 1, n - 2
            const int first_stored = span >= 2 ? n + span - 2 : n;  // sweeps store their last two
            int l = 0;
            for (int q = first_stored; q < n + span; ++q) {
                while (l == live[0] || l == live[1]) ++l;
                W3D_REQUIRE(l < L_, "level plan needs more time levels than allocated");
                slot_[q + 1] = l;
                first_write_[q + 1] = !used[l];
                used[l] = 1;
                ++l;
            }
            for (int q = n; q < first_stored; ++q) slot_[q + 1] = slot_[n + span];  // unstored layers
            n += span;
        }
    }
    const Wrap& wrap_depth(const DevRank<T>& R, int d) const {
        return d >= 4 ? R.wrap4 : (d == 3 ? R.wrap3 : (d == 2 ? R.wrap2 : R.wrap));
    }

    int send_plane(const DevRank<T>& R, int side) const {
        return side ? R.topo.x_send_plus() : R.topo.x_send_minus();
    }

    void* send_ptr(DevRank<T>& R, size_t m, int n) {
        const auto& f = R.plan.sends[m];
        if (f.axis == 0) return plane(R, lvl(n), send_plane(R, f.side));
        return R.sbuf[m];
    }
    void* recv_ptr(DevRank<T>& R, size_t m, int n) {
        const auto& f = R.plan.recvs[m];
        if (f.axis == 0) return plane(R, lvl(n), f.side ? R.topo.X() + 1 : 0);
        return R.rbuf[m];
    }

    StepCoefs coefs(int n) const {
        StepCoefs c;
        c.hx2 = prob_.hx2;
        c.hy2 = prob_.hy2;
        c.hz2 = prob_.hz2;
        c.coef = n == 1 ? prob_.coef_first : prob_.coef;
        c.ct = ct_[n];
        return c;
    }

    void step_boxes(DevRank<T>& R, int n, const Box* boxes, int nbox, const KernelVariant& kind,
                    hipStream_t s) {
        const T* u1 = R.g[lvl(n - 1)];
        const T* u2 = R.g[lvl(n - 2)];
        launch_step<T>(kind, n == 1, u1, u2, R.g[lvl(n)], R.gv, boxes, nbox, R.error.i0,
                       R.error.i1, R.wrap, R.pack, R.tx, R.ty, R.tz, coefs(n),
                       R.err + size_t(n) * kSlotsPerLayer, cfg_.chunk, s);
    }

    // Halo plan of the temporal-blocking paths (depth dA = layers per sweep):
    //  x up:   newest level planes ending at X (last x-rank: at X-1) -> peer ghosts 1-dA..0,
    //          the level before at depth dA-1, [last: plane X -> peer alias plane(s)]
    //  x down: mirrored -> peer ghosts X+1..X+dA, [first: plane 1 -> peer alias]
    //  y, z:   rows / columns staged through buffers, after the x planes, over the full extent
    //          of the axes exchanged before (edges without diagonal messages)
    // Sends are listed up then down, receives from-down then from-up: per-peer FIFO order
    // matches on both ends also when up == down (dims[0] == 2).
    void build_tb_plan(DevRank<T>& R) {
        R.tb_sends.clear();
        R.tb_recvs.clear();
        const auto& t = R.topo;
        const int X = t.X(), Y = t.Y(), Z = t.Z();
        R.tb_interior = R.compute;
        R.tb_shell.clear();
        const bool ysplit = t.dims[1] > 1, zsplit = t.dims[2] > 1;
        if (!tb_ || (R.plan.self_x && !ysplit && !zsplit)) return;
        using M = typename DevRank<T>::PlaneMsg;
        using BM = typename DevRank<T>::BoxMsg;
        // ---- x: whole planes (contiguous, sent in place) ----------------------------------
        // depth dA of the newest level (next A), dB = dA - 1 of the one before (next B); the
        // periodic duplicate plane x = N is skipped (mpi_new.cpp:186-187) and shipped to the
        // other end of the ring as the seam alias plane instead (tags 12/14, 22/24)
        const int dA = tbd_, dB = tbd_ - 1;
        if (!R.plan.self_x) {
            W3D_REQUIRE(X >= 2 * dA, "temporal blocking needs >= 2 x depth planes per rank");
            // one x rank messaging itself (--x-self-transport): the seam partner planes are
            // its own planes X and 1 (see sweep), no alias messages
            const bool first = t.first(0) && t.dims[0] > 1, last = t.last(0) && t.dims[0] > 1;
            const bool lastx = t.last(0), firstx = t.first(0);
            const int up = t.nbr[0][1], dn = t.nbr[0][0];
            const bool aliasB = tbd_ >= 3;
            R.tb_sends.push_back(M{up, 11, 0, lastx ? X - dA : X - dA + 1, dA});
            if (last) R.tb_sends.push_back(M{up, 12, 0, X, 1});
            R.tb_sends.push_back(M{up, 13, 1, lastx ? X - dB : X - dB + 1, dB});
            if (last && aliasB) R.tb_sends.push_back(M{up, 14, 1, X, 1});
            R.tb_sends.push_back(M{dn, 21, 0, firstx ? 2 : 1, dA});
            if (first) R.tb_sends.push_back(M{dn, 22, 0, 1, 1});
            R.tb_sends.push_back(M{dn, 23, 1, firstx ? 2 : 1, dB});
            if (first && aliasB) R.tb_sends.push_back(M{dn, 24, 1, 1, 1});
            R.tb_recvs.push_back(M{dn, 11, 0, 1 - dA, dA});
            if (first) R.tb_recvs.push_back(M{dn, 12, 0, kAliasPlane, 1});
            R.tb_recvs.push_back(M{dn, 13, 1, 1 - dB, dB});
            if (first && aliasB) R.tb_recvs.push_back(M{dn, 14, 1, kAliasPlane, 1});
            R.tb_recvs.push_back(M{up, 21, 0, X + 1, dA});
            if (last) R.tb_recvs.push_back(M{up, 22, 0, kAliasPlane, 1});
            R.tb_recvs.push_back(M{up, 23, 1, X + 1, dB});
            if (last && aliasB) R.tb_recvs.push_back(M{up, 24, 1, kAliasPlane, 1});
            if (first || last) {
                HIP_CHECK(hipMalloc(&R.alias_buf, R.gv.si * sizeof(T)));
                HIP_CHECK(hipMemset(R.alias_buf, 0, R.gv.si * sizeof(T)));
                if (aliasB) {
                    HIP_CHECK(hipMalloc(&R.alias_bufB, R.gv.si * sizeof(T)));
                    HIP_CHECK(hipMemset(R.alias_bufB, 0, R.gv.si * sizeof(T)));
                }
            }
        }
        // ---- y (round 0) and z (round 1): next A depth dA, next B depth dB ---------------
        const int G = G_;
        if (direct_) build_tb_direct(R);
        for (int ax = 1; ax <= 2 && !direct_; ++ax) {
            if (t.dims[ax] == 1) continue;
            const int n = ax == 1 ? Y : Z;
            auto box = [&](int lo, int hi) {
                // full extent (ghosts included) on the axes exchanged before this one
                Box b{1 - G, X + G, 1, Y, 1, Z};
                if (ax == 1) b.j0 = lo, b.j1 = hi;
                else b.j0 = 1 - G, b.j1 = Y + G, b.k0 = lo, b.k1 = hi;
                return b;
            };
            auto add = [&](std::vector<BM>& v, int peer, int tag, int level, Box b) {
                const size_t cnt = size_t(b.i1 - b.i0 + 1) * (b.j1 - b.j0 + 1) * (b.k1 - b.k0 + 1);
                T* buf = nullptr;
                HIP_CHECK(hipMalloc(&buf, cnt * sizeof(T)));
                v.push_back(BM{peer, tag, level, b, buf});
            };
            const int base = ax == 1 ? 30 : 50;
            const int dn = t.nbr[ax][0], up = t.nbr[ax][1];
            auto& S = R.tb_bsends[ax - 1];
            auto& V = R.tb_brecvs[ax - 1];
            // sends: down (to dn) then up; receives: from down then from up — the same
            // per-peer order on both sides (tag-less RCCL matching)
            W3D_REQUIRE(n >= 2 * dA, "temporal blocking needs >= 2 x depth nodes per rank on split axes");
            if (dn >= 0) add(S, dn, base + 1, 0, box(1, dA)), add(S, dn, base + 2, 1, box(1, dB));
            if (up >= 0)
                add(S, up, base + 11, 0, box(n - dA + 1, n)), add(S, up, base + 12, 1, box(n - dB + 1, n));
            if (dn >= 0) add(V, dn, base + 11, 0, box(1 - dA, 0)), add(V, dn, base + 12, 1, box(1 - dB, 0));
            if (up >= 0)
                add(V, up, base + 1, 0, box(n + 1, n + dA)), add(V, up, base + 2, 1, box(n + 1, n + dB));
            // three-layer sweeps also evaluate C on the seam alias plane (k_seam_c), whose
            // j/k neighbours at the subdomain edge are ghosts: the alias planes of the y/z
            // neighbours (same x coordinate, so they hold the same global plane) supply them
            if (tbd_ >= 3 && R.alias_buf) {
                auto abox = [&](int lo, int hi) {
                    Box b = box(lo, hi);
                    b.i0 = b.i1 = 0;
                    return b;
                };
                if (dn >= 0) add(S, dn, base + 3, 2, abox(1, dA));
                if (up >= 0) add(S, up, base + 13, 2, abox(n - dA + 1, n));
                if (dn >= 0) add(V, dn, base + 13, 2, abox(1 - dA, 0));
                if (up >= 0) add(V, up, base + 3, 2, abox(n + 1, n + dA));
            }
        }
        // the last layer within dA nodes of a received ghost depends on it (through the rings).
        // The j/k shells are widened to whole tiles — TJ rows from the compute box's edge, k on
        // the global 64-column tile grid — so the shell launch runs no partially filled tiles
        // (a 2-column z shell used 2 of 64 lanes per tile and cost ~20 % of a sweep); the
        // interior shrinks by the same nodes, so the total work is that of one full sweep. x
        // shells stay dA planes thin: the march along i handles thin boxes at a small prologue.
        // The shells also contain every plane / row / column the next exchange sends (the first
        // and last x-ranks send one plane deeper, skipping the periodic duplicate plane), so the
        // exchange can start as soon as the shells are done, while the interior still runs.
        Box c = R.compute, in = c;
        const int TJ = tb_rows_ * tb_waves_ / tb_nwk_, TKs = kTileK * tb_nwk_;
        if (!R.plan.self_x) {
            const int xs = t.dims[0] > 1 ? 1 : 0;  // one x rank messaging itself: both ends
            in.i0 = std::max(in.i0, 1 + dA + ((t.first(0) || !xs) ? 1 : 0));
            in.i1 = std::min(in.i1, X - dA - ((t.last(0) || !xs) ? 1 : 0));
        }
        if (t.nbr[1][0] >= 0) in.j0 = std::max(in.j0, std::max(1 + dA, c.j0 + TJ));
        if (t.nbr[1][1] >= 0) in.j1 = std::min(in.j1, std::min(Y - dA, c.j1 - TJ));
        if (t.nbr[2][0] >= 0) in.k0 = std::max(in.k0, 1 + TKs * ((dA + TKs - 1) / TKs));
        if (t.nbr[2][1] >= 0) in.k1 = std::min(in.k1, TKs * ((Z - dA) / TKs));
        R.tb_interior = in;
        auto add = [&](Box b) {
            if (!b.empty()) R.tb_shell.push_back(b);
        };
        if (in.empty()) {
            add(c);
        } else {
            add({c.i0, in.i0 - 1, c.j0, c.j1, c.k0, c.k1});
            add({in.i1 + 1, c.i1, c.j0, c.j1, c.k0, c.k1});
            add({in.i0, in.i1, c.j0, in.j0 - 1, c.k0, c.k1});
            add({in.i0, in.i1, in.j1 + 1, c.j1, c.k0, c.k1});
            add({in.i0, in.i1, in.j0, in.j1, c.k0, in.k0 - 1});
            add({in.i0, in.i1, in.j0, in.j1, in.k1 + 1, c.k1});
        }
    }

    // Single-round deep-halo plan (--halo direct, the default). The round plan above needs three
    // dependent rounds (x planes, then y boxes over the received x ghosts, then z boxes over both)
    // so that edges and corners arrive without diagonal messages. On a fully connected xGMI node
    // every diagonal neighbour has its own link, so here every ghost region — faces, edges,
    // corners, of A (depth dA) and B (depth dB), and of the seam alias planes — comes straight
    // from the rank that owns it, all in one transport group: one latency instead of three, all
    // links busy at once (2x2x2: 7 peers, one link each). Region rules per axis a, receiver R,
    // sender S = R + d: d_a = -1 -> R's ghosts 1-D..0 from S's top D owned nodes, +1 -> R's
    // ghosts E+1..E+D from S's bottom D, 0 -> the owned range (and the x ghosts as well when x
    // wraps inside the rank: the fused wrap fills them). Across the periodic seam the duplicate
    // plane is skipped (mpi_new.cpp:186-187): the last x-rank sends X-D..X-1, the first 2..D+1,
    // and the planes x = N / x = 0 themselves travel as the alias planes. Messages are listed
    // by (level, direction) on both ends, so per-peer FIFO order matches for tag-less RCCL.
    void build_tb_direct(DevRank<T>& R) {
        using BM = typename DevRank<T>::BoxMsg;
        const auto& t = R.topo;
        const int E[3] = {t.X(), t.Y(), t.Z()};
        const int dA = tbd_, dB = tbd_ - 1;
        const bool selfx = R.plan.self_x;  // dims[0] == 1, wrap fused into the kernels
        const bool seam = t.dims[0] > 1;   // alias planes exist (first / last x-rank)
        auto peer = [&](const int d[3]) -> int {  // rank at coords + d, -1 outside y/z
            int c[3];
            for (int a = 0; a < 3; ++a) {
                c[a] = t.coords[a] + d[a];
                if (a == 0) c[a] = ((c[a] % t.dims[0]) + t.dims[0]) % t.dims[0];
                else if (c[a] < 0 || c[a] >= t.dims[a]) return -1;
            }
            return t.rank_of(c[0], c[1], c[2]);
        };
        auto add = [&](std::vector<BM>& v, int pr, int tag, int level, Box b) {
            v.push_back(BM{pr, tag, level, b, nullptr});  // buffer: the peer's packed message
        };
        // receive box of R for direction d (ghost region), depth D
        auto rbox = [&](const int d[3], int D, bool alias) {
            int lo[3], hi[3];
            for (int a = 0; a < 3; ++a) {
                if (d[a] < 0) lo[a] = 1 - D, hi[a] = 0;
                else if (d[a] > 0) lo[a] = E[a] + 1, hi[a] = E[a] + D;
                else if (a == 0 && selfx) lo[a] = 1 - D, hi[a] = E[a] + D;
                else lo[a] = 1, hi[a] = E[a];
            }
            if (alias) lo[0] = hi[0] = 0;  // the alias buffer's one plane (logical i = 0)
            return Box{lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]};
        };
        // source box of R for a receiver Q = R - d (R fills Q's ghosts in direction d)
        auto sbox = [&](const int d[3], int D, bool alias) {
            int lo[3], hi[3];
            for (int a = 0; a < 3; ++a) {
                // crossing the periodic seam from Q to R: Q first and R last x-rank (d = -1),
                // or Q last and R first (d = +1); with one x rank messaging itself both hold
                const int tw = a == 0 && ((d[a] < 0 && t.last(0)) || (d[a] > 0 && t.first(0))) ? 1 : 0;
                if (d[a] < 0) lo[a] = E[a] - D + 1 - tw, hi[a] = E[a] - tw;
                else if (d[a] > 0) lo[a] = 1 + tw, hi[a] = D + tw;
                else if (a == 0 && selfx) lo[a] = 1 - D, hi[a] = E[a] + D;
                else lo[a] = 1, hi[a] = E[a];
            }
            if (alias) lo[0] = hi[0] = d[0] < 0 ? E[0] : 1;  // plane x = N (last) / x = 0 (first)
            return Box{lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]};
        };
        for (int level = 0; level < (tbd_ >= 3 ? 4 : 3); ++level) {
            const bool alias = level >= 2;
            if (alias && !seam) continue;
            const int D = (level == 0 || level == 2) ? dA : dB;
            int q = 0;
            for (int dx = -1; dx <= 1; ++dx)
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dz = -1; dz <= 1; ++dz, ++q) {
                        if (!dx && !dy && !dz) continue;
                        if (selfx && dx) continue;  // x ghosts: fused wrap
                        if (alias && !dx) continue;  // alias planes cross the x seam only
                        if (!dy && !dz) continue;    // x faces: whole planes in place (x list)
                        const int tag = 200 + q * 4 + level;
                        const int d[3] = {dx, dy, dz}, md[3] = {-dx, -dy, -dz};
                        // receive: from S = R + d into R's ghosts (alias: R first x-rank <- last
                        // for d_x = -1, R last <- first for d_x = +1)
                        const int S = peer(d);
                        const bool ra = !alias || (dx < 0 ? t.first(0) : t.last(0));
                        if (S >= 0 && ra) add(R.tb_drecvs, S, tag, level, rbox(d, D, alias));
                        // send: to Q = R - d from R's own nodes (alias: R last x-rank -> first
                        // for d_x = -1, R first -> last for d_x = +1)
                        const int Q = peer(md);
                        const bool sa = !alias || (dx < 0 ? t.last(0) : t.first(0));
                        if (Q >= 0 && sa) add(R.tb_dsends, Q, tag, level, sbox(d, D, alias));
                    }
        }
        // one buffer per peer: its boxes back to back in (level, direction) order — the order
        // in which both ends list them, so the packed messages have the same layout
        auto aggregate = [&](std::vector<BM>& v, std::vector<typename DevRank<T>::PeerBuf>& agg) {
            std::vector<int> peers;
            for (auto& m : v)
                if (std::find(peers.begin(), peers.end(), m.peer) == peers.end()) peers.push_back(m.peer);
            std::sort(peers.begin(), peers.end());
            for (int pr : peers) {
                size_t n = 0;
                for (auto& m : v)
                    if (m.peer == pr) n += size_t(m.box.count());
                T* buf = nullptr;
                HIP_CHECK(hipMalloc(&buf, n * sizeof(T)));
                size_t off = 0;
                for (auto& m : v)
                    if (m.peer == pr) m.buf = buf + off, off += size_t(m.box.count());
                agg.push_back({pr, buf, n});
            }
        };
        aggregate(R.tb_dsends, R.tb_psends);
        aggregate(R.tb_drecvs, R.tb_precvs);
    }

    // single-step overlap: y/z shells as whole tiles of the march kernel (else flat shells)
    bool shells_tiled() const { return kind_.march && !kind_.flat; }

    bool tb_halo(const DevRank<T>& R) const {
        return !R.tb_sends.empty() || !R.tb_bsends[0].empty() || !R.tb_bsends[1].empty() ||
               !R.tb_brecvs[0].empty() || !R.tb_brecvs[1].empty() || !R.tb_dsends.empty() ||
               !R.tb_drecvs.empty();
    }

    void* tb_ptr(DevRank<T>& R, const typename DevRank<T>::PlaneMsg& m, int mD) {
        if (m.plane == kAliasPlane) return m.level == 0 ? R.alias_buf : R.alias_bufB;
        return plane(R, lvl(m.level == 0 ? mD : mD - 1), m.plane);
    }

    // exchange after a sweep whose D layer is mD (A level = mD, B level = mD-1)
    // --halo direct: pack every message, one transport group (or loopback copies), unpack.
    // Grid of a message's box: levels 0 / 1 are the A / B levels; the seam alias levels 2 / 3 are
    // sent from the sender's own A / B planes (x = N or x = 0) and received into the alias
    // buffers (one plane, logical i = 0).
    T* direct_grid(DevRank<T>& R, int level, int mD, bool send) {
        if (level == 2 && !send) return R.alias_buf + R.plane_off;
        if (level == 3 && !send) return R.alias_bufB + R.plane_off;
        return R.g[lvl(level % 2 == 0 ? mD : mD - 1)];
    }
    void box_copies(DevRank<T>& R, std::vector<typename DevRank<T>::BoxMsg>& v, int mD, bool to_buf, hipStream_t s) {
        for (size_t q0 = 0; q0 < v.size(); q0 += kMaxBoxCopy) {
            BoxCopy<T> o[kMaxBoxCopy];
            int n = 0;
            for (size_t q = q0; q < v.size() && n < kMaxBoxCopy; ++q, ++n) {
                // an alias buffer holds one plane: never let a box index another (host check)
                W3D_REQUIRE(v[q].level < 2 || to_buf || (v[q].box.i0 == 0 && v[q].box.i1 == 0),
                            "direct halo: alias box outside its one-plane buffer");
                o[n].grid = direct_grid(R, v[q].level, mD, to_buf), o[n].buf = v[q].buf, o[n].b = v[q].box;
            }
            launch_box_copy<T>(o, n, R.gv, to_buf, s);
        }
    }
    void exchange_direct(int mD, hipStream_t s) {
        for (auto& R : ranks_) box_copies(R, R.tb_dsends, mD, true, s);
        auto bytes = [](const typename DevRank<T>::BoxMsg& m) { return size_t(m.box.count()) * sizeof(T); };
        mark(s, 6);
        (void)bytes;
        constexpr int kPeerTag = 199;  // one packed message per peer and direction of travel
        if (ext_) {
            // x faces as whole planes sent and received in place (their y/z ghost rows are
            // overwritten by the edge boxes unpacked after the group), then one packed message
            // per peer — the same order on both ends
            auto& R = ranks_[0];
            std::vector<Message> snd, rcv;
            for (auto& m : R.tb_sends)
                snd.push_back({m.peer, m.tag, tb_ptr(R, m, mD), size_t(m.nplanes) * R.gv.si * sizeof(T)});
            for (auto& m : R.tb_recvs)
                rcv.push_back({m.peer, m.tag, tb_ptr(R, m, mD), size_t(m.nplanes) * R.gv.si * sizeof(T)});
            for (auto& m : R.tb_psends) snd.push_back({m.peer, kPeerTag, m.buf, m.count * sizeof(T)});
            for (auto& m : R.tb_precvs) rcv.push_back({m.peer, kPeerTag, m.buf, m.count * sizeof(T)});
            model_link_ext(snd, s);
            if (!snd.empty() || !rcv.empty()) ext_->exchange(snd, rcv, s);
        } else {
            std::map<std::pair<int, int>, size_t> link;
            for (auto& S : ranks_) {
                for (auto& m : S.tb_sends) link[{S.topo.rank, m.peer}] += size_t(m.nplanes) * S.gv.si * sizeof(T);
                for (auto& m : S.tb_psends) link[{S.topo.rank, m.peer}] += m.count * sizeof(T);
            }
            model_link(link, s);
            for (auto& S : ranks_)
                for (auto& m : S.tb_sends) {
                    auto& D = ranks_[m.peer];
                    bool done = false;
                    for (auto& g : D.tb_recvs)
                        if (g.peer == S.topo.rank && g.tag == m.tag) {
                            W3D_REQUIRE(g.nplanes == m.nplanes, "tb halo size mismatch");
                            loop_copy(tb_ptr(D, g, mD), tb_ptr(S, m, mD), size_t(m.nplanes) * S.gv.si * sizeof(T),
                                      S.topo.rank, D.topo.rank, m.tag, s);
                            done = true;
                            break;
                        }
                    W3D_REQUIRE(done, "unmatched tb halo message");
                }
            for (auto& S : ranks_)
                for (auto& m : S.tb_psends) {
                    bool done = false;
                    for (auto& g : ranks_[m.peer].tb_precvs)
                        if (g.peer == S.topo.rank) {
                            W3D_REQUIRE(g.count == m.count, "direct halo size mismatch between ranks " +
                                                                std::to_string(S.topo.rank) + " and " +
                                                                std::to_string(m.peer));
                            loop_copy(g.buf, m.buf, m.count * sizeof(T), S.topo.rank, m.peer, kPeerTag, s);
                            done = true;
                            break;
                        }
                    W3D_REQUIRE(done, "unmatched direct halo message to rank " + std::to_string(m.peer));
                }
        }
        mark(s, 7);
        for (auto& R : ranks_) box_copies(R, R.tb_drecvs, mD, false, s);
        for (auto& R : ranks_) inject_after_exchange(R, mD, s);
    }

    void exchange_tb(int mD, hipStream_t s) {
        if (direct_) {
            exchange_direct(mD, s);
            return;
        }
        if (ext_) {
            auto& R = ranks_[0];
            std::vector<Message> snd, rcv;
            for (auto& m : R.tb_sends)
                snd.push_back({m.peer, m.tag, tb_ptr(R, m, mD), size_t(m.nplanes) * R.gv.si * sizeof(T)});
            for (auto& m : R.tb_recvs)
                rcv.push_back({m.peer, m.tag, tb_ptr(R, m, mD), size_t(m.nplanes) * R.gv.si * sizeof(T)});
            if (!snd.empty() || !rcv.empty()) {
                mark(s, 6);
                model_link_ext(snd, s);
                ext_->exchange(snd, rcv, s);
                mark(s, 7);
            }
        } else {
            mark(s, 6);
            for (auto& S : ranks_)
                for (auto& m : S.tb_sends) {
                    auto& D = ranks_[m.peer];
                    bool done = false;
                    for (auto& g : D.tb_recvs)
                        if (g.peer == S.topo.rank && g.tag == m.tag) {
                            W3D_REQUIRE(g.nplanes == m.nplanes, "tb halo size mismatch");
                            loop_copy(tb_ptr(D, g, mD), tb_ptr(S, m, mD), size_t(m.nplanes) * S.gv.si * sizeof(T),
                                      S.topo.rank, D.topo.rank, m.tag, s);
                            done = true;
                            break;
                        }
                    W3D_REQUIRE(done, "unmatched tb halo message");
                }
            mark(s, 7);
        }
        // y then z rounds: pack -> transport / D2D -> unpack, strictly after the x planes
        for (int rd = 0; rd < 2; ++rd) {
            bool any = false;
            for (auto& R : ranks_) any |= !R.tb_bsends[rd].empty() || !R.tb_brecvs[rd].empty();
            if (!any) continue;
            auto ops = [&](DevRank<T>& R, std::vector<typename DevRank<T>::BoxMsg>& v) {
                std::vector<BoxCopy<T>> o;
                for (auto& m : v) {
                    BoxCopy<T> b;
                    // level 2 = the seam alias plane (a one-plane buffer at logical i = 0)
                    b.grid = m.level == 2 ? R.alias_buf + R.plane_off
                                          : R.g[lvl(m.level == 0 ? mD : mD - 1)];
                    b.buf = m.buf;
                    b.b = m.box;
                    o.push_back(b);
                }
                return o;
            };
            for (auto& R : ranks_) {
                auto o = ops(R, R.tb_bsends[rd]);
                launch_box_copy<T>(o.data(), int(o.size()), R.gv, true, s);
            }
            auto bytes = [](const typename DevRank<T>::BoxMsg& m) {
                const Box& b = m.box;
                return size_t(b.i1 - b.i0 + 1) * (b.j1 - b.j0 + 1) * (b.k1 - b.k0 + 1) * sizeof(T);
            };
            if (ext_) {
                auto& R = ranks_[0];
                std::vector<Message> snd, rcv;
                for (auto& m : R.tb_bsends[rd]) snd.push_back({m.peer, m.tag, m.buf, bytes(m)});
                for (auto& m : R.tb_brecvs[rd]) rcv.push_back({m.peer, m.tag, m.buf, bytes(m)});
                mark(s, 6);
                model_link_ext(snd, s);
                ext_->exchange(snd, rcv, s);
                mark(s, 7);
            } else {
                mark(s, 6);
                for (auto& S : ranks_)
                    for (auto& m : S.tb_bsends[rd]) {
                        bool done = false;
                        for (auto& g : ranks_[m.peer].tb_brecvs[rd])
                            if (g.peer == S.topo.rank && g.tag == m.tag) {
                                W3D_REQUIRE(bytes(g) == bytes(m), "tb box halo size mismatch");
                                loop_copy(g.buf, m.buf, bytes(m), S.topo.rank, m.peer, m.tag, s);
                                done = true;
                                break;
                            }
                        W3D_REQUIRE(done, "unmatched tb box halo message");
                    }
                mark(s, 7);
            }
            for (auto& R : ranks_) {
                auto o = ops(R, R.tb_brecvs[rd]);
                launch_box_copy<T>(o.data(), int(o.size()), R.gv, false, s);
            }
        }
        for (auto& R : ranks_) inject_after_exchange(R, mD, s);
    }

    // temporal-blocking sweep: layers m (C) and m+1 (D) from m-1 (A) and m-2 (B)
    void sweep(DevRank<T>& R, int m, hipStream_t s, const Box* boxes = nullptr, int nbox = 0) {
        const T* A = R.g[lvl(m - 1)];
        const T* B = R.g[lvl(m - 2)];
        SeamAlias<T> al;
        if (R.topo.dims[0] == 1) {  // self-wrap, fused or through the transport
            al.next_i = 0;  // ghost copy of N-1 sees x=N (own plane X) as its x+ neighbour
            al.next = A + i64(R.topo.X()) * R.gv.si;
            al.prev_i = R.topo.X() + 1;  // ghost copy of 1 sees x=0 (own plane 1) as x-
            al.prev = A + i64(1) * R.gv.si;
        } else if (R.topo.first(0)) {   // alias = x=N received from the last x-rank
            al.next_i = 0;
            al.next = R.alias_buf + R.plane_off;
        } else if (R.topo.last(0)) {    // alias = x=0 received from the first x-rank
            al.prev_i = R.topo.X() + 1;
            al.prev = R.alias_buf + R.plane_off;
        }
        if (!boxes) boxes = &R.compute, nbox = 1;
        // two-layer tails of a tb3 run whose tile has no tb2 instantiation (1-row tiles) use
        // the default tb2 tile
        const bool own = tb2_supported(tb_rows_, tb_waves_, tb_occ_, tb_nwk_);
        // (--math fma tails of a tb3 run: the r2w8 fma instantiation)
        launch_tb2<T>(own ? tb_rows_ : 2, own ? tb_waves_ : 8, own ? tb_occ_ : 0, own ? tb_nwk_ : 1, cfg_.delta,
                      cfg_.fma && tb2_fma_supported(own ? tb_rows_ : 2, own ? tb_waves_ : 8, own ? tb_nwk_ : 1, cfg_.delta),
                      m == 1, A, B, R.g[lvl(m)], R.g[lvl(m + 1)], R.gv, boxes, nbox,
                      R.cdom, R.error.i0, R.error.i1, R.wrap, R.wrap2, al, R.txy, R.tz, R.rtxy, R.rtz,
                      coefs(m), coefs(m + 1), R.err + size_t(m) * kSlotsPerLayer,
                      R.err + size_t(m + 1) * kSlotsPerLayer, cfg_.chunk, s);
    }

    // Three-layer sweep m: C = u^m (registers only), D = u^{m+1}, E = u^{m+2}.
    SeamPartners<T> seam_partners(DevRank<T>& R, int m, std::vector<SeamCPlane<T>>* ops) {
        const T* A = R.g[lvl(m - 1)];
        const T* B = R.g[lvl(m - 2)];
        const i64 si = R.gv.si;
        const int X = R.topo.X();
        SeamPartners<T> sp;
        auto scratch = [&](int q) { return R.seamc_buf + i64(q) * si + R.plane_off; };
        auto add = [&](int q, const T* Ac, const T* Am, const T* Ap, const T* Bc) {
            W3D_REQUIRE(R.seamc_buf, "seam C scratch not allocated");
            SeamCPlane<T> o;
            o.out = scratch(q), o.Ac = Ac, o.Am = Am, o.Ap = Ap, o.Bc = Bc;
            if (ops) ops->push_back(o);
            return scratch(q);
        };
        const T* aA = R.alias_buf ? R.alias_buf + R.plane_off : nullptr;
        const T* aB = R.alias_bufB ? R.alias_bufB + R.plane_off : nullptr;
        if (R.topo.dims[0] == 1) {
            // ghost copy of N-1 (plane 0) sees x=N (plane X); ghost copy of 1 (X+1) sees x=0
            sp.next_i = 0, sp.nA = A + X * si;
            sp.nC = add(0, A + X * si, A + (X - 1) * si, A + (X + 1) * si, B + X * si);
            sp.prev_i = X + 1, sp.pA = A + 1 * si;
            sp.pC = add(1, A + 1 * si, A + 0 * si, A + 2 * si, B + 1 * si);
        } else if (R.topo.first(0)) {  // partner x=N lives on the last x-rank (alias planes)
            sp.next_i = 0, sp.nA = aA;
            sp.nC = add(0, aA, A + 0 * si, A + 2 * si, aB);
        } else if (R.topo.last(0)) {   // partner x=0 lives on the first x-rank
            sp.prev_i = X + 1, sp.pA = aA;
            sp.pC = add(1, aA, A + (X - 1) * si, A + (X + 1) * si, aB);
        }
        return sp;
    }

    // seam C planes: after the halo of u^{m-1} (they read its ghost / alias planes)
    void seam_c(DevRank<T>& R, int m, hipStream_t s) {
        std::vector<SeamCPlane<T>> ops;
        seam_partners(R, m, &ops);
        launch_seam_c<T>(m == 1, cfg_.delta, cfg_.fma, ops.data(), int(ops.size()), R.gv, R.cdom, coefs(m), s);
    }

    // Four-layer sweep m (k_tbn): layers m, m+1 in registers only, m+2 and m+3 stored. The seam
    // partners are layers m-1 (A), m and m+1 at the partner planes; layer m+1 there needs layer m
    // at the partner and at both its x neighbours — with the seam rule at the one across the seam
    // (the ghost copy of global 1 sees x = 0, of N-1 sees x = N): stage 1 evaluates layer m on
    // those planes (C ops), stage 2 layer m+1 at each partner (D ops), both before the sweep.
    TbnSeam<T> seam_partners4(DevRank<T>& R, int m, std::vector<SeamCPlane<T>>* c_ops,
                              std::vector<SeamCPlane<T>>* d_ops) {
        const T* A = R.g[lvl(m - 1)];
        const T* B = R.g[lvl(m - 2)];
        const i64 si = R.gv.si;
        const int X = R.topo.X();
        TbnSeam<T> sp;
        auto scratch = [&](int q) { return R.seamc_buf + i64(q) * si + R.plane_off; };
        // increment form: B holds d^{m-1}; the partner planes' layer-m ops also keep their d
        // (scratch 8 / 9), which stage 2 takes as its Bc in place of the leapfrog's u^{m-1} = A
        const bool dl = cfg_.delta;
        auto op = [&](std::vector<SeamCPlane<T>>* v, int q, const T* c, const T* xm, const T* xp, const T* pw,
                      int dq = -1) {
            W3D_REQUIRE(R.seamc_buf, "seam scratch not allocated");
            SeamCPlane<T> o;
            o.out = scratch(q), o.Ac = c, o.Am = xm, o.Ap = xp, o.Bc = pw;
            if (dl && dq >= 0) o.dout = scratch(dq);
            if (v) v->push_back(o);
            return scratch(q);
        };
        auto dpl = [&](int q, const T* leap) { return dl ? static_cast<const T*>(scratch(q)) : leap; };
        auto Ap = [&](int i) { return A + i64(i) * si; };
        auto Bp = [&](int i) { return B + i64(i) * si; };
        const T* aA = R.alias_buf ? R.alias_buf + R.plane_off : nullptr;
        const T* aB = R.alias_bufB ? R.alias_bufB + R.plane_off : nullptr;
        if (R.topo.dims[0] == 1) {
            // next side (ghost 0 = copy of N-1): partner x = N = plane X
            const T* cX = op(c_ops, 0, Ap(X), Ap(X - 1), Ap(X + 1), Bp(X), 8);
            const T* cXm = op(c_ops, 1, Ap(X - 1), Ap(X - 2), Ap(X), Bp(X - 1));
            const T* cXp = op(c_ops, 2, Ap(X + 1), Ap(1), Ap(X + 2), Bp(X + 1));  // copy of 1: x- = x=0
            sp.next_i = 0, sp.nP[0] = Ap(X), sp.nP[1] = cX, sp.nP[2] = op(d_ops, 6, cX, cXm, cXp, dpl(8, Ap(X)));
            // prev side (ghost X+1 = copy of 1): partner x = 0 = plane 1
            const T* c1 = op(c_ops, 3, Ap(1), Ap(0), Ap(2), Bp(1), 9);
            const T* c0 = op(c_ops, 4, Ap(0), Ap(-1), Ap(X), Bp(0));  // copy of N-1: x+ = x=N
            const T* c2 = op(c_ops, 5, Ap(2), Ap(1), Ap(3), Bp(2));
            sp.prev_i = X + 1, sp.pP[0] = Ap(1), sp.pP[1] = c1, sp.pP[2] = op(d_ops, 7, c1, c0, c2, dpl(9, Ap(1)));
        } else if (R.topo.first(0)) {
            // partner x = N lives on the last x-rank (alias planes); ghost 0 = N-1, plane 2 = global 1
            const T* cN = op(c_ops, 0, aA, Ap(0), Ap(2), aB, 8);
            const T* cNm = op(c_ops, 1, Ap(0), Ap(-1), aA, Bp(0));
            const T* c1 = op(c_ops, 2, Ap(2), Ap(1), Ap(3), Bp(2));
            sp.next_i = 0, sp.nP[0] = aA, sp.nP[1] = cN, sp.nP[2] = op(d_ops, 6, cN, cNm, c1, dpl(8, aA));
        } else if (R.topo.last(0)) {
            // partner x = 0 lives on the first x-rank; plane X-1 = N-1, ghost X+1 = global 1
            const T* c0 = op(c_ops, 3, aA, Ap(X - 1), Ap(X + 1), aB, 9);
            const T* cm = op(c_ops, 4, Ap(X - 1), Ap(X - 2), Ap(X), Bp(X - 1));
            const T* cp = op(c_ops, 5, Ap(X + 1), aA, Ap(X + 2), Bp(X + 1));  // copy of 1: x- = x=0
            sp.prev_i = X + 1, sp.pP[0] = aA, sp.pP[1] = c0, sp.pP[2] = op(d_ops, 7, c0, cm, cp, dpl(9, aA));
        }
        return sp;
    }

    void seam4(DevRank<T>& R, int m, hipStream_t s) {
        std::vector<SeamCPlane<T>> c_ops, d_ops;
        seam_partners4(R, m, &c_ops, &d_ops);
        launch_seam_c<T>(m == 1, cfg_.delta, cfg_.fma, c_ops.data(), int(c_ops.size()), R.gv, R.cdom, coefs(m), s);
        launch_seam_c<T>(false, cfg_.delta, cfg_.fma, d_ops.data(), int(d_ops.size()), R.gv, R.cdom, coefs(m + 1), s);
    }

    void sweep4(DevRank<T>& R, int m, hipStream_t s, const Box* boxes = nullptr, int nbox = 0) {
        const T* A = R.g[lvl(m - 1)];
        const T* B = R.g[lvl(m - 2)];
        const TbnSeam<T> sp = seam_partners4(R, m, nullptr, nullptr);
        if (!boxes) boxes = &R.compute, nbox = 1;
        StepCoefs c[4];
        u64* err[4];
        for (int l = 0; l < 4; ++l) c[l] = coefs(m + l), err[l] = R.err + size_t(m + l) * kSlotsPerLayer;
        launch_tbn<T>(4, tb_rows_, tb_waves_, cfg_.fma, m == 1, A, B, R.g[lvl(m + 2)], R.g[lvl(m + 3)], R.gv, boxes,
                      nbox, R.cdom, R.error.i0, R.error.i1, R.wrap3, R.wrap4, sp, R.txy, R.tz, R.rtxy, R.rtz, c,
                      err, cfg_.chunk, s, cfg_.delta);
    }

    // the seam pre-kernels of the sweep that starts at layer m (span 3 or 4); `in`: into the
    // interior's own scratch copy (overlapped self-wrap runs: the interior and the shells run
    // concurrently on two streams)
    void seam_pre(DevRank<T>& R, int m, int span, hipStream_t s, bool in = false) {
        SeamScratch use(R, in);
        if (span == 4) seam4(R, m, s);
        else seam_c(R, m, s);
    }
    void sweep_deep(DevRank<T>& R, int m, int span, hipStream_t s, const Box* boxes = nullptr, int nbox = 0,
                    bool in = false) {
        SeamScratch use(R, in);
        if (span == 4) sweep4(R, m, s, boxes, nbox);
        else sweep3(R, m, s, boxes, nbox);
    }
    // selects the seam scratch set for the calls in its scope
    struct SeamScratch {
        DevRank<T>& R;
        T* saved;
        SeamScratch(DevRank<T>& r, bool in) : R(r), saved(r.seamc_buf) {
            if (in && r.seamc_in) r.seamc_buf = r.seamc_in;
        }
        ~SeamScratch() { R.seamc_buf = saved; }
    };

    void sweep3(DevRank<T>& R, int m, hipStream_t s, const Box* boxes = nullptr, int nbox = 0) {
        const T* A = R.g[lvl(m - 1)];
        const T* B = R.g[lvl(m - 2)];
        const SeamPartners<T> sp = seam_partners(R, m, nullptr);
        if (!boxes) boxes = &R.compute, nbox = 1;
        if (tbn_ && tbd_ == 3) {  // the depth-generic kernel at depth 3 (A/B against k_tb3)
            TbnSeam<T> ts;
            ts.next_i = sp.next_i, ts.prev_i = sp.prev_i;
            ts.nP[0] = sp.nA, ts.nP[1] = sp.nC, ts.pP[0] = sp.pA, ts.pP[1] = sp.pC;
            StepCoefs c[3];
            u64* err[3];
            for (int l = 0; l < 3; ++l) c[l] = coefs(m + l), err[l] = R.err + size_t(m + l) * kSlotsPerLayer;
            launch_tbn<T>(3, tb_rows_, tb_waves_, cfg_.fma, m == 1, A, B, R.g[lvl(m + 1)], R.g[lvl(m + 2)], R.gv,
                          boxes, nbox, R.cdom, R.error.i0, R.error.i1, R.wrap2, R.wrap3, ts, R.txy, R.tz, R.rtxy,
                          R.rtz, c, err, cfg_.chunk, s);
            return;
        }
        launch_tb3<T>(tb_rows_, tb_waves_, cfg_.delta, cfg_.fma, m == 1, A, B, R.g[lvl(m + 1)], R.g[lvl(m + 2)], R.gv, boxes,
                      nbox, R.cdom, R.error.i0, R.error.i1, R.wrap2, R.wrap3, sp, R.txy, R.tz, R.rtxy, R.rtz,
                      coefs(m), coefs(m + 1), coefs(m + 2), R.err + size_t(m) * kSlotsPerLayer,
                      R.err + size_t(m + 1) * kSlotsPerLayer, R.err + size_t(m + 2) * kSlotsPerLayer,
                      cfg_.chunk, s);
    }

    void pack_faces(DevRank<T>& R, int n, hipStream_t s, bool to_buf) {
        FaceOp<T> ops[4];
        int k = 0;
        const auto& list = to_buf ? R.plan.sends : R.plan.recvs;
        for (size_t m = 0; m < list.size(); ++m) {
            const auto& f = list[m];
            if (f.axis == 0) continue;
            FaceOp<T>& o = ops[k++];
            o.buf = to_buf ? R.sbuf[m] : R.rbuf[m];
            o.axis = f.axis;
            if (to_buf) o.index = f.side ? R.topo.ext[f.axis] : 1;
            else o.index = f.side ? R.topo.ext[f.axis] + 1 : 0;
        }
        launch_faces<T>(R.g[lvl(n)], R.gv, ops, k, to_buf, s);
    }

    void inject_after_exchange(DevRank<T>& R, int n, hipStream_t s) {
        if (selftest_) return;
        // exchanges follow every sweep: a fault layer inside the sweep hits its exchange
        const int lo = tb_ ? n - tbd_ : n - 1;
        if (fault_.kind == "drop_face" && fault_.hits_range(R.topo.rank, lo, n))
            HIP_CHECK(hipMemsetAsync(plane(R, lvl(n), 0), 0, R.gv.si * sizeof(T), s));
    }
    void inject_after_compute(DevRank<T>& R, int n, hipStream_t s, int from = -1) {
        if (fault_.kind == "nan" && fault_.hits_range(R.topo.rank, (from < 0 ? n : from) - 1, n)) {
            const Box& b = R.compute;
            if (b.empty()) return;
            T* p = R.g[lvl(n)] + i64((b.i0 + b.i1) / 2) * R.gv.si + i64((b.j0 + b.j1) / 2) * R.gv.sj +
                   (b.k0 + b.k1) / 2;
            HIP_CHECK(hipMemsetAsync(p, 0xFF, sizeof(T), s));
        }
    }

    // Exchange of layer n, issued on stream s (loopback: all ranks; transport: this rank).
    void exchange(int n, hipStream_t s) {
        if (ext_) {
            auto& R = ranks_[0];
            std::vector<Message> snd, rcv;
            for (size_t m = 0; m < R.plan.sends.size(); ++m)
                snd.push_back({R.plan.sends[m].peer, R.plan.sends[m].tag, send_ptr(R, m, n),
                               size_t(R.plan.sends[m].count) * sizeof(T)});
            for (size_t m = 0; m < R.plan.recvs.size(); ++m)
                rcv.push_back({R.plan.recvs[m].peer, R.plan.recvs[m].tag, recv_ptr(R, m, n),
                               size_t(R.plan.recvs[m].count) * sizeof(T)});
            if (!snd.empty() || !rcv.empty()) {
                mark(s, 6);
                model_link_ext(snd, s);
                ext_->exchange(snd, rcv, s);
                mark(s, 7);
            }
            pack_faces(R, n, s, false);
            inject_after_exchange(R, n, s);
            return;
        }
        mark(s, 6);
        {
            std::map<std::pair<int, int>, size_t> link;
            for (auto& S : ranks_)
                for (auto& f : S.plan.sends) link[{S.topo.rank, f.peer}] += size_t(f.count) * sizeof(T);
            model_link(link, s);
        }
        for (auto& S : ranks_)
            for (size_t m = 0; m < S.plan.sends.size(); ++m) {
                const auto& f = S.plan.sends[m];
                auto& D = ranks_[f.peer];
                bool done = false;
                for (size_t q = 0; q < D.plan.recvs.size(); ++q) {
                    const auto& g = D.plan.recvs[q];
                    if (g.peer == S.topo.rank && g.tag == f.tag) {
                        W3D_REQUIRE(g.count == f.count, "halo size mismatch");
                        loop_copy(recv_ptr(D, q, n), send_ptr(S, m, n), f.count * sizeof(T), S.topo.rank,
                                  D.topo.rank, f.tag, s);
                        done = true;
                        break;
                    }
                }
                W3D_REQUIRE(done, "unmatched halo message");
            }
        mark(s, 7);
        for (auto& R : ranks_) {
            pack_faces(R, n, s, false);
            inject_after_exchange(R, n, s);
        }
    }

    // --model-link: the loopback transfer of one exchange round also waits the time the
    // busiest link of the round needs — every (sender, receiver) pair has its own xGMI link on a
    // fully connected node and every rank sends at once, so a round lasts max over pairs of
    // bytes / bandwidth, plus one latency. One wave spins that long on the exchange stream (one
    // CU, as a remote transfer's kernels), so overlap experiments on one GPU see a halo that
    // costs wall time without costing the interior sweep its CUs.
    // ... and for a rank of a distributed job (one process per GPU, or processes sharing one GPU
    // through the staged transport): its own busiest outgoing link — every rank sends at once, so
    // the exchange lasts about that long on every rank (bench.py --model-link rehearses the
    // 8-GPU decompositions on one GPU with a link cost)
    void model_link_ext(const std::vector<Message>& snd, hipStream_t s) {
        if (cfg_.model_link_gbps <= 0 || snd.empty()) return;
        std::map<std::pair<int, int>, size_t> link;
        for (const auto& m : snd) link[{ranks_[0].topo.rank, m.peer}] += m.bytes;
        model_link(link, s);
    }
    void model_link(const std::map<std::pair<int, int>, size_t>& link_bytes, hipStream_t s) {
        if (cfg_.model_link_gbps <= 0) return;
        size_t most = 0;
        for (const auto& kv : link_bytes) most = std::max(most, kv.second);
        const double sec = double(most) / (cfg_.model_link_gbps * 1e9) + cfg_.model_link_lat_us * 1e-6;
        launch_spin(u64(sec * clock_khz_ * 1e3), s);
    }

    // ---- loopback copies and the RCCL mirror ------------------------------------------------
    // One halo message between two in-process ranks: a D2D copy. With --rccl-mirror every such
    // message also travels through a 1-rank RCCL communicator (ncclSend/ncclRecv to itself, the
    // same group call, bytes and stream order as a real multi-GPU rank) into a scratch buffer,
    // and a device compare against the loopback copy counts differing words per message kind:
    // every message shape of the multi-GPU plan runs through RCCL on one GPU, bit for bit.
    // Loopback halo copies of simulated ranks: WAVE3D_LOOP_COPY=sdma issues them to the DMA
    // engines (hipMemcpyDeviceToDeviceNoCU: no CU taken from a concurrent interior sweep, as a
    // remote peer's xGMI traffic takes none), blit = HIP's copy kernels
    static hipMemcpyKind loop_copy_kind() {
        static const hipMemcpyKind k = [] {
            const char* e = std::getenv("WAVE3D_LOOP_COPY");
            return e && std::string(e) == "sdma" ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToDevice;
        }();
        return k;
    }
    void loop_copy(void* dst, const void* src, size_t bytes, int src_rank, int dst_rank, int tag, hipStream_t s) {
        HIP_CHECK(hipMemcpyAsync(dst, src, bytes, loop_copy_kind(), s));
        if (!mirror_) return;
        W3D_REQUIRE(bytes <= mirror_bytes_, "rccl mirror scratch too small");
        mirror_->exchange({Message{0, tag, const_cast<void*>(src), bytes}}, {Message{0, tag, mirror_buf_, bytes}}, s);
        launch_compare_bytes(mirror_buf_, dst, bytes, mirror_res_ + 2 * mirror_slot(src_rank, dst_rank, tag), s);
        ++mirror_msgs_;
    }

    int mirror_slot(int src, int dst, int tag) {
        const i64 key = (i64(src) << 40) | (i64(dst) << 20) | i64(tag & 0xFFFFF);
        auto it = mirror_index_.find(key);
        if (it != mirror_index_.end()) return it->second;
        W3D_REQUIRE(mirror_keys_.size() < kMirrorSlots, "too many distinct halo messages for the rccl mirror");
        mirror_keys_.push_back("rank " + std::to_string(src) + " -> rank " + std::to_string(dst) + " tag " +
                               std::to_string(tag));
        const int slot = int(mirror_keys_.size()) - 1;
        mirror_index_[key] = slot;
        return slot;
    }

    void setup_mirror() {
        size_t most = 8 * (size_t(prob_.K) + 1) * kSlotsPerLayer;  // the error-key allreduce
        for (auto& R : ranks_) {
            for (auto& f : R.plan.sends) most = std::max(most, size_t(f.count) * sizeof(T));
            for (auto& m : R.tb_sends) most = std::max(most, size_t(m.nplanes) * size_t(R.gv.si) * sizeof(T));
            for (int rd = 0; rd < 2; ++rd)
                for (auto& m : R.tb_bsends[rd]) most = std::max(most, size_t(m.box.count()) * sizeof(T));
            for (auto& m : R.tb_psends) most = std::max(most, m.count * sizeof(T));
        }
        int dev = 0;
        HIP_CHECK(hipGetDevice(&dev));
        mirror_ = std::make_unique<RcclTransport>(0, 1, rccl_unique_id(), dev);
        mirror_bytes_ = most;
        HIP_CHECK(hipMalloc(&mirror_buf_, most));
        HIP_CHECK(hipMalloc(&mirror_res_, sizeof(u64) * 2 * kMirrorSlots));
        reset_mirror();
    }

    void reset_mirror() {
        std::vector<u64> init(2 * kMirrorSlots);
        for (size_t q = 0; q < init.size(); ++q) init[q] = q % 2 ? ~0ull : 0ull;
        HIP_CHECK(hipMemcpy(mirror_res_, init.data(), init.size() * sizeof(u64), hipMemcpyHostToDevice));
    }

    // after a solve: the error keys through a 1-rank ncclAllReduce(max) too, then every count
    void check_mirror(const u64* err, size_t n, hipStream_t s) {
        HIP_CHECK(hipMemcpyAsync(mirror_buf_, err, n * sizeof(u64), hipMemcpyDeviceToDevice, s));
        mirror_->allreduce_max_u64(static_cast<u64*>(mirror_buf_), n, s);
        launch_compare_bytes(mirror_buf_, err, n * sizeof(u64), mirror_res_ + 2 * mirror_slot(0, 0, -1), s);
        ++mirror_msgs_;
        std::vector<u64> res(2 * kMirrorSlots);
        HIP_CHECK(hipMemcpyAsync(res.data(), mirror_res_, res.size() * sizeof(u64), hipMemcpyDeviceToHost, s));
        sync(s);
        std::string bad;
        for (size_t q = 0; q < mirror_keys_.size(); ++q)
            if (res[2 * q])
                bad += "\n  " + (mirror_keys_[q] == "rank 0 -> rank 0 tag -1" ? std::string("error-key allreduce")
                                                                            : mirror_keys_[q]) +
                       ": " + std::to_string(res[2 * q]) + " words differ (first word " +
                       std::to_string(res[2 * q + 1]) + ")";
        reset_mirror();
        if (!bad.empty()) throw Error("wave3d: RCCL mirror differs from the loopback copies:" + bad);
    }

    // ---- init-time halo self-test ---------------------------------------------------------
    // One real exchange of position-encoded patterns (hip_selftest.hpp) through this run's
    // plan and transport — x planes, seam alias planes, y/z box rounds, or the single-step
    // faces — and a device check of every cell each message delivered. A wrong peer, tag,
    // size, level or placement fails at setup with the rank, peer and tag of the message; the
    // failure count is max-reduced over the ranks so every rank stops at once (the reference
    // only ever sees a halo bug as a wrong error table, cuda_sol.cpp:245-310).
    struct CheckRegion {
        int peer = -1, tag = 0;
        const T* origin = nullptr;  // logical (0,0,0) of the level / alias plane
        Box box;
        PatternCoords pc;
        std::string what;
    };

    std::vector<CheckRegion> check_regions(DevRank<T>& R, bool deep, int lA, int lB, unsigned sA, unsigned sB) {
        std::vector<CheckRegion> out;
        const auto& t = R.topo;
        const int X = t.X(), Y = t.Y(), Z = t.Z();
        PatternCoords base;
        for (int a = 0; a < 3; ++a) base.off[a] = t.off[a];
        base.N = prob_.N;
        auto region = [&](int peer, int tag, const T* origin, Box b, unsigned salt, i64 gi, std::string what) {
            CheckRegion c;
            c.peer = peer, c.tag = tag, c.origin = origin, c.box = b, c.pc = base;
            c.pc.salt = salt, c.pc.gi_fixed = gi, c.what = std::move(what);
            out.push_back(c);
        };
        if (!deep) {
            const int l = lvl(1);
            for (const auto& f : R.plan.recvs) {
                Box b{1, X, 1, Y, 1, Z};
                const int ghost = f.side ? t.ext[f.axis] + 1 : 0;
                if (f.axis == 0) b.i0 = b.i1 = ghost;
                else if (f.axis == 1) b.j0 = b.j1 = ghost;
                else b.k0 = b.k1 = ghost;
                region(f.peer, f.tag, R.g[l], b, sA, -1, std::string("face axis ") + "xyz"[f.axis]);
            }
            return out;
        }
        const i64 alias_gi = t.first(0) ? prob_.N : 0;  // first x-rank holds x=N, last x=0
        for (const auto& m : R.tb_recvs) {
            const unsigned salt = m.level == 0 ? sA : sB;
            if (m.plane == kAliasPlane) {
                const T* o = (m.level == 0 ? R.alias_buf : R.alias_bufB) + R.plane_off;
                region(m.peer, m.tag, o, Box{0, 0, 1, Y, 1, Z}, salt, alias_gi, "seam alias plane");
            } else {
                region(m.peer, m.tag, R.g[m.level == 0 ? lA : lB],
                       Box{m.plane, m.plane + m.nplanes - 1, 1, Y, 1, Z}, salt, -1, "x planes");
            }
        }
        for (const auto& m : R.tb_drecvs) {  // --halo direct: every message is one box
            Box b = m.box;
            if (R.plan.self_x && m.level < 2) b.i0 = std::max(b.i0, 1), b.i1 = std::min(b.i1, X);
            const unsigned salt = (m.level == 0 || m.level == 2) ? sA : sB;
            const bool al = m.level >= 2;
            region(m.peer, m.tag, direct_grid(R, m.level, 2, false), b, salt, al ? alias_gi : -1,
                   al ? "direct alias box" : "direct box");
        }
        const int dA = tbd_, dB = tbd_ - 1;
        for (int rd = 0; rd < 2; ++rd)
            for (const auto& m : R.tb_brecvs[rd]) {
                // only what the sender itself held valid: ghosts of depth dA (A) / dB (B) on
                // the axes exchanged before; a fused local x wrap is not part of the exchange
                const int d = m.level == 1 ? dB : dA;
                Box b = m.box;
                if (m.level != 2) {
                    b.i0 = std::max(b.i0, R.plan.self_x ? 1 : 1 - d);
                    b.i1 = std::min(b.i1, R.plan.self_x ? X : X + d);
                }
                b.j0 = std::max(b.j0, 1 - d), b.j1 = std::min(b.j1, Y + d);
                b.k0 = std::max(b.k0, 1 - d), b.k1 = std::min(b.k1, Z + d);
                if (m.level == 2)
                    region(m.peer, m.tag, R.alias_buf + R.plane_off, b, sA, alias_gi, "alias plane box");
                else
                    region(m.peer, m.tag, R.g[m.level == 0 ? lA : lB], b, m.level == 0 ? sA : sB, -1,
                           rd == 0 ? "y box" : "z box");
            }
        return out;
    }

    void halo_self_test() {
        TraceRange tr("wave3d.halo_selftest");
        const bool deep = tb_ && tb_halo(ranks_[0]);
        const int mD = 2;  // deep: A level = lvl(2), B = lvl(1) (as exchange_tb); faces: lvl(1)
        // a fixed slot plan for the test (layers -1..2 -> slots 2, 3, 1, 0), independent of K
        const std::vector<int> run_slots = slot_;
        slot_ = {2, 3, 1, 0};
        const int lA = deep ? lvl(mD) : lvl(1), lB = lvl(mD - 1);
        const unsigned sA = 0xA11CEu, sB = 0xB0B5u;
        hipStream_t s = s_comp_;
        std::vector<std::vector<CheckRegion>> regs;
        size_t nreg = 0;
        for (auto& R : ranks_) {
            PatternCoords pc;
            for (int a = 0; a < 3; ++a) pc.off[a] = R.topo.off[a];
            pc.N = prob_.N;
            const Box all{1 - G_, R.topo.X() + G_, 1 - G_, R.topo.Y() + G_, 1 - G_, R.topo.Z() + G_};
            pc.salt = sA;
            launch_pattern_fill<T>(R.g[lA], R.gv, all, pc, 0, 0.0, s);
            if (deep) {
                pc.salt = sB;
                launch_pattern_fill<T>(R.g[lB], R.gv, all, pc, 0, 0.0, s);
                if (R.alias_buf) HIP_CHECK(hipMemsetAsync(R.alias_buf, 0, R.gv.si * sizeof(T), s));
                if (R.alias_bufB) HIP_CHECK(hipMemsetAsync(R.alias_bufB, 0, R.gv.si * sizeof(T), s));
            } else {
                pack_faces(R, 1, s, true);
            }
            regs.push_back(check_regions(R, deep, lA, lB, sA, sB));
            nreg += regs.back().size();
        }
        selftest_ = true;  // no --fault drop_face injection into the test exchange
        if (deep) exchange_tb(mD, s);
        else exchange(1, s);
        selftest_ = false;
        // fault hook (--fault corrupt_tag:RANK:TAG): what the message of that tag delivered to
        // RANK is overwritten, as a transport that lost or misrouted it would leave it
        for (size_t q = 0; q < ranks_.size(); ++q)
            if (fault_.kind == "corrupt_tag" && ranks_[q].topo.rank == fault_.rank)
                for (auto& c : regs[q])
                    if (c.tag == fault_.layer)
                        launch_pattern_fill<T>(const_cast<T*>(c.origin), ranks_[q].gv, c.box, c.pc, 1, 0.0, s);
        u64* dres = nullptr;
        HIP_CHECK(hipMalloc(&dres, sizeof(u64) * 2 * std::max<size_t>(1, nreg)));
        std::vector<u64> init(2 * std::max<size_t>(1, nreg));
        for (size_t q = 0; q < init.size(); ++q) init[q] = q % 2 ? ~0ull : 0ull;
        HIP_CHECK(hipMemcpyAsync(dres, init.data(), init.size() * sizeof(u64), hipMemcpyHostToDevice, s));
        size_t idx = 0;
        for (size_t q = 0; q < ranks_.size(); ++q)
            for (auto& c : regs[q]) launch_pattern_check<T>(c.origin, ranks_[q].gv, c.box, c.pc, dres + 2 * idx++, s);
        std::vector<u64> res(init.size());
        HIP_CHECK(hipMemcpyAsync(res.data(), dres, res.size() * sizeof(u64), hipMemcpyDeviceToHost, s));
        sync(s);
        std::string report;
        int nbad = 0;
        idx = 0;
        for (size_t q = 0; q < ranks_.size(); ++q)
            for (auto& c : regs[q]) {
                const u64 bad = res[2 * idx], first = res[2 * idx + 1];
                ++idx;
                if (!bad) continue;
                ++nbad;
                const Box& b = c.box;
                const i64 nk = b.k1 - b.k0 + 1, nj = b.j1 - b.j0 + 1;
                const int k = b.k0 + int(i64(first) % nk), j = b.j0 + int(i64(first) / nk % nj),
                          i = b.i0 + int(i64(first) / nk / nj);
                T got{};
                HIP_CHECK(hipMemcpy(&got, c.origin + i64(i) * ranks_[q].gv.si + i64(j) * ranks_[q].gv.sj + k,
                                    sizeof(T), hipMemcpyDeviceToHost));
                i64 gi = c.pc.gi_fixed >= 0 ? c.pc.gi_fixed : c.pc.off[0] + i - 1;
                const i64 gj = c.pc.off[1] + j - 1, gk = c.pc.off[2] + k - 1, N = prob_.N;
                gi = gi < 0 ? gi + N : (gi > N ? gi - N : gi);
                const double want = (gj < 0 || gj > N || gk < 0 || gk > N)
                                        ? kPatternSentinel
                                        : double(T(halo_pattern_value(gi, gj, gk, c.pc.salt)));
                if (nbad <= 8)
                    report += "\n  rank " + std::to_string(ranks_[q].topo.rank) + ": message from peer " +
                              std::to_string(c.peer) + " tag " + std::to_string(c.tag) + " (" + c.what + "): " +
                              std::to_string(bad) + " of " + std::to_string(b.count()) +
                              " cells wrong, first at local (" + std::to_string(i) + "," + std::to_string(j) +
                              "," + std::to_string(k) + "): got " + std::to_string(double(got)) + " expected " +
                              std::to_string(want);
            }
        (void)hipFree(dres);
        double v = nbad;
        if (ext_) ext_->allreduce_max_host(&v, 1);  // every rank fails together, fast
        // restore the post-allocation state the solve relies on (zeroed levels and alias planes)
        for (auto& R : ranks_) {
            for (int l = 0; l < L_; ++l) HIP_CHECK(hipMemsetAsync(R.alloc[l], 0, R.elems * sizeof(T), s));
            if (R.alias_buf) HIP_CHECK(hipMemsetAsync(R.alias_buf, 0, R.gv.si * sizeof(T), s));
            if (R.alias_bufB) HIP_CHECK(hipMemsetAsync(R.alias_bufB, 0, R.gv.si * sizeof(T), s));
        }
        sync(s);
        slot_ = run_slots;
        if (v > 0)
            throw Error("wave3d: halo self-test failed" +
                        (report.empty() ? std::string(" on another rank (this rank's messages were correct)")
                                        : ":" + report));
        halo_checked_ = int(nreg);
        log_msg(LogLevel::Info, "halo self-test: ", nreg, " messages verified");
    }

    // Phase timers (the reference's C26 breakdown, mpi_new.cpp:33-34,368-371, in every run).
    // Slots: 0/1 compute (loop), 2/3 halo exchange incl. pack/unpack (comm stream when
    // overlapped), 4/5 final error reduction, 6/7 the transport itself (RCCL group / loopback
    // copies: the reference's "MPI exchange" time; 2/3 minus 6/7 is its "host-device
    // exchange"). Per-sweep ("fine") marks whenever halos move; a run without any exchange gets
    // one loop interval around the IC + time loop instead (nothing between its kernels).
    // Direct launches record timing events (a stream marker, no kernel); inside a hipGraph
    // capture — where event records carry no timestamps on this HIP — a one-lane kernel stamps
    // the device wall clock into pinned host memory instead. WAVE3D_NO_TIMERS=1 drops every
    // fine mark (the A/B baseline of the timer cost).
    enum MarkMode { kAlways, kFine, kCoarse };
    void mark(hipStream_t s, int slot, MarkMode m = kFine) {
        if ((m == kFine && !fine_) || (m == kCoarse && fine_)) return;
        if (no_timers_ && m != kAlways) return;
        if (tn_ >= ts_cap_) return;  // capacity is sized for every mark of a solve
        if (capturing_ || stamped_) launch_stamp(ts_dev_, int(tn_), s);
        else HIP_CHECK(hipEventRecord(ev_marks_[tn_], s));
        if (tn_ < tslot_.size()) tslot_[tn_] = slot;
        else tslot_.push_back(slot);
        ++tn_;
    }

    // device progress for the transport watchdog: marks of this solve completed so far
    long progress() {
        if (stamped_) {
            while (prog_seen_ < tn_ && reinterpret_cast<volatile u64*>(ts_host_)[prog_seen_] != 0) ++prog_seen_;
        } else {
            while (prog_seen_ < tn_ && hipEventQuery(ev_marks_[prog_seen_]) == hipSuccess) ++prog_seen_;
        }
        return long(prog_seen_);
    }

    // ---- time loop --------------------------------------------------------------------
    void solve(RunResult& res, Timings& tm) {
        TraceRange tr("wave3d.solve");
        const int K = prob_.K;
        prog_seen_ = 0;
        std::fill(ts_host_, ts_host_ + ts_cap_, u64(0));
        // No per-solve clear of the levels: every cell the stencil reads is written first
        // in this solve (IC, fused wrap / halo exchange, Dirichlet faces at n <= 3); the
        // buffers are zeroed once at allocation.
        for (auto& R : ranks_) launch_init_err(R.err, K + 1, s_comp_);
        sync(s_comp_);
        if (ext_) ext_->barrier();

        res.resumed_from = -1;
        res.aborted = false;
        plan_slots(1);  // a resume re-plans from its checkpoint layer (load_checkpoints)
        if (graph_eligible() && !gexec_ && !graph_failed_) build_graph(res);  // host-only work
        HIP_CHECK(hipEventRecord(ev_start_, s_comp_));
        if (gexec_) {
            // the whole IC + time loop as one graph launch (no per-kernel host overhead); its
            // timer marks were captured with it
            tn_ = graph_tn_;
            stamped_ = true;
            HIP_CHECK(hipGraphLaunch(gexec_, s_comp_));
            res.layers_done = K;
        } else {
            tn_ = 0;
            stamped_ = false;
            int start = 1;
            if (!cfg_.resume_dir.empty()) {
                start = load_checkpoints() + 1;
                res.resumed_from = start - 1;
                mark(s_comp_, 0, kCoarse);
            } else {
                enqueue_ic();
            }
            res.layers_done = enqueue_layers(res, start);
        }
        res.graph = gexec_ != nullptr;

        // final max-reduction of the per-layer slots (mpi_new.cpp:358-361)
        TraceRange trr("wave3d.reduce");
        mark(s_comp_, 4, kAlways);
        const size_t nslot = size_t(K + 1) * kSlotsPerLayer;
        std::vector<u64> acc(nslot, 0);
        if (ext_) {
            HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_halo_, 0));
            ext_->allreduce_max_u64(ranks_[0].err, nslot, s_comp_);
        }
        for (auto& R : ranks_) {
            HIP_CHECK(hipMemcpyAsync(host_err_.data(), R.err, nslot * sizeof(u64),
                                     hipMemcpyDeviceToHost, s_comp_));
            sync(s_comp_);
            for (size_t q = 0; q < nslot; ++q) acc[q] = std::max(acc[q], host_err_[q]);
        }
        mark(s_comp_, 5, kAlways);
        HIP_CHECK(hipEventRecord(ev_end_, s_comp_));
        if (mirror_) check_mirror(ranks_[0].err, nslot, s_comp_);  // outside the timed interval
        HIP_CHECK(hipEventSynchronize(ev_end_));
        // graph replay: the progress lines once the layers are done (one launch runs them all)
        if (res.graph && cfg_.print_layers && !cfg_.quiet && ranks_[0].topo.rank == 0)
            for (int q = 1; q <= K; ++q) std::cout << "calculating layer " << q << "\n";
        finish_checkpoint();  // files complete when solve() returns
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, ev_start_, ev_end_));
        tm.total_ms = ms;
        res.max_abs.assign(K + 1, kErrInit);
        res.max_rel.assign(K + 1, kErrInit);
        for (int n = 0; n <= K; ++n) {
            res.max_abs[n] = decode_max_key(acc[size_t(n) * 3 + 0]);
            res.max_rel[n] = decode_max_key(acc[size_t(n) * 3 + 1]);
        }
        if (res.resumed_from >= 0)
            for (int n = 0; n <= res.resumed_from && n < int(ckpt_abs_.size()); ++n)
                res.max_abs[n] = ckpt_abs_[n], res.max_rel[n] = ckpt_rel_[n];
        collect_profile(tm);
        res.rccl_mirror_msgs = mirror_msgs_;
    }

    // ---- time loop ----------------------------------------------------------------------
    void enqueue_ic() {
        TraceRange tr("wave3d.ic");
        mark(s_comp_, 0, kAlways);
        for (auto& R : ranks_) {
            launch_init<T>(R.g[lvl(0)], R.gv, R.owned, wrap_depth(R, G_), R.tx, R.ty, R.tz, ct_[0],
                           R.err, s_comp_);
            pack_faces(R, 0, s_comp_, true);
        }
        mark(s_comp_, 1);
        if (prob_.K >= 1) issue_exchange(0);
    }

    // Layers start..K on the streams; host work only for --check-every / checkpoints.
    // Returns the last layer computed.
    int enqueue_layers(RunResult& res, int start) {
        TraceRange tr("wave3d.layers");
        // the order this enqueue (or the graph captured from it) runs: checked against the
        // reported order by tests (a replayed graph of another arm would show here)
        order_enqueued_ = !overlap_ ? "none" : shells_first_ ? "shells_first" : "beside";
        CuReserveScope cu_scope(s_comp_ == s_comp_cu_ ? comm_cus_ : 0);  // work items for the CUs kept
        const int K = prob_.K;
        int done = start - 1;
        for (int n = start; n <= K;) {
            // temporal blocking: 3 (tb3) or 2 layers per sweep; shorter tails use the
            // two-layer sweep / a single step (the storage has ghosts for the deepest)
            const int span = span_at(n);
            bool comm_follows = false;  // the comm stream already runs behind this layer's shells
            for (int q = n; q < n + span; ++q) guard_checkpoint_level(lvl(q), s_comp_);
            if (cfg_.print_layers && !cfg_.quiet && !capturing_ && ranks_[0].topo.rank == 0)
                for (int q = n; q < n + span; ++q) std::cout << "calculating layer " << q << "\n";
            mark(s_comp_, 0);
            // Dirichlet faces of each level buffer on its first write of the solve (the kernels
            // never store to them; a tb3 C layer is not stored)
            for (int q = n; q < n + span; ++q)
                for (auto& R : ranks_)
                    if ((first_write_[q + 1] || q == start) && !(span >= 3 && q < n + span - 2))
                        launch_zero_faces<T>(R.g[lvl(q)], R.gv, R.zero_mask, s_comp_);
            bool exchanged = false;  // the exchange of this sweep's last layer is already enqueued
            if (span >= 3 && overlap_ && shells_first_) {
                // Shells first (WAVE3D_OVERLAP_SHELLS_FIRST): after the previous halo, the shells run
                // on the compute stream as one launch over the whole GPU (work items sized for it),
                // then the next exchange starts on the comm stream while the interior sweeps. The
                // shells no longer share the GPU with the interior for the whole sweep, which a
                // full-length tile band in j or k otherwise does (the z shell is a 64-column band).
                HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_halo_, 0));
                for (auto& R : ranks_) {
                    seam_pre(R, n, span, s_comp_);
                    if (!R.tb_shell.empty())
                        sweep_deep(R, n, span, s_comp_, R.tb_shell.data(), int(R.tb_shell.size()));
                }
                const int last = n + span - 1;
                if (last < K) {
                    HIP_CHECK(hipEventRecord(ev_shell_, s_comp_));
                    HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_shell_, 0));
                    issue_exchange(last, true);
                    exchanged = true;
                }
                for (auto& R : ranks_)
                    if (!R.tb_interior.empty()) sweep_deep(R, n, span, s_comp_, &R.tb_interior, 1);
            } else if (span >= 3 && overlap_) {
                // Shells on the (high-priority) comm stream right behind the previous halo,
                // concurrently with the interior on the compute stream, as the two-layer path:
                // the shells need that halo and the previous sweep's interior; the interior reads
                // only owned nodes of the previous sweep (it stays `span` nodes away from every
                // remote ghost), so it never waits for a halo. The next exchange follows the
                // shells on the comm stream; the compute stream waits for the shells before the
                // next interior (whose rings reach into them).
                HIP_CHECK(hipEventRecord(ev_layer_, s_comp_));
                HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_layer_, 0));
                for (auto& R : ranks_) {
                    seam_pre(R, n, span, s_comm_);
                    if (!R.tb_shell.empty())
                        sweep_deep(R, n, span, s_comm_, R.tb_shell.data(), int(R.tb_shell.size()));
                }
                HIP_CHECK(hipEventRecord(ev_shell_, s_comm_));
                for (auto& R : ranks_) {
                    // periodic self-wrap: the interior spans every x plane, so it reads the seam
                    // partner planes too (at positions that need no remote halo) — from its own
                    // copy, the shells' copy is rewritten concurrently on the comm stream
                    if (R.plan.self_x && !R.tb_interior.empty()) seam_pre(R, n, span, s_comp_, true);
                    if (!R.tb_interior.empty()) sweep_deep(R, n, span, s_comp_, &R.tb_interior, 1, true);
                }
                HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_shell_, 0));
                comm_follows = true;
            } else if (span >= 3) {
                for (auto& R : ranks_) {
                    seam_pre(R, n, span, s_comp_);
                    sweep_deep(R, n, span, s_comp_);
                }
            } else if (span == 2 && overlap_) {
                // Shells on the (high-priority) comm stream right behind the previous halo,
                // concurrently with the interior on the compute stream: both read only levels
                // of earlier sweeps and write disjoint nodes. The shells need the interior of
                // the previous sweep (their rings reach into it); the compute stream waits for
                // the shells before the next interior (whose rings reach into them). The next
                // exchange follows the shells on the comm stream without waiting for the
                // interior — the shells contain every node it sends.
                HIP_CHECK(hipEventRecord(ev_layer_, s_comp_));
                HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_layer_, 0));
                for (auto& R : ranks_)
                    if (!R.tb_shell.empty())
                        sweep(R, n, s_comm_, R.tb_shell.data(), int(R.tb_shell.size()));
                HIP_CHECK(hipEventRecord(ev_shell_, s_comm_));
                for (auto& R : ranks_)
                    if (!R.tb_interior.empty()) sweep(R, n, s_comp_, &R.tb_interior, 1);
                HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_shell_, 0));
                comm_follows = true;
            } else if (span == 2) {
                for (auto& R : ranks_) sweep(R, n, s_comp_);
            } else if (overlap_) {
                // as the two-layer sweep: shells on the comm stream behind the previous halo,
                // concurrently with the interior; the exchange follows the shells
                HIP_CHECK(hipEventRecord(ev_layer_, s_comp_));
                HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_layer_, 0));
                for (auto& R : ranks_) {
                    const int nx = R.shell_x, ny = int(R.shell.size()) - nx;
                    if (nx > 0) step_boxes(R, n, R.shell.data(), nx, naive_, s_comm_);
                    if (ny > 0)
                        step_boxes(R, n, R.shell.data() + nx, ny, shells_tiled() ? kind_ : naive_, s_comm_);
                }
                HIP_CHECK(hipEventRecord(ev_shell_, s_comm_));
                for (auto& R : ranks_)
                    if (!R.interior.empty()) step_boxes(R, n, &R.interior, 1, kind_, s_comp_);
                HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_shell_, 0));
                comm_follows = true;
            } else {
                for (auto& R : ranks_) step_boxes(R, n, &R.compute, 1, kind_, s_comp_);
            }
            // deep sweeps never store their first span-2 layers: a fault there goes to the first
            // stored layer
            const int first_stored = span >= 3 ? n + span - 2 : n;
            for (int q = first_stored; q < n + span; ++q)
                for (auto& R : ranks_) inject_after_compute(R, q, s_comp_, q == first_stored ? n : q);
            mark(s_comp_, 1);
            const int last = n + span - 1;
            if (last < K && !exchanged) issue_exchange(last, comm_follows);
            done = last;
            bool ck = false, stop = false;
            for (int q = n; q <= last; ++q) {
                ck |= cfg_.checkpoint_every > 0 && q % cfg_.checkpoint_every == 0;
                if (cfg_.check_every > 0 && (q % cfg_.check_every == 0 || q == K) && !stop)
                    stop = check_layer(q, res);
            }
            if (stop) break;
            if (ck && last < K) save_checkpoints(last);
            n += span;
        }
        mark(s_comp_, 1, kCoarse);
        return done;
    }

    // hipGraph replay (HIP's answer to a tracing compiler): the IC and every layer — kernels,
    // loopback D2D halo copies and the cross-stream event joins — are captured once per
    // session and replayed with one hipGraphLaunch per solve. Only for runs without host
    // interaction inside the loop (no external transport, checks, checkpoints, profiling,
    // faults); a failed capture falls back to direct launches.
    // With overlap on, --graph auto launches directly: a replayed capture of the two-stream
    // overlap ran its branches serialised (8 simulated ranks with modelled 50 GB/s links: 347k
    // Mpts/s replayed vs 408k launched directly; 2 ranks 348k vs 446k, profiles/overlap_model_r4.txt)
    bool graph_eligible() const {
        return cfg_.graph != 0 && !ext_ && !mirror_ && cfg_.check_every == 0 && cfg_.checkpoint_every == 0 &&
               cfg_.resume_dir.empty() && fault_.kind.empty() && (cfg_.graph == 1 || !overlap_);
    }

    void build_graph(RunResult& res) {
        TraceRange tr("wave3d.graph_capture");
        hipGraph_t g = nullptr;
        try {
            HIP_CHECK(hipStreamBeginCapture(s_comp_, hipStreamCaptureModeThreadLocal));
            capturing_ = true;
            tn_ = 0;
            enqueue_ic();
            enqueue_layers(res, 1);
            graph_tn_ = tn_;
            capturing_ = false;
            HIP_CHECK(hipStreamEndCapture(s_comp_, &g));
            HIP_CHECK(hipGraphInstantiate(&gexec_, g, nullptr, nullptr, 0));
            HIP_CHECK(hipGraphDestroy(g));
            log_msg(LogLevel::Info, "captured IC + ", prob_.K, " layers as one hipGraph");
        } catch (const Error& e) {
            capturing_ = false;
            hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
            if (hipStreamIsCapturing(s_comp_, &st) == hipSuccess && st != hipStreamCaptureStatusNone) {
                hipGraph_t h = nullptr;
                (void)hipStreamEndCapture(s_comp_, &h);
                if (h) (void)hipGraphDestroy(h);
            }
            if (g) (void)hipGraphDestroy(g);
            (void)hipStreamSynchronize(s_comp_);
            (void)hipGetLastError();
            (void)hipGetLastError();
            gexec_ = nullptr;
            graph_failed_ = true;
            if (cfg_.graph == 1) throw;
            if (!cfg_.quiet)
                log_msg(LogLevel::Warn, "hipGraph capture failed (", e.what(),
                        "), using direct launches");
        }
    }

    // exchange of layer n: overlapped on the comm stream, or inline on the compute stream
    void any_exchange(int n, hipStream_t s) {
        if (tb_ && tb_halo(ranks_[0])) exchange_tb(n, s);  // deep halos
        else exchange(n, s);
    }

    void issue_exchange(int n, bool comm_follows = false) {
        if (overlap_) {
            if (!comm_follows) {
                HIP_CHECK(hipEventRecord(ev_layer_, s_comp_));
                HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_layer_, 0));
            }
            mark(s_comm_, 2);
            any_exchange(n, s_comm_);
            mark(s_comm_, 3);
            HIP_CHECK(hipEventRecord(ev_halo_, s_comm_));
        } else {
            bool any = false;
            for (auto& R : ranks_)
                any |= !R.plan.sends.empty() || tb_halo(R) || fault_.kind == "drop_face";
            if (!any) return;
            mark(s_comp_, 2);
            any_exchange(n, s_comp_);
            mark(s_comp_, 3);
            HIP_CHECK(hipEventRecord(ev_halo_, s_comp_));
        }
    }

    void collect_profile(Timings& tm) {
        HIP_CHECK(hipDeviceSynchronize());
        double sum[4] = {0, 0, 0, 0};  // loop, exchange, error, transport
        for (size_t q = 0; q + 1 < tn_; ++q) {
            const int a = tslot_[q];
            if (a % 2) continue;
            for (size_t r = q + 1; r < tn_; ++r)
                if (tslot_[r] == a + 1) {
                    float ms = 0;
                    if (stamped_) ms = float(double(i64(ts_host_[r] - ts_host_[q])) / clock_khz_);
                    else HIP_CHECK(hipEventElapsedTime(&ms, ev_marks_[q], ev_marks_[r]));
                    sum[a / 2] += ms;
                    break;
                }
        }
        tm.loop_ms = sum[0];
        tm.exchange_ms = sum[1];
        tm.comm_ms = sum[3];
        tm.error_ms = sum[2];
    }

    // Both streams idle: host-side collectives (side stream of the transport) must never run
    // concurrently with an in-flight halo exchange on the same communicator.
    void quiesce() {
        sync(s_comp_);
        sync(s_comm_);
    }

    // stream drain; with an external transport under its watchdog (RcclTransport)
    void sync(hipStream_t s) {
        const std::function<long()> prog = [this] { return progress(); };
        if (!(ext_ && ext_->wait_stream(s, &prog))) HIP_CHECK(hipStreamSynchronize(s));
    }

    bool check_layer(int n, RunResult& res) {
        quiesce();
        double v[2] = {kErrInit, 0.0};
        for (auto& R : ranks_) {
            u64 h[3];
            HIP_CHECK(hipMemcpy(h, R.err + size_t(n) * 3, sizeof(h), hipMemcpyDeviceToHost));
            v[0] = std::max(v[0], decode_max_key(h[0]));
            v[1] = std::max(v[1], double(h[2]));
        }
        if (ext_) ext_->allreduce_max_host(v, 2);
        if (layer_diverged(v[0], v[1] != 0.0)) {
            res.aborted = true;
            res.abort_layer = n;
            res.abort_reason = v[1] != 0.0 ? "non-finite values" : "error out of range";
            return true;
        }
        return false;
    }

    // ---- checkpoint / resume ------------------------------------------------------------
    std::vector<double> global_errors_upto(int n) {
        const size_t nslot = size_t(prob_.K + 1) * 3;
        std::vector<u64> h(nslot);
        std::vector<double> a(prob_.K + 1, kErrInit), r(prob_.K + 1, kErrInit);
        quiesce();
        for (auto& R : ranks_) {
            HIP_CHECK(hipMemcpy(h.data(), R.err, nslot * sizeof(u64), hipMemcpyDeviceToHost));
            for (int q = 0; q <= n; ++q) {
                a[q] = std::max(a[q], decode_max_key(h[size_t(q) * 3]));
                r[q] = std::max(r[q], decode_max_key(h[size_t(q) * 3 + 1]));
            }
        }
        if (ext_) {
            ext_->allreduce_max_host(a.data(), a.size());
            ext_->allreduce_max_host(r.data(), r.size());
        }
        a.insert(a.end(), r.begin(), r.end());
        return a;
    }

    HostLevel host_level(DevRank<T>& R, std::vector<T>& h, int level) { return host_level(R, h.data(), level); }
    HostLevel host_level(DevRank<T>& R, T* h, int level) {
        HostLevel L;
        L.origin = h + (R.g[level] - R.alloc[level]);
        L.X = R.topo.X();
        L.Y = R.topo.Y();
        L.Z = R.topo.Z();
        L.sj = R.gv.sj;
        L.si = R.gv.si;
        return L;
    }

    // Checkpoint after layer n: the error maxima so far are reduced now (small,
    // synchronous), the two newest levels are copied device -> pinned host memory on their own
    // stream while the time loop continues, and a background thread writes the files. The
    // compute stream only waits for the copy before it overwrites one of those two levels; the
    // next checkpoint (or the end of the solve) waits for the previous write.
    void save_checkpoints(int n) {
        TraceRange tr("wave3d.checkpoint");
        finish_checkpoint();
        std::vector<double> ar = global_errors_upto(n);
        std::vector<double> a(ar.begin(), ar.begin() + prob_.K + 1), r(ar.begin() + prob_.K + 1, ar.end());
        if (!s_ckpt_) {
            HIP_CHECK(hipStreamCreateWithFlags(&s_ckpt_, hipStreamNonBlocking));
            HIP_CHECK(hipEventCreateWithFlags(&ev_ckpt_, hipEventDisableTiming));
        }
        std::vector<CheckpointHeader> hs;
        std::vector<HostLevel> lps, lcs;
        for (auto& R : ranks_) {
            const int lp = lvl(n - 1), lc = lvl(n);
            if (!R.pinned) {
                void* h = nullptr;
                HIP_CHECK(hipHostMalloc(&h, 2 * R.elems * sizeof(T), hipHostMallocDefault));
                R.pinned = static_cast<T*>(h);
            }
            HIP_CHECK(hipMemcpyAsync(R.pinned, R.alloc[lp], R.elems * sizeof(T), hipMemcpyDeviceToHost, s_ckpt_));
            HIP_CHECK(hipMemcpyAsync(R.pinned + R.elems, R.alloc[lc], R.elems * sizeof(T),
                                     hipMemcpyDeviceToHost, s_ckpt_));
            hs.push_back(make_header(cfg_, R.topo, n, sizeof(T)));
            lps.push_back(host_level(R, R.pinned, lp));
            lcs.push_back(host_level(R, R.pinned + R.elems, lc));
        }
        HIP_CHECK(hipEventRecord(ev_ckpt_, s_ckpt_));
        ckpt_levels_[0] = lvl(n - 1), ckpt_levels_[1] = lvl(n);
        ckpt_pending_ = true;
        int dev = 0;
        HIP_CHECK(hipGetDevice(&dev));
        const std::string dir = cfg_.checkpoint_dir;
        std::vector<int> rk;
        for (auto& R : ranks_) rk.push_back(R.topo.rank);
        hipEvent_t ev = ev_ckpt_;
        ckpt_thread_ = std::thread([=]() {
            try {
                (void)hipSetDevice(dev);
                HIP_CHECK(hipEventSynchronize(ev));
                for (size_t q = 0; q < hs.size(); ++q) {
                    write_checkpoint(dir, hs[q], lps[q], lcs[q], a, r);
                    prune_checkpoints(dir, hs[q], n, 2);
                    log_msg(LogLevel::Info, "rank ", rk[q], ": checkpoint after layer ", n, " -> ",
                            checkpoint_path(dir, rk[q], n));
                }
            } catch (const std::exception& e) {
                ckpt_error_ = e.what();
            }
        });
    }

    // the compute stream is about to write `level`: keep the checkpoint copy consistent
    void guard_checkpoint_level(int level, hipStream_t s) {
        if (ckpt_pending_ && (level == ckpt_levels_[0] || level == ckpt_levels_[1])) {
            HIP_CHECK(hipStreamWaitEvent(s, ev_ckpt_, 0));
            ckpt_pending_ = false;
        }
    }

    void finish_checkpoint() {
        if (ckpt_thread_.joinable()) ckpt_thread_.join();
        ckpt_pending_ = false;
        if (!ckpt_error_.empty()) {
            std::string e = ckpt_error_;
            ckpt_error_.clear();
            throw Error("checkpoint write failed: " + e);
        }
    }

    void copy_plane(DevRank<T>& R, int level, int src, int dst) {
        HIP_CHECK(hipMemcpy(plane(R, level, dst), plane(R, level, src), R.gv.si * sizeof(T),
                            hipMemcpyDeviceToDevice));
    }

    int load_checkpoints() {
        HIP_CHECK(hipDeviceSynchronize());
        std::vector<CheckpointHeader> ex;
        for (auto& R : ranks_) ex.push_back(make_header(cfg_, R.topo, 0, sizeof(T)));
        const int n = agree_resume_layer(cfg_.resume_dir, ex, ext_);  // same layer on every rank
        plan_slots(n + 1);  // the resumed run's own schedule from layer n + 1
        for (auto& R : ranks_) {
            const int lp = lvl(n - 1), lc = lvl(n);
            std::vector<T> prev(R.elems, T(0)), cur(R.elems, T(0));
            CheckpointHeader h = make_header(cfg_, R.topo, n, sizeof(T));
            read_checkpoint(cfg_.resume_dir, h, host_level(R, prev, lp), host_level(R, cur, lc),
                            ckpt_abs_, ckpt_rel_);
            HIP_CHECK(hipMemcpy(R.alloc[lp], prev.data(), R.elems * sizeof(T), hipMemcpyHostToDevice));
            HIP_CHECK(hipMemcpy(R.alloc[lc], cur.data(), R.elems * sizeof(T), hipMemcpyHostToDevice));
            if (R.plan.self_x) {  // periodic self-wrap ghosts of both levels
                const Wrap& wc = wrap_depth(R, G_);        // u^n is the next A
                const Wrap& wp = wrap_depth(R, std::max(1, G_ - 1));
                for (int q = 0; q < kMaxWrap; ++q)
                    if (wc.src[q] >= 1) copy_plane(R, lc, wc.src[q], wc.dst[q]);
                for (int q = 0; q < kMaxWrap; ++q)
                    if (wp.src[q] >= 1) copy_plane(R, lp, wp.src[q], wp.dst[q]);
            }
        }
        // device-to-device hipMemcpy need not block the host, and the sweeps run on
        // non-blocking streams: the restored levels must be complete before the first one
        HIP_CHECK(hipDeviceSynchronize());
        if (tb_ && tb_halo(ranks_[0])) {
            exchange_tb(n, s_comp_);  // A level = u^n (2 deep + alias), B level = u^{n-1}
        } else {
            for (int l : {n - 1, n}) {
                for (auto& R : ranks_) pack_faces(R, l, s_comp_, true);
                exchange(l, s_comp_);
            }
        }
        HIP_CHECK(hipEventRecord(ev_halo_, s_comp_));
        return n;
    }

    Config cfg_;
    Transport* ext_;
    Problem prob_;
    FaultSpec fault_;
    KernelVariant kind_, naive_;
    bool tb_ = false;   // temporal blocking (2 layers per sweep)
    int tb_rows_ = 2;
    int tb_waves_ = 4;
    int tb_occ_ = 0;
    int tb_nwk_ = 1;    // tb2 waves along k (tile width 64 * tb_nwk_)
    int tbd_ = 1;       // layers per sweep (1, 2, 3 or 4)
    bool tbn_ = false;  // deep sweeps through k_tbn (tb4; "tbn3": the depth-generic kernel at 3)
    hipGraphExec_t gexec_ = nullptr;  // captured IC + time loop (graph_eligible())
    const char* order_enqueued_ = "none";  // overlap order of the last enqueue / captured graph
    bool graph_failed_ = false;
    int G_ = 1;         // ghost depth
    int L_ = 3;         // time levels kept
    std::vector<int> slot_;          // level buffer of layer n at [n + 1] (plan_slots)
    std::vector<char> first_write_;  // layer n is the first write of its buffer in the solve
    bool overlap_ = false;
    bool overlap_auto_ = false;   // --overlap auto with a remote halo
    bool shells_first_ = overlap_shells_first();  // deep sweeps: shells, then exchange || interior
    // overlap auto trial solves: on (shells beside), off, on (shells first), twice each
    static constexpr int kOverlapTrials = kOverlapTrialSolves;
    int trials_done_ = 0;         // overlap auto trials run
    int solves_ = 0;              // solves of this session
    double trial_ms_[kOverlapTrials] = {};
    // best (smallest) trial time of an arm (0 on beside, 1 off, 2 on shells first) so far, 0 before
    // its first trial
    double best_trial(int arm) const {
        double b = 0;
        for (int q = arm; q < trials_done_; q += 3) b = b > 0 ? std::min(b, trial_ms_[q]) : trial_ms_[q];
        return b;
    }
    bool xself_ = false;  // --x-self-transport
    bool direct_ = true;  // --halo direct: single-round deep-halo plan (build_tb_direct)
    static constexpr size_t kMirrorSlots = 2048;
    std::unique_ptr<RcclTransport> mirror_;  // --rccl-mirror: 1-rank communicator
    void* mirror_buf_ = nullptr;
    size_t mirror_bytes_ = 0;
    u64* mirror_res_ = nullptr;              // per message kind: differing words, first word
    std::vector<std::string> mirror_keys_;
    std::map<i64, int> mirror_index_;
    long mirror_msgs_ = 0;                   // messages mirrored (all solves)
    bool selftest_ = false;  // inside halo_self_test()
    int halo_checked_ = 0;   // messages verified by the init-time halo self-test
    int world_ = 1;
    std::vector<int> local_;
    std::vector<DevRank<T>> ranks_;
    std::vector<double> ct_;
    std::vector<u64> host_err_;
    std::thread ckpt_thread_;       // background checkpoint writer
    std::string ckpt_error_;
    hipStream_t s_ckpt_ = nullptr;  // device -> pinned host copies of checkpointed levels
    hipEvent_t ev_ckpt_ = nullptr;
    bool ckpt_pending_ = false;
    int ckpt_levels_[2] = {-1, -1};
    std::vector<double> ckpt_abs_, ckpt_rel_;
    hipStream_t s_comp_ = nullptr, s_comm_ = nullptr;
    hipStream_t s_comp_full_ = nullptr, s_comp_cu_ = nullptr;  // s_comp_ is one of them
    int comm_cus_ = 0;  // CUs the masked compute stream leaves to the halo stream
    hipEvent_t ev_start_ = nullptr, ev_end_ = nullptr, ev_layer_ = nullptr, ev_halo_ = nullptr;
    hipEvent_t ev_shell_ = nullptr;  // shells of the current sweep done (comm stream)
    u64* ts_host_ = nullptr;       // timer-mark stamps (pinned, coherent host memory)
    u64* ts_dev_ = nullptr;        // its device address
    size_t ts_cap_ = 0;
    double clock_khz_ = 1e5;       // device wall-clock rate
    std::vector<int> tslot_;       // slot of each mark, in record order
    size_t tn_ = 0;                // marks recorded for the current solve
    size_t graph_tn_ = 0;          // marks captured in the hipGraph
    size_t prog_seen_ = 0;         // marks known complete (watchdog progress)
    bool fine_ = false;            // per-sweep marks (halos move, or --profile)
    bool capturing_ = false;       // inside the hipGraph capture: marks are stamp kernels
    bool stamped_ = false;         // this solve's marks are stamps (graph replay), not events
    bool no_timers_ = false;       // WAVE3D_NO_TIMERS=1: fine marks off (timer-cost A/B)
    std::vector<hipEvent_t> ev_marks_;  // timing events of the direct-launch marks
    double init_ms_ = 0;
};

template <class T>
class HipSession : public Session {
public:
    HipSession(const Config& c, Transport* ext) : s_(c, ext) { s_.init(); }
    RunResult solve() override { return s_.solve_one(); }
    double init_ms() const override { return s_.init_ms(); }
    std::vector<FieldBlock> field(int layer) override { return s_.field(layer); }

private:
    HipSolver<T> s_;
};

}  // namespace

std::unique_ptr<Session> make_hip_session(const Config& c, Transport* external) {
    if (c.device >= 0) HIP_CHECK(hipSetDevice(c.device));
    if (c.dtype == DType::F64) return std::make_unique<HipSession<double>>(c, external);
    return std::make_unique<HipSession<float>>(c, external);
}

RunResult run_hip(const Config& c, Transport* external) {
    auto s = make_hip_session(c, external);
    return run_session(*s, c);
}

}  // namespace wave3d
