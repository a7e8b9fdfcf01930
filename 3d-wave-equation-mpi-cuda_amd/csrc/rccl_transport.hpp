// RCCL point-to-point halo transport over xGMI.
//
// Replaces the reference's host-staged blocking MPI_Sendrecv chain (cuda_sol.cpp:230-312):
// every face of one exchange is posted inside one ncclGroupStart/End on the caller's
// stream, straight from device memory — no pinned staging, no host sync. The final error
// reduction is one ncclAllReduce(ncclMax) on the order-preserving u64 keys.
#pragma once

#include <memory>
#include <string>

#include "halo.hpp"

namespace wave3d {

constexpr int kRcclIdBytes = 128;  // sizeof(ncclUniqueId)

std::string rccl_unique_id();  // 128 raw bytes

// CTA budget (ncclConfig_t::maxCTAs) of the halo communicator, fixed when it is created:
// WAVE3D_RCCL_MAX_CTAS when set (<= 0: RCCL's own budget), else by the run's overlap mode —
//   off, auto -> 0: RCCL's own budget. Nothing runs beside the exchange with overlap off, so a
//                cap could only slow it (a 2x2x2 rank posts 7 peers' messages in one group);
//                auto keeps it too: the budget is fixed for the communicator's life, and on 2x2x2
//                blocks the overlap-off arm is the expected winner of the auto trials (the shell
//                tax outweighs the hidden exchange, profiles/overlap_model_r4.txt).
//   on        -> kRcclOverlapMaxCtas: the interior sweep runs concurrently on the compute
//                stream, and each halo CTA holds a CU the sweep's workgroups then wait for.
// One MI355X cannot tell the budgets apart (profiles/rccl_ctas_r3.txt: a 1-rank self-send
// costs the same at 1..8 CTAs and at the default); the JSON records the budget of every run.
constexpr int kRcclOverlapMaxCtas = 8;
int rccl_max_ctas(const std::string& overlap_mode = "auto");
// Watchdog limit of host-level collectives (WAVE3D_HOST_WATCHDOG_S, default 1800 s)
double host_collective_limit_s();

class RcclTransport : public Transport {
public:
    // Must be called with `device` as the current device on this thread.
    // max_ctas < 0: rccl_max_ctas("auto")
    RcclTransport(int rank, int size, const std::string& unique_id, int device, int max_ctas = -1);
    ~RcclTransport() override;
    std::string name() const override { return "rccl"; }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    bool device() const override { return true; }
    int comm_size() const override;  // ncclCommCount
    void exchange(const std::vector<Message>& sends, const std::vector<Message>& recvs,
                  void* stream) override;
    void allreduce_max_u64(u64* data, size_t n, void* stream) override;
    void allreduce_max_host(double* data, size_t n) override;
    void barrier() override;
    // Async-error watchdog: throws if the communicator reported an error.
    void check_async() const;
    // Polls the stream and the communicator's async error; aborts the communicator and throws
    // after WAVE3D_WATCHDOG_S seconds (default 120, below the benchmark driver's timeout)
    // without progress — measured from the last growth of `progress` when given — so a dead
    // peer ends the run with an error instead of a hang.
    bool wait_stream(void* stream, const std::function<long()>* progress = nullptr) override;
    int max_ctas() const;  // CTA budget the communicator was created with (0 = RCCL default)
    int cta_budget() const override { return max_ctas(); }
    static double init_limit_s();  // WAVE3D_RCCL_INIT_S, default 120 s

private:
    void settle(int nccl_result, double limit_s, const char* what);
    void wait_stream_limit(void* stream, const std::function<long()>* progress, double limit_s);
    struct Impl;
    std::unique_ptr<Impl> impl_;
    int rank_, size_;
};

// Minimal TCP rendezvous for the standalone program (torchrun-style env: RANK, WORLD_SIZE,
// MASTER_ADDR, MASTER_PORT): rank 0 generates the RCCL id and serves it to the others.
std::string tcp_share_unique_id(int rank, int size, const std::string& addr, int port);

}  // namespace wave3d
