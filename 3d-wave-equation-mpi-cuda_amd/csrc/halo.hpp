// Face-halo exchange plan and the transport interface (P6).
//
// Each rank sends the owned plane next to each existing neighbour and receives into the
// ghost plane on that side. Tags follow the reference (mpi_new.cpp:201-238): a message
// travelling towards +axis carries tag 2a+1, towards -axis tag 2a+2. Sends and receives
// are listed in one canonical order (axis, then tag), so transports without tags (RCCL)
// match messages by per-peer FIFO order.
//
// Payloads are contiguous:
//   x: the whole padded (j,k) plane — already contiguous in the [i][j][k] layout, sent and
//      received in place, no pack/unpack;
//   y: rows i=1..X of the (i,k) face, k over the full padded row -> X*pitch elements;
//   z: i=1..X, j=0..Y+1 of the (i,j) face                       -> X*(Y+2) elements.
// A rank that is its own x-neighbour (dims[0] == 1) wraps locally instead of messaging,
// unless `self_msg` is set: then the wrap is two messages to this rank (the same plan a
// rank of a dims[0] >= 2 ring has, both ends being itself).
#pragma once

#include <functional>
#include <string>
#include <vector>

#include "common.hpp"
#include "topology.hpp"

namespace wave3d {

struct FaceMsg {
    int axis = 0;
    int side = 0;   // 0 = minus face, 1 = plus face of *this* rank
    int peer = -1;
    int tag = 0;
    i64 count = 0;  // elements
};

struct HaloPlan {
    std::vector<FaceMsg> sends;  // canonical order
    std::vector<FaceMsg> recvs;  // canonical order
    bool self_x = false;         // periodic x neighbour is this rank
};

// `x_plane` = elements of one padded (j,k) plane, `row` = elements of a y-face row.
HaloPlan make_halo_plan(const Topology& t, i64 x_plane, int row, bool self_msg = false);

// Description of one message for a transport.
struct Message {
    int peer = -1;
    int tag = 0;
    void* ptr = nullptr;
    size_t bytes = 0;
};

// Watchdog loop shared by the device transports: polls `done` until it returns
// true; `async_error` returns a non-empty message when the communicator failed; `progress`
// (optional) grows while the device makes progress, and the clock restarts whenever it does.
// On an error or `limit_s` seconds (> 0) without progress it calls `abort` and throws
// wave3d::Error naming the cause. Host-only (unit-tested on the CPU).
void watch_until(const std::function<bool()>& done, const std::function<std::string()>& async_error,
                 const std::function<long()>* progress, double limit_s,
                 const std::function<void()>& abort, const std::string& what);
// WAVE3D_WATCHDOG_S, default 120 s (below the benchmark driver's timeout)
double watchdog_limit_s();

// Job-wide abort flag of one process (thread-per-GPU ranks): the first rank thread that fails
// raises it, and every watch_until() loop of the other ranks — waits on RCCL streams and
// communicator initialisation — aborts its communicator and throws within a poll interval
// instead of sitting in a collective until the watchdog limit.
void raise_job_abort(const std::string& why);
bool job_aborted(std::string* why = nullptr);
void clear_job_abort();  // before a new job in the same process (tests)

// Runs body(r) for r = 0..n-1 on n threads (thread-per-GPU ranks) and returns each rank's
// error message ("" = success). A rank that throws raises the job abort flag, so ranks blocked
// in watch_until() on it fail within a poll interval. The flag is cleared before and after.
std::vector<std::string> run_rank_threads(int n, const std::function<void(int)>& body);

// A transport moves the messages of one exchange. Device transports order the operation
// on `stream` (a hipStream_t) and return without host synchronisation; host transports
// complete before returning.
class Transport {
public:
    virtual ~Transport() = default;
    virtual std::string name() const = 0;
    virtual int rank() const = 0;
    virtual int size() const = 0;
    virtual bool device() const = 0;
    // Ranks of the underlying communicator as the library itself reports them (RCCL:
    // ncclCommCount), so a run can prove which world the halos travelled in.
    virtual int comm_size() const { return size(); }
    // CTA budget of a GPU collective library's communicator (RCCL maxCTAs; 0 = the library's
    // own), -1 when the transport has none
    virtual int cta_budget() const { return -1; }
    virtual void exchange(const std::vector<Message>& sends, const std::vector<Message>& recvs,
                          void* stream) = 0;
    // In-place max over ranks of n order-preserving error keys (see encode_max_key).
    virtual void allreduce_max_u64(u64* data, size_t n, void* stream) = 0;
    // Host doubles, max over ranks (timers).
    virtual void allreduce_max_host(double* data, size_t n) = 0;
    virtual void barrier() = 0;
    // Wait for `stream` to drain. A transport with asynchronous failure modes (RCCL) polls
    // its error state and enforces a watchdog timeout here instead of blocking forever;
    // returns false when the caller should simply synchronise the stream itself.
    // `progress` (optional) returns a count that grows while the device makes progress (e.g.
    // completed per-sweep events): the watchdog measures time since it last grew.
    virtual bool wait_stream(void* /*stream*/, const std::function<long()>* /*progress*/ = nullptr) {
        return false;
    }
};

}  // namespace wave3d
