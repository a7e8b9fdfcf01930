#include "rccl_transport.hpp"
#include "trace.hpp"

#include <arpa/inet.h>
#include <hip/hip_runtime.h>
#include <netdb.h>
#include <netinet/in.h>
#include <rccl/rccl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace wave3d {

#define NCCL_CHECK(x)                                                                     \
    do {                                                                                  \
        ncclResult_t r_ = (x);                                                            \
        if (r_ != ncclSuccess)                                                            \
            throw ::wave3d::Error(std::string("RCCL error ") + ncclGetErrorString(r_) +  \
                                  " at " __FILE__ ":" + std::to_string(__LINE__));        \
    } while (0)
#define HIP_CHECK_T(x)                                                                 \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess)                                                          \
            throw ::wave3d::Error(std::string("HIP error ") + hipGetErrorString(e_) + \
                                  " at " __FILE__ ":" + std::to_string(__LINE__));     \
    } while (0)

static_assert(sizeof(ncclUniqueId) == kRcclIdBytes, "unexpected ncclUniqueId size");

std::string rccl_unique_id() {
    ncclUniqueId id;
    NCCL_CHECK(ncclGetUniqueId(&id));
    return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

struct RcclTransport::Impl {
    ncclComm_t comm = nullptr;
    hipStream_t side = nullptr;   // for host-value collectives
    double* scratch = nullptr;    // device scratch for allreduce_max_host
    size_t scratch_n = 0;
    int max_ctas = 0;             // configured CTA budget (0 = RCCL default)
};

int RcclTransport::max_ctas() const { return impl_->max_ctas; }

namespace {
int env_int(const char* k, int dflt) {
    const char* v = std::getenv(k);
    return v && *v ? std::atoi(v) : dflt;
}
}  // namespace

int rccl_max_ctas(const std::string& overlap_mode) {
    const char* e = std::getenv("WAVE3D_RCCL_MAX_CTAS");
    if (e && *e) return std::max(0, std::atoi(e));
    return overlap_mode == "on" ? kRcclOverlapMaxCtas : 0;
}

// The communicator is non-blocking (config.blocking = 0): initialisation and every enqueue
// may return ncclInProgress, and settle() polls ncclCommGetAsyncError under the watchdog, so a
// peer that never arrives at ncclCommInitRank, or a failed rank thread of this process (job
// abort flag), ends the wait with an error instead of a hang. The CTA budget (maxCTAs,
// WAVE3D_RCCL_MAX_CTAS) caps how many CUs the halo kernels take from the interior sweep
// that runs concurrently: a face of a few MB needs a few channels, not RCCL's default.
RcclTransport::RcclTransport(int rank, int size, const std::string& uid, int device, int max_ctas)
    : impl_(new Impl), rank_(rank), size_(size) {
    W3D_REQUIRE(uid.size() == sizeof(ncclUniqueId), "bad RCCL unique id");
    HIP_CHECK_T(hipSetDevice(device));
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    const int mx = max_ctas >= 0 ? max_ctas : rccl_max_ctas("auto");
    if (mx > 0) {
        cfg.maxCTAs = mx;
        cfg.minCTAs = std::min(mx, env_int("WAVE3D_RCCL_MIN_CTAS", 1));
    }
    impl_->max_ctas = mx;
    const ncclResult_t r = ncclCommInitRankConfig(&impl_->comm, size, id, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
        if (impl_->comm) (void)ncclCommAbort(impl_->comm);
        impl_->comm = nullptr;
        NCCL_CHECK(r);
    }
    settle(r, init_limit_s(), "RCCL init");
    HIP_CHECK_T(hipStreamCreateWithFlags(&impl_->side, hipStreamNonBlocking));
}

double RcclTransport::init_limit_s() {
    const char* e = std::getenv("WAVE3D_RCCL_INIT_S");
    return e ? std::atof(e) : 120.0;
}

// ncclInProgress: poll until the communicator's state leaves it (watchdog, job abort)
void RcclTransport::settle(int r0, double limit_s, const char* what) {
    ncclResult_t r = ncclResult_t(r0);
    if (r == ncclSuccess) return;
    if (r != ncclInProgress) NCCL_CHECK(r);
    W3D_REQUIRE(impl_->comm, "RCCL communicator missing");
    ncclResult_t st = ncclInProgress;
    watch_until(
        [&] {
            NCCL_CHECK(ncclCommGetAsyncError(impl_->comm, &st));
            return st != ncclInProgress;
        },
        [&] { return st == ncclSuccess || st == ncclInProgress ? std::string() : std::string(ncclGetErrorString(st)); },
        nullptr, limit_s,
        [&] {
            (void)ncclCommAbort(impl_->comm);
            impl_->comm = nullptr;
        },
        what);
    if (st != ncclSuccess) {
        (void)ncclCommAbort(impl_->comm);
        impl_->comm = nullptr;
        throw Error(std::string(what) + " failed: " + ncclGetErrorString(st));
    }
}

RcclTransport::~RcclTransport() {
    if (impl_->scratch) (void)hipFree(impl_->scratch);
    if (impl_->side) (void)hipStreamDestroy(impl_->side);
    if (!impl_->comm) return;
    // non-blocking communicator: finalize (flushes outstanding work), wait for it, destroy;
    // any failure or a stuck finalize falls back to abort
    ncclResult_t r = ncclCommFinalize(impl_->comm), st = r;
    const auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress || r == ncclSuccess) {
        if (ncclCommGetAsyncError(impl_->comm, &st) != ncclSuccess || st != ncclInProgress) break;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) break;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    if ((r == ncclSuccess || r == ncclInProgress) && st == ncclSuccess) (void)ncclCommDestroy(impl_->comm);
    else (void)ncclCommAbort(impl_->comm);
}

void RcclTransport::exchange(const std::vector<Message>& sends, const std::vector<Message>& recvs,
                             void* stream) {
    TraceRange tr("rccl.exchange");
    hipStream_t s = static_cast<hipStream_t>(stream);
    W3D_REQUIRE(impl_->comm, "RCCL communicator was aborted");
    NCCL_CHECK(ncclGroupStart());
    for (const auto& m : sends)
        NCCL_CHECK(ncclSend(m.ptr, m.bytes, ncclChar, m.peer, impl_->comm, s));
    for (const auto& m : recvs)
        NCCL_CHECK(ncclRecv(m.ptr, m.bytes, ncclChar, m.peer, impl_->comm, s));
    settle(ncclGroupEnd(), watchdog_limit_s(), "RCCL group");
}

int RcclTransport::comm_size() const {
    int n = 0;
    if (!impl_->comm) return 0;
    NCCL_CHECK(ncclCommCount(impl_->comm, &n));
    return n;
}

void RcclTransport::allreduce_max_u64(u64* data, size_t n, void* stream) {
    W3D_REQUIRE(impl_->comm, "RCCL communicator was aborted");
    settle(ncclAllReduce(data, data, n, ncclUint64, ncclMax, impl_->comm, static_cast<hipStream_t>(stream)),
           watchdog_limit_s(), "RCCL allreduce");
}

void RcclTransport::allreduce_max_host(double* data, size_t n) {
    if (impl_->scratch_n < n) {
        if (impl_->scratch) HIP_CHECK_T(hipFree(impl_->scratch));
        HIP_CHECK_T(hipMalloc(&impl_->scratch, n * sizeof(double)));
        impl_->scratch_n = n;
    }
    HIP_CHECK_T(hipMemcpyAsync(impl_->scratch, data, n * sizeof(double), hipMemcpyHostToDevice,
                               impl_->side));
    W3D_REQUIRE(impl_->comm, "RCCL communicator was aborted");
    settle(ncclAllReduce(impl_->scratch, impl_->scratch, n, ncclFloat64, ncclMax, impl_->comm, impl_->side),
           host_collective_limit_s(), "RCCL allreduce");
    HIP_CHECK_T(hipMemcpyAsync(data, impl_->scratch, n * sizeof(double), hipMemcpyDeviceToHost,
                               impl_->side));
    wait_stream_limit(impl_->side, nullptr, host_collective_limit_s());
}

void RcclTransport::barrier() {
    double v = 0;
    allreduce_max_host(&v, 1);
}

void RcclTransport::check_async() const {
    W3D_REQUIRE(impl_->comm, "RCCL communicator was aborted");
    ncclResult_t st = ncclSuccess;
    NCCL_CHECK(ncclCommGetAsyncError(impl_->comm, &st));
    if (st != ncclSuccess) throw Error(std::string("RCCL async error: ") + ncclGetErrorString(st));
}

bool RcclTransport::wait_stream(void* stream, const std::function<long()>* progress) {
    wait_stream_limit(stream, progress, watchdog_limit_s());
    return true;
}

// Host-level collectives (timers, the per-checkpoint error reduction, barriers) wait for the
// slowest rank's host work — e.g. its checkpoint writer finishing an fsync of many GB — not for
// device progress: they get the longer WAVE3D_HOST_WATCHDOG_S limit (default 1800 s).
double host_collective_limit_s() {
    static const double limit = [] {
        const char* e = std::getenv("WAVE3D_HOST_WATCHDOG_S");
        return e ? std::atof(e) : std::max(1800.0, watchdog_limit_s());
    }();
    return limit;
}

void RcclTransport::wait_stream_limit(void* stream, const std::function<long()>* progress, double limit_s) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    watch_until(
        [&] {
            const hipError_t q = hipStreamQuery(s);
            if (q != hipErrorNotReady) HIP_CHECK_T(q);
            return q == hipSuccess;
        },
        [&] {
            ncclResult_t st = ncclSuccess;
            if (!impl_->comm) return std::string("communicator aborted");
            NCCL_CHECK(ncclCommGetAsyncError(impl_->comm, &st));
            return st == ncclSuccess || st == ncclInProgress ? std::string() : std::string(ncclGetErrorString(st));
        },
        progress, limit_s,
        [&] {
            if (impl_->comm) (void)ncclCommAbort(impl_->comm);
            impl_->comm = nullptr;
        },
        "RCCL");
}

// ---- TCP rendezvous -------------------------------------------------------------------
std::string tcp_share_unique_id(int rank, int size, const std::string& addr, int port) {
    if (size == 1) return rccl_unique_id();
    if (rank == 0) {
        std::string id = rccl_unique_id();
        int fd = socket(AF_INET, SOCK_STREAM, 0);
        W3D_REQUIRE(fd >= 0, "socket() failed");
        int one = 1;
        setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_port = htons(uint16_t(port));
        a.sin_addr.s_addr = htonl(INADDR_ANY);
        W3D_REQUIRE(bind(fd, (sockaddr*)&a, sizeof(a)) == 0, "bind() failed on port " + std::to_string(port));
        W3D_REQUIRE(listen(fd, size) == 0, "listen() failed");
        for (int q = 1; q < size; ++q) {
            int c = accept(fd, nullptr, nullptr);
            W3D_REQUIRE(c >= 0, "accept() failed");
            size_t off = 0;
            while (off < id.size()) {
                ssize_t w = send(c, id.data() + off, id.size() - off, 0);
                W3D_REQUIRE(w > 0, "send() failed");
                off += size_t(w);
            }
            close(c);
        }
        close(fd);
        return id;
    }
    std::string id(kRcclIdBytes, '\0');
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    W3D_REQUIRE(getaddrinfo(addr.c_str(), std::to_string(port).c_str(), &hints, &res) == 0,
                "cannot resolve " + addr);
    int fd = -1;
    for (int attempt = 0; attempt < 600; ++attempt) {  // up to ~60 s for rank 0 to listen
        fd = socket(AF_INET, SOCK_STREAM, 0);
        if (connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
        close(fd);
        fd = -1;
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
    freeaddrinfo(res);
    W3D_REQUIRE(fd >= 0, "cannot connect to rank 0 at " + addr + ":" + std::to_string(port));
    size_t off = 0;
    while (off < id.size()) {
        ssize_t r = recv(fd, &id[off], id.size() - off, 0);
        W3D_REQUIRE(r > 0, "recv() failed");
        off += size_t(r);
    }
    close(fd);
    return id;
}

}  // namespace wave3d
