#include "halo.hpp"

#include <atomic>
#include <chrono>
#include <mutex>
#include <cstdlib>
#include <thread>

namespace wave3d {

double watchdog_limit_s() {
    static const double limit = [] {
        const char* e = std::getenv("WAVE3D_WATCHDOG_S");
        return e ? std::atof(e) : 120.0;
    }();
    return limit;
}

namespace {
std::mutex g_abort_mu;
std::atomic<bool> g_abort{false};
std::string g_abort_why;
}  // namespace

void raise_job_abort(const std::string& why) {
    std::lock_guard<std::mutex> g(g_abort_mu);
    if (!g_abort.load()) g_abort_why = why;
    g_abort.store(true);
}

bool job_aborted(std::string* why) {
    if (!g_abort.load(std::memory_order_relaxed)) return false;
    if (why) {
        std::lock_guard<std::mutex> g(g_abort_mu);
        *why = g_abort_why;
    }
    return true;
}

void clear_job_abort() {
    std::lock_guard<std::mutex> g(g_abort_mu);
    g_abort.store(false);
    g_abort_why.clear();
}

std::vector<std::string> run_rank_threads(int n, const std::function<void(int)>& body) {
    clear_job_abort();
    std::vector<std::string> errs(n);
    std::vector<std::thread> th;
    for (int r = 0; r < n; ++r)
        th.emplace_back([&, r] {
            try {
                body(r);
            } catch (const std::exception& e) {
                errs[r] = e.what();
                raise_job_abort("rank " + std::to_string(r) + ": " + e.what());
            }
        });
    for (auto& t : th) t.join();
    clear_job_abort();
    return errs;
}

void watch_until(const std::function<bool()>& done, const std::function<std::string()>& async_error,
                 const std::function<long()>* progress, double limit_s,
                 const std::function<void()>& abort, const std::string& what) {
    using clk = std::chrono::steady_clock;
    auto t0 = clk::now();
    long seen = progress ? (*progress)() : 0;
    for (int spin = 0;; ++spin) {
        if (done()) return;
        std::string why;
        if (job_aborted(&why)) {
            abort();
            throw Error(what + " aborted: another rank failed (" + why + ")");
        }
        const std::string err = async_error();
        const auto now = clk::now();
        if (progress && (spin & 63) == 0) {
            const long p = (*progress)();
            if (p != seen) seen = p, t0 = now;  // the device moved on: restart the clock
        }
        const double el = std::chrono::duration<double>(now - t0).count();
        if (!err.empty() || (limit_s > 0 && el > limit_s)) {
            abort();
            throw Error(!err.empty() ? what + " async error: " + err
                                     : what + " watchdog: no progress for " + std::to_string(int(el)) +
                                           " s (WAVE3D_WATCHDOG_S), communicator aborted");
        }
        if (spin > 1000) std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

HaloPlan make_halo_plan(const Topology& t, i64 x_plane, int row, bool self_msg) {
    HaloPlan p;
    const i64 X = t.ext[0], Y = t.ext[1];
    const i64 count[3] = {x_plane, X * row, X * (Y + 2)};
    p.self_x = t.nbr[0][0] == t.rank && !self_msg;
    for (int a = 0; a < 3; ++a) {
        if (a == 0 && p.self_x) continue;
        // travelling +a: send from the plus face to nbr[a][1] (tag 2a+1)
        if (t.nbr[a][1] >= 0) p.sends.push_back({a, 1, t.nbr[a][1], 2 * a + 1, count[a]});
        // travelling -a: send from the minus face to nbr[a][0] (tag 2a+2)
        if (t.nbr[a][0] >= 0) p.sends.push_back({a, 0, t.nbr[a][0], 2 * a + 2, count[a]});
        // receive the +a traveller from the minus neighbour into the minus ghost
        if (t.nbr[a][0] >= 0) p.recvs.push_back({a, 0, t.nbr[a][0], 2 * a + 1, count[a]});
        // receive the -a traveller from the plus neighbour into the plus ghost
        if (t.nbr[a][1] >= 0) p.recvs.push_back({a, 1, t.nbr[a][1], 2 * a + 2, count[a]});
    }
    return p;
}

}  // namespace wave3d
