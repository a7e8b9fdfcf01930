// wave3d — MI355X program with the reference CLI (cuda_sol.cpp:447-597):
//     wave3d N Np Lx Ly Lz [T] [timesteps] [options]
// Launch modes:
//  * torchrun-style multi-process (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT
//    in the environment): one process per GPU, RCCL bootstrap over a small TCP rendezvous;
//  * single process, Np > 1: one host thread per GPU (Np GPUs of this node);
//  * single process, Np == 1: one GPU, or `--ranks P` simulated ranks on it.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <iostream>
#include <mutex>
#include <thread>

#include "cli_common.hpp"
#include "rccl_transport.hpp"
#include "sizing.hpp"
#include "solver.hpp"

using namespace wave3d;

static int env_int(const char* k, int dflt) {
    const char* v = std::getenv(k);
    return v ? std::atoi(v) : dflt;
}

int main(int argc, char** argv) {
    try {
        Config c = parse_cli(argc, argv);
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
            std::cerr << "wave3d: no HIP device found (use wave3d_cpu for the OpenMP backend)\n";
            return 1;
        }
        const int world = env_int("WORLD_SIZE", 1);
        if (c.fill_hbm > 0) {
            // size the grid to the device: every rank of the job has the
            // same HBM; simulated ranks share one device
            const int dev = c.device >= 0 ? c.device : (world > 1 ? env_int("LOCAL_RANK", 0) % ndev : 0);
            size_t freeb = 0, total = 0;
            if (hipSetDevice(dev) != hipSuccess || hipMemGetInfo(&freeb, &total) != hipSuccess)
                throw Error("hipMemGetInfo failed");
            const int nr = world > 1 ? world : (c.Np > 1 && c.ranks == 0 ? c.Np : std::max(1, c.ranks));
            const double budget = c.fill_hbm * double(total) / (world > 1 || c.ranks == 0 ? 1 : c.ranks);
            c.N = fill_hbm_N(c, nr, budget);
            if (!c.quiet && env_int("RANK", 0) == 0)
                std::cout << "fill-hbm: N = " << c.N << " (" << device_bytes_per_rank(c, nr) / 1e9
                          << " GB per GPU of " << total / 1e9 << " GB)" << std::endl;
        }
        Problem p = Problem::from_config(c);
        if (world > 1) {
            const int rank = env_int("RANK", 0);
            const int local = env_int("LOCAL_RANK", rank);
            if (!courant_check(c, p, rank == 0)) return 2;
            c.device = c.device >= 0 ? c.device : local % ndev;
            if (hipSetDevice(c.device) != hipSuccess) throw Error("hipSetDevice failed");
            const char* addr = std::getenv("MASTER_ADDR");
            int port = env_int("WAVE3D_BOOT_PORT", env_int("MASTER_PORT", 29500) + 17);
            std::string id = tcp_share_unique_id(rank, world, addr ? addr : "127.0.0.1", port);
            if (!c.quiet)
                std::cout << "Process " << rank << " local rank = " << local << " local size = "
                          << env_int("LOCAL_WORLD_SIZE", world) << " hostname = " << host_name()
                          << " device = " << c.device << std::endl;
            RcclTransport tr(rank, world, id, c.device, rccl_max_ctas(overlap_mode(c)));
            RunResult r = run_hip(c, &tr);
            finish(c, r, rank == 0);
            return r.aborted ? 3 : 0;
        }
        if (!courant_check(c, p, true)) return 2;
        if (!c.quiet) std::cout << "number of devices on node " << host_name() << ": " << ndev << std::endl;
        if (c.Np > 1 && c.ranks == 0) {
            // one host thread per GPU, RCCL between them
            W3D_REQUIRE(c.Np <= ndev, "Np = " + std::to_string(c.Np) + " GPUs requested, " +
                                          std::to_string(ndev) +
                                          " present (use --ranks P to simulate ranks on one GPU)");
            std::string id = rccl_unique_id();
            std::vector<RunResult> res(c.Np);
            std::mutex io;
            // a failing rank thread raises the job abort flag: the others' RCCL waits return
            // at once (run_rank_threads, halo.cpp) instead of waiting for the watchdog
            const std::vector<std::string> errs = run_rank_threads(c.Np, [&](int r) {
                Config cr = c;
                cr.device = r;
                if (hipSetDevice(r) != hipSuccess) throw Error("hipSetDevice failed");
                if (!c.quiet) {
                    std::lock_guard<std::mutex> g(io);
                    std::cout << "Process " << r << " local rank = " << r << " local size = " << c.Np
                              << " hostname = " << host_name() << " device = " << r << std::endl;
                }
                RcclTransport tr(r, c.Np, id, r, rccl_max_ctas(overlap_mode(c)));
                res[r] = run_hip(cr, &tr);
            });
            for (int r = 0; r < c.Np; ++r)  // the first failure is the cause, the rest followed it
                if (!errs[r].empty() && errs[r].find("another rank failed") == std::string::npos)
                    throw Error("rank " + std::to_string(r) + ": " + errs[r]);
            for (int r = 0; r < c.Np; ++r)
                if (!errs[r].empty()) throw Error("rank " + std::to_string(r) + ": " + errs[r]);
            finish(c, res[0], true);
            return res[0].aborted ? 3 : 0;
        }
        if (!c.quiet) {
            int P = std::max(1, c.ranks);
            for (int r = 0; r < P; ++r)
                std::cout << "Process " << r << " local rank = " << r << " local size = " << P
                          << " hostname = " << host_name() << std::endl;
        }
        RunResult r = run_hip(c);
        finish(c, r, true);
        return r.aborted ? 3 : 0;
    } catch (const std::exception& e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
}
