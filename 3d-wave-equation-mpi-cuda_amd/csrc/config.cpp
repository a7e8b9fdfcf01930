#include "config.hpp"

#include <cstdlib>
#include <sstream>

namespace wave3d {

std::string usage() {
    return "usage: wave3d N Np Lx Ly Lz [T=1] [timesteps=20] [options]\n"
           "  Lx|Ly|Lz: number or the literal 'pi'\n"
           "options:\n"
           "  --dtype fp64|fp32      compute precision (default fp64)\n"
           "  --math exact|fma       exact = the reference's operation order, bit for bit (default);\n"
           "                         fma = coef/h^2 folded into fused multiply-adds (tb3 kernels)\n"
           "  --pi ref|exact         ref = 3.1415926535 as the reference CPU programs (default)\n"
           "  --scheme leapfrog|delta  delta = increment form (fp32 accuracy; tb2 / tb3 kernels, CPU)\n"
           "  --ic ref|shifted       shifted = sin(2*pi*x/Lx + 0.7) periodic-BC check\n"
           "  --dims a,b,c           override the Cartesian process grid\n"
           "  --ranks P              simulate P ranks in-process (loopback transport)\n"
           "  --transport auto|rccl|loopback\n"
           "  --halo direct|rounds   temporal-blocking deep halos in one round (faces, edges, corners\n"
           "                         straight from their owners; default) or three dependent rounds\n"
           "  --x-self-transport     one x rank: send the periodic wrap through the transport\n"
           "                         to this rank (exercises RCCL send/recv on a single GPU)\n"
           "  --overlap auto|on|off  interior/shell split with the halo on a second stream; auto\n"
           "                         (default) times solves 2-7: on / off / on with the shells first, twice\n"
           "                         each, and keeps the fastest\n"
           "  --no-overlap           = --overlap off\n"
           "  --kernel K             auto (leapfrog: tb4; increment form: tb3) |\n"
           "                         tb4 | tb3[r<R>w<W>] | tbn3 | tb2[r<R>][w<W>]\n"
           "                         | march[2|4|8][nt|p|f]\n"
           "                         | naive | flat   (temporal blocking / single-step variants)\n"
           "  --chunk C              i-planes per marching work item\n"
           "  --format new|omp|cuda|none      output file flavour (default new)\n"
           "  --out-dir D  --out-name F\n"
           "  --json                 one-line JSON summary on stdout\n"
           "  --check-every k        abort if a layer's error is NaN/Inf/>1 (checked every k layers)\n"
           "  --strict-cfl           refuse unstable Courant numbers (C > 1/sqrt(3))\n"
           "  --checkpoint-every k --checkpoint-dir D   --resume D\n"
           "  --repeat R --warmup W  timed / untimed solves (benchmarking)\n"
           "  --profile              per-phase timers\n"
           "  --graph on|off|auto    replay the time loop as one hipGraph (auto: when eligible)\n"
           "  --fill-hbm FRAC        GPU program: largest N whose per-GPU footprint fits FRAC of HBM\n"
           "  --dump PATH            write the final layer u^K as float64 .npy\n"
           "  --fault SPEC           fault injection (drop_face:RANK:LAYER | nan:RANK:LAYER |\n"
           "                         corrupt_tag:RANK:TAG = halo self-test delivery of TAG to RANK)\n"
           "  --rccl-mirror          with --ranks P: also send every halo message (and the error\n"
           "                         allreduce) through a 1-rank RCCL communicator, compare bitwise\n"
           "  --no-halo-check        skip the init-time halo self-test (patterns through the real plan)\n"
           "  --model-link G[,L]     every halo exchange also waits the time its busiest peer link\n"
           "                         needs at G GB/s (+ L us latency), on one CU (an xGMI link model\n"
           "                         for overlap experiments on one GPU: --ranks P, or processes\n"
           "                         sharing it through the staged transport)\n"
           "  --device d  --threads t  --no-print-layers  --quiet\n";
}

namespace {

double parse_len(const std::string& s, bool& is_pi) {
    is_pi = (s == "pi");
    if (is_pi) return 0.0;  // resolved once the pi mode is known
    size_t pos = 0;
    double v = std::stod(s, &pos);
    W3D_REQUIRE(pos == s.size(), "bad length '" + s + "'");
    W3D_REQUIRE(v > 0, "lengths must be positive");
    return v;
}

int parse_int(const std::string& s, const char* what) {
    size_t pos = 0;
    int v = 0;
    try {
        v = std::stoi(s, &pos);
    } catch (...) {
        throw Error(std::string("wave3d: bad ") + what + " '" + s + "'");
    }
    W3D_REQUIRE(pos == s.size(), std::string("bad ") + what + " '" + s + "'");
    return v;
}

}  // namespace

Config parse_cli(const std::vector<std::string>& a) {
    Config c;
    std::vector<std::string> pos;
    size_t i = 0;
    for (; i < a.size(); ++i) {
        if (a[i].rfind("--", 0) == 0) break;
        pos.push_back(a[i]);
    }
    if (pos.size() < 5 || pos.size() > 7)
        throw Error("wave3d: expected 5-7 positional arguments\n" + usage());
    try {
        c.N = parse_int(pos[0], "N");
        c.Np = parse_int(pos[1], "Np");
        c.Lx = parse_len(pos[2], c.Lx_is_pi);
        c.Ly = parse_len(pos[3], c.Ly_is_pi);
        c.Lz = parse_len(pos[4], c.Lz_is_pi);
        if (pos.size() >= 6) c.T = std::stod(pos[5]);
        if (pos.size() >= 7) c.timesteps = parse_int(pos[6], "timesteps");
    } catch (const Error&) {
        throw;
    } catch (const std::exception& e) {
        throw Error(std::string("wave3d: bad positional argument (") + e.what() + ")\n" + usage());
    }
    W3D_REQUIRE(c.N >= 2 || c.N == 0, "N must be >= 2 (0 only with --fill-hbm)");
    W3D_REQUIRE(c.Np >= 1, "Np must be >= 1");
    W3D_REQUIRE(c.timesteps >= 1, "timesteps must be >= 1");
    W3D_REQUIRE(c.T > 0, "T must be positive");

    auto need = [&](size_t k) -> const std::string& {
        W3D_REQUIRE(k + 1 < a.size(), "option " + a[k] + " needs a value");
        return a[k + 1];
    };
    for (; i < a.size(); ++i) {
        const std::string& o = a[i];
        if (o == "--dtype") {
            const std::string& v = need(i++);
            if (v == "fp64" || v == "f64" || v == "double") c.dtype = DType::F64;
            else if (v == "fp32" || v == "f32" || v == "float") c.dtype = DType::F32;
            else throw Error("wave3d: bad --dtype " + v);
        } else if (o == "--scheme") {
            const std::string& v = need(i++);
            if (v == "leapfrog") c.delta = false;
            else if (v == "delta") c.delta = true;
            else throw Error("wave3d: bad --scheme " + v);
        } else if (o == "--math") {
            const std::string& v = need(i++);
            if (v == "exact") c.fma = false;
            else if (v == "fma") c.fma = true;
            else throw Error("wave3d: bad --math " + v);
        } else if (o == "--pi") {
            const std::string& v = need(i++);
            if (v == "ref") c.pi = PiMode::Ref;
            else if (v == "exact") c.pi = PiMode::Exact;
            else throw Error("wave3d: bad --pi " + v);
        } else if (o == "--ic") {
            const std::string& v = need(i++);
            if (v == "ref") c.ic = ICMode::Ref;
            else if (v == "shifted") c.ic = ICMode::Shifted;
            else throw Error("wave3d: bad --ic " + v);
        } else if (o == "--dims") {
            std::stringstream ss(need(i++));
            std::string tok;
            int d = 0;
            while (std::getline(ss, tok, ',')) {
                W3D_REQUIRE(d < 3, "--dims takes 3 values");
                c.dims[d++] = parse_int(tok, "dims");
            }
            W3D_REQUIRE(d == 3, "--dims takes 3 values");
        } else if (o == "--ranks") {
            c.ranks = parse_int(need(i++), "ranks");
        } else if (o == "--transport") {
            c.transport = need(i++);
        } else if (o == "--halo") {
            const std::string& v = need(i++);
            if (v == "direct") c.halo_direct = true;
            else if (v == "rounds") c.halo_direct = false;
            else throw Error("wave3d: bad --halo " + v);
        } else if (o == "--x-self-transport") {
            c.x_self_transport = true;
        } else if (o == "--no-overlap") {
            c.overlap = false;
            c.overlap_auto = false;
        } else if (o == "--overlap") {
            // --overlap [on|off|auto]; bare --overlap = on
            std::string v = "on";
            if (i + 1 < a.size() && (a[i + 1] == "on" || a[i + 1] == "off" || a[i + 1] == "auto")) v = a[++i];
            c.overlap = v != "off";
            c.overlap_auto = v == "auto";
        } else if (o == "--kernel") {
            c.kernel = need(i++);
        } else if (o == "--chunk") {
            c.chunk = parse_int(need(i++), "chunk");
        } else if (o == "--format") {
            const std::string& v = need(i++);
            if (v == "new" || v == "mpi") c.format = ReportFormat::New;
            else if (v == "omp") c.format = ReportFormat::Omp;
            else if (v == "cuda") c.format = ReportFormat::Cuda;
            else if (v == "none") c.format = ReportFormat::None;
            else throw Error("wave3d: bad --format " + v);
        } else if (o == "--out-dir") {
            c.out_dir = need(i++);
        } else if (o == "--out-name") {
            c.out_name = need(i++);
        } else if (o == "--json") {
            c.json = true;
        } else if (o == "--check-every") {
            c.check_every = parse_int(need(i++), "check-every");
        } else if (o == "--strict-cfl") {
            c.strict_cfl = true;
        } else if (o == "--checkpoint-every") {
            c.checkpoint_every = parse_int(need(i++), "checkpoint-every");
        } else if (o == "--checkpoint-dir") {
            c.checkpoint_dir = need(i++);
        } else if (o == "--resume") {
            c.resume_dir = need(i++);
        } else if (o == "--repeat") {
            c.repeat = parse_int(need(i++), "repeat");
        } else if (o == "--warmup") {
            c.warmup = parse_int(need(i++), "warmup");
        } else if (o == "--profile") {
            c.profile = true;
        } else if (o == "--dump") {
            c.dump = need(i++);
        } else if (o == "--fill-hbm") {
            c.fill_hbm = std::stod(need(i++));
            if (!(c.fill_hbm > 0 && c.fill_hbm <= 0.98)) throw Error("--fill-hbm needs 0 < FRAC <= 0.98");
        } else if (o == "--graph") {
            const std::string& v = need(i++);
            if (v == "on") c.graph = 1;
            else if (v == "off") c.graph = 0;
            else if (v == "auto") c.graph = -1;
            else throw Error("--graph must be on, off or auto");
        } else if (o == "--rccl-mirror") {
            c.rccl_mirror = true;
        } else if (o == "--model-link") {
            const std::string v = need(i++);
            const size_t cm = v.find(',');
            c.model_link_gbps = std::stod(v.substr(0, cm));
            c.model_link_lat_us = cm == std::string::npos ? 0.0 : std::stod(v.substr(cm + 1));
            W3D_REQUIRE(c.model_link_gbps > 0 && c.model_link_lat_us >= 0, "--model-link needs GBPS > 0[,LAT_US >= 0]");
        } else if (o == "--no-halo-check") {
            c.halo_check = false;
        } else if (o == "--fault") {
            c.fault = need(i++);
        } else if (o == "--device") {
            c.device = parse_int(need(i++), "device");
        } else if (o == "--threads") {
            c.threads = parse_int(need(i++), "threads");
        } else if (o == "--print-layers") {
            c.print_layers = true;
        } else if (o == "--no-print-layers") {
            c.print_layers = false;
        } else if (o == "--quiet") {
            c.quiet = true;
        } else {
            throw Error("wave3d: unknown option " + o + "\n" + usage());
        }
    }
    W3D_REQUIRE(c.repeat >= 1 && c.warmup >= 0, "bad --repeat/--warmup");
    W3D_REQUIRE(c.checkpoint_every == 0 || !c.checkpoint_dir.empty(),
                "--checkpoint-every needs --checkpoint-dir");
    if (c.fault.empty()) {
        if (const char* e = std::getenv("WAVE_FI")) c.fault = e;
    }
    W3D_REQUIRE(c.N >= 2 || c.fill_hbm > 0, "N must be >= 2 (0 only with --fill-hbm)");
    return c;
}

Config parse_cli(int argc, const char* const* argv) {
    std::vector<std::string> a;
    for (int i = 1; i < argc; ++i) a.emplace_back(argv[i]);
    return parse_cli(a);
}

}  // namespace wave3d
