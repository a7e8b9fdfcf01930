// Python binding of libwave3d (pybind11; deliberately no libtorch dependency — tensors
// cross the boundary as raw device pointers + the caller's HIP stream).
//
//   run(args, backend, transport)  whole solver runs (CLI-equivalent), returns a dict
//   RcclTransport / rccl_unique_id native RCCL halo transport (bootstrapped from Python)
//   Transport                      subclassable from Python (e.g. torch.distributed/gloo)
//   k_* functions                  the individual HIP kernels, for numerics tests
#include <hip/hip_runtime.h>
#include <algorithm>

#include <pybind11/functional.h>
#include <pybind11/pybind11.h>

#include <chrono>
#include <thread>
#include <pybind11/stl.h>

#include "checkpoint.hpp"
#include "hip_kernels.hpp"
#include "problem.hpp"
#include "rccl_transport.hpp"
#include "sizing.hpp"
#include "solver.hpp"

namespace py = pybind11;
using namespace wave3d;

namespace {

// Host transport implemented in Python. `exchange(sends, recvs)` receives lists of
// (peer, tag, address, nbytes); the Python side must complete all transfers.
class PyTransport : public Transport {
public:
    using Transport::Transport;
    std::string name() const override { PYBIND11_OVERRIDE_PURE(std::string, Transport, name); }
    int rank() const override { PYBIND11_OVERRIDE_PURE(int, Transport, rank); }
    int size() const override { PYBIND11_OVERRIDE_PURE(int, Transport, size); }
    bool device() const override { PYBIND11_OVERRIDE_PURE(bool, Transport, device); }
    void exchange(const std::vector<Message>& s, const std::vector<Message>& r, void* stream) override {
        py::gil_scoped_acquire g;
        py::function f = py::get_override(static_cast<const Transport*>(this), "exchange");
        if (!f) throw Error("Transport.exchange not implemented");
        py::list ls, lr;
        for (auto& m : s) ls.append(py::make_tuple(m.peer, m.tag, (uintptr_t)m.ptr, m.bytes));
        for (auto& m : r) lr.append(py::make_tuple(m.peer, m.tag, (uintptr_t)m.ptr, m.bytes));
        f(ls, lr, (uintptr_t)stream);
    }
    void allreduce_max_u64(u64* data, size_t n, void* stream) override {
        py::gil_scoped_acquire g;
        py::function f = py::get_override(static_cast<const Transport*>(this), "allreduce_max_u64");
        if (!f) throw Error("Transport.allreduce_max_u64 not implemented");
        f((uintptr_t)data, n, (uintptr_t)stream);
    }
    void allreduce_max_host(double* data, size_t n) override {
        py::gil_scoped_acquire g;
        py::function f = py::get_override(static_cast<const Transport*>(this), "allreduce_max_host");
        if (!f) throw Error("Transport.allreduce_max_host not implemented");
        py::list v;
        for (size_t q = 0; q < n; ++q) v.append(data[q]);
        py::list out = f(v);
        W3D_REQUIRE(out.size() == n, "allreduce_max_host returned a wrong length");
        for (size_t q = 0; q < n; ++q) data[q] = out[q].cast<double>();
    }
    void barrier() override { PYBIND11_OVERRIDE_PURE(void, Transport, barrier); }
};

py::dict result_dict(const Config& c, const RunResult& r) {
    py::dict d;
    d["N"] = r.N;
    d["timesteps"] = r.K;
    d["nprocs"] = r.nprocs;
    d["Np"] = r.Np;
    d["dims"] = std::vector<int>{r.dims[0], r.dims[1], r.dims[2]};
    d["dtype"] = dtype_name(r.dtype);
    d["backend"] = r.backend;
    d["kernel"] = r.kernel;
    d["scheme"] = r.scheme;
    d["math"] = r.math;
    d["transport"] = r.transport;
    d["courant"] = r.courant;
    d["max_abs"] = r.max_abs;
    d["max_rel"] = r.max_rel;
    d["linf_abs"] = r.linf_final();
    d["init_ms"] = r.t.init_ms;
    d["total_ms"] = r.t.total_ms;
    d["loop_ms"] = r.t.loop_ms;
    d["exchange_ms"] = r.t.exchange_ms;
    d["comm_ms"] = r.t.comm_ms;
    d["error_ms"] = r.t.error_ms;
    d["solve_ms"] = r.solve_ms;
    d["mpts_per_s"] = r.mpts_per_s();
    d["mpts_per_s_best"] = r.mpts_per_s_best();
    d["aborted"] = r.aborted;
    d["abort_layer"] = r.abort_layer;
    d["abort_reason"] = r.abort_reason;
    d["layers_done"] = r.layers_done;
    d["resumed_from"] = r.resumed_from;
    d["graph"] = r.graph;
    d["overlap"] = r.overlap;
    d["overlap_mode"] = r.overlap_mode;
    d["overlap_trial_ms"] = py::make_tuple(r.overlap_trial_ms[0], r.overlap_trial_ms[1], r.overlap_trial_ms[2]);
    py::list trials;
    for (int q = 0; q < kOverlapTrialSolves; ++q) trials.append(r.overlap_trials[q]);
    d["overlap_trials_ms"] = py::tuple(trials);
    d["overlap_order"] = r.overlap_order;
    d["overlap_order_run"] = r.overlap_order_run;
    d["comm_size"] = r.comm_size;
    d["rccl_max_ctas"] = r.rccl_max_ctas;
    d["halo_checked"] = r.halo_checked;
    d["overlap_interior"] = r.overlap_interior;
    d["rccl_mirror_msgs"] = r.rccl_mirror_msgs;
    d["report"] = format_report(c, r);
    d["output_file"] = output_filename(c, r);
    d["json"] = json_summary(c, r);
    return d;
}

// The in-process API is quiet by default: the programs' per-layer progress lines
// ("calculating layer n", cuda_sol.cpp:385) only with an explicit --print-layers.
Config parse_api(const std::vector<std::string>& args) {
    Config c = parse_cli(args);
    if (std::find(args.begin(), args.end(), "--print-layers") == args.end()) c.print_layers = false;
    return c;
}

py::dict run(const std::vector<std::string>& args, const std::string& backend,
             Transport* transport, bool write, bool root) {
    Config c = parse_api(args);
    RunResult r;
    {
        py::gil_scoped_release nogil;
        if (backend == "cpu") r = run_cpu(c, transport);
        else if (backend == "hip") r = run_hip(c, transport);
        else throw Error("unknown backend " + backend);
    }
    if (write && root) write_report(c, r);
    return result_dict(c, r);
}

template <class T>
T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }

GridView gview(const std::vector<i64>& g) {
    W3D_REQUIRE(g.size() == 5, "grid view = (nx, ny, nz, sj, si)");
    GridView v;
    v.X = int(g[0]) - 2;
    v.Y = int(g[1]) - 2;
    v.Z = int(g[2]) - 2;
    v.G = 1;
    v.sj = int(g[3]);
    v.si = g[4];
    return v;
}

Box tobox(const std::vector<int>& b) {
    W3D_REQUIRE(b.size() == 6, "box = (i0, i1, j0, j1, k0, k1)");
    return Box{b[0], b[1], b[2], b[3], b[4], b[5]};
}

// flat (src, dst, src, dst, ...) list of at most kMaxWrap pairs
Wrap towrap(const std::vector<int>& v) {
    W3D_REQUIRE(v.size() % 2 == 0 && v.size() <= 2 * kMaxWrap, "wrap = (src, dst, ...) pairs");
    Wrap w;
    for (size_t q = 0; q < v.size() / 2; ++q) w.src[q] = v[2 * q], w.dst[q] = v[2 * q + 1];
    return w;
}

template <class T>
void k_step(const std::string& kind, bool first, uintptr_t u1, uintptr_t u2, uintptr_t u,
            const std::vector<i64>& g, const std::vector<std::vector<int>>& boxes, int ei0,
            int ei1, const std::vector<int>& wrap, uintptr_t tx, uintptr_t ty, uintptr_t tz,
            const std::vector<double>& coefs, uintptr_t err, int chunk, uintptr_t stream,
            const std::vector<uintptr_t>& packbuf, const std::vector<int>& packidx) {
    std::vector<Box> bx;
    for (auto& b : boxes) bx.push_back(tobox(b));
    Wrap w = towrap(wrap);
    FusedPack<T> fp;
    if (packbuf.size() == 4 && packidx.size() == 4) {
        fp.zbuf[0] = P<T>(packbuf[0]), fp.zbuf[1] = P<T>(packbuf[1]);
        fp.ybuf[0] = P<T>(packbuf[2]), fp.ybuf[1] = P<T>(packbuf[3]);
        fp.zk[0] = packidx[0], fp.zk[1] = packidx[1], fp.yj[0] = packidx[2], fp.yj[1] = packidx[3];
    }
    W3D_REQUIRE(coefs.size() == 5, "coefs = (hx2, hy2, hz2, coef, ct)");
    StepCoefs c{coefs[0], coefs[1], coefs[2], coefs[3], coefs[4]};
    launch_step<T>(parse_kernel_variant(kind), first, P<T>(u1),
                   P<T>(u2), P<T>(u), gview(g), bx.data(), int(bx.size()), ei0, ei1, w, fp,
                   P<T>(tx), P<T>(ty), P<T>(tz), c, P<u64>(err), chunk, (hipStream_t)stream);
}

// Dense [nx][ny][nz] tensor with G ghost layers per side: logical (i,j,k) at tensor index
// (i+G-1, j+G-1, k+G-1); returns the view and the logical-origin offset (elements).
GridView gview_g(const std::vector<i64>& g, i64& origin) {
    W3D_REQUIRE(g.size() == 4, "grid view = (nx, ny, nz, G)");
    GridView v;
    v.G = int(g[3]);
    W3D_REQUIRE(v.G >= 1, "ghost depth >= 1");
    v.X = int(g[0]) - 2 * v.G;
    v.Y = int(g[1]) - 2 * v.G;
    v.Z = int(g[2]) - 2 * v.G;
    W3D_REQUIRE(v.X >= 1 && v.Y >= 1 && v.Z >= 1, "grid smaller than its ghosts");
    v.sj = int(g[2]);
    v.si = g[1] * g[2];
    v.poff = (v.G - 1) * (v.sj + 1);
    origin = i64(v.G - 1) * (v.si + v.sj + 1);
    return v;
}

StepCoefs tocoefs(const std::vector<double>& c) {
    W3D_REQUIRE(c.size() == 5, "coefs = (hx2, hy2, hz2, coef, ct)");
    return StepCoefs{c[0], c[1], c[2], c[3], c[4]};
}

// One temporal-blocking sweep (k_tb2) on dense tensors: C = u^m, D = u^{m+1} from A, B.
template <class T>
void k_tb2_dense(int rows, int waves, int nwk, bool delta, bool first, uintptr_t A, uintptr_t B, uintptr_t Cc, uintptr_t D,
                 const std::vector<i64>& g, const std::vector<std::vector<int>>& boxes,
                 const std::vector<int>& cdom, int ei0, int ei1, const std::vector<int>& wrapC,
                 const std::vector<int>& wrapD, uintptr_t tx, uintptr_t ty, uintptr_t tz,
                 const std::vector<double>& cC, const std::vector<double>& cD, uintptr_t errC,
                 uintptr_t errD, int chunk, uintptr_t stream) {
    i64 o = 0;
    const GridView v = gview_g(g, o);
    W3D_REQUIRE(v.G >= 2, "k_tb2 needs ghost depth >= 2");
    std::vector<Box> bx;
    for (auto& b : boxes) bx.push_back(tobox(b));
    // the kernel reads sx*sy from a product table (the solver builds it once per run)
    const hipStream_t s = (hipStream_t)stream;
    T* txy = nullptr;
    if (hipMalloc(&txy, txy_elems(v.X, v.Y) * sizeof(T)) != hipSuccess) throw Error("k_tb2: hipMalloc failed");
    try {
        launch_txy<T>(txy, P<T>(tx), P<T>(ty), v.X, v.Y, s);
        launch_tb2<T>(rows, waves, 0, nwk, delta, false, first, P<T>(A) + o, P<T>(B) + o, P<T>(Cc) + o, P<T>(D) + o, v,
                      bx.data(), int(bx.size()), tobox(cdom), ei0, ei1, towrap(wrapC), towrap(wrapD),
                      SeamAlias<T>{}, txy, P<T>(tz), nullptr, nullptr, tocoefs(cC), tocoefs(cD),
                      P<u64>(errC), P<u64>(errD), chunk, s);
    } catch (...) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(txy);
        throw;
    }
    const hipError_t e = hipStreamSynchronize(s);
    (void)hipFree(txy);
    if (e != hipSuccess) throw Error(std::string("k_tb2: ") + hipGetErrorString(e));
}

// One three-layer sweep (k_tb3): C = u^m (errors only), D = u^{m+1}, E = u^{m+2}.
template <class T>
void k_tb3_dense(int rows, int waves, bool fm, bool first, uintptr_t A, uintptr_t B, uintptr_t D, uintptr_t E,
                 const std::vector<i64>& g, const std::vector<std::vector<int>>& boxes,
                 const std::vector<int>& cdom, int ei0, int ei1, uintptr_t tx, uintptr_t ty,
                 uintptr_t tz, const std::vector<double>& cC, const std::vector<double>& cD,
                 const std::vector<double>& cE, uintptr_t errC, uintptr_t errD, uintptr_t errE,
                 int chunk, uintptr_t stream) {
    i64 o = 0;
    const GridView v = gview_g(g, o);
    W3D_REQUIRE(v.G >= 3, "k_tb3 needs ghost depth >= 3");
    std::vector<Box> bx;
    for (auto& b : boxes) bx.push_back(tobox(b));
    const hipStream_t s = (hipStream_t)stream;
    T* txy = nullptr;
    T* rt = nullptr;  // --math fma: 1/|txy| then 1/|tz|
    const size_t ntxy = txy_elems(v.X, v.Y), ntz = size_t(v.Z) + 2;
    if (hipMalloc(&txy, ntxy * sizeof(T)) != hipSuccess) throw Error("k_tb3: hipMalloc failed");
    if (fm && hipMalloc(&rt, (2 * ntxy + ntz) * sizeof(T)) != hipSuccess) {
        (void)hipFree(txy);
        throw Error("k_tb3: hipMalloc failed");
    }
    try {
        launch_txy<T>(txy, P<T>(tx), P<T>(ty), v.X, v.Y, s);
        if (fm) {
            launch_txr<T>(rt, txy, ntxy, s);
            launch_recip_abs<T>(rt + 2 * ntxy, P<T>(tz), ntz, s);
        }
        launch_tb3<T>(rows, waves, false, fm, first, P<T>(A) + o, P<T>(B) + o, P<T>(D) + o, P<T>(E) + o, v,
                      bx.data(), int(bx.size()), tobox(cdom), ei0, ei1, Wrap{}, Wrap{},
                      SeamPartners<T>{}, txy, P<T>(tz), rt, fm ? rt + 2 * ntxy : nullptr, tocoefs(cC), tocoefs(cD),
                      tocoefs(cE), P<u64>(errC), P<u64>(errD), P<u64>(errE), chunk, s);
    } catch (...) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(txy);
        (void)hipFree(rt);
        throw;
    }
    const hipError_t e = hipStreamSynchronize(s);
    (void)hipFree(txy);
    (void)hipFree(rt);
    if (e != hipSuccess) throw Error(std::string("k_tb3: ") + hipGetErrorString(e));
}

// One deep sweep (k_tbn, `depth` layers): layers m .. m+depth-3 errors only, O0 = u^{m+depth-2},
// O1 = u^{m+depth-1}; coefs[l] = (hx2, hy2, hz2, coef, ct) and err[l] of layer m+l.
template <class T>
void k_tbn_dense(int depth, int rows, int waves, bool fm, bool first, uintptr_t A, uintptr_t B, uintptr_t O0,
                 uintptr_t O1, const std::vector<i64>& g, const std::vector<std::vector<int>>& boxes,
                 const std::vector<int>& cdom, int ei0, int ei1, uintptr_t tx, uintptr_t ty, uintptr_t tz,
                 const std::vector<std::vector<double>>& coefs, const std::vector<uintptr_t>& err, int chunk,
                 uintptr_t stream, bool delta) {
    i64 o = 0;
    const GridView v = gview_g(g, o);
    W3D_REQUIRE(int(coefs.size()) == depth && int(err.size()) == depth, "k_tbn: one coefficient set / slot per layer");
    std::vector<Box> bx;
    for (auto& b : boxes) bx.push_back(tobox(b));
    StepCoefs cs[kTbnMaxDepth];
    u64* es[kTbnMaxDepth] = {};
    for (int l = 0; l < depth; ++l) cs[l] = tocoefs(coefs[l]), es[l] = P<u64>(err[l]);
    const hipStream_t s = (hipStream_t)stream;
    T* txy = nullptr;
    T* rt = nullptr;
    const size_t ntxy = txy_elems(v.X, v.Y), ntz = size_t(v.Z) + 2;
    if (hipMalloc(&txy, ntxy * sizeof(T)) != hipSuccess) throw Error("k_tbn: hipMalloc failed");
    if (fm && hipMalloc(&rt, (2 * ntxy + ntz) * sizeof(T)) != hipSuccess) {
        (void)hipFree(txy);
        throw Error("k_tbn: hipMalloc failed");
    }
    try {
        launch_txy<T>(txy, P<T>(tx), P<T>(ty), v.X, v.Y, s);
        if (fm) {
            launch_txr<T>(rt, txy, ntxy, s);
            launch_recip_abs<T>(rt + 2 * ntxy, P<T>(tz), ntz, s);
        }
        launch_tbn<T>(depth, rows, waves, fm, first, P<T>(A) + o, P<T>(B) + o, P<T>(O0) + o, P<T>(O1) + o, v,
                      bx.data(), int(bx.size()), tobox(cdom), ei0, ei1, Wrap{}, Wrap{}, TbnSeam<T>{}, txy, P<T>(tz),
                      rt, fm ? rt + 2 * ntxy : nullptr, cs, es, chunk, s, delta);
    } catch (...) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(txy);
        (void)hipFree(rt);
        throw;
    }
    const hipError_t e = hipStreamSynchronize(s);
    (void)hipFree(txy);
    (void)hipFree(rt);
    if (e != hipSuccess) throw Error(std::string("k_tbn: ") + hipGetErrorString(e));
}

template <class T>
void k_init(uintptr_t u, const std::vector<i64>& g, const std::vector<int>& box,
            const std::vector<int>& wrap, uintptr_t tx, uintptr_t ty, uintptr_t tz, double ct0,
            uintptr_t err, uintptr_t stream) {
    Wrap w = towrap(wrap);
    launch_init<T>(P<T>(u), gview(g), tobox(box), w, P<T>(tx), P<T>(ty), P<T>(tz), ct0,
                   P<u64>(err), (hipStream_t)stream);
}

template <class T>
void k_faces(uintptr_t u, const std::vector<i64>& g, const std::vector<std::tuple<uintptr_t, int, int>>& ops,
             bool to_buf, uintptr_t stream) {
    std::vector<FaceOp<T>> o;
    for (auto& t : ops) o.push_back({P<T>(std::get<0>(t)), std::get<1>(t), std::get<2>(t)});
    launch_faces<T>(P<T>(u), gview(g), o.data(), int(o.size()), to_buf, (hipStream_t)stream);
}

template <class T>
void k_zero_faces(uintptr_t u, const std::vector<i64>& g, int mask, uintptr_t stream) {
    launch_zero_faces<T>(P<T>(u), gview(g), mask, (hipStream_t)stream);
}

}  // namespace

PYBIND11_MODULE(_wave3d_C, m) {
    m.doc() = "wave3d native runtime (C++/HIP for MI355X)";
    py::register_exception<Error>(m, "Wave3dError");

    py::class_<Message>(m, "Message");
    py::class_<Transport, PyTransport>(m, "Transport")
        .def(py::init<>())
        .def("name", &Transport::name)
        .def("rank", &Transport::rank)
        .def("size", &Transport::size)
        .def("device", &Transport::device);

    py::class_<RcclTransport, Transport>(m, "RcclTransport")
        .def(py::init([](int rank, int size, py::bytes uid, int device, int max_ctas) {
                 std::string s = uid;
                 py::gil_scoped_release nogil;
                 return new RcclTransport(rank, size, s, device, max_ctas);
             }),
             py::arg("rank"), py::arg("size"), py::arg("uid"), py::arg("device"), py::arg("max_ctas") = -1)
        .def("max_ctas", &RcclTransport::max_ctas)
        .def("barrier", [](RcclTransport& t) {
            py::gil_scoped_release nogil;
            t.barrier();
        })
        .def("check_async", &RcclTransport::check_async)
        .def("comm_size", &RcclTransport::comm_size);
    m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
    m.def("rccl_max_ctas", &rccl_max_ctas, py::arg("overlap_mode") = "auto",
          "CTA budget a halo communicator gets for an overlap mode (WAVE3D_RCCL_MAX_CTAS overrides)");

    py::class_<Session>(m, "Session", "Persistent solver: allocate once, solve() many times")
        .def(py::init([](const std::vector<std::string>& args, const std::string& backend,
                         Transport* tr) {
                 Config c = parse_api(args);
                 py::gil_scoped_release nogil;
                 if (backend == "cpu") return make_cpu_session(c, tr).release();
                 if (backend == "hip") return make_hip_session(c, tr).release();
                 throw Error("unknown backend " + backend);
             }),
             py::arg("args"), py::arg("backend") = "hip", py::arg("transport") = nullptr,
             py::keep_alive<1, 4>())
        .def("solve", [](Session& s, const std::vector<std::string>& args) {
            Config c = parse_cli(args);
            RunResult r;
            {
                py::gil_scoped_release nogil;
                r = s.solve();
            }
            return result_dict(c, r);
        }, py::arg("args"))
        .def_property_readonly("init_ms", &Session::init_ms)
        .def("field", [](Session& s, int layer) {
            std::vector<FieldBlock> bl;
            {
                py::gil_scoped_release nogil;
                bl = s.field(layer);
            }
            py::list out;
            for (auto& b : bl) {
                py::dict d;
                d["rank"] = b.rank;
                d["off"] = std::vector<int>{b.off[0], b.off[1], b.off[2]};
                d["ext"] = std::vector<int>{b.ext[0], b.ext[1], b.ext[2]};
                d["data"] = b.data;
                out.append(d);
            }
            return out;
        }, py::arg("layer"),
           "Owned blocks (k fastest) of layer K or K-1 after a solve (print_layer analogue).");

    m.def("run", &run, py::arg("args"), py::arg("backend") = "hip",
          py::arg("transport") = nullptr, py::arg("write") = true, py::arg("root") = true,
          "Run the solver with reference-style CLI arguments; returns a result dict.");
    m.def("parse", [](const std::vector<std::string>& a) {
        Config c = parse_cli(a);
        Problem p = Problem::from_config(c);
        py::dict d;
        d["N"] = c.N, d["Np"] = c.Np, d["T"] = c.T, d["timesteps"] = c.timesteps;
        d["Lx"] = p.Lx, d["Ly"] = p.Ly, d["Lz"] = p.Lz, d["pi"] = p.pi;
        d["a2"] = p.a2, d["a_t"] = p.a_t, d["tau"] = p.tau;
        d["hx"] = p.hx, d["hy"] = p.hy, d["hz"] = p.hz;
        d["coef"] = p.coef, d["coef_first"] = p.coef_first, d["courant"] = p.courant;
        d["dtype"] = dtype_name(c.dtype), d["ranks"] = c.ranks, d["overlap"] = c.overlap;
        d["overlap_auto"] = c.overlap_auto, d["rccl_mirror"] = c.rccl_mirror, d["halo_check"] = c.halo_check;
        d["kernel"] = c.kernel, d["chunk"] = c.chunk;
        d["dims"] = std::vector<int>{c.dims[0], c.dims[1], c.dims[2]};
        d["table_x"] = p.table_x(), d["table_y"] = p.table_y(), d["table_z"] = p.table_z();
        d["table_t"] = p.table_t();
        return d;
    });
    m.def("usage", &usage);
    m.def("memory_plan", [](const std::vector<std::string>& a, int world) {
        Config c = parse_cli(a);
        Layout l = plan_layout(c, world);
        py::dict d;
        d["tb"] = l.tb, d["ghost"] = l.G, d["levels"] = l.L, d["rows"] = l.rows, d["waves"] = l.waves;
        d["dims"] = std::vector<int>{l.dims[0], l.dims[1], l.dims[2]};
        d["bytes_per_rank"] = device_bytes_per_rank(c, world);
        return d;
    }, py::arg("args"), py::arg("world") = 1,
       "Device-memory plan of the HIP solver for a CLI configuration (sizing.hpp).");
    m.def("fill_hbm_N", [](const std::vector<std::string>& a, int world, double budget) {
        return fill_hbm_N(parse_cli(a), world, budget);
    }, py::arg("args"), py::arg("world"), py::arg("budget_bytes"),
       "Largest N whose per-rank footprint fits budget_bytes (--fill-hbm).");
    m.def("topology", [](int N, int nprocs, int rank, std::vector<int> dims) {
        int d[3] = {0, 0, 0};
        for (size_t q = 0; q < dims.size() && q < 3; ++q) d[q] = dims[q];
        Topology t = Topology::make(N, nprocs, rank, d);
        py::dict r;
        r["dims"] = std::vector<int>{t.dims[0], t.dims[1], t.dims[2]};
        r["coords"] = std::vector<int>{t.coords[0], t.coords[1], t.coords[2]};
        r["ext"] = std::vector<int>{t.ext[0], t.ext[1], t.ext[2]};
        r["off"] = std::vector<int>{t.off[0], t.off[1], t.off[2]};
        r["nbr"] = std::vector<std::vector<int>>{{t.nbr[0][0], t.nbr[0][1]},
                                                 {t.nbr[1][0], t.nbr[1][1]},
                                                 {t.nbr[2][0], t.nbr[2][1]}};
        auto bx = [](const Box& b) { return std::vector<int>{b.i0, b.i1, b.j0, b.j1, b.k0, b.k1}; };
        r["compute_box"] = bx(t.compute_box());
        r["error_box"] = bx(t.error_box());
        r["owned_box"] = bx(t.owned_box());
        HaloPlan hp = make_halo_plan(t, i64(t.ext[1] + 2) * (t.ext[2] + 2), t.ext[2] + 2);
        auto msgs = [](const std::vector<FaceMsg>& v) {
            py::list l;
            for (auto& f : v) l.append(py::make_tuple(f.axis, f.side, f.peer, f.tag, f.count));
            return l;
        };
        r["sends"] = msgs(hp.sends);
        r["recvs"] = msgs(hp.recvs);
        r["self_x"] = hp.self_x;
        return r;
    });
    m.def("dims_create", [](int n, std::vector<int> dims) {
        int d[3] = {0, 0, 0};
        for (size_t q = 0; q < dims.size() && q < 3; ++q) d[q] = dims[q];
        Topology::dims_create(n, d);
        return std::vector<int>{d[0], d[1], d[2]};
    });
    // host-side watchdog probe for tests: the device "finishes" after `done_after_s`; progress
    // grows every poll until `progress_until_s`, then stalls; returns the wait or raises
    m.def("watchdog_probe", [](double limit_s, double done_after_s, double progress_until_s) {
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        auto el = [&] { return std::chrono::duration<double>(clk::now() - t0).count(); };
        long p = 0;
        const std::function<long()> prog = [&] { return el() < progress_until_s ? ++p : p; };
        bool aborted = false;
        py::gil_scoped_release nogil;
        watch_until([&] { return el() >= done_after_s; }, [] { return std::string(); }, &prog,
                    limit_s, [&] { aborted = true; }, "probe");
        return el();
    }, py::arg("limit_s"), py::arg("done_after_s"), py::arg("progress_until_s"));
    // thread-per-GPU failure handling without a GPU: rank `fail_rank` throws after
    // `fail_after_s`, every other rank waits in watch_until (as on an RCCL stream) with a
    // `limit_s` watchdog; returns (seconds, error) per rank
    m.def("abort_probe", [](int n, int fail_rank, double fail_after_s, double limit_s) {
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        auto el = [&] { return std::chrono::duration<double>(clk::now() - t0).count(); };
        std::vector<double> t(n, 0.0);
        std::vector<std::string> errs;
        {
            py::gil_scoped_release nogil;
            errs = run_rank_threads(n, [&](int r) {
                if (r == fail_rank) {
                    std::this_thread::sleep_for(std::chrono::duration<double>(fail_after_s));
                    t[r] = el();
                    throw Error("injected failure");
                }
                try {
                    watch_until([] { return false; }, [] { return std::string(); }, nullptr, limit_s, [] {},
                                "probe");
                } catch (...) {
                    t[r] = el();
                    throw;
                }
            });
        }
        py::list out;
        for (int r = 0; r < n; ++r) out.append(py::make_tuple(t[r], errs[r]));
        return out;
    }, py::arg("n"), py::arg("fail_rank"), py::arg("fail_after_s"), py::arg("limit_s"));
    m.def("checkpoint_layers", [](const std::string& dir, int rank) { return checkpoint_layers(dir, rank); },
          py::arg("dir"), py::arg("rank"),
          "Layers with a complete checkpoint file of `rank` in `dir` (ascending).");
    m.def("encode_max_key", &encode_max_key);
    m.def("decode_max_key", &decode_max_key);
    m.def("march_rows_per_thread", &march_rows_per_thread);

    // kernel-level entry points (device pointers as ints, explicit stream)
    m.def("k_step_f64", &k_step<double>);
    m.def("k_step_f32", &k_step<float>);
    m.def("k_tb2_f64", &k_tb2_dense<double>);
    m.def("k_tb2_f32", &k_tb2_dense<float>);
    m.def("k_tb3_f64", &k_tb3_dense<double>);
    m.def("k_tb3_f32", &k_tb3_dense<float>);
    m.def("k_tbn_f64", &k_tbn_dense<double>);
    m.def("k_tbn_f32", &k_tbn_dense<float>);
    m.def("tbn_supported", &tbn_supported);
    m.def("tbn_delta_supported", &tbn_delta_supported);
    m.def("tb_supported", [](int depth, int rows, int waves, int nwk, bool fm) {
        return depth == 3 ? tb3_supported(rows, waves, fm) : tb2_supported(rows, waves, 0, nwk);
    }, py::arg("depth"), py::arg("rows"), py::arg("waves"), py::arg("nwk") = 1, py::arg("fm") = false);
    m.def("k_init_f64", &k_init<double>);
    m.def("k_init_f32", &k_init<float>);
    m.def("k_faces_f64", &k_faces<double>);
    m.def("k_faces_f32", &k_faces<float>);
    m.def("k_zero_faces_f64", &k_zero_faces<double>);
    m.def("k_zero_faces_f32", &k_zero_faces<float>);
    m.def("k_init_err", [](uintptr_t err, int layers, uintptr_t s) {
        launch_init_err(P<u64>(err), layers, (hipStream_t)s);
    });
    m.def("k_encode_keys", [](uintptr_t v, uintptr_t k, int n, uintptr_t s) {
        launch_encode_keys(P<double>(v), P<u64>(k), n, (hipStream_t)s);
    });
    // raw HIP helpers for Python-side device transports (staged halos in tests/tools)
    m.def("hip_memcpy", [](uintptr_t dst, uintptr_t src, size_t bytes, uintptr_t stream) {
        py::gil_scoped_release nogil;
        hipError_t e = hipMemcpyAsync((void*)dst, (const void*)src, bytes, hipMemcpyDefault,
                                      (hipStream_t)stream);
        if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
        if (e != hipSuccess) throw Error(std::string("hip_memcpy: ") + hipGetErrorString(e));
    });
    m.def("hip_stream_sync", [](uintptr_t stream) {
        py::gil_scoped_release nogil;
        hipError_t e = hipStreamSynchronize((hipStream_t)stream);
        if (e != hipSuccess) throw Error(std::string("hip_stream_sync: ") + hipGetErrorString(e));
    });
    m.def("device_count", []() {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        return n;
    });
}
