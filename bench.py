#!/usr/bin/env python3
"""wave3d benchmark — the reference's headline metric on MI355X.

Metric (BASELINE.json): Mpoints/s (whole node) + L-inf error vs the analytic solution,
N=512^3 fp64. One benchmark *step* is one complete solve exactly as timed by the reference
(`numerical solution calculated in`, mpi_new.cpp:325-357): initial condition, Taylor first
layer, `timesteps` leapfrog layers, the fused per-layer max-error evaluation and the final
cross-rank MAX reduction. Mpoints/s = (N+1)^3 * timesteps * steps / t_wall.

`--gpus n` runs the BASELINE.json config for that GPU count, each with a golden L-inf from
the reference (the reference's errors are identical for every P):

    1 GPU : N=512,  1x1x1          (config 2)      golden 6.03381e-07
    2 GPUs: N=512,  2x1x1 slabs    (config 3)      golden 6.03381e-07   strong vs 1 GPU
    4 GPUs: N=1024, 2x2x1          (config 4 grid) golden 8.04265e-08   strong vs 8 GPUs
    8 GPUs: N=1024, 2x2x2 blocks   (config 4)      golden 8.04265e-08   weak vs 1 GPU

The decomposition is MPI_Dims_create's, as in the reference (mpi_new.cpp:409-433); `--dims`
overrides it. The default kernel is four-layer temporal blocking (tb4: 4 layers per sweep,
~8 instead of 24 B/node/layer, 4 time levels) with 4-deep RCCL halos; the fp32 increment form
runs three layers per sweep (tb3); `--kernel tb3|tb2` selects three- / two-layer blocking,
`--kernel march2` the single-step kernel.
The JSON line states what ran: N and dtype in the metric, dims, the effective overlap,
the transport and the ranks RCCL itself reports (ncclCommCount), and whether the L-inf
matches the golden. Data: the analytic initial condition on a synthetic grid (the
reference's own test problem).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "Mpoints/sec (whole node) + L∞ error vs analytic, N={N}³ {dtype}"  # BASELINE.json at N=512


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5, help="timed solves")
    ap.add_argument("--warmup", type=int, default=3,
                    help="untimed solves (with halos, solves 2-7 are the --overlap auto trials)")
    ap.add_argument("--N", type=int, default=0, help="override global N (default: the BASELINE config)")
    ap.add_argument("--config", default="",
                    help="run a named BASELINE config instead (models/presets.py CONFIGS, e.g. "
                         "gpu2048x8_fp32 = config 5: N, timesteps, dtype, decomposition)")
    ap.add_argument("--dims", default="", help="process grid a,b,c (default: the BASELINE config's)")
    ap.add_argument("--timesteps", type=int, default=None,
                    help="layers per solve (default 100; with --fill-hbm 0; 0: smallest stable count with "
                         "margin, C <= 0.5)")
    ap.add_argument("--fill-hbm", type=float, default=0.0,
                    help="size N to this fraction of each GPU's HBM (SURVEY §7.3; e.g. 0.9)")
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"])
    ap.add_argument("--scheme", default="auto", choices=["auto", "leapfrog", "delta"],
                    help="time stepping: leapfrog (the reference's), delta (increment form, same scheme "
                         "without the 2u-u cancellation); auto = leapfrog for fp64, delta for fp32 "
                         "(profiles/fp32_accuracy_r2.txt, fp32_scheme_r4.txt)")
    ap.add_argument("--math", default="auto", choices=["auto", "exact", "fma"],
                    help="stencil arithmetic: exact = the reference CPU programs' operation order, bit for "
                         "bit; fma = coef/h^2 folded into fused multiply-adds (same scheme, same L-inf abs to "
                         "9 digits at the headline config, profiles/math_fma_r3.txt); auto = fma on the GPU")
    ap.add_argument("--fp64-ref", default="auto", choices=["auto", "on", "off"],
                    help="fp32 runs: after timing, solve the same N/K/decomposition in fp64 and report "
                         "its L-inf as linf_fp64_ref (BASELINE.md §4 config 5); auto = on for fp32")
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--overlap", default="auto", choices=["auto", "on", "off"],
                    help="interior/shell split with the halo on a second stream; auto times the first "
                         "two solves (warmup) on and off and keeps the faster")
    ap.add_argument("--no-overlap", action="store_true", help="= --overlap off")
    ap.add_argument("--backend", default="hip", choices=["hip", "cpu"])
    ap.add_argument("--profile", action="store_true", help="per-phase timers (slower)")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "staged"],
                    help="halo transport for N>1 (staged = rehearsal on one shared GPU)")
    ap.add_argument("--shared-device", action="store_true", help="all ranks on device 0 (rehearsal)")
    ap.add_argument("--model-link", default="",
                    help="GBPS[,LAT_US]: each halo exchange also waits its busiest link's time at that "
                         "bandwidth (the 8-GPU rehearsal on one GPU with an xGMI-like link cost)")
    ap.add_argument("--launch-timeout", type=float, default=1000.0,
                    help="self-launch (--gpus N without torchrun): kill every rank after this many s")
    a = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # one command, N ranks (the reference's `mpirun -n Np`, README.txt:43): spawn the ranks
        # as child processes before this process touches torch or the GPU
        return launch_ranks(a.gpus, sys.argv[1:], a.launch_timeout)

    import torch
    import torch.distributed as dist

    import wave3d
    from wave3d.models import presets
    from wave3d.parallel import dist as wdist

    C = wave3d.load_native()
    rank, world, local = wdist.env_rank()
    if world != a.gpus and world > 1:
        print(f"bench: WORLD_SIZE={world} but --gpus {a.gpus}", file=sys.stderr)
    n_gpus = world if world > 1 else a.gpus

    transport = None
    if world > 1:
        if a.backend == "hip":
            # preflight before any communicator exists: one GPU per rank (RCCL refuses two
            # ranks on one device; --shared-device rehearses on one GPU with --transport staged)
            ndev = torch.cuda.device_count()
            if ndev == 0 or (not a.shared_device and ndev < world):
                print(f"bench: rank {rank}: {world} ranks need {world} GPUs, {ndev} visible "
                      "(--shared-device --transport staged rehearses on one GPU)", file=sys.stderr)
                return 2
            if a.shared_device and a.transport == "rccl":
                print("bench: --shared-device needs --transport staged (RCCL refuses duplicate GPUs)",
                      file=sys.stderr)
                return 2
            torch.cuda.set_device(0 if a.shared_device else local % ndev)
        nccl = a.backend == "hip" and a.transport == "rccl"
        wdist.init_from_env("nccl" if nccl else "gloo")
        if os.environ.get("WAVE3D_BENCH_FAIL_RANK") == str(rank):  # test hook: a rank dies
            print(f"bench: rank {rank}: WAVE3D_BENCH_FAIL_RANK", file=sys.stderr)
            return 3
        if a.backend == "hip":
            transport = wdist.make_transport(a.transport, overlap="off" if a.no_overlap else a.overlap)
        else:
            transport = wdist.TorchHostTransport()
    elif a.backend == "hip":
        torch.cuda.set_device(0)

    plan = presets.bench_plan(n_gpus)
    if a.config:
        if a.config not in presets.CONFIGS:
            print(f"bench: unknown --config {a.config} ({', '.join(presets.CONFIGS)})", file=sys.stderr)
            return 2
        named = presets.CONFIGS[a.config]
        if named["backend"] == "hip" and named["Np"] != n_gpus:
            print(f"bench: --config {a.config} is a {named['Np']}-GPU config (running on {n_gpus})",
                  file=sys.stderr)
        np_ = named["problem"]
        a.N, a.timesteps, a.dtype = np_.N, np_.timesteps, np_.dtype
        if a.scheme == "auto":
            a.scheme = np_.scheme
        if named["dims"] and not a.dims and named["Np"] == n_gpus:
            a.dims = ",".join(str(x) for x in named["dims"])
        plan = dict(plan, config=a.config, golden=presets.GOLDEN_LINF.get((np_.N, np_.timesteps)))
    N = a.N or plan["N"]
    dims = [int(x) for x in a.dims.split(",")] if a.dims else (None if a.N else plan["dims"])
    if a.timesteps is None:  # --fill-hbm moves N: keep the run stable unless K is given
        a.timesteps = 0 if a.fill_hbm > 0 else 100
    if a.fill_hbm > 0:
        if a.backend != "hip":
            print("bench: --fill-hbm needs the hip backend", file=sys.stderr)
            return 2
        total = torch.cuda.mem_get_info()[1]
        probe = wave3d.WaveSolver(wave3d.WaveProblem(N, timesteps=max(1, a.timesteps), dtype=a.dtype),
                                  a.backend, Np=n_gpus, kernel=a.kernel).args()
        N = C.fill_hbm_N(probe, n_gpus, a.fill_hbm * total)
    K = a.timesteps
    if K <= 0:
        K = wave3d.WaveProblem(N, dtype=a.dtype).min_stable_timesteps()
        K = max(20, int(K * 0.577 / 0.5) + 1)  # C <= 0.5
    a.timesteps = K
    if a.scheme == "auto":
        a.scheme = presets.default_scheme(a.dtype)
    if a.math == "auto":
        a.math = presets.default_math(a.backend, a.dtype)
    prob = wave3d.WaveProblem(N, timesteps=a.timesteps, dtype=a.dtype, scheme=a.scheme, math=a.math)
    if not prob.stable():
        print(f"bench: warning: C={prob.courant:.3f} > 1/sqrt(3) (unstable)", file=sys.stderr)
    solver = wave3d.WaveSolver(prob, a.backend, transport=transport, Np=n_gpus, kernel=a.kernel, dims=dims,
                               chunk=a.chunk, overlap="off" if a.no_overlap else a.overlap, profile=a.profile,
                               device=(torch.cuda.current_device() if a.backend == "hip" else None),
                               model_link=a.model_link or None)
    args = solver.args()
    sess = C.Session(args, a.backend, transport)

    def sync():
        if a.backend == "hip":
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    res = None
    # --overlap auto with remote halos times its three arms (on with the shells beside the
    # interior, off, on with the shells first) twice each on solves 2-7 (solve 1 warms up): with
    # fewer than 7 warm-up solves the missing trial solves run here, untimed, so the timed solves
    # all use the chosen arm (reported as "tuning_solves")
    tuning = (max(0, 7 - a.warmup) if a.backend == "hip" and world > 1 and not a.no_overlap
              and a.overlap == "auto" else 0)
    for _ in range(tuning + a.warmup):
        res = sess.solve(args)
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = sess.solve(args)
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        on_gpu = a.backend == "hip" and a.transport == "rccl"
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if on_gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    pts = (N + 1) ** 3
    value = pts * a.timesteps * a.steps / elapsed / 1e6
    base = presets.BASELINE_MPTS.get(N, presets.BASELINE_MPTS[512])
    golden = presets.GOLDEN_LINF.get((N, a.timesteps)) if a.dtype == "fp64" else None
    dims = res["dims"]
    out = {
        "metric": METRIC.format(N=N, dtype=a.dtype),
        "value": round(value, 3),
        "unit": "Mpoints/s",
        "n_gpus": n_gpus,
        "steps": a.steps,
        "warmup": a.warmup,
        "tuning_solves": tuning,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if a.N else plan["scaling"],  # --N fixes the global grid
        "vs_baseline": round(value / base, 3),
        "dtype": a.dtype,
        "scheme": res.get("scheme", a.scheme),
        "math": res.get("math", a.math),
        "data": "synthetic (analytic initial condition u=sin(2pi x/Lx)sin(pi y/Ly)sin(pi z/Lz))",
        "config": {
            "model": f"wave3d {a.scheme} 7-point, N={N}^3, L=pi, T=1, timesteps={a.timesteps}",
            "global_batch": 1,
            "seq_len": N + 1,
            "parallelism": f"dd{dims[0]}x{dims[1]}x{dims[2]}-{res['kernel']}"
                           + ("" if n_gpus == 1 else f"-{res['transport']}"),
            "baseline_config": a.config or (None if a.N else plan["config"]),
            "N": N,
            "timesteps": a.timesteps,
            "dims": dims,
            "kernel": res["kernel"],
            "overlap": bool(res["overlap"]),  # effective (off when there is no remote halo)
            "overlap_mode": res.get("overlap_mode"),
            "overlap_order": res.get("overlap_order"),  # beside | shells_first (with overlap on)
            "overlap_trial_ms": list(res.get("overlap_trial_ms", (0, 0, 0))),  # best of two per arm
            "overlap_trials_ms": list(res.get("overlap_trials_ms", (0,) * 6)),
            "model_link": a.model_link or None,  # rehearsal link model (GBPS[,LAT_US]), None = real links
            "transport": res["transport"],
            "hip_graph": bool(res.get("graph", False)),
            "fill_hbm": a.fill_hbm or None,
            "device_bytes_per_gpu": C.memory_plan(args, n_gpus)["bytes_per_rank"]
                                     if a.backend == "hip" else None,
        },
        # ranks the halo communicator spans as RCCL reports them (ncclCommCount), None without one
        "rccl_nranks": res["comm_size"] if res["transport"] == "rccl" else None,
        # CTA budget the halo communicator was created with (0 = RCCL's own; rccl_transport.hpp)
        "rccl_max_ctas": res.get("rccl_max_ctas") if res["transport"] == "rccl" else None,
        # halo messages checked at setup with position-encoded patterns (hip_solver.hip)
        "halo_checked": res.get("halo_checked", 0),
        "launch": "self" if os.environ.get("WAVE3D_SELF_LAUNCH") else ("torchrun" if world > 1 else "single"),
        "linf_abs": res["linf_abs"],
        "linf_final_layer": res["timesteps"],
        "linf_golden": golden,
        "linf_ok": None if golden is None else f"{res['linf_abs']:.6g}" == f"{golden:.6g}",
        "courant": round(prob.courant, 4),
        "solver_ms_per_step": round(sum(res["solve_ms"]) / max(1, len(res["solve_ms"])), 4),
        # the reference's timer breakdown of the last solve, max over ranks (mpi_new.cpp:368-371)
        "timers_ms": {k: round(res[k], 4) for k in ("loop_ms", "exchange_ms", "comm_ms", "error_ms", "total_ms")},
        "baseline_mpts": base,
    }
    # explicit teardown while HIP and the process group are alive: the session (which keeps the
    # transport alive) first, then the transport (ncclCommDestroy), then the torch group
    del sess
    import gc
    gc.collect()
    want_ref = a.fp64_ref == "on" or (a.dtype == "fp32" and a.fp64_ref == "auto" and not a.fill_hbm)
    if want_ref:
        # the fp64 L-inf of the same N, K and decomposition (config 5 compares
        # against its own fp64 run), after the timed region and after the fp32 session is freed.
        # auto skips it with --fill-hbm (N is sized to the fp32 footprint, fp64 needs twice that)
        # and when the fp64 levels do not fit the free HBM; a failed reference solve leaves
        # linf_fp64_ref null — the timed result is printed either way.
        out["linf_fp64_ref"] = None
        p64 = wave3d.WaveProblem(N, timesteps=a.timesteps, dtype="fp64", math=presets.default_math(a.backend, "fp64"))
        try:
            s64 = wave3d.WaveSolver(p64, a.backend, transport=transport, Np=n_gpus, kernel="auto", dims=dims,
                                    overlap="off" if a.no_overlap else a.overlap,
                                    device=(torch.cuda.current_device() if a.backend == "hip" else None))
            need = C.memory_plan(s64.args(), n_gpus)["bytes_per_rank"] if a.backend == "hip" else 0
            free = torch.cuda.mem_get_info()[0] if a.backend == "hip" else 1 << 62
            fits = torch.tensor([1.0 if need < 0.95 * free else 0.0])
            if world > 1:  # every rank runs the reference solve, or none does
                fits = fits.cuda() if a.backend == "hip" and a.transport == "rccl" else fits
                dist.all_reduce(fits, op=dist.ReduceOp.MIN)
            if float(fits.item()) < 1.0:
                out["linf_fp64_ref_skipped"] = f"fp64 levels need {need / 1e9:.1f} GB, {free / 1e9:.1f} GB free"
            else:
                r64 = s64.run()
                out["linf_fp64_ref"] = r64.linf_abs
                out["linf_fp64_ref_kernel"] = r64.kernel
                out["linf_vs_fp64"] = round(out["linf_abs"] / r64.linf_abs, 3) if r64.linf_abs > 0 else None
            del s64
        except Exception as e:  # noqa: BLE001 — the reference is an extra, never the result
            # ... on one rank; with several, a rank that failed inside the solve would leave its
            # peers waiting in the exchange until the launcher's timeout: fail the job at once
            if world > 1:
                raise
            out["linf_fp64_ref_skipped"] = f"reference solve failed: {e}"[:300]
        gc.collect()
    if rank == 0:
        print(json.dumps(out), flush=True)
    transport = None
    gc.collect()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv: list[str], timeout: float) -> int:
    """Run this script as `n` ranks (children with torchrun's env: RANK, WORLD_SIZE,
    LOCAL_RANK, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) and relay rank 0's stdout.
    The parent never imports torch or touches a GPU. The first rank to fail (or the timeout)
    ends the job: the other ranks are terminated at once instead of waiting in a collective,
    and the exit status is the failed rank's. The ranks run in their own sessions (a rank's
    process group is killed as a whole), so they never outlive this launcher: SIGINT / SIGTERM
    and any exit path stop them, and each rank gets SIGKILL from the kernel if the launcher
    itself dies (PR_SET_PDEATHSIG)."""
    import signal
    import subprocess
    import threading

    def die_with_parent():  # runs in the child between fork and exec
        try:
            import ctypes

            libc = ctypes.CDLL(None, use_errno=True)
            libc.prctl(1, signal.SIGKILL, 0, 0, 0)  # PR_SET_PDEATHSIG
        except Exception:  # noqa: BLE001 — best effort (non-Linux)
            pass

    port = _free_port()
    procs = []

    def relay():
        for line in procs[0].stdout:
            sys.stdout.write(line)
            sys.stdout.flush()

    def stop_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        t_end = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()

    def on_signal(signum, _frame):
        raise KeyboardInterrupt(f"signal {signum}")

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGINT, signal.SIGTERM)}
    t0 = time.time()
    rc = 0
    th = None
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r),
                       LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=str(port), WAVE3D_SELF_LAUNCH="1")
            procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env,
                                          stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                          start_new_session=True, text=True, preexec_fn=die_with_parent))
        th = threading.Thread(target=relay, daemon=True)
        th.start()
        while True:
            codes = [p.poll() for p in procs]
            failed = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if failed:
                r, rc = failed[0]
                print(f"bench: rank {r} exited with status {rc}; stopping the other ranks", file=sys.stderr)
                break
            if all(c == 0 for c in codes):
                break
            if time.time() - t0 > timeout:
                print(f"bench: ranks still running after {timeout:.0f} s; stopping them", file=sys.stderr)
                rc = 124
                break
            time.sleep(0.05)
    except KeyboardInterrupt as e:
        print(f"bench: interrupted ({e}); stopping the ranks", file=sys.stderr)
        rc = 130
    finally:
        stop_all()  # no-op for ranks that already exited
        for s, h in old.items():
            signal.signal(s, h)
    if th is not None:
        th.join(timeout=5)
    return rc if rc > 0 else (1 if rc < 0 else 0)


if __name__ == "__main__":
    sys.exit(main())
