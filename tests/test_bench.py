"""bench.py output contract: one JSON line with the driver's fields, the BASELINE.json metric,
and an L-inf that equals the reference golden for the config it ran."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
          "scaling", "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(extra, nproc=1, timeout=300, self_launch=False):
    if self_launch:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(nproc)] + extra
    elif nproc == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + extra
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()),
               os.path.join(ROOT, "bench.py"), "--gpus", str(nproc)] + extra
    out = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, timeout=timeout)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def _check(r, n, steps, warmup):
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        metric = json.load(f)["metric"]
    assert FIELDS <= set(r)
    N = r["config"]["N"]
    # BASELINE.json's metric, stating the N that actually ran (identical at N=512 fp64)
    assert r["metric"] == metric.replace("N=512³", f"N={N}³") and r["unit"] == "Mpoints/s"
    assert r["higher_is_better"] is True
    assert r["n_gpus"] == n and r["steps"] == steps and r["warmup"] == warmup
    assert r["value"] > 0 and r["ms_per_step"] > 0 and r["dtype"] == "fp64"
    cfg = r["config"]
    pts = (cfg["N"] + 1) ** 3 * cfg["timesteps"]
    # value = whole-job points per second over the timed solves (ms_per_step is one solve)
    assert r["value"] == pytest.approx(pts / (r["ms_per_step"] * 1e3), rel=1e-3)


def test_bench_cpu_single_process():
    r = _bench(["--backend", "cpu", "--N", "32", "--timesteps", "20", "--steps", "1", "--warmup", "0"])
    _check(r, 1, 1, 0)
    assert f"{r['linf_abs']:.6g}" == "0.000175963"  # golden N=32 K=20


def test_bench_cpu_two_ranks_gloo():
    r = _bench(["--backend", "cpu", "--N", "32", "--timesteps", "20", "--steps", "1", "--warmup", "0"],
               nproc=2)
    _check(r, 2, 1, 0)
    assert r["scaling"] == "strong"  # global N fixed by --N
    assert f"{r['linf_abs']:.6g}" == "0.000175963"
    assert r["tuning_solves"] == 0  # no overlap trials on the CPU backend


@pytest.mark.parametrize("sig", ["SIGTERM", "SIGKILL"])
def test_bench_self_launch_ranks_die_with_launcher(sig):
    """ranks of a self-launched job (own sessions) never outlive the launcher. SIGTERM:
    the launcher's handler stops every rank's process group; SIGKILL (no handler runs): the
    kernel kills each rank (PR_SET_PDEATHSIG)."""
    import signal
    import time

    import psutil

    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "cpu", "--N", "96",
           "--timesteps", "400", "--steps", "50", "--warmup", "0"]
    p = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        kids, t_end = [], time.time() + 60
        while time.time() < t_end and len(kids) < 2:
            kids = psutil.Process(p.pid).children()
            time.sleep(0.1)
        assert len(kids) == 2
        time.sleep(3)  # the ranks are up and solving
        assert all(k.is_running() for k in kids)
        os.kill(p.pid, getattr(signal, sig))
        p.wait(timeout=60)
        _, alive = psutil.wait_procs(kids, timeout=30)
        assert not alive, f"ranks outlived the launcher: {[k.pid for k in alive]}"
    finally:
        if p.poll() is None:
            p.kill()


@pytest.mark.gpu
def test_bench_gpu_default_config_short():
    r = _bench(["--steps", "1", "--warmup", "1"])
    _check(r, 1, 1, 1)
    assert r["scaling"] == "weak" and r["config"]["N"] == 512 and r["config"]["timesteps"] == 100
    assert r["math"] == "fma" and r["config"]["kernel"] == "tb4"  # the GPU default (presets)
    assert f"{r['linf_abs']:.6g}" == "6.03381e-07"  # golden N=512 K=100
    assert r["linf_golden"] == 6.03381e-07 and r["linf_ok"] is True
    assert r["config"]["dims"] == [1, 1, 1] and r["config"]["overlap"] is False  # no remote halo
    assert r["config"]["baseline_config"] == "gpu512" and r["rccl_nranks"] is None


def test_bench_plan_maps_gpu_counts_to_baseline_configs(C):
    from wave3d.models import presets

    assert presets.bench_plan(1) == dict(N=512, dims=None, scaling="weak", config="gpu512",
                                         golden=6.03381e-07)
    p2, p4, p8 = presets.bench_plan(2), presets.bench_plan(4), presets.bench_plan(8)
    assert (p2["N"], p2["dims"], p2["golden"]) == (512, [2, 1, 1], 6.03381e-07)
    assert (p4["N"], p4["dims"], p4["golden"]) == (1024, [2, 2, 1], 8.04265e-08)
    assert (p8["N"], p8["dims"], p8["golden"]) == (1024, [2, 2, 2], 8.04265e-08)
    assert p8["scaling"] == "weak" and p2["scaling"] == "strong"
    assert C.dims_create(4, [0, 0, 0]) == p4["dims"] and C.dims_create(8, [0, 0, 0]) == p8["dims"]


@pytest.mark.gpu
@pytest.mark.parametrize("n,N,dims,golden", [(2, 512, [2, 1, 1], 6.03381e-07), (4, 1024, [2, 2, 1], 8.04265e-08),
                                             (8, 1024, [2, 2, 2], 8.04265e-08)])
def test_bench_gpu_multirank_plan_staged(n, N, dims, golden):
    """The multi-GPU benchmark path end to end with n processes on one MI355X (staged device
    transport; RCCL refuses duplicate GPUs): each n runs its BASELINE config and decomposition
    at the benchmark's K=100 and must reproduce the reference's golden L-inf; the halo plan is
    verified at setup (halo_checked) and --overlap auto records both trial times."""
    r = _bench(["--steps", "1", "--warmup", "2", "--transport", "staged", "--shared-device"], nproc=n,
               timeout=900)
    assert r["n_gpus"] == n and r["config"]["N"] == N and r["config"]["dims"] == dims
    assert r["config"]["transport"] == "staged.gloo" and r["rccl_nranks"] is None
    assert r["config"]["timesteps"] == 100 and r["linf_golden"] == golden and r["linf_ok"] is True
    assert r["halo_checked"] > 0 and r["value"] > 0
    assert r["config"]["overlap_mode"] == "auto" and min(r["config"]["overlap_trial_ms"]) > 0
    assert r["warmup"] == 2 and r["tuning_solves"] == 5  # trial solves 3-7 ran untimed
    assert r["timers_ms"]["exchange_ms"] > 0 and r["timers_ms"]["comm_ms"] > 0


@pytest.mark.gpu
def test_bench_gpu_model_link_rehearsal_records_the_arms():
    """The 8-GPU bench shape rehearsed on one MI355X with an xGMI-like link cost (--model-link
    50,5: every exchange also waits its busiest link's bytes at 50 GB/s + 5 us): 8 processes,
    N=1024 on 2x2x2 at the golden L-inf; the JSON carries every --overlap auto trial, the arm kept
    (overlap / overlap_order agree with the fastest best-of-two, ties to the earlier arm), the
    link model and the RCCL CTA budget field (None without RCCL)."""
    r = _bench(["--steps", "1", "--warmup", "7", "--transport", "staged", "--shared-device",
                "--model-link", "50,5"], nproc=8, timeout=900)
    c = r["config"]
    assert c["dims"] == [2, 2, 2] and r["linf_ok"] is True and c["model_link"] == "50,5"
    trials, (on, off, first) = c["overlap_trials_ms"], c["overlap_trial_ms"]
    assert len(trials) == 6 and min(trials) > 0
    assert on == min(trials[0], trials[3]) and off == min(trials[1], trials[4]) and first == min(trials[2], trials[5])
    best = min(on, off, first)
    kept = "beside" if on == best else ("none" if off == best else "shells_first")
    assert c["overlap_order"] == kept and c["overlap"] == (kept != "none")
    assert "rccl_max_ctas" in r and r["rccl_max_ctas"] is None


@pytest.mark.gpu
@pytest.mark.parametrize("scheme,linf", [("leapfrog", "4.47035e-06"), ("auto", "1.3113e-06")])
def test_bench_gpu_fp32_two_ranks_staged(scheme, linf):
    """fp32 runs the three-layer sweep (tb3, 3-deep halos) through the multi-process bench path:
    2 processes on one MI355X, staged transport, N=512 on 2x1x1 slabs, K=100 (stable): the fp32
    L-inf of the single-GPU run (leapfrog 4.47035e-06, profiles/fp32_accuracy_r2.txt; the fp32
    default, the increment form, 1.3113e-06), and the fp64 L-inf of the same run (the golden)."""
    r = _bench(["--steps", "1", "--warmup", "0", "--dtype", "fp32", "--transport", "staged",
                "--shared-device", "--overlap", "on", "--scheme", scheme, "--math", "exact"], nproc=2, timeout=600)
    assert r["dtype"] == "fp32" and r["n_gpus"] == 2 and r["config"]["dims"] == [2, 1, 1]
    # the leapfrog runs four layers per sweep (tb4), the increment form three (tb3)
    assert r["config"]["kernel"] == ("tb3" if scheme == "auto" else "tb4") and r["config"]["overlap"] is True
    assert r["scheme"] == ("delta" if scheme == "auto" else scheme)
    assert f"{r['linf_abs']:.6g}" == linf
    assert f"{r['linf_fp64_ref']:.6g}" == "6.03381e-07"


def test_bench_named_config_cpu128():
    """--config runs a BASELINE config by name (config 1: N=128 fp64 K=20 on the CPU backend)."""
    r = _bench(["--backend", "cpu", "--config", "cpu128", "--steps", "1", "--warmup", "0"])
    _check(r, 1, 1, 0)
    assert r["config"]["N"] == 128 and r["config"]["timesteps"] == 20
    assert r["config"]["baseline_config"] == "cpu128"
    assert f"{r['linf_abs']:.6g}" == "8.81051e-06" and r["linf_ok"] is True


def test_bench_self_launch_cpu_two_ranks():
    """`python bench.py --gpus 2` without torchrun spawns its own two ranks (the reference's
    one-command `mpirun -n Np`, README.txt:43) and relays rank 0's JSON line."""
    r = _bench(["--backend", "cpu", "--N", "32", "--timesteps", "20", "--steps", "1", "--warmup", "0"],
               nproc=2, self_launch=True)
    _check(r, 2, 1, 0)
    assert r["launch"] == "self" and r["config"]["dims"] == [2, 1, 1]
    assert f"{r['linf_abs']:.6g}" == "0.000175963" and r["linf_ok"] is True


def test_bench_self_launch_fails_fast():
    """One rank dying makes the self-launched job exit with that rank's status at once (the
    other ranks sit in a collective and are terminated instead of waiting for a timeout)."""
    import time

    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--backend", "cpu", "--N", "32",
           "--timesteps", "20", "--steps", "1", "--warmup", "0"]
    t0 = time.time()
    out = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, timeout=120,
                         env=dict(os.environ, WAVE3D_BENCH_FAIL_RANK="1"))
    assert out.returncode == 3, out.stderr[-2000:]
    assert "rank 1 exited with status 3" in out.stderr
    assert time.time() - t0 < 60


@pytest.mark.gpu
def test_bench_gpu_self_launch_two_ranks_staged():
    """The multi-GPU bench as one command: 2 self-launched ranks on one MI355X (staged
    transport), the BASELINE 2-GPU config (N=512, 2x1x1, K=100) at the golden L-inf, with the
    init-time halo self-test through the real plan."""
    r = _bench(["--steps", "1", "--warmup", "0", "--transport", "staged", "--shared-device"], nproc=2,
               timeout=600, self_launch=True)
    _check(r, 2, 1, 0)
    assert r["tuning_solves"] == 7  # overlap auto: warm-up + two trials of each of 3 arms, then timed
    assert r["launch"] == "self" and r["config"]["N"] == 512 and r["config"]["dims"] == [2, 1, 1]
    assert r["config"]["timesteps"] == 100 and r["linf_ok"] is True
    assert r["halo_checked"] > 0
