"""Multi-process runs through torch.distributed.run (the launcher the benchmark uses).

CPU: OpenMP backend, gloo host transport, world 2/4/8.
GPU (marked): HIP backend with P processes sharing one MI355X through the staged device
transport (the reference's MPS-oversubscription test mode, P5), with and without the
interior/shell overlap; and the native RCCL transport in a single-rank world.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def torchrun(nproc, flags, args, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tools", "dist_solve.py")] + flags + ["--"] + args
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("RESULT ")]
    assert line, out.stdout[-2000:] + out.stderr[-2000:]
    return json.loads(line[0][7:])


ARGS = ["27", "1", "1.3", "pi", "2.1", "1", "11", "--ic", "shifted", "--threads", "1"]


@pytest.fixture(scope="module")
def single_cpu(C):
    return C.run(ARGS, "cpu", None, False, True)


@pytest.mark.parametrize("P", [2, 4, 8])
def test_cpu_gloo_matches_single_process(C, single_cpu, P):
    r = torchrun(P, ["--backend", "cpu", "--transport", "gloo"], ARGS)
    assert r["nprocs"] == P and r["transport"] == "torch.gloo"
    assert r["max_abs"] == single_cpu["max_abs"] and r["max_rel"] == single_cpu["max_rel"]


@pytest.mark.gpu
@pytest.mark.parametrize("P,overlap", [(2, True), (4, True), (8, True), (2, False), (4, False)])
def test_hip_multiprocess_shared_gpu(C, single_cpu, P, overlap):
    """Single-step kernel on the 3-D decomposition (2x2x2 at P=8), 6-face halos."""
    extra = ["--kernel", "march2"] + ([] if overlap else ["--no-overlap"])
    r = torchrun(P, ["--backend", "hip", "--transport", "staged", "--shared-device"], ARGS + extra)
    assert r["nprocs"] == P and r["transport"] == "staged.gloo"
    assert r["max_abs"] == single_cpu["max_abs"] and r["max_rel"] == single_cpu["max_rel"]


@pytest.mark.gpu
@pytest.mark.parametrize("P,kernel", [(2, "tb2r4"), (4, "tb2")])
def test_hip_multiprocess_temporal_blocking(C, single_cpu, P, kernel):
    r = torchrun(P, ["--backend", "hip", "--transport", "staged", "--shared-device"],
                 ARGS + ["--kernel", kernel, "--dims", f"{P},1,1"])
    assert r["dims"] == [P, 1, 1] and r["kernel"] == kernel
    assert r["max_abs"] == single_cpu["max_abs"] and r["max_rel"] == single_cpu["max_rel"]


@pytest.mark.gpu
@pytest.mark.parametrize("P,dims,kernel", [(8, "2,2,2", "auto"), (4, "1,2,2", "tb2r2w8")])
def test_hip_multiprocess_temporal_blocking_3d(C, single_cpu, P, dims, kernel):
    """Temporal blocking on the reference's 3-D block decomposition (6-face deep halos), P
    processes through the tag-less FIFO staged transport: the fp64 auto kernel (tb4) and tb2."""
    r = torchrun(P, ["--backend", "hip", "--transport", "staged", "--shared-device"],
                 ARGS + ["--dims", dims, "--kernel", kernel])
    assert r["dims"] == [int(x) for x in dims.split(",")]
    assert r["kernel"] == {"auto": "tb4"}.get(kernel, kernel)  # fp64 auto = tb4
    assert r["max_abs"] == single_cpu["max_abs"] and r["max_rel"] == single_cpu["max_rel"]


@pytest.mark.gpu
def test_rccl_transport_single_rank(C, single_cpu):
    r = torchrun(1, ["--backend", "hip", "--transport", "rccl"], ARGS)
    assert r["transport"] == "rccl" and r["comm_size"] == 1
    assert r["max_abs"] == single_cpu["max_abs"] and r["max_rel"] == single_cpu["max_rel"]


@pytest.mark.gpu
@pytest.mark.parametrize("kernel,overlap", [("march2", True), ("march2", False), ("tb2", True),
                                            ("tb2", False), ("tb3", True)])
def test_rccl_self_send(C, single_cpu, kernel, overlap):
    """--x-self-transport: the periodic x wrap of the one x rank travels as ncclSend/ncclRecv
    to itself (x planes, the deep temporal-blocking planes) instead of the fused local wrap,
    so the RCCL point-to-point path of the multi-GPU halo runs on a one-GPU lease; the
    per-layer errors must equal the OpenMP oracle's bit for bit."""
    extra = ["--kernel", kernel, "--x-self-transport"] + ([] if overlap else ["--no-overlap"])
    r = torchrun(1, ["--backend", "hip", "--transport", "rccl"], ARGS + extra)
    assert r["transport"] == "rccl" and r["comm_size"] == 1 and r["kernel"] == kernel
    assert r["overlap"] == overlap
    assert r["rccl_max_ctas"] == (C.rccl_max_ctas("auto") if overlap else 0)
    assert r["exchange_ms"] > 0  # halo messages were timed on the stream
    assert r["max_abs"] == single_cpu["max_abs"] and r["max_rel"] == single_cpu["max_rel"]



def test_rccl_cta_budget_follows_overlap(C, monkeypatch):
    """the halo communicator's CTA budget is RCCL's own (0) unless the interior
    sweep is known to run beside the exchange (overlap on: a cap). --overlap auto keeps RCCL's
    own: the budget is fixed for the communicator's life and the overlap-off arm is the expected
    winner on 2x2x2 blocks. WAVE3D_RCCL_MAX_CTAS overrides. Every run's JSON records the budget."""
    monkeypatch.delenv("WAVE3D_RCCL_MAX_CTAS", raising=False)
    assert C.rccl_max_ctas("off") == 0 and C.rccl_max_ctas("auto") == 0
    assert C.rccl_max_ctas("on") == 8
    monkeypatch.setenv("WAVE3D_RCCL_MAX_CTAS", "3")
    assert C.rccl_max_ctas("off") == 3 and C.rccl_max_ctas("auto") == 3
    monkeypatch.setenv("WAVE3D_RCCL_MAX_CTAS", "0")
    assert C.rccl_max_ctas("on") == 0


def test_watchdog_is_progress_based(C):
    """The transport watchdog (halo.cpp watch_until, used by RcclTransport::wait_stream) measures
    time since the device last made progress, not since the wait began: a wait that keeps
    progressing outlives the limit, a stalled one is aborted with a message naming the cause."""
    # progress for 0.6 s, done at 0.7 s, limit 0.3 s: never 0.3 s without progress -> no abort
    assert 0.69 < C.watchdog_probe(0.3, 0.7, 0.65) < 2.0
    # progress stalls at 0.1 s, never done: aborted ~0.3 s later
    with pytest.raises(Exception, match="no progress"):
        C.watchdog_probe(0.3, 100.0, 0.1)


def test_thread_ranks_fail_fast(C):
    """Thread-per-GPU ranks (`wave3d N 8 ...`): when one rank thread throws, the others — blocked
    in the RCCL watchdog loop, here with a 60 s limit — see the job abort flag and fail within a
    poll interval, naming the failed rank, instead of waiting out the watchdog."""
    out = C.abort_probe(4, 1, 0.2, 60.0)
    assert out[1][1] == "injected failure"
    for r in (0, 2, 3):
        t, err = out[r]
        assert "another rank failed" in err and "rank 1: injected failure" in err
        assert 0.15 < t < 5.0
    # the flag is cleared when the job ends: a later wait is unaffected
    assert 0.2 < C.watchdog_probe(5.0, 0.25, 0.25) < 2.0
