"""Init-time halo self-test (hip_solver.hip halo_self_test, hip_selftest.hip).

Every run that moves halos first sends position-encoded patterns through its real plan and
transport and checks every delivered cell on the device. These tests run it on the plans of
every decomposition shape and kernel family (single-step faces, two- and three-layer deep
halos with seam alias planes and y/z box rounds) and check that a corrupted delivery fails the
run at setup, naming the rank, peer and tag, within seconds."""
import json
import subprocess
import time

import pytest

pytestmark = pytest.mark.gpu

ARGS = ["40", "1", "pi", "pi", "pi", "1", "12"]

CASES = [
    # (dims, kernel, dtype, a tag the plan delivers to rank 1, deep-halo plan)
    ("2,1,1", "march2", "fp64", 1, "direct"),
    ("2,2,2", "march2", "fp64", 4, "direct"),
    ("1,2,2", "march2", "fp64", 5, "direct"),
    ("2,1,1", "tb2", "fp64", 11, "rounds"),
    ("2,2,2", "tb2", "fp64", 61, "rounds"),
    ("1,2,2", "tb2", "fp64", 32, "rounds"),
    ("4,1,1", "tb3", "fp64", 13, "rounds"),
    ("2,2,2", "tb3", "fp32", 63, "rounds"),
    ("1,2,2", "tb3", "fp32", 31, "rounds"),
    # --halo direct (default): x faces as whole planes in place (the x round's tags); edges, corners
    # and y/z faces packed, tag = 200 + 4 * direction + level, direction = 9(dx+1)+3(dy+1)+(dz+1)
    ("2,1,1", "tb2", "fp64", 11, "direct"),    # x face planes, in place (as the x round)
    ("2,1,1", "tb2", "fp64", 22, "direct"),    # seam alias plane from the first x-rank
    ("2,2,2", "tb2", "fp64", 296, "direct"),   # corner (+1,+1,-1), level A
    ("1,2,2", "tb3", "fp32", 261, "direct"),   # y/z edge (0,+1,-1), level B, x ghosts by wrap
    ("2,2,2", "tb3", "fp64", 226, "direct"),   # alias A corner (-1,+1,-1)
    ("2,2,2", "tb3", "fp64", 227, "direct"),   # alias B corner (-1,+1,-1)
    ("4,1,1", "tb3r1w8", "fp64", 13, "direct"),   # x face planes of the B level
    # the default leapfrog kernel (tb4: 4-deep A halos, 3-deep B halos, alias planes of A and B)
    ("2,2,2", "tb4", "fp64", 296, "direct"),   # depth-4 corner (+1,+1,-1), level A
    ("2,2,2", "tb4", "fp64", 227, "direct"),   # alias B corner (-1,+1,-1)
    ("2,1,1", "tb4", "fp64", 24, "direct"),    # seam alias plane of B, to the last x-rank
    ("1,2,2", "tb4", "fp32", 261, "direct"),   # y/z edge (0,+1,-1), level B, x ghosts by wrap
]


def _run(gpu_prog, dims, kernel, dtype, extra=(), halo="direct"):
    P = 1
    for d in dims.split(","):
        P *= int(d)
    cmd = [gpu_prog] + ARGS + ["--ranks", str(P), "--dims", dims, "--kernel", kernel, "--dtype", dtype,
                               "--halo", halo, "--json", "--quiet", "--format", "none"] + list(extra)
    t0 = time.time()
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    return out, time.time() - t0


@pytest.mark.parametrize("dims,kernel,dtype,tag,halo", CASES)
def test_halo_selftest_passes(gpu_prog, dims, kernel, dtype, tag, halo):
    out, _ = _run(gpu_prog, dims, kernel, dtype, halo=halo)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert r["halo_checked"] > 0 and r["kernel"].startswith(kernel[:3])


@pytest.mark.parametrize("dims,kernel,dtype,tag,halo", CASES)
def test_halo_selftest_names_corrupted_tag(gpu_prog, dims, kernel, dtype, tag, halo):
    out, dt = _run(gpu_prog, dims, kernel, dtype, ["--fault", f"corrupt_tag:1:{tag}"], halo=halo)
    assert out.returncode != 0
    assert "halo self-test failed" in out.stderr, out.stderr[-2000:]
    assert f"rank 1: message from peer" in out.stderr and f" tag {tag} " in out.stderr, out.stderr[-2000:]
    assert dt < 60


def test_halo_selftest_can_be_skipped(gpu_prog):
    out, _ = _run(gpu_prog, "2,1,1", "tb2", "fp64", ["--no-halo-check", "--fault", "corrupt_tag:1:11"])
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert r["halo_checked"] == 0


MIRROR = [("2,2,2", "tb2", "fp64"), ("1,2,2", "tb2", "fp64"), ("2,2,2", "tb3", "fp64"), ("1,2,2", "tb3", "fp32"),
          ("2,2,2", "march2", "fp64"), ("1,2,2", "march2", "fp64"), ("2,1,1", "tb3", "fp64"),
          # the leapfrog default since round 4: 4-deep halos, seam alias planes of A and B
          ("2,2,2", "tb4", "fp64"), ("1,2,2", "tb4", "fp32"), ("2,1,1", "tb4", "fp64")]


@pytest.mark.parametrize("dims,kernel,dtype", MIRROR)
@pytest.mark.parametrize("overlap", ["on", "off"])
@pytest.mark.parametrize("halo", ["direct", "rounds"])
def test_rccl_mirror_every_message_shape(gpu_prog, cpu_prog, dims, kernel, dtype, overlap, halo):
    """--rccl-mirror: every halo message of the multi-GPU plan (x planes, seam alias planes,
    y/z box rounds, faces) and the error-key allreduce also run through a 1-rank RCCL
    communicator and are compared bitwise on the device with the loopback copy; the per-layer
    errors equal the OpenMP oracle's (same decomposition)."""
    out, _ = _run(gpu_prog, dims, kernel, dtype, ["--rccl-mirror", "--overlap", overlap, "--repeat", "2"], halo=halo)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert r["rccl_mirror_msgs"] > 0 and r["halo_checked"] > 0 and r["overlap"] == (overlap == "on")
    P = 1
    for d in dims.split(","):
        P *= int(d)
    ref = subprocess.run([cpu_prog] + ARGS + ["--ranks", str(P), "--dims", dims, "--dtype", dtype, "--json",
                                              "--quiet", "--format", "none", "--threads", "4"],
                         capture_output=True, text=True, timeout=120)
    o = json.loads([l for l in ref.stdout.splitlines() if l.startswith("{")][0])
    assert r["linf_abs"] == o["linf_abs"] and r["max_rel_final"] == o["max_rel_final"]


def test_overlap_auto_trials_then_keeps_the_faster(gpu_prog):
    """--overlap auto (the default): solve 1 warms up, solves 2-7 run the three arms twice each
    (overlapped with the shells beside the interior / not / overlapped with the shells first),
    later solves use the arm with the shortest best-of-two (max-over-ranks) time; the JSON records
    every trial, the best per arm and the order kept."""
    out, _ = _run(gpu_prog, "2,2,2", "tb4", "fp64", ["--repeat", "8"])
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    on, off, first = r["overlap_trial_ms"]
    trials = r["overlap_trials_ms"]
    assert r["overlap_mode"] == "auto" and len(trials) == 6 and min(trials) > 0
    assert on == min(trials[0], trials[3]) and off == min(trials[1], trials[4]) and first == min(trials[2], trials[5])
    best = min(on, off, first)  # ties keep the earlier arm
    assert r["overlap_order_run"] == r["overlap_order"]
    if on == best:
        assert r["overlap"] and r["overlap_order"] == "beside"
    elif off == best:
        assert not r["overlap"]
    else:
        assert r["overlap"] and r["overlap_order"] == "shells_first"


@pytest.mark.parametrize("graph", ["on", "auto"])
def test_overlap_auto_graph_replays_the_reported_order(gpu_prog, graph):
    """--overlap auto with captured graphs (--graph on): every change of arm — the overlap on/off
    state or only the shell order — drops the captured graph, so the order that actually runs
    (recorded when the layers are enqueued, i.e. at capture) is the order reported, at every
    solve count through the trials and after them."""
    for repeat in (3, 4, 7, 9):
        out, _ = _run(gpu_prog, "2,1,1", "tb4", "fp64", ["--repeat", str(repeat), "--graph", graph])
        assert out.returncode == 0, out.stderr[-2000:]
        r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
        assert r["overlap_mode"] == "auto"
        assert r["overlap_order_run"] == r["overlap_order"], (repeat, r["overlap_order_run"], r["overlap_order"])
