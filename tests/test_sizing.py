"""Device-memory planning (sizing.cpp) and small CLI knobs
(--graph, --fill-hbm, WAVE_LOG levels)."""
import os
import subprocess

import pytest

ARGS = ["512", "1", "pi", "pi", "pi", "1", "100"]


def test_layout_auto_is_temporal_blocking_on_dims_create(C):
    p1 = C.memory_plan(ARGS, 1)
    assert p1["tb"] and p1["ghost"] == 4 and p1["levels"] == 4  # fp64 auto = tb4, 4-level ring
    p8 = C.memory_plan(ARGS, 8)  # no override: MPI_Dims_create's 2x2x2, as the reference
    assert p8["tb"] and p8["dims"] == [0, 0, 0]
    s8 = C.memory_plan(ARGS + ["--dims", "8,1,1"], 8)  # x slabs on request
    assert s8["tb"] and s8["dims"] == [8, 1, 1]
    m = C.memory_plan(ARGS + ["--kernel", "march2"], 8)
    assert not m["tb"] and m["ghost"] == 1 and m["levels"] == 3 and m["dims"] == [0, 0, 0]
    y = C.memory_plan(ARGS + ["--dims", "2,2,2"], 8)  # temporal blocking with y/z halos
    assert y["tb"] and y["dims"] == [2, 2, 2]


def test_bytes_per_rank_matches_level_formula(C):
    # one rank, N=512 fp64, four-layer blocking (tb4): 4 levels of (513+8)^2 x
    # roundup(16+513+4, 16)
    sj = ((16 + 513 + 4 + 15) // 16) * 16
    level = (513 + 8) * (513 + 8) * sj * 8
    b = C.memory_plan(ARGS, 1)["bytes_per_rank"]
    assert 4 * level <= b < 4 * level * 1.01
    # fp32 halves the level size (rows padded to 32 elements); leapfrog also tb4: 4 levels, 4-deep
    p32 = C.memory_plan(ARGS + ["--dtype", "fp32", "--scheme", "leapfrog"], 1)
    assert p32["tb"] and p32["ghost"] == 4 and p32["levels"] == 4
    b32 = p32["bytes_per_rank"]
    assert 0.50 * b < b32 < 0.56 * b
    # the fp64 increment form: three-layer blocking (tb3, 4 levels, 3-deep ghosts)
    pd = C.memory_plan(ARGS + ["--scheme", "delta"], 1)
    assert pd["ghost"] == 3 and pd["levels"] == 4
    # the fp32 increment form: three-layer blocking (tb3, no tb4 increment form), 3-deep ghosts
    p32d = C.memory_plan(ARGS + ["--dtype", "fp32", "--scheme", "delta"], 1)
    assert p32d["ghost"] == 3 and p32d["levels"] == 4 and p32d["bytes_per_rank"] < b32
    assert C.memory_plan(ARGS, 8)["bytes_per_rank"] < b / 7


@pytest.mark.parametrize("extra,world", [([], 1), (["--dtype", "fp32"], 8),
                                         (["--kernel", "march2", "--dims", "2,2,2"], 8)])
def test_fill_hbm_is_tight(C, extra, world):
    budget = 0.9 * 288e9
    N = C.fill_hbm_N(ARGS + extra, world, budget)
    at = lambda n: C.memory_plan([str(n)] + ARGS[1:] + extra, world)["bytes_per_rank"]
    assert at(N) <= budget < at(N + 1)
    # 0.9 x 288e9 B holds ~1996^3 fp64 nodes with 4 levels (5 levels: ~1850^3); the
    # program takes the budget from hipMemGetInfo's total (288 GiB on an MI355X): ~2040^3
    assert N > 1950


def test_fill_hbm_survey_estimate(C):
    # 3 fp64 levels per GPU on 2x2x2 -> ~4,400^3 global
    N = C.fill_hbm_N(ARGS + ["--kernel", "march2", "--dims", "2,2,2"], 8, 0.9 * 288e9)
    assert 4300 <= N <= 4500


def test_cli_graph_and_fill_flags(C):
    C.parse(ARGS + ["--graph", "off"])
    C.parse(ARGS + ["--fill-hbm", "0.9"])
    with pytest.raises(Exception):
        C.parse(ARGS + ["--graph", "sometimes"])
    with pytest.raises(Exception):
        C.parse(ARGS + ["--fill-hbm", "1.5"])


def test_wave_log_levels(cpu_prog):
    env = dict(os.environ, WAVE_LOG="info")
    r = subprocess.run([cpu_prog, "12", "1", "pi", "pi", "pi", "1", "3", "--format", "none",
                        "--ranks", "2", "--quiet"], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0
    assert "wave3d[info] rank 0/2 dims 2x1x1" in r.stderr
    env["WAVE_LOG"] = "warn"
    r = subprocess.run([cpu_prog, "12", "1", "pi", "pi", "pi", "1", "3", "--format", "none",
                        "--quiet"], env=env, capture_output=True, text=True, timeout=60)
    assert "wave3d[info]" not in r.stderr
