"""Host sanitizers: the OpenMP oracle built with ASan + UBSan runs a
multi-rank solve, a checkpoint/resume cycle and a fault-injection abort without reports;
built with TSan against LLVM's libomp + the Archer OMPT tool (which makes OpenMP
synchronisation visible to TSan) its threaded paths run race-free, while a negative control
with the reference's unsynchronised running maximum (hybrid_new.cpp:281-291, Appendix B4) is
reported. (Device-side ASan / xnack builds are not available on the MI355X pool.)"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "3d-wave-equation-mpi-cuda_amd")
BIN = os.path.join(PKG, "build", "san", "wave3d_cpu_address_undefined")
TSAN_BIN = os.path.join(PKG, "build", "san", "wave3d_cpu_tsan")
RACY_BIN = os.path.join(PKG, "build", "san", "racy_max_tsan")
ARCHER = "/opt/rocm/lib/llvm/lib/libarcher.so"

pytestmark = pytest.mark.slow


@pytest.fixture(scope="module")
def san_prog():
    r = subprocess.run(["make", "-C", PKG, "sanitize", "SAN=address,undefined"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return BIN


def _run(prog, args, tmp_path, code=0):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="2")
    r = subprocess.run([prog] + args + ["--format", "none", "--quiet"], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=300)
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == code, r.stderr[-2000:]
    return r


def test_asan_ubsan_multirank_checkpoint_fault(san_prog, tmp_path):
    base = ["22", "2", "1.3", "pi", "2.1", "1", "9", "--ic", "shifted"]
    _run(san_prog, base + ["--ranks", "4", "--dims", "1,2,2"], tmp_path)
    ck = str(tmp_path / "ck")
    os.makedirs(ck)
    _run(san_prog, base + ["--ranks", "2", "--checkpoint-every", "4", "--checkpoint-dir", ck], tmp_path)
    _run(san_prog, base + ["--ranks", "2", "--resume", ck], tmp_path)
    _run(san_prog, base + ["--ranks", "2", "--fault", "nan:1:3", "--check-every", "1"], tmp_path, code=3)


@pytest.fixture(scope="module")
def tsan_progs():
    if not os.path.exists(ARCHER):
        pytest.skip("LLVM Archer (libarcher.so) not installed")
    r = subprocess.run(["make", "-C", PKG, "tsan"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return TSAN_BIN, RACY_BIN


def _run_tsan(prog, args, cwd):
    env = dict(os.environ, OMP_TOOL_LIBRARIES=ARCHER,
               TSAN_OPTIONS="ignore_noninstrumented_modules=1:halt_on_error=0")
    return subprocess.run([prog] + args, cwd=cwd, env=env, capture_output=True, text=True,
                          timeout=600)


def test_tsan_archer_openmp_paths_race_free(tsan_progs, tmp_path):
    prog, _ = tsan_progs
    base = ["20", "4", "1.3", "pi", "2.1", "1", "8", "--ic", "shifted", "--format", "none", "--quiet"]
    ck = str(tmp_path / "ck")
    os.makedirs(ck)
    for extra in ([], ["--ranks", "2", "--threads", "2"], ["--ranks", "4", "--dims", "1,2,2"],
                  ["--ranks", "2", "--checkpoint-every", "3", "--checkpoint-dir", ck],
                  ["--ranks", "2", "--resume", ck]):
        r = _run_tsan(prog, base + extra, tmp_path)
        assert "ThreadSanitizer" not in r.stderr, (extra, r.stderr[-3000:])
        assert r.returncode == 0, (extra, r.stderr[-2000:])


def test_tsan_archer_flags_reference_race(tsan_progs, tmp_path):
    """The detector is live: the reference's racy max pattern is reported."""
    _, racy = tsan_progs
    r = _run_tsan(racy, [], tmp_path)
    assert "WARNING: ThreadSanitizer: data race" in r.stderr
    assert "racy_max.cpp" in r.stderr
