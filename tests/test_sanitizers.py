"""Host sanitizers: the OpenMP oracle built with ASan + UBSan runs a
multi-rank solve, a checkpoint/resume cycle and a fault-injection abort without reports.
(Device-side ASan / xnack builds are not available on the MI355X pool; TSan is not used on
the OpenMP paths because libgomp is not instrumented and reports its own barriers.)"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "3d-wave-equation-mpi-cuda_amd")
BIN = os.path.join(PKG, "build", "san", "wave3d_cpu_address_undefined")

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
