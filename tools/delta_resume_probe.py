"""Repeat the fp32 increment-form checkpoint/resume comparison and print where the layer maxima
differ (debug aid for tests/test_gpu_solver.py::test_delta_scheme_checkpoint_resume)."""
import sys
import tempfile

sys.path.insert(0, ".")
import wave3d  # noqa: E402


def solve(p, backend="hip", **kw):
    return wave3d.WaveSolver(p, backend, **kw).run()


def main():
    p = wave3d.WaveProblem(29, Lx=1.3, Ly="pi", Lz=2.0, timesteps=16, ic="shifted", dtype="fp32",
                           scheme="delta")
    ref = solve(p, backend="cpu", threads=4)
    for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        full = solve(p)
        with tempfile.TemporaryDirectory() as d:
            solve(p, checkpoint_every=6, checkpoint_dir=d)
            res = solve(p, resume=d)
        for name, r in (("full", full), ("resumed", res)):
            da = [q for q, (x, y) in enumerate(zip(r.max_abs, ref.max_abs)) if x != y]
            dr = [q for q, (x, y) in enumerate(zip(r.max_rel, ref.max_rel)) if x != y]
            if da or dr or rep == 0:
                print(rep, name, "abs differs at", da, "rel differs at", dr,
                      [(r.max_rel[q], ref.max_rel[q]) for q in dr][:3], flush=True)


if __name__ == "__main__":
    main()
