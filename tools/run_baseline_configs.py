#!/usr/bin/env python3
"""Run the BASELINE.json configurations that fit this machine and print one table.

    python tools/run_baseline_configs.py [--only NAME ...] [--repeat 3]

CPU configs run the OpenMP program; 1-GPU configs run in-process; multi-GPU configs are
launched with torch.distributed.run (one rank per GPU, RCCL) when enough GPUs are visible and
skipped otherwise. Each row: Mpoints/s, final-layer L-inf vs the reference golden.
"""
import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--simulate", action="store_true",
                    help="run multi-GPU configs that do not fit as simulated ranks on ONE GPU "
                         "(loopback halos, subdomains serialised: checks accuracy and "
                         "decomposition cost, NOT a scaling number; rows are marked 'sim')")
    ap.add_argument("--math", default="exact", choices=["exact", "fma"], help="the GPU configs' arithmetic")
    a = ap.parse_args()

    import wave3d
    from wave3d.models import presets

    ngpu = 0
    try:
        import torch

        ngpu = torch.cuda.device_count()
    except Exception:
        pass
    print(f"{'config':16s} {'backend':7s} {'Np':>3s} {'dims':9s} {'Mpts/s':>12s} {'L_inf abs':>13s} {'golden':>12s}")
    for name, cfg in presets.CONFIGS.items():
        if a.only and name not in a.only:
            continue
        p, be, Np, dims = cfg["problem"], cfg["backend"], cfg["Np"], cfg["dims"]
        if be == "hip":
            p.math = a.math
        golden = presets.GOLDEN_LINF.get((p.N, p.timesteps))
        sim = be == "hip" and Np > ngpu and a.simulate and ngpu >= 1
        if be == "hip" and Np > ngpu and not sim:
            print(f"{name:16s} {be:7s} {Np:3d} {'-':9s} {'skipped (needs %d GPUs)' % Np:>26s}")
            continue
        if be == "cpu" or Np == 1:
            r = wave3d.WaveSolver(p, be, Np=Np, dims=dims).run(repeat=a.repeat, warmup=1)
            mpts, linf, d = r.mpts_per_s_best, r.linf_abs, r.dims
        elif sim:
            # --overlap auto as bench.py: solves 2-7 time the arms (untimed warm-ups here)
            r = wave3d.WaveSolver(p, be, ranks=Np, dims=dims, overlap="auto").run(repeat=a.repeat, warmup=7)
            mpts, linf, d = r.mpts_per_s_best, r.linf_abs, r.dims
            be = "hip-sim"
        else:
            args = p.args(Np) + (["--dims", ",".join(map(str, dims))] if dims else []) + \
                ["--repeat", str(a.repeat), "--warmup", "1"]
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={Np}",
                   "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                   os.path.join(ROOT, "tools", "dist_solve.py"), "--backend", "hip", "--transport", "rccl",
                   "--"] + args
            out = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
            line = [l for l in out.stdout.splitlines() if l.startswith("RESULT ")]
            if out.returncode or not line:
                print(f"{name:16s} failed: {out.stderr[-500:]}")
                continue
            d0 = json.loads(line[0][7:])
            pts = (p.N + 1) ** 3 * p.timesteps
            mpts, linf, d = pts / (d0["total_ms"] * 1e3), d0["max_abs"][-1], d0["dims"]
        gs = f"{golden:.6g}" if golden else "-"
        print(f"{name:16s} {be:7s} {Np:3d} {'x'.join(map(str, d)):9s} {mpts:12.1f} {linf:13.6g} {gs:>12s}")


if __name__ == "__main__":
    main()
