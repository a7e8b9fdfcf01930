#!/usr/bin/env python3
"""One rank of a distributed wave3d solve (launch with torch.distributed.run).

    python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 \\
        --master-port 29611 tools/dist_solve.py --backend hip --transport rccl -- 32 1 pi pi pi 1 20

--transport rccl   native RCCL halos, one GPU per rank (production path)
--transport staged device halos staged through gloo: several ranks may share one GPU
--transport gloo   host halos over gloo (OpenMP backend)
Rank 0 prints one JSON line with the per-layer errors and timings.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="hip", choices=["hip", "cpu"])
    ap.add_argument("--transport", default="rccl", choices=["rccl", "staged", "gloo"])
    ap.add_argument("--shared-device", action="store_true", help="all ranks on device 0")
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    args = [x for x in a.rest if x != "--"]

    import torch
    import torch.distributed as dist

    import wave3d
    from wave3d.parallel import dist as wdist

    C = wave3d.load_native()
    rank, world, local = wdist.env_rank()
    if a.backend == "hip":
        dev = 0 if a.shared_device else local % torch.cuda.device_count()
        torch.cuda.set_device(dev)
        args += ["--device", str(dev)]
    wdist.init_from_env("nccl" if a.transport == "rccl" else "gloo", force=True)
    mode = "auto"
    for q, x in enumerate(args):
        if x == "--no-overlap":
            mode = "off"
        elif x == "--overlap":
            mode = args[q + 1] if q + 1 < len(args) and args[q + 1] in ("on", "off", "auto") else "on"
    tr = wdist.make_transport(a.transport, a.backend, overlap=mode)
    r = C.run(args, a.backend, tr, False, rank == 0)
    if rank == 0:
        keep = ("N", "timesteps", "nprocs", "dims", "transport", "kernel", "max_abs", "max_rel",
                "total_ms", "loop_ms", "exchange_ms", "comm_ms", "overlap", "comm_size", "rccl_max_ctas",
                "solve_ms", "mpts_per_s_best",
                "aborted", "abort_layer", "resumed_from")
        print("RESULT " + json.dumps({k: r[k] for k in keep}), flush=True)
    dist.barrier()
    del tr
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
