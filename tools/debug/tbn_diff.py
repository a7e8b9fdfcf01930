"""Debug: one k_tbn<4> sweep on random fields vs the chained oracle; prints where O0/O1 differ."""
import sys
import torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from test_gpu_tb_kernels import _rand, _tables, _mask, _sl, COEF, TBN_CASES  # noqa: E402
from wave3d.ops import kernels, reference  # noqa: E402

DEV = "cuda"
for dtype in (torch.float64, torch.float32):
    for first in (False, True):
        for fma in (False, True):
            for case in (3,):
                (X, Y, Z), boxes, cdom, chunk = TBN_CASES[case]
                G = 4
                shape = (X + 2 * G, Y + 2 * G, Z + 2 * G)
                A, B = _rand(shape, dtype, 24), _rand(shape, dtype, 25)
                tx, ty, tz = _tables(max(shape), dtype, 26)
                c = 2.9e-4
                c4 = (3.1e-4, 2.9e-4, 2.7e-4, 2.6e-4) if not fma else ((3.1e-4 if first else c), c, c, c)
                ct4 = (-0.83, 0.47, 0.21, -0.66)
                dO0, dO1 = (torch.full(shape, v, dtype=dtype, device=DEV) for v in (-7.0, -9.0))
                errs = [kernels.new_err(1) for _ in range(4)]
                ei = (min(b[0] for b in boxes), max(b[1] for b in boxes))
                co = [(*COEF.values(), c4[q], ct4[q]) for q in range(4)]
                kernels.tbn_sweep(A.to(DEV), B.to(DEV), dO0, dO1, boxes, depth=4, first=first, cdom=cdom, err_i=ei,
                                  tx=tx.to(DEV), ty=ty.to(DEV), tz=tz.to(DEV), coefs=co, errs=errs, chunk=chunk, fma=fma)
                torch.cuda.synchronize()
                L = reference.chained_layers(A, B, 4, first=first, mask=_mask(shape, G, cdom), coefs=list(c4), **COEF)
                for name, g, e in (("O0", dO0.cpu(), L[2]), ("O1", dO1.cpu(), L[3])):
                    s = _sl(boxes[0], G)
                    d = (g[s].double() - e[s].double()).abs()
                    bad = (d > (1e-9 if dtype == torch.float64 else 1e-4)) | d.isnan()
                    idx = bad.nonzero()
                    print(f"{dtype} first={first} fma={fma} case={case} {name}: box {boxes[0]} bad {int(bad.sum())}/{bad.numel()}",
                          "first bad (i,j,k) rel box:", idx[:6].tolist(), "max", float(d[~d.isnan()].max()) if (~d.isnan()).any() else None)
                    if bad.any():
                        # per-i and per-j and per-k counts
                        print("   bad per i:", bad.sum(dim=(1, 2)).tolist())
                        print("   bad per j:", bad.sum(dim=(0, 2)).tolist())
                        print("   bad per k (first 70):", bad.sum(dim=(0, 1)).tolist()[:70])
