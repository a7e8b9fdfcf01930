"""Parsing of the reference-format output files and golden data.

The golden tables are the reference's own outputs captured by the survey (Appendix C):
the whole ``output_N32_Np8_MPI.txt`` error table and spot values at N=128/512/1024 plus
the phase-shifted initial condition.
"""
from __future__ import annotations

import re

_ERR = re.compile(r"max abs and rel errors on layer (\d+): (\S+) (\S+)")
_NUM = re.compile(r"numerical solution calculated in ([0-9.eE+-]+)\s*ms")


def parse_output(text: str) -> dict:
    """Parse an output_N*.txt file into {'layers': [(abs, rel)], 'numerical_ms': t, ...}."""
    layers = {}
    for m in _ERR.finditer(text):
        layers[int(m.group(1))] = (float(m.group(2)), float(m.group(3)))
    out = {"layers": [layers[k] for k in sorted(layers)], "raw_layers": {}}
    for m in _ERR.finditer(text):
        out["raw_layers"][int(m.group(1))] = (m.group(2), m.group(3))
    m = _NUM.search(text)
    if m:
        out["numerical_ms"] = float(m.group(1))
    for key, pat in (("init_ms", r"(?:grids initialized|initialization done) in ([0-9.]+)\s*ms"),
                     ("comm_ms", r"total MPI exchange time: ([0-9.eE+-]+)\s*ms"),
                     ("loop_ms", r"total loop time: ([0-9.eE+-]+)\s*ms")):
        mm = re.search(pat, text)
        if mm:
            out[key] = float(mm.group(1))
    return out


# Appendix C.1: `mpirun -n 8 mpi_new 32 1 pi pi pi 1 20` (identical for omp / mpi_sol /
# mpi_new / hybrid_* at P = 1, 2, 4, 8) — printed with default ostream precision.
GOLDEN_N32_K20 = [
    ("0", "0"),
    ("4.51206e-07", "4.53838e-07"),
    ("1.80449e-06", "1.81508e-06"),
    ("4.05882e-06", "4.09001e-06"),
    ("7.21249e-06", "7.284e-06"),
    ("1.12631e-05", "1.14042e-05"),
    ("1.62076e-05", "1.64602e-05"),
    ("2.20422e-05", "2.24634e-05"),
    ("2.87625e-05", "2.94321e-05"),
    ("3.63633e-05", "3.73818e-05"),
    ("4.48389e-05", "4.63243e-05"),
    ("5.41829e-05", "5.62857e-05"),
    ("6.4388e-05", "6.7304e-05"),
    ("7.54467e-05", "7.93753e-05"),
    ("8.73503e-05", "9.2518e-05"),
    ("0.00010009", "0.000106751"),
    ("0.000113656", "0.00012209"),
    ("0.000128037", "0.000138557"),
    ("0.000143223", "0.000156169"),
    ("0.000159203", "0.000174945"),
    ("0.000175963", "0.000194911"),
]

# Appendix C.2 spot values {(N, K, ic): {layer: (abs, rel)}} as printed (6 significant digits).
GOLDEN_SPOTS = {
    (128, 20, "ref"): {1: ("2.25895e-08", "2.9261e-07"), 10: ("2.24513e-06", "2.28846e-06"),
                       20: ("8.81051e-06", "1.247e-05")},
    (512, 100, "ref"): {1: ("6.12008e-11", "2.1262e-09"), 10: ("6.18154e-09", "2.99143e-06"),
                        100: ("6.03381e-07", "3.77041e-05")},
    (1024, 100, "ref"): {1: ("7.55696e-12", "4.68365e-09"), 50: ("2.04773e-08", "2.11704e-05"),
                         100: ("8.04265e-08", "0.000151774")},
    (32, 20, "shifted"): {1: ("4.49562e-07", "4.51292e-07"), 10: ("4.46755e-05", "4.57045e-05"),
                          20: ("0.000175322", "0.000190237")},
}

# BASELINE.md §3 (final-layer L-inf abs / max rel, 6 significant digits)
GOLDEN_FINAL = {
    (32, 20): ("0.000175963", "0.000194911"),
    (64, 20): ("4.22698e-05", "4.94014e-05"),
    (128, 20): ("8.81051e-06", "1.247e-05"),
    (256, 40): ("2.20262e-06", "1.07382e-05"),
    (512, 100): ("6.03381e-07", "3.77041e-05"),
    (1024, 100): ("8.04265e-08", "0.000151774"),
}


def fmt6(v: float) -> str:
    """C++ default ostream formatting of a double (%g with 6 significant digits)."""
    return "%g" % v
