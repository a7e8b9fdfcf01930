"""Report parsing, golden data and small helpers."""
from .report import (GOLDEN_FINAL, GOLDEN_N32_K20, GOLDEN_SPOTS, fmt6,  # noqa: F401
                     parse_output)
