#!/usr/bin/env python3
"""Print the measured device log2/exp2 errors (gs_fastmath_check) against the budget."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gibbssampling_amd import _native  # noqa: E402

ctx = _native.Context(0)
el, ee = ctx.fastmath_check()
print(f"log2 abs err {el:.3e} ({el / 2**-24:.2f} x 2^-24), budget {_native.LOG2_ERR_BUDGET:.3e}")
print(f"exp2 rel err {ee:.3e} ({ee / 2**-24:.2f} x 2^-24), budget {_native.EXP2_ERR_BUDGET:.3e}")
ctx.close()
