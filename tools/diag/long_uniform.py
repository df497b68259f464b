"""Stats breakdown of the long kernel's first sweep from uniform starts
(tests/test_gpu_long_kernel.py::test_long_uniform_starts_background_picks cases)."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np
from conftest import init_positions, make_dataset
from gibbssampling_amd import Context

lib = sys.argv[1] if len(sys.argv) > 1 else None
print("lib", lib)
ctx = Context(0, lib_path=lib, tuning={"dna_mode": 1, "long_mode": 1})
for W, L, ragged in [(15, 500, False), (12, 420, True)]:
    for N in (900, 20000):
        codes, offsets = make_dataset(N, L, W, b"ACGT", seed=40 + W, ragged=ragged, planted=False)
        pos = init_positions(offsets, W, 41 + W)
        u = np.random.default_rng(42 + W).random(N)
        ctx.set_sequences(codes, offsets, b"ACGT")
        s0 = ctx.stats()
        gpos, _ = ctx.motif_sweep(W, 1e-4, 1.0, pos, u)
        s1 = ctx.stats()
        d = {k: s1[k] - s0[k] for k in s1 if s1[k] != s0[k]}
        print(W, L, ragged, N, ctx.sweep_kernel_name(), "bg frac", round(float((gpos == -1).mean()), 3), d, flush=True)
