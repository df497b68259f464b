import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from conftest import make_dataset
from gibbssampling_amd import Context
from gibbssampling_amd._native import GibbsError
for alpha, L, W in [(b"ACDEFGHIKLMNPQRSTVWY", 1500, 20), (b"ACDEFGHIKLMNPQRSTVWY", 2500, 20), (b"ACDEFGHIKLMNPQRSTVWY", 4000, 20),
                    (b"ACGT", 8000, 12), (b"ACGT", 12000, 12), (b"ACGT", 30000, 12)]:
    codes, offsets = make_dataset(6, L, W, alpha, seed=3)
    ctx = Context(0)
    ctx.set_sequences(codes, offsets, alpha)
    res = {}
    for name, f in [("starts0", lambda: ctx.random_starts(W, 1e-4, 1, 0)),
                    ("starts1", lambda: ctx.random_starts(W, 1e-4, 1, 1)),
                    ("sweep", lambda: ctx.motif_sweep(W, 1e-4, 1.0, np.zeros(6, np.int32), np.full(6, 0.5))),
                    ("motif_sampling", lambda: ctx.motif_sampling(W, 1e-4, 1.0, 5)),
                    ("site_sampling", lambda: ctx.site_sampling(W, 1e-4, 5)),
                    ("multi2", lambda: ctx.motif_sampling_multi(2, W, 1e-4, 1.0, 5))]:
        try:
            f(); res[name] = "ok"
        except GibbsError as e:
            res[name] = f"E{e.status}"
    ctx.close()
    print(len(alpha), L, W, res, flush=True)
