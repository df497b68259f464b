import sys, time
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np
from conftest import make_dataset
from gibbssampling_amd import Context
for name, (N, L, W, al) in {"cfg2": (10000, 200, 12, b"ACGT"), "cfg5": (50000, 300, 20, b"ACDEFGHIKLMNPQRSTVWY")}.items():
    codes, offsets = make_dataset(N, L, W, al, seed=5)
    for rnd in range(2):
        for lib in ["gibbssampling_amd/libgibbs_hip_prev.so", None]:
            c = Context(0, lib) if lib else Context(0)
            c.set_sequences(codes, offsets, al)
            sc, p = c.random_starts(W, 1e-4, 7, 1)
            c.site_scan(W, 1e-4, p)
            t = time.perf_counter(); r = c.site_scan(W, 1e-4, p); t1 = time.perf_counter() - t
            t = time.perf_counter(); c.random_starts(W, 1e-4, 7, 1); t2 = time.perf_counter() - t
            t = time.perf_counter(); c.random_starts(W, 1e-4, 7, 0); t3 = time.perf_counter() - t
            print(name, lib or "new", f"scan {t1*1e3:.2f} ms shared-starts {t2*1e3:.2f} ms exact-starts {t3*1e3:.1f} ms", flush=True)
            c.close()
