import sys, time
sys.path.insert(0,'.'); sys.path.insert(0,'tests')
import numpy as np
from conftest import make_dataset
from gibbssampling_amd import Context
from oracle import oracle_lib as ol
N,L,W=10000,200,12
codes, offsets = make_dataset(N, L, W, b"ACGT", seed=5)
ctx = Context(0); ctx.set_sequences(codes, offsets, b"ACGT")
sc, p = ctx.random_starts(W, 1e-4, 7, 1)
u = np.array([ol.uniform(7, ol.stream_sweep(0), n) for n in range(N)])
p1, w1 = ctx.motif_sweep(W, 1e-4, 1.0, p, u)
for rep in range(2):
    t=time.perf_counter(); s = ctx.motif_greedy(W, 1e-4, 1.0, p1, w1); ts=time.perf_counter()-t
    cnt = (p1 >= 0).astype(np.int32); lst = np.where(p1 >= 0, p1, -1).reshape(N, 1).astype(np.int32)
    t=time.perf_counter(); l = ctx.motif_greedy_multi(1, W, 1e-4, 1.0, cnt, lst, w1); tl=time.perf_counter()-t
    same = np.array_equal(np.where(l[0] > 0, l[1][:, 0], -1), s[0]) and np.array_equal(l[2], s[1])
    print(f"star {ts*1e3:.1f} ms ({s[2]} passes)  list-spec {tl*1e3:.1f} ms  identical={same}")
# hybrid estimate: star engine for the first k passes, then the speculative list path
for k in (1, 2, 3):
    t = time.perf_counter()
    s1 = ctx.motif_greedy(W, 1e-4, 1.0, p1, w1, max_passes=k)
    t1 = time.perf_counter() - t
    cnt = (s1[0] >= 0).astype(np.int32)
    lst = np.where(s1[0] >= 0, s1[0], -1).reshape(N, 1).astype(np.int32)
    t = time.perf_counter()
    l = ctx.motif_greedy_multi(1, W, 1e-4, 1.0, cnt, lst, s1[1])
    t2 = time.perf_counter() - t
    s = ctx.motif_greedy(W, 1e-4, 1.0, p1, w1)
    same = np.array_equal(np.where(l[0] > 0, l[1][:, 0], -1), s[0]) and np.array_equal(l[2], s[1])
    print(f"hybrid k={k}: star {t1*1e3:.1f} ms + spec {t2*1e3:.1f} ms ({l[3]} passes) identical={same}")
