"""The library's shard entry points in two processes (world_size 2), with gloo as the
transport: each rank holds a Context over its contiguous shard (n_global /
global_offset), and after every sweep the ranks sum their partial aggregates
(gs_agg_download -> gloo all-reduce -> gs_agg_upload), the host-staged form of the
in-stream RCCL all-reduce.  Both ranks share the one GPU of the box (RCCL needs a
GPU per rank; the exchange protocol is what is under test).  The gathered chain
must equal the oracle's single-process chain bit for bit, for the general sweep
kernel and for the DNA kernel."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import init_positions, make_dataset, uniforms

pytestmark = pytest.mark.gpu

N, L, W, SEED, SWEEPS = 3000, 160, 12, 4242, 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


MODES = {"general": ({"dna_mode": 0}, "gs_sweep_kernel"),
         "dna": ({"dna_mode": 1, "live_mode": 0}, "gs_sweep_dna_kernel"),
         "live": ({"dna_mode": 1}, "gs_sweep_live_kernel"),
         "long": ({"dna_mode": 1, "long_mode": 1}, "gs_sweep_long_kernel")}


def _worker(rank, world, port, mode, out_dir, start="uniform", bounds=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gibbssampling_amd import Context
        from gibbssampling_amd.dist import shard_bounds
        codes, offsets = make_dataset(N, L, W, seed=5, ragged=True, mut=0.15)
        pos = _start(codes, offsets, start)
        lo, hi = (bounds or shard_bounds(np.diff(offsets), world))[rank]
        ctx = Context(0, tuning=MODES[mode][0])
        ctx.set_sequences(codes[offsets[lo]:offsets[hi]], offsets[lo:hi + 1] - offsets[lo],
                          b"ACGT", n_global=N, global_offset=lo)

        def exchange():
            agg = torch.from_numpy(ctx.agg_download())
            dist.all_reduce(agg)
            ctx.agg_upload(agg.numpy())

        ctx.set_positions(W, pos[lo:hi])
        exchange()
        trail = []
        for t in range(SWEEPS):
            ctx.run_sweeps(1e-4, 1.0, 1, SEED, t)
            exchange()
            trail.append(ctx.get_state()[0])
        p, w = ctx.get_state()
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), lo=lo, p=p, w=w,
                 trail=np.array(trail, np.int32).reshape(SWEEPS, hi - lo),
                 kernel=ctx.sweep_kernel_name(), oob=ctx.stats()["desc_oob"])
        ctx.close()
    finally:
        dist.destroy_process_group()


def _start(codes, offsets, start):
    """'uniform': uniform random starts (5 % of them []); 'init': getPWMOfRandomStarts'
    output (.fs:589-611, shared draws), the snapshot doMotifSampling sweeps
    (.fs:1035-1037), in which every target keeps a motif through the chain."""
    if start == "uniform":
        return init_positions(offsets, W, 6, 0.05)
    from oracle import oracle_lib as ol
    return ol.random_starts(ol.Seqs(codes, offsets, b"ACGT"), W, 1e-4, seed=77, mode=1)[1]


def _run(tmp_path, mode, start="uniform", bounds=None):
    from oracle import oracle_lib as ol
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, str(tmp_path), start, bounds))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs)
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(2)]
    assert all(int(x["oob"]) == 0 for x in parts)  # descriptor index audit (gs_stats [13])
    got_p = np.concatenate([x["p"] for x in parts])
    got_w = np.concatenate([x["w"] for x in parts])
    trail = np.concatenate([x["trail"] for x in parts], axis=1)
    codes, offsets = make_dataset(N, L, W, seed=5, ragged=True, mut=0.15)
    S = ol.Seqs(codes, offsets, b"ACGT")
    ref = _start(codes, offsets, start)
    keep = []
    for t in range(SWEEPS):
        ref, rw, _ = ol.sweep(S, W, 1e-4, 1.0, ref, uniforms(SEED, ol.stream_sweep(t), N))
        assert np.array_equal(trail[t], ref), f"sweep {t}"
        keep.append(float((trail[t] >= 0).mean()))
    assert np.array_equal(got_p, ref)
    assert np.array_equal(got_w, rw) or np.allclose(got_w, rw, rtol=1e-12, atol=0)
    return parts, keep


@pytest.mark.parametrize("mode", sorted(MODES))
def test_two_rank_gloo_exchange_matches_oracle(tmp_path, mode):
    parts, _ = _run(tmp_path, mode)
    assert {str(x["kernel"]) for x in parts} == {MODES[mode][1]}


@pytest.mark.parametrize("mode", sorted(MODES))
def test_two_rank_gloo_live_chain_init_regime(tmp_path, mode):
    """The exchange of LIVE aggregates: the chain from the initialiser's output, in
    which every target keeps a motif (a chain from uniform starts drops them all in
    its first sweep and exchanges zeros from then on).  Positions equal the oracle's
    after every sweep."""
    parts, keep = _run(tmp_path, mode, start="init")
    assert {str(x["kernel"]) for x in parts} == {MODES[mode][1]}
    assert min(keep) > 0.9, keep


@pytest.mark.parametrize("mode", ["live", "general", "long"])
def test_two_rank_gloo_empty_shard(tmp_path, mode):
    """One rank holds every sequence, the other none (n_local = 0): the empty rank
    still sweeps (its done counter reached) and contributes zero aggregates.  The
    kernels audit every descriptor load's index (gs_stats [13] counts loads outside
    [0, n_local)): the empty rank's sweeps, which once read len[-1] / doff[-1] for the
    first sequence's prefetch, and the full rank's must load none."""
    parts, keep = _run(tmp_path, mode, start="init", bounds=[(0, N), (N, N)])
    assert str(parts[0]["kernel"]) == MODES[mode][1]
    assert len(parts[1]["p"]) == 0
    assert [int(x["oob"]) for x in parts] == [0, 0]
    assert min(keep) > 0.9, keep
