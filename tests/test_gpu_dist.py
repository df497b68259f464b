"""The multi-GPU code path on one MI355X: a real RCCL communicator (one rank) runs
the per-sweep in-stream all-reduce; results must equal the communicator-free run
bit for bit.  (Two or more ranks need a GPU each; the decomposition itself is
covered by test_two_shards_bit_identical and tests/test_dist_cpu.py.)"""
import os
import socket

import numpy as np
import pytest

from conftest import init_positions, make_dataset

pytestmark = pytest.mark.gpu


def test_rccl_one_rank_matches_plain(gpu_ctx):
    from gibbssampling_amd import Context
    N, L, W, seed = 2000, 150, 10, 77
    codes, offsets = make_dataset(N, L, W, seed=201, mut=0.1)
    pos = init_positions(offsets, W, 202)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    ref = gpu_ctx.motif_run(W, 1e-4, 1.0, 5, seed, pos)
    c = Context(0)
    c.set_sequences(codes, offsets, b"ACGT")
    c.comm_init(Context.unique_id(), 1, 0)
    got = c.motif_run(W, 1e-4, 1.0, 5, seed, pos)
    c.profile(True)
    c.set_positions(W, pos)
    c.run_sweeps(1e-4, 1.0, 3, seed)
    c.synchronize()
    kms, nk, arms, nar = c.profile_read()
    c.close()
    assert np.array_equal(ref[0], got[0]) and np.array_equal(ref[1], got[1])
    assert nk == 3 and nar >= 3 and kms > 0 and arms > 0


def test_sharded_sampler_world_one():
    import torch.distributed as dist
    from gibbssampling_amd.dist import ShardedSampler
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        N, W = 500, 8
        codes, offsets = make_dataset(N, 90, W, seed=211, ragged=True)
        pos = init_positions(offsets, W, 212)
        sh = ShardedSampler(codes, offsets, b"ACGT", 0, 1, 0)
        sh.set_positions(W, pos)
        sh.run_sweeps(1e-4, 1.0, 3, 5)
        p, w = sh.gather_state()
        from gibbssampling_amd import Context
        c = Context(0)
        c.set_sequences(codes, offsets, b"ACGT")
        rp, rw = c.motif_run(W, 1e-4, 1.0, 3, 5, pos)
        c.close()
        sh.ctx.close()
        assert np.array_equal(p, rp) and np.array_equal(w, rw)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("first_sweep,sweeps", [(0, 13), (4, 12), (7, 5)])
def test_graph_chain_matches_direct(first_sweep, sweeps, monkeypatch):
    """hipGraph replay of sweep chains (6 sweeps per graph, the counter-RNG stream
    from the device sweep counter) gives the direct launches' chain bit for bit."""
    from gibbssampling_amd import Context
    N, L, W, seed = 3000, 120, 9, 91
    codes, offsets = make_dataset(N, L, W, seed=221, mut=0.1, ragged=True)
    pos = init_positions(offsets, W, 222, 0.1)
    out = []
    for mode in ("0", "1"):
        tuning = {"graph_mode": float(mode)}
        c = Context(0, tuning=tuning)
        c.set_sequences(codes, offsets, b"ACGT")
        out.append(c.motif_run(W, 1e-4, 1.0, sweeps, seed, pos, first_sweep=first_sweep))
        # a second chain on the same context reuses the captured graph
        c.run_sweeps(1e-4, 1.0, sweeps, seed, first_sweep + sweeps)
        out.append(c.get_state())
        c.close()
    for a, b in ((out[0], out[2]), (out[1], out[3])):
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_rccl_one_rank_graph_chain(gpu_ctx):
    """With a communicator the chain is replayed as graphs with the all-reduces
    captured in them (RCCL under stream capture)."""
    from gibbssampling_amd import Context
    N, L, W, seed = 2000, 150, 10, 78
    codes, offsets = make_dataset(N, L, W, seed=231, mut=0.1)
    pos = init_positions(offsets, W, 232)
    gpu_ctx.set_sequences(codes, offsets, b"ACGT")
    ref = gpu_ctx.motif_run(W, 1e-4, 1.0, 20, seed, pos)
    c = Context(0)
    c.set_sequences(codes, offsets, b"ACGT")
    c.comm_init(Context.unique_id(), 1, 0)
    got = c.motif_run(W, 1e-4, 1.0, 20, seed, pos)
    c.close()
    assert np.array_equal(ref[0], got[0]) and np.array_equal(ref[1], got[1])


def test_prepare_sweeps_then_chain(monkeypatch):
    """gs_prepare_sweeps captures the graph ahead of time without running a sweep."""
    from gibbssampling_amd import Context
    N, L, W, seed = 1500, 100, 8, 93
    codes, offsets = make_dataset(N, L, W, seed=241, mut=0.1)
    pos = init_positions(offsets, W, 242)
    out = []
    for mode in ("0", "1"):
        tuning = {"graph_mode": float(mode)}
        c = Context(0, tuning=tuning)
        c.set_sequences(codes, offsets, b"ACGT")
        c.set_positions(W, pos)
        c.run_sweeps(1e-4, 1.0, 5, seed)
        c.prepare_sweeps(1e-4, 1.0, seed)
        before = c.get_state()
        c.run_sweeps(1e-4, 1.0, 12, seed, 5)
        out.append((before, c.get_state()))
        c.close()
    (b0, a0), (b1, a1) = out
    assert np.array_equal(b0[0], b1[0]) and np.array_equal(a0[0], a1[0])
    assert np.array_equal(a0[1], a1[1])
