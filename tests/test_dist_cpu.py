"""The N>1 path on CPU: world_size-2 gloo processes run the sharded protocol.

Each rank takes its shard (gibbssampling_amd.dist.shard_bounds), computes its
partial aggregates, all-reduces them (here gloo; on MI355X the library's RCCL
all-reduce), and sweeps its own targets against the global aggregates with
uniforms keyed by the global sequence index.  The gathered result must equal the
single-process sweep bit for bit, sweep after sweep.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import init_positions, make_dataset


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gibbssampling_amd.dist import shard_bounds
        from oracle import oracle_lib as ol
        N, W, seed = 90, 8, 31337
        codes, offsets = make_dataset(N, 70, W, seed=3, ragged=True, mut=0.1)
        pos = init_positions(offsets, W, 4, 0.1)
        lo, hi = shard_bounds(np.diff(offsets), world)[rank]
        S = ol.Seqs(codes[offsets[lo]:offsets[hi]], offsets[lo:hi + 1] - offsets[lo], b"ACGT")
        p = pos[lo:hi].copy()
        # the RCCL unique id travels the same way (broadcast_object_list, dist.py)
        obj = [b"\x01" * 128 if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        assert obj[0] == b"\x01" * 128
        for t in range(4):
            C, T = ol.counts(S, W, p)
            agg = torch.from_numpy(np.concatenate([C.reshape(-1), T]))
            dist.all_reduce(agg)  # the per-sweep aggregate all-reduce
            agg = agg.numpy()
            Cg, Tg = agg[:4 * W].reshape(4, W), agg[4 * W:]
            u = np.array([ol.uniform(seed, ol.stream_sweep(t), lo + n) for n in range(hi - lo)])
            p, w = ol.sweep_shard(S, N, W, 1e-4, 1.0, Cg, Tg, p, u)
        parts = [None] * world
        dist.all_gather_object(parts, (lo, p, w))
        if rank == 0:
            Sf = ol.Seqs(codes, offsets, b"ACGT")
            ref = pos.copy()
            for t in range(4):
                u = np.array([ol.uniform(seed, ol.stream_sweep(t), n) for n in range(N)])
                ref, rw, _ = ol.sweep(Sf, W, 1e-4, 1.0, ref, u)
            got_p = np.concatenate([x[1] for x in sorted(parts, key=lambda x: x[0])])
            got_w = np.concatenate([x[2] for x in sorted(parts, key=lambda x: x[0])])
            q.put(bool(np.array_equal(got_p, ref) and np.array_equal(got_w, rw)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_sweeps_bit_identical(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True
