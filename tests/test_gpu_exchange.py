"""The in-kernel exchange of the aggregate vector (include/gibbs_hip.h gs_exchange_*)
in two processes (world_size 2) on the box's one GPU: each rank's context exports its
exchange buffer as a HIP IPC handle, the ranks all-gather the handles over gloo and
open them, and from then on the live and long sweeps end with their last workgroup
writing the rank's partial aggregates into both ranks' buffers and summing both
(.fs:940-942: every target reads only the shared snapshot) -- no all-reduce after the
sweeps, neither RCCL's nor the host-staged one.  Only the snapshot set from outside is
exchanged by the caller (gloo).  The gathered chain of several sweeps run in ONE
chain call must equal the oracle's single-process chain (positions exactly, PWMS
within 1e-12), both ranks must end with the same global aggregates, and the kernels'
bounded paths must have run (few exact rescans).  (The xGMI latency of the exchange
between GPUs is not measured here: one GPU.)"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import init_positions, make_dataset, uniforms

pytestmark = pytest.mark.gpu

N, L, W, SEED, SWEEPS = 3000, 160, 12, 4343, 6
MODES = {"live": ({"dna_mode": 1}, "gs_sweep_live_kernel"),
         "long": ({"dna_mode": 1, "long_mode": 1}, "gs_sweep_long_kernel")}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _start(codes, offsets, start):
    if start == "uniform":
        return init_positions(offsets, W, 6, 0.05)
    from oracle import oracle_lib as ol
    return ol.random_starts(ol.Seqs(codes, offsets, b"ACGT"), W, 1e-4, seed=77, mode=1)[1]


def _worker(rank, world, port, mode, out_dir, start, bounds, per_call):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gibbssampling_amd import Context
        from gibbssampling_amd.dist import shard_bounds
        codes, offsets = make_dataset(N, L, W, seed=15, ragged=True, mut=0.15)
        pos = _start(codes, offsets, start)
        lo, hi = (bounds or shard_bounds(np.diff(offsets), world))[rank]
        ctx = Context(0, tuning=MODES[mode][0])
        ctx.set_sequences(codes[offsets[lo]:offsets[hi]], offsets[lo:hi + 1] - offsets[lo],
                          b"ACGT", n_global=N, global_offset=lo)
        # the IPC handles, all-gathered over gloo, opened, agreed on (dist.open_exchange)
        from gibbssampling_amd.dist import open_exchange
        assert open_exchange(ctx, rank, world) == ""
        # the snapshot set from outside: its aggregates exchanged by the caller
        ctx.set_positions(W, pos[lo:hi])
        agg = torch.from_numpy(ctx.agg_download())
        dist.all_reduce(agg)
        ctx.agg_upload(agg.numpy())
        ctx.synchronize()
        r0 = ctx.stats()["exact_rescans"]
        dist.barrier()  # every rank's buffer open (and zeroed) before any rank sweeps
        if per_call:
            for t in range(SWEEPS):
                ctx.run_sweeps(1e-4, 1.0, 1, SEED, t)
        else:
            ctx.run_sweeps(1e-4, 1.0, SWEEPS, SEED, 0)
        ctx.synchronize()
        p, w = ctx.get_state()
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), lo=lo, p=p, w=w,
                 kernel=ctx.sweep_kernel_name(), agg=ctx.agg_download(),
                 rescans=ctx.stats()["exact_rescans"] - r0)
        dist.barrier()
        ctx.exchange_close()
        ctx.close()
    finally:
        dist.destroy_process_group()


def _run(tmp_path, mode, start="init", bounds=None, per_call=False):
    from oracle import oracle_lib as ol
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, str(tmp_path), start, bounds, per_call))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(2)]
    got_p = np.concatenate([x["p"] for x in parts])
    got_w = np.concatenate([x["w"] for x in parts])
    codes, offsets = make_dataset(N, L, W, seed=15, ragged=True, mut=0.15)
    S = ol.Seqs(codes, offsets, b"ACGT")
    ref = _start(codes, offsets, start)
    for t in range(SWEEPS):
        ref, rw, _ = ol.sweep(S, W, 1e-4, 1.0, ref, uniforms(SEED, ol.stream_sweep(t), N))
    assert np.array_equal(got_p, ref)
    assert np.array_equal(got_w, rw) or np.allclose(got_w, rw, rtol=1e-12, atol=0)
    # both ranks hold the same (global) aggregates of the last snapshot
    assert np.array_equal(parts[0]["agg"], parts[1]["agg"])
    # the kernels' bounded paths ran (a table fault would rescan every target exactly
    # and still match)
    assert sum(int(x["rescans"]) for x in parts) <= 0.05 * N * SWEEPS
    return parts


@pytest.mark.parametrize("mode", sorted(MODES))
def test_exchange_chain_matches_oracle(tmp_path, mode):
    parts = _run(tmp_path, mode)
    assert {str(x["kernel"]) for x in parts} == {MODES[mode][1]}


def test_exchange_one_sweep_calls(tmp_path):
    """The same with one chain call a sweep (the exchange count runs across calls)."""
    _run(tmp_path, "live", per_call=True)


def test_exchange_empty_shard(tmp_path):
    """One rank holds every sequence, the other none: the empty rank's sweep still
    reaches its last workgroup and exchanges zeros."""
    parts = _run(tmp_path, "live", bounds=[(0, N), (N, N)])
    assert len(parts[1]["p"]) == 0


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("graph", [0, 1])
def test_exchange_one_rank_with_communicator(mode, graph):
    """One rank, a one-rank RCCL communicator and the exchange open: the chain (replayed
    as hipGraphs with graph_mode 1 -- the sweeps captured without an all-reduce -- or
    launched directly) equals the communicator-free chain bit for bit, the exchange
    count advancing inside the captured kernels."""
    from gibbssampling_amd import Context
    codes, offsets = make_dataset(N, L, W, seed=15, ragged=True, mut=0.15)
    pos = _start(codes, offsets, "init")
    r = Context(0, tuning=MODES[mode][0])  # (the same kernel without communicator or exchange)
    r.set_sequences(codes, offsets, b"ACGT")
    ref = r.motif_run(W, 1e-4, 1.0, 14, SEED, pos)
    r.close()
    c = Context(0, tuning={**MODES[mode][0], "graph_mode": float(graph)})
    c.set_sequences(codes, offsets, b"ACGT")
    c.comm_init(Context.unique_id(), 1, 0)
    c.exchange_open([c.exchange_handle()], 0)
    if not graph:
        c.profile(True)  # (per-launch events: direct launches only)
    got = c.motif_run(W, 1e-4, 1.0, 14, SEED, pos)
    c.synchronize()
    _, nk, _, nar = c.profile_read() if not graph else (0, 0, 0, 0)
    name = c.sweep_kernel_name()
    c.exchange_close()
    c.close()
    assert name == MODES[mode][1]
    assert np.array_equal(ref[0], got[0]) and np.array_equal(ref[1], got[1])
    # no all-reduce of the aggregate vector after the sweeps (the snapshot's own may run)
    assert nar <= 2, (nk, nar)
