"""gibbssampling_amd.dist.open_exchange's agreement, on the CPU with gloo (world 2): the
ranks all-gather their exchange handles and agree on the outcome before any sweep, so a
rank that cannot export or open its exchange makes every rank fall back to the
communicator's all-reduce together (bench.py --exchange auto relies on it), and no
rank is left waiting in a collective the other skipped.  The context is a stand-in
recording the calls (the library's entry points need a GPU)."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class FakeCtx:
    def __init__(self, rank, fail_handle=False, fail_open=False):
        self.rank, self.fail_handle, self.fail_open = rank, fail_handle, fail_open
        self.opened = None
        self.closed = False

    def exchange_handle(self):
        if self.fail_handle:
            raise RuntimeError("hipIpcGetMemHandle: invalid argument")
        return bytes([self.rank]) * 64

    def exchange_open(self, handles, rank):
        if self.fail_open:
            raise RuntimeError("hipIpcOpenMemHandle: invalid argument")
        self.opened = (list(handles), rank)

    def exchange_close(self):
        self.closed = True

    def synchronize(self):
        pass


def _worker(rank, world, port, fails, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gibbssampling_amd.dist import open_exchange
        what = fails.get(rank, "")
        ctx = FakeCtx(rank, fail_handle=what == "handle", fail_open=what == "open")
        err = open_exchange(ctx, rank, world)
        q.put((rank, err, ctx.opened, ctx.closed))
    finally:
        dist.destroy_process_group()


def _run(fails):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, fails, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    return out


def test_open_exchange_all_ranks():
    out = _run({})
    for rank, err, opened, closed in out:
        assert err == "" and not closed
        assert opened == ([bytes([0]) * 64, bytes([1]) * 64], rank)


@pytest.mark.parametrize("what", ["handle", "open"])
def test_open_exchange_one_rank_fails(what):
    out = _run({1: what})
    (_, err0, opened0, closed0), (_, err1, opened1, closed1) = out
    assert err0 and err1  # both ranks fall back
    assert opened1 is None
    if what == "open":
        assert opened0 is not None and closed0  # rank 0 opened, then closed it again
    else:
        assert opened0 is None  # nothing was opened: a handle was missing
