"""bench.py under torch.distributed.run with one rank and a real one-rank communicator:
--exchange ipc opens the in-kernel exchange, checks it on the warmup chain and times
the chain with it (the line says "exchange": "ipc"), the default (auto) keeps RCCL at
one rank.  Config 3 (the long kernel, one of the two kernels that exchange in-kernel)."""
import json
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _bench(*extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--gpus", "1", "--steps", "6", "--warmup", "2", "--config", "cfg3", "--no-side",
           "--no-cpu-baseline", *extra]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_bench_exchange_ipc_one_rank():
    out = _bench("--exchange", "ipc")
    assert out["exchange"] == "ipc"
    assert "HIP IPC" in out["config"]["parallelism"]
    assert out["roofline"]["kernel"] == "gs_sweep_long_kernel"
    assert out["chain"]["keep_motif"] > 0.9 and out["chain"]["rescans_per_sweep"] < 100


def test_bench_exchange_auto_one_rank_is_rccl():
    out = _bench()
    assert "exchange" not in out
    assert "RCCL" in out["config"]["parallelism"]
