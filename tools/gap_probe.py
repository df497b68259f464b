"""Wall time per sweep of back-to-back resident sweeps with and without the
kernel-attached timing events (does the event bookkeeping widen the dispatch gap?).
    python tools/gap_probe.py cfg2 400"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import _native, synthetic  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    w = synthetic.CONFIGS[name]
    codes, offsets = synthetic.generate(w)
    ctx = _native.Context(0)
    ctx.set_sequences(codes, offsets, w.alphabet)
    ctx.set_positions(w.W, synthetic.initial_positions(w))
    ctx.run_sweeps(w.pc, w.cutoff, 20, seed=1)
    ctx.synchronize()
    out = {}
    for prof in (False, True, False, True):
        ctx.profile(prof)
        ctx.profile_read()
        t = time.perf_counter()
        ctx.run_sweeps(w.pc, w.cutoff, n, seed=1, first_sweep=20)
        ctx.synchronize()
        dt = (time.perf_counter() - t) / n * 1e6
        kms, nk, _, _ = ctx.profile_read()
        out.setdefault("events" if prof else "plain", []).append(
            {"us_per_sweep": dt, "kernel_us": kms * 1e3 / nk if nk else None})
    ctx.profile(False)
    print(json.dumps({name: out}))


if __name__ == "__main__":
    main()
