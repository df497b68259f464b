"""Diagnostics for the live-chain sweep (gs_sweep_live.hip): one test-suite case run
through several kernel settings; the targets that differ from the oracle are printed
with their inputs and the oracle's categories (diagnostic tool, not a test)."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import init_positions, make_dataset  # noqa: E402
from oracle import oracle_lib as ol  # noqa: E402
from gibbssampling_amd import Context  # noqa: E402


def dbg_main(lib):
    """With the GS_LIVE_DEBUG variant: per target, the filter's block mask and threshold
    (live_force 0) or the refinement's list length / passing count and list sum (1),
    against the oracle's passing windows."""
    N, L, W, alpha, ragged, none_rate, seed = 300, 120, 12, b"ACGT", True, 0.1, 2
    codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=ragged)
    S = ol.Seqs(codes, offsets, alpha)
    pos = ol.random_starts(S, W, 1e-4, seed=seed + 1, mode=1)[1].astype(np.int32)
    pos[np.random.default_rng(seed).random(N) < none_rate] = -1
    u = np.random.default_rng(seed + 200).random(N)
    rows = []
    for G in (1, 4):
        for force in (0, 1):
            ctx = Context(0, lib_path=lib, tuning={"live_G": G, "live_force": force})
            ctx.set_sequences(codes, offsets, alpha)
            gpos, gpw = ctx.motif_sweep(W, 1e-4, 1.0, pos, u)
            ctx.close()
            for n in (10, 12, 28, 31, 111, 112):
                d = ol.target_detail(S, W, 1e-4, pos, n)
                l2 = np.log(d["S"]) / np.log(2.0)
                passing = [int(k) for k in np.nonzero(l2 > 1.0)[0]]
                rows.append({"G": G, "force": force, "n": n, "pos_out": int(gpos[n]),
                             "pwms": float(gpw[n]), "passing": passing,
                             "Msum": float(l2[l2 > 1.0].sum())})
    print(json.dumps(rows, indent=0))


def main():
    N, L, W, alpha, ragged, none_rate, seed = 300, 120, 12, b"ACGT", True, 0.1, 2
    codes, offsets = make_dataset(N, L, W, alpha, seed=seed, ragged=ragged)
    S = ol.Seqs(codes, offsets, alpha)
    pos = ol.random_starts(S, W, 1e-4, seed=seed + 1, mode=1)[1].astype(np.int32)
    pos[np.random.default_rng(seed).random(N) < none_rate] = -1
    u = np.random.default_rng(seed + 200).random(N)
    opos, opw, _ = ol.sweep(S, W, 1e-4, 1.0, pos, u, threads=8)
    lib = sys.argv[1] if len(sys.argv) > 1 else None
    out = {}
    for name, tun in [("live1", {"live_G": 1}), ("live2", {"live_G": 2}), ("live4", {"live_G": 4}),
                      ("live8", {"live_G": 8}), ("force", {"live_G": 1, "live_force": 1}),
                      ("dna1", {"dna_mode": 1, "live_mode": 0, "dna_G": 1})]:
        ctx = Context(0, lib_path=lib, tuning=tun)
        ctx.set_sequences(codes, offsets, alpha)
        s0 = ctx.stats()
        gpos, gpw = ctx.motif_sweep(W, 1e-4, 1.0, pos, u)
        s1 = ctx.stats()
        bad = np.nonzero(gpos != opos)[0]
        rec = {"ndiff": int(bad.size), "stats": {k: s1[k] - s0[k] for k in s1}, "diff": []}
        for n in bad[:6]:
            d = ol.target_detail(S, W, 1e-4, pos, int(n))
            Sk = d["S"]
            M = np.where(np.log(Sk) / np.log(2.0) > 1.0, np.log(Sk) / np.log(2.0), np.nan)
            tot = d["G"].sum() + np.nansum(M)
            passing = [(int(k), float(M[k])) for k in np.nonzero(np.isfinite(M))[0]]
            rec["diff"].append({"n": int(n), "L": int(offsets[n + 1] - offsets[n]), "pos_in": int(pos[n]),
                                "u": float(u[n]), "gpos": int(gpos[n]), "opos": int(opos[n]),
                                "gpw": float(gpw[n]), "opw": float(opw[n]), "Gsum": float(d["G"].sum()),
                                "total": float(tot), "passing": passing,
                                "u_total": float(u[n] * tot)})
        out[name] = rec
        ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "dbg":
        dbg_main(sys.argv[1])
    else:
        main()
