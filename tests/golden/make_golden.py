#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/*.npz from the CPU oracle.

Every fixture is produced by oracle/gibbs_oracle.c in BOTH its reference-faithful
O(N^2) mode and its hold-one-out mode (asserted identical) and, where small enough,
cross-checked against the pure-Python literal restatement oracle/gibbs_ref.py.
Inputs: BASELINE config 1 (synthetic) and the data sets of GibbsSampling.fsx
(tests/golden/fsx_sets.json).  Parity against reference-produced numbers is
unpinned (the F# reference cannot run here).
"""
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))

from gibbssampling_amd import synthetic  # noqa: E402
from gibbssampling_amd.bioarray import AMINO20, DNA_BASES, pack  # noqa: E402
from oracle import gibbs_ref as gr  # noqa: E402
from oracle import oracle_lib as ol  # noqa: E402

SEED = 20241015


def sweep_fixture(name, codes, offsets, alphabet, W, pc, cutoff, pos, u, detail=(0,),
                  python_check=False):
    S = ol.Seqs(codes, offsets, alphabet)
    p1, w1, m1 = ol.sweep(S, W, pc, cutoff, pos, u, faithful=True)
    p2, w2, m2 = ol.sweep(S, W, pc, cutoff, pos, u, faithful=False)
    assert np.array_equal(p1, p2) and np.array_equal(w1, w2)
    if python_check:
        seqs = [list(codes[offsets[i]:offsets[i + 1]]) for i in range(len(offsets) - 1)]
        mem = [(0.0, [int(p)] if p >= 0 else []) for p in pos]
        ref = gr.findBestMotifIndicesByWithStartPositions(1, W, pc, cutoff, list(alphabet), seqs,
                                                          mem, list(u))
        assert [r[1][0] if r[1] else -1 for r in ref] == list(p1)
        assert [r[0] for r in ref] == list(w1)
    C, T = ol.counts(S, W, pos)
    out = dict(codes=codes, offsets=offsets, alphabet=np.frombuffer(alphabet, np.uint8),
               W=np.int32(W), pc=np.float64(pc), cutoff=np.float64(cutoff), pos_in=pos, u=u,
               pos_out=p1, pwms_out=w1, margin=m1, C=C, T=T,
               detail_targets=np.array(detail, np.int32))
    for t in detail:
        d = ol.target_detail(S, W, pc, pos, t)
        for k, v in d.items():
            out[f"t{t}_{k}"] = v
    np.savez(HERE / f"{name}.npz", **out)
    print(name, len(pos), "targets, picks:", int((p1 >= 0).sum()), "motif,",
          int((p1 < 0).sum()), "background; min margin", float(m1.min()))


def main():
    sets = json.loads((HERE / "fsx_sets.json").read_text())

    # BASELINE config 1: 100 synthetic DNA sequences x 50 bp, W = 8
    w = synthetic.CONFIGS["cfg1"]
    codes, offsets = synthetic.generate(w)
    pos = synthetic.initial_positions(w)
    u = np.array([ol.uniform(SEED, ol.stream_sweep(0), n) for n in range(w.N)])
    sweep_fixture("cfg1_sweep", codes, offsets, w.alphabet, w.W, w.pc, w.cutoff, pos, u,
                  detail=(0, 1, 57), python_check=True)

    # chained sweeps with counter-RNG uniforms (gs_run_sweeps semantics)
    S = ol.Seqs(codes, offsets, w.alphabet)
    p = pos.copy()
    for t in range(5):
        uu = np.array([ol.uniform(SEED, ol.stream_sweep(t), n) for n in range(w.N)])
        p, pw, _ = ol.sweep(S, w.W, w.pc, w.cutoff, p, uu)
    np.savez(HERE / "cfg1_chain5.npz", codes=codes, offsets=offsets,
             alphabet=np.frombuffer(w.alphabet, np.uint8), W=np.int32(w.W), pc=np.float64(w.pc),
             cutoff=np.float64(w.cutoff), pos_in=pos, seed=np.uint64(SEED), sweeps=np.int32(5),
             pos_out=p, pwms_out=pw)

    # .fsx toy sets with dnaBases (|A| = 5): starts from getPWMOfRandomStarts (exact mode)
    for key, W in [("tests", 6), ("bioTestsWithMultipleSamples", 6), ("bioTestsII", 7)]:
        c, o = pack([s.encode() for s in sets[key]["seqs"]])
        Sx = ol.Seqs(c, o, DNA_BASES)
        sc, ps = ol.random_starts(Sx, W, 1e-4, seed=SEED, mode=0)
        np.savez(HERE / f"fsx_{key}_starts.npz", codes=c, offsets=o,
                 alphabet=np.frombuffer(DNA_BASES, np.uint8), W=np.int32(W), pc=np.float64(1e-4),
                 seed=np.uint64(SEED), mode=np.int32(0), score=sc, pos=ps)
        uu = np.array([ol.uniform(SEED, ol.stream_sweep(0), n) for n in range(len(ps))])
        sweep_fixture(f"fsx_{key}_sweep", c, o, DNA_BASES, W, 1e-4, 1.0, ps, uu, detail=(0,),
                      python_check=True)

    # the 31-gene Chlamydomonas dataSet (62 sequences, 29,616 bp), W = 10
    c, o = pack([s.encode() for s in sets["dataSet"]["seqs"]])
    Sx = ol.Seqs(c, o, DNA_BASES)
    sc, ps = ol.random_starts(Sx, 10, 1e-4, seed=SEED, mode=1)
    uu = np.array([ol.uniform(SEED, ol.stream_sweep(0), n) for n in range(len(ps))])
    sweep_fixture("fsx_dataSet_sweep", c, o, DNA_BASES, 10, 1e-4, 1.0, ps, uu, detail=(0, 61))

    # protein mini-set: ragged 40-90 aa, 20 standard amino acids plus '*', W = 8
    rng = np.random.default_rng(SEED)
    a = np.frombuffer(AMINO20, np.uint8)
    seqs = []
    for _ in range(30):
        s = a[rng.integers(0, 20, rng.integers(40, 91))]
        s[rng.random(len(s)) < 0.01] = ord("*")
        seqs.append(bytes(s))
    c, o = pack(seqs)
    lens = np.diff(o)
    ps = (rng.random(30) * (lens - 8 + 1)).astype(np.int32)
    ps[[3, 11]] = -1
    uu = rng.random(30)
    sweep_fixture("protein_mini_sweep", c, o, AMINO20, 8, 1e-4, 1.0, ps, uu, detail=(3, 4),
                  python_check=True)


if __name__ == "__main__":
    main()
