"""GPU parity of the four-symbol sweep's finished workgroup tables (gs_sweep.hip
ek4_build_tables; gs_set_tuning ftab_mode): built by every workgroup (0, the default),
by a one-workgroup kernel before each sweep (1), or handed over by the previous
sweep's last workgroup through the two-level done counter (2).  Every mode must give
the chain the oracle gives (.fs:935-970, normalizePPM .fs:257-260 and the PCV logs
.fs:119 computed once a sweep instead of once a workgroup), also across calls that
drop the handed-over tables (positions or aggregates set from outside).  Modes 1 and 2
are a build of their own (-DGS_FTAB: libgibbs_hip_ftab.so, built beside the default
library): the default library rejects them."""
import numpy as np
import pytest

from conftest import ROOT, make_dataset, uniforms
from oracle import oracle_lib as ol

pytestmark = pytest.mark.gpu


FTAB_LIB = ROOT / "gibbssampling_amd" / "libgibbs_hip_ftab.so"


def chain(mode, codes, offsets, W, pos, sweeps, seed, split=None):
    from gibbssampling_amd import Context
    c = Context(0, FTAB_LIB, tuning={"ftab_mode": float(mode)})
    try:
        c.set_sequences(codes, offsets, b"ACGT")
        if split is None:
            out = c.motif_run(W, 1e-4, 1.0, sweeps, seed, pos)
        else:
            # two chain calls, the aggregates downloaded and uploaded in between (an
            # entry point that drops the handed-over tables)
            c.set_positions(W, pos)
            c.run_sweeps(1e-4, 1.0, split, seed=seed, first_sweep=0)
            c.agg_upload(c.agg_download())
            c.run_sweeps(1e-4, 1.0, sweeps - split, seed=seed, first_sweep=split)
            out = c.get_state()
        assert c.last_sweep_launch()["ek"] == 4
        return out
    finally:
        c.close()


@pytest.mark.parametrize("W,N,L", [(12, 3000, 200), (8, 2000, 120), (20, 1500, 260)])
def test_ftab_modes_same_chain(W, N, L):
    codes, offsets = make_dataset(N, L, W, b"ACGT", seed=500 + W)
    S = ol.Seqs(codes, offsets, b"ACGT")
    pos = ol.random_starts(S, W, 1e-4, seed=7, mode=1)[1].astype(np.int32)
    sweeps, seed = 6, 77
    ref = chain(0, codes, offsets, W, pos, sweeps, seed)
    for mode in (1, 2):
        got = chain(mode, codes, offsets, W, pos, sweeps, seed)
        assert np.array_equal(got[0], ref[0]), f"mode {mode}: positions differ"
        assert np.array_equal(got[1], ref[1]), f"mode {mode}: PWMS differ"
    got = chain(2, codes, offsets, W, pos, sweeps, seed, split=2)
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
    opos, opw = pos, None
    for t in range(sweeps):
        opos, opw, _ = ol.sweep(S, W, 1e-4, 1.0, opos, uniforms(seed, ol.stream_sweep(t), N), threads=8)
    assert np.array_equal(ref[0], opos)
    fin = np.isfinite(opw)
    rel = np.abs(ref[1][fin] - opw[fin]) / np.maximum(np.abs(opw[fin]), 1e-300)
    assert rel.max() <= 1e-12


def test_ftab_modes_need_their_build():
    from gibbssampling_amd import Context
    from gibbssampling_amd._native import GS_E_UNSUPPORTED, GibbsError
    N, L, W = 300, 120, 12
    codes, offsets = make_dataset(N, L, W, seed=520)
    c = Context(0, tuning={"ftab_mode": 2.0})
    try:
        c.set_sequences(codes, offsets, b"ACGT")
        with pytest.raises(GibbsError) as e:
            c.motif_run(W, 1e-4, 1.0, 2, 5, np.zeros(N, np.int32))
        assert e.value.status == GS_E_UNSUPPORTED
    finally:
        c.close()
