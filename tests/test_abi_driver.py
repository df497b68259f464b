"""The F# shim's C call sequence, run as a separate C program (tests/abi_driver.c,
dlopen + dlsym like .NET P/Invoke) for the reference driver's own calls:

  GibbsSampling.fsx:384  getMotifsWithBestInformationContent 1 6 0.0001 dnaBases bioTests
  GibbsSampling.fsx:407  getMotifsWithBestInformationContents 1 2 6 0.0001 1. dnaBases
                         bioTestsWithMultipleSamples

(with fixed seeds; also 5 repetitions and motifAmount 1).  Every result must equal
the Python mirror of the same entry points (gibbssampling_amd/sampler.py) for the
same seeds, which the other GPU tests hold to the oracle.
"""
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

from gibbssampling_amd.bioarray import DNA_BASES

ROOT = Path(__file__).resolve().parents[1]
DRIVER = ROOT / "tests" / "abi_driver"
LIB = ROOT / "gibbssampling_amd" / "libgibbs_hip.so"
SETS = json.loads((Path(__file__).parent / "golden" / "fsx_sets.json").read_text())


def test_driver_built():
    """build() compiles the driver (CPU check: present and executable)."""
    assert DRIVER.exists(), "run __graft_entry__.build()"


def run_driver(args, seqs):
    stdin = DNA_BASES.decode() + "\n" + "\n".join(seqs) + "\n"
    r = subprocess.run([str(DRIVER), str(LIB), *map(str, args)], input=stdin, text=True,
                       capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = []
    for line in r.stdout.splitlines():
        f = line.split()
        out.append((float(f[0]), [int(x) for x in f[1:]]))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("reps,seed", [(1, 11), (5, 300)])
def test_fsx384_site_sampler(reps, seed):
    from gibbssampling_amd.sampler import SiteSampler
    seqs = SETS["tests"]["seqs"]
    got = run_driver(["site", reps, 6, 1e-4, seed], seqs)
    ref = SiteSampler.getMotifsWithBestInformationContent(reps, 6, 1e-4, DNA_BASES,
                                                          [s.encode() for s in seqs], seed=seed)
    assert [p for _, p in got] == [[p] for _, p in ref]
    np.testing.assert_array_equal([w for w, _ in got], [s for s, _ in ref])


@pytest.mark.gpu
@pytest.mark.parametrize("reps,M,seed", [(1, 2, 21), (5, 2, 400), (3, 1, 500)])
def test_fsx407_motif_sampler(reps, M, seed):
    from gibbssampling_amd.sampler import MotifSampler
    seqs = SETS["bioTestsWithMultipleSamples"]["seqs"]
    got = run_driver(["motif", reps, M, 6, 1e-4, 1.0, seed], seqs)
    ref = MotifSampler.getMotifsWithBestInformationContents(
        reps, M, 6, 1e-4, 1.0, DNA_BASES, [s.encode() for s in seqs], seed=seed)
    assert [p for _, p in got] == [list(m.Positions) for m in ref]
    np.testing.assert_array_equal([w for w, _ in got], [m.PWMS for m in ref])
