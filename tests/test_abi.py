"""CPU-side checks of the drop-in boundary and the host logic (no GPU compute)."""
import ctypes as C
import re
import subprocess

import numpy as np
import pytest

from gibbssampling_amd import _native, bioarray, synthetic
from gibbssampling_amd.dist import shard_bounds
from oracle import oracle_lib as ol


def test_library_exports_every_header_symbol():
    lib = _native.load_library()
    declared = _native.header_symbols()
    assert len(declared) >= 20
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    # and nothing with gs_ linkage that the header does not declare (public surface)
    out = subprocess.run(["nm", "-D", "--defined-only", str(_native.LIB_PATH)],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (gs_\w+)$", out, re.M))
    assert exported == set(declared), exported ^ set(declared)


def test_header_is_plain_c():
    """C ABI: compiles as C99 with no C++ or torch types."""
    src = '#include "gibbs_hip.h"\nint main(void){ gs_ctx *c = 0; (void)c; return 0; }\n'
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-x", "c", "-",
                        "-I", str(_native.HEADER_PATH.parent), "-o", "/dev/null"],
                       input=src, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    text = _native.HEADER_PATH.read_text()
    assert "torch" not in text and "std::" not in text


def test_version_and_host_rng():
    lib = _native.load_library()
    assert b"gfx950" in lib.gs_version()
    for seed, stream, idx in [(0, 0, 0), (7, _native.stream_sweep(3), 99), (2**63, 1, 2**33)]:
        assert _native.uniform(seed, stream, idx) == ol.uniform(seed, stream, idx)
        assert 0.0 <= _native.uniform(seed, stream, idx) < 1.0


def test_create_without_gpu_fails_cleanly():
    """In a GPU-less container gs_create reports GS_E_HIP instead of crashing."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = _native.load_library()
    h = C.c_void_p()
    assert lib.gs_create(0, C.byref(h)) == _native.GS_E_HIP
    assert not h.value


def test_native_raises_on_missing_library(tmp_path):
    with pytest.raises(ImportError):
        _native.load_library(tmp_path / "nope.so")


def test_bioarray_parsing_rules():
    # BioArray.ofNucleotideString: upper-case, drop whitespace / non-symbols (App. C)
    assert bioarray.of_nucleotide_string("acg t\nN-*xE1") == b"ACGTN-*"
    assert bioarray.of_amino_acid_string("mkl vz*-1\t") == b"MKLVZ*-"
    codes, off = bioarray.pack([b"ACGT", "GG", [65, 67]])
    assert codes.tobytes() == b"ACGTGGAC" and list(off) == [0, 4, 6, 8]
    assert bioarray.DNA_BASES == b"ATGC-"  # dnaBases of .fsx:368-369


def test_shard_bounds():
    lens = np.array([10, 10, 10, 10, 100, 10, 10, 10])
    b = shard_bounds(lens, 2)
    assert b[0][0] == 0 and b[-1][1] == 8 and b[0][1] == b[1][0]
    assert all(hi > lo for lo, hi in b)
    for world in (1, 2, 3, 8):
        b = shard_bounds(np.full(1000, 200), world)
        sizes = [hi - lo for lo, hi in b]
        assert sum(sizes) == 1000 and max(sizes) - min(sizes) <= 1
    assert shard_bounds([5, 5], 4)[-1] == (2, 2)


def test_synthetic_shards_are_consistent():
    w = synthetic.CONFIGS["cfg2"]
    c, o = synthetic.generate(w)
    c2, o2 = synthetic.generate(w, 3000, 5100)
    assert np.array_equal(c2, c[3000 * w.L:5100 * w.L])
    assert set(np.unique(c)) <= set(w.alphabet)
    p = synthetic.initial_positions(w)
    assert p.min() >= 0 and p.max() <= w.L - w.W
