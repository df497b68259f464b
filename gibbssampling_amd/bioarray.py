"""Input-format layer: BioFSharp's string parsers and symbol codes, restated.

The sampler consumes `BioItem.symbol` codes (ASCII, slot = code - 42, .fs:17).
The parsing rules below were recovered from the vendored BioFSharp.dll IL
(SURVEY.md Appendix C); they are the contract the F# caller's data obeys.
"""
from __future__ import annotations

from typing import Iterable, Sequence

import numpy as np

# Nucleotides.charToParsedNucleotideChar: everything here maps to Some(symbol).
_NUC_ACCEPT = set("ACGTUI" "BDHKMNRSVWY" "*-")
# BioArray.ofAminoAcidSymbolString: A-Z, '-' and '*'.
_AA_ACCEPT = set("ABCDEFGHIJKLMNOPQRSTUVWXYZ" "*-")

#: dnaBases of GibbsSampling.fsx:368-369 = [A; T; G; C; Gap]  (|A| = 5)
DNA_BASES = b"ATGC-"
#: plain ACGT alphabet used by BASELINE.json's synthetic configs (|A| = 4)
ACGT = b"ACGT"
#: aminoAcids of GibbsSampling.fsx:372-382 (24 symbols, one-letter codes)
AMINO_ACIDS = b"ARNDBCJQEZGHILKMFPOUSTWV"
#: the 20 standard amino acids (BASELINE config 5)
AMINO20 = b"ACDEFGHIKLMNPQRSTVWY"


def of_nucleotide_string(s: str) -> bytes:
    """BioArray.ofNucleotideString: upper-case, keep parsable symbols, drop the rest."""
    return bytes(ord(ch) for ch in s.upper() if ch in _NUC_ACCEPT)


def of_amino_acid_string(s: str) -> bytes:
    """BioArray.ofAminoAcidSymbolString: upper-case, keep A-Z, '-', '*'."""
    return bytes(ord(ch) for ch in s.upper() if ch in _AA_ACCEPT)


def pack(sources: Sequence[bytes | str | Iterable[int]]) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate sequences into (codes uint8, offsets int64[N+1])."""
    parts = []
    for s in sources:
        if isinstance(s, str):
            s = s.encode("ascii")
        parts.append(np.frombuffer(bytes(s), np.uint8) if isinstance(s, (bytes, bytearray))
                     else np.asarray(list(s), np.uint8))
    lens = np.array([len(p) for p in parts], np.int64)
    offsets = np.zeros(len(parts) + 1, np.int64)
    np.cumsum(lens, out=offsets[1:])
    codes = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return codes.astype(np.uint8, copy=False), offsets


def alphabet_codes(alphabet: bytes | str | Iterable[int]) -> bytes:
    if isinstance(alphabet, str):
        return alphabet.encode("ascii")
    if isinstance(alphabet, (bytes, bytearray)):
        return bytes(alphabet)
    return bytes(int(x) for x in alphabet)
