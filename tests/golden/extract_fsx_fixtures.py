#!/usr/bin/env python3
"""Extract the sequence data sets of the reference's driver script as fixtures.

Reads /root/reference/GibbsSampling/GibbsSampling.fsx AS TEXT (nothing of the
reference is executed) and writes tests/golden/fsx_sets.json: the planted-motif
toy sets (.fsx:29-79), the heat-shock gene collection (.fsx:223-365) and the
31-gene Chlamydomonas `dataSet` (.fsx:546-1153), each parsed with the
BioArray.ofNucleotideString rules (gibbssampling_amd/bioarray.py).  Only the
data travels with the repo; this script is how it was made.
"""
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from gibbssampling_amd.bioarray import of_nucleotide_string  # noqa: E402

FSX = Path("/root/reference/GibbsSampling/GibbsSampling.fsx")


def strip_comments(text: str) -> str:
    # DNA literals never contain '//', so a line comment starts at the first '//'
    return "\n".join(line.split("//", 1)[0] for line in text.splitlines())


def let_block(text: str, name: str) -> str:
    m = re.search(r"^let %s\s*=" % re.escape(name), text, re.M)
    if not m:
        raise KeyError(name)
    nxt = re.search(r"^let ", text[m.end():], re.M)
    return text[m.end(): m.end() + (nxt.start() if nxt else len(text))]


def literals(block: str) -> list[str]:
    return re.findall(r'"([^"]*)"', strip_comments(block), re.S)


def names_in(block: str) -> list[str]:
    inner = strip_comments(block)
    inner = inner[inner.index("[|") + 2: inner.index("|]")]
    return [x.strip() for x in re.split(r"[;\s]+", inner) if x.strip()]


def main() -> None:
    text = FSX.read_text()
    out = {"source": "GibbsSampling/GibbsSampling.fsx (reference), parsed with "
                     "BioArray.ofNucleotideString rules; whitespace inside literals dropped"}
    for key, line in [("tests", ".fsx:29-35"), ("bioTestsWithMultipleSamples", ".fsx:49-57"),
                      ("bioTestsII", ".fsx:59-76")]:
        out[key] = {"cite": line,
                    "seqs": [of_nucleotide_string(s).decode() for s in literals(let_block(text, key))]}
    genes = names_in(let_block(text, "geneCollection"))
    out["geneCollection"] = {
        "cite": ".fsx:223-360",
        "seqs": [of_nucleotide_string(s).decode() for g in genes for s in literals(let_block(text, g))]}
    members = names_in(let_block(text, "dataSet"))
    out["dataSet"] = {
        "cite": ".fsx:546-1153",
        "seqs": [of_nucleotide_string(s).decode() for g in members for s in literals(let_block(text, g))]}
    for k in ("tests", "bioTestsWithMultipleSamples", "bioTestsII", "geneCollection", "dataSet"):
        print(k, len(out[k]["seqs"]), sum(len(s) for s in out[k]["seqs"]))
    (Path(__file__).parent / "fsx_sets.json").write_text(json.dumps(out, indent=0))


if __name__ == "__main__":
    main()
