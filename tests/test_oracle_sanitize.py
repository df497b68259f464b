"""The CPU oracle (the checker every parity claim rests on) under host
AddressSanitizer + UndefinedBehaviorSanitizer: oracle/sanitize_main.c runs the
faithful and hold-one-out restatements, the greedy, initialiser and site passes on
seeded data sets shaped like the golden fixtures and cross-checks them; any memory
error, UB, or difference fails the run.  CPU only."""
import os
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "asan"], check=True, timeout=300)
    env = dict(os.environ, OMP_NUM_THREADS="2",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(ROOT / "oracle" / "_build" / "oracle_sanitize")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "all checks passed" in r.stdout
