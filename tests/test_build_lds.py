"""The built library's live and long sweep kernels allocate no static LDS
(tools/lds_static.py): they address their tables from LDS offset 0 and take a nonzero
dynamic base as a table fault, which would send every target to the exact rescan --
parity would still hold, so only this check (and the rescan counters) would see it."""
import shutil
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))


@pytest.mark.skipif(not (ROOT / "gibbssampling_amd/libgibbs_hip.so").exists() or shutil.which("objcopy") is None,
                    reason="library not built")
def test_live_long_kernels_no_static_lds():
    from lds_static import static_lds
    sizes = static_lds(str(ROOT / "gibbssampling_amd/libgibbs_hip.so"))
    zero = {k: v for k, v in sizes.items() if "gs_sweep_live_kernel" in k or "gs_sweep_long_kernel" in k}
    assert len(zero) >= 10, sorted(sizes)
    assert all(v == 0 for v in zero.values()), zero
