"""Host-side unit test of the native C++ runtime (slab partition invariants, TCP star
collectives across forked ranks, summary block), compiled with AddressSanitizer and
UBSan (`make -C csrc check`).  GPU sanitizers are unavailable on the pool, so the host
code is where ASan runs (race detection / sanitizers)."""
import shutil
import subprocess
from pathlib import Path

import pytest

CSRC = Path(__file__).resolve().parent.parent / "csrc"


@pytest.mark.skipif(shutil.which("g++") is None or not Path("/opt/rocm/include").exists(),
                    reason="needs g++ and the ROCm headers")
def test_runtime_host_asan():
    lib = CSRC.parent / "multigpu_advectiondiffusion_amd" / "lib" / "libadvdiff.so"
    if not lib.exists():
        pytest.skip("libadvdiff.so not built")
    r = subprocess.run(["make", "-C", str(CSRC), "check"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "runtime host tests: OK" in r.stdout


def test_library_matches_tree():
    """The in-tree libadvdiff.so must be built from the kernel sources in this tree: its
    compiled-in source hash (csrc/Makefile SRC_HASH) equals the hash of csrc/ now, and the
    Makefile and the Python loader compute that hash identically."""
    from multigpu_advectiondiffusion_amd.ops import _lib
    r = subprocess.run(["make", "-s", "-C", str(CSRC), "hash"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == _lib.source_hash()
    if not _lib.LIB_PATH.exists():
        pytest.skip("libadvdiff.so not built")
    if not _lib.available():
        err = _lib.load_error() or ""
        assert "stale" not in err, err
        pytest.skip(f"library not loadable here: {err}")
    assert _lib.library_hash() == _lib.source_hash()
