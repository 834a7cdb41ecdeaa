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
