"""Packaging (setup.py / pyproject.toml): the console scripts resolve to callables, the
version is the package's, and the wheel ships the kernel library."""
import importlib
import re
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def _entry_points():
    src = (ROOT / "setup.py").read_text()
    pkg = re.search(r'PKG = "([^"]+)"', src).group(1)
    eps = re.findall(r'f"([\w-]+) = \{PKG\}([\w.]*):(\w+)"', src)
    assert eps, "no console_scripts found in setup.py"
    return [(name, pkg + mod, fn) for name, mod, fn in eps]


@pytest.mark.parametrize("name,mod,fn", _entry_points())
def test_console_script_resolves(name, mod, fn):
    assert callable(getattr(importlib.import_module(mod), fn)), f"{name} -> {mod}:{fn}"


def test_setup_metadata():
    import multigpu_advectiondiffusion_amd as m
    out = subprocess.run([sys.executable, "setup.py", "--version"], cwd=ROOT,
                         capture_output=True, text=True, check=True).stdout.split()
    assert out[-1] == m.__version__
    assert "lib/libadvdiff.so" in (ROOT / "setup.py").read_text()
