"""Packaging: ``pip install .`` / ``pip install -e .``.

The build_py hook builds lib/libadvdiff.so (csrc/Makefile, hipcc --offload-arch=gfx950)
before the Python files are collected, so a wheel or an editable install carries the
kernels.  ADVDIFF_SKIP_NATIVE_BUILD=1 packages whatever library is already in the tree."""
import os
import re
import subprocess
from pathlib import Path

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py
from setuptools.dist import Distribution

ROOT = Path(__file__).resolve().parent
PKG = "multigpu_advectiondiffusion_amd"
VERSION = re.search(r'__version__ = "([^"]+)"', (ROOT / PKG / "__init__.py").read_text()).group(1)


class BuildWithKernels(build_py):
    def run(self):
        if os.environ.get("ADVDIFF_SKIP_NATIVE_BUILD") != "1":
            jobs = str(min(16, os.cpu_count() or 4))
            subprocess.run(["make", "-C", str(ROOT / "csrc"), f"-j{jobs}", "lib"], check=True)
        super().run()


class BinaryDistribution(Distribution):
    """The wheel carries a gfx950 / x86-64 shared library: tag it for the platform."""

    def has_ext_modules(self):
        return True


setup(
    name="multigpu-advectiondiffusion-amd",
    version=VERSION,
    description="MI355X-native (gfx950) multi-GPU heat / Burgers stencil framework: "
                "hand-written HIP kernels, RCCL or peer-mapped halos",
    long_description=(ROOT / "README.md").read_text(),
    long_description_content_type="text/markdown",
    python_requires=">=3.10",
    packages=find_packages(include=[PKG, PKG + ".*"]),
    package_data={PKG: ["lib/libadvdiff.so"]},
    install_requires=["torch", "numpy"],
    extras_require={"test": ["pytest", "pytest-timeout", "hypothesis", "scipy"],
                    "plot": ["matplotlib"]},
    entry_points={"console_scripts": [
        f"advdiff = {PKG}.cli:main",
        f"advdiff-launch = {PKG}.launch:main",
        f"advdiff-runall = {PKG}.runall:main",
        f"advdiff-devices = {PKG}.devices:main",
        f"advdiff-sizing = {PKG}.utils.sizing:main",
    ]},
    cmdclass={"build_py": BuildWithKernels},
    distclass=BinaryDistribution,
)
