"""The banded z-schedule model of the fused heat step (diffusion_fused.hip step_bands,
host-only, queried through advdiff_step_bands_plan): its splits cover the launch's planes
exactly, never model worse than the best uniform chunking, and pin the choices the round-5
A/Bs measured (512^3 FD4: 387 + 121 planes, profiles/r5/ab/band_sweep.log)."""
import ctypes

import pytest

from multigpu_advectiondiffusion_amd.ops import _lib


def _plan(n, tiles, slots=256, warm=8, minc=16):
    try:
        lib = _lib.require()
    except RuntimeError as e:  # pragma: no cover - the library is built in-tree
        pytest.skip(str(e))
    out = (ctypes.c_longlong * 5)()
    assert lib.advdiff_step_bands_plan(n, tiles, slots, warm, minc, out) == 0
    return tuple(int(v) for v in out)


@pytest.mark.parametrize("n,tiles,warm", [(508, 189, 8), (510, 144, 4), (116, 817, 8),
                                          (122, 544, 4), (244, 418, 8), (1020, 817, 8),
                                          (17, 9, 8), (64, 2000, 4), (300, 1, 8)])
def test_band_plan_covers_the_range_and_beats_uniform(n, tiles, warm):
    first, rest, nb, span, uni = _plan(n, tiles, warm=warm)
    assert 1 <= first <= n and nb >= 1 and rest >= 1
    covered = first + (nb - 1) * rest
    assert covered >= n  # every plane in some band
    if nb > 1:
        assert first + (nb - 2) * rest < n  # no empty band
    assert span <= uni  # never modelled worse than uniform chunks


def test_band_plan_pins_the_measured_choices():
    assert _plan(508, 189)[:3] == (387, 121, 2)      # 512^3 FD4 (band_sweep.log best)
    assert _plan(116, 817)[:3] == (91, 25, 2)        # 8-GPU slab rank, FD4 interior


def test_band_plan_rejects_bad_arguments():
    lib = _lib.require()
    out = (ctypes.c_longlong * 5)()
    assert lib.advdiff_step_bands_plan(0, 10, 256, 8, 16, out) != 0
    assert lib.advdiff_step_bands_plan(10, 10, 256, 8, 16, None) != 0
