"""utils/sizing.py: the pitch rule is applied to the global cells per rank, as the Solver
does (round-5 advisor finding: with the ghost-inclusive allocation the rule could flip
near its 128 MiB threshold).  The GPU comparison with Solver.memory_bytes() is
tests/test_pitch_gpu.py::test_sizing_matches_solver_memory_at_the_pitch_threshold."""
from multigpu_advectiondiffusion_amd.utils.sizing import max_cube, row_pitch, solver_bytes


def test_threshold_uses_cells_per_rank():
    n = 256                      # 256^3 fp64 = 128 MiB: exactly at the threshold, dense
    alloc = (n + 12, n, n)       # + 2 x 3R ghost planes: past the threshold
    dense = 2 * (n + 12) * n * row_pitch(n, 8) * 8
    assert solver_bytes(alloc, 8, 2, cells_per_rank=n ** 3) == dense
    pitched = 2 * (n + 12) * (n + 1) * (row_pitch(n, 8) + 4) * 8
    assert solver_bytes(alloc, 8, 2, cells_per_rank=n ** 3 + 1) == pitched


def test_max_cube_fits():
    n = max_cube(288 * 10 ** 9, 8, 2, 6)
    assert n % 64 == 0 and solver_bytes((n + 12, n, n), 8, 2, cells_per_rank=n ** 3) < 288e9
