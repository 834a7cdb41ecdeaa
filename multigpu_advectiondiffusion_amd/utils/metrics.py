"""Throughput metrics and the reference's summary block.

Reference formulas (BASELINE.md "Metric definitions"):
* "Total effective GFLOPs" = 3·it·cells·FLOPS·1e-9 / t for MultiGPU and SingleGPU-Burgers
  (`MultiGPU/Diffusion3d_Baseline/Tools.c:247-250`, `SingleGPU/Burgers3d_WENO5/tools.cpp:145-148`),
  it·cells·FLOPS·1e-9 / t for SingleGPU diffusion (no ×3,
  `SingleGPU/Diffusion3d_baselineCode/tools.cpp:148-151`); FLOPS = 8.
* MLUPS = cells·steps / t / 1e6 with one step = one full SSP-RK3 step (3 stages).

The summary printers reproduce the reference labels byte-for-byte
(`MultiGPU/Diffusion3d_Baseline/Tools.c:255-270`, `SingleGPU/.../tools.cpp:185-199`) and
append the MLUPS / bandwidth lines the reference lacks.
"""
from __future__ import annotations

FLOPS = 8.0
SEP = "=" * 67


def gflops_reference(seconds: float, iterations: int, cells: int, times3: bool = True) -> float:
    if seconds <= 0:
        return 0.0
    return (3 if times3 else 1) * iterations * cells * 1e-9 * FLOPS / seconds


def mlups(seconds: float, steps: int, cells: int) -> float:
    return cells * steps / seconds / 1e6 if seconds > 0 else 0.0


def summary_multigpu(title: str, optimization: str, compute_s: float, htod_s: float,
                     dtoh_s: float, gflops: float, iterations: int, grid, extra=None,
                     stages: int = 3) -> str:
    nx, ny = grid[0], grid[1]
    lines = [f"======================={title}=====================",
             f"Optimization                                 :  {optimization}",
             f"Kernel time ex. data transfers               :  {compute_s:f} seconds",
             f"Data transfer(s) HtD                         :  {htod_s:f} seconds",
             f"Data transfer(s) DtH                         :  {dtoh_s:f} seconds",
             SEP,
             f"Total effective GFLOPs                       :  {gflops:f}",
             SEP]
    if len(grid) == 3:
        lines.append(f"3D Grid Size                                 :  {nx} x {ny} x {grid[2]}")
    else:
        lines.append(f"2D Grid Size                                 :  {nx} x {ny}")
    lines.append(f"Iterations                                   :  {iterations} x {stages} RK steps")
    lines.append(SEP)
    for k, v in (extra or {}).items():
        lines.append(f"{k:<45}:  {v}")
    if extra:
        lines.append(SEP)
    return "\n".join(lines)


def summary_singlegpu(title: str, optimization: str, compute_s: float, gflops: float,
                      iterations: int, grid, final_time: float, extra=None) -> str:
    nx, ny = grid[0], grid[1]
    lines = [f"=========================== {title} =======================",
             f"Optimization                                 :  {optimization}",
             f"Kernel time ex. data transfers               :  {compute_s:f} seconds",
             SEP,
             f"Total effective GFLOPs                       :  {gflops:f}",
             SEP]
    if len(grid) == 3:
        lines.append(f"3D Grid Size                                 :  {nx} x {ny} x {grid[2]} ")
    else:
        lines.append(f"2D Grid Size                                 :  {nx} x {ny} ")
    lines.append(f"Iterations                                   :  {iterations}")
    lines.append(f"Final Time                                   :  {final_time:g}")
    lines.append(SEP)
    for k, v in (extra or {}).items():
        lines.append(f"{k:<45}:  {v}")
    if extra:
        lines.append(SEP)
    return "\n".join(lines)


def error_norms_block(l1: float, l2: float, linf: float) -> str:
    """`CalcError` output (`SingleGPU/Diffusion3d_baselineCode/tools.cpp:177-179`)."""
    return "\n".join([f"L1 norm                                       :  {l1:e}",
                      f"L2 norm                                       :  {l2:e}",
                      f"Linf norm                                     :  {linf:e}"])
