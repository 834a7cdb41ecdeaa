"""Visualisation helpers — the reference's L6 plotting layer (`*/myplot.m`, the slice
plots at the end of every `Run.m`, and the k-Wave colour map of `*/getColorMap.m`).

Reads the raw float32 ``result.bin`` (x fastest) and renders orthogonal mid-plane slices
(3-D) or the field (2-D) to PNG with matplotlib (Agg, no display needed).
"""
from __future__ import annotations

import numpy as np


def kwave_colormap(n: int = 256):
    """Bone for the negative half, reversed hot for the positive half (k-Wave style,
    `getColorMap('kwave')`), rebuilt from matplotlib's bone/hot maps."""
    from matplotlib import colormaps
    from matplotlib.colors import ListedColormap
    pad = 48 * n // 256
    bone = colormaps["bone"](np.linspace(0, 1, n // 2 + pad))[pad:]
    hot = colormaps["hot"](np.linspace(0, 1, n // 2))[::-1]
    return ListedColormap(np.vstack([bone, hot]), name="kwave")


def plot_slices(arr: np.ndarray, path: str, title: str = "", lengths=None, cmap=None):
    """Save mid-plane slices of a [z][y][x] array (or the [y][x] field in 2-D)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    cmap = cmap or kwave_colormap()
    if arr.ndim == 2:
        fig, ax = plt.subplots(figsize=(5, 4))
        ext = None if lengths is None else (0, lengths[0], 0, lengths[1])
        im = ax.imshow(arr, origin="lower", cmap=cmap, extent=ext, aspect="auto")
        fig.colorbar(im, ax=ax)
        ax.set_xlabel("x")
        ax.set_ylabel("y")
    else:
        nz, ny, nx = arr.shape
        fig, axes = plt.subplots(1, 3, figsize=(13, 4))
        vmin, vmax = float(arr.min()), float(arr.max())
        for ax, sl, lab in ((axes[0], arr[nz // 2], "z mid-plane (x-y)"),
                            (axes[1], arr[:, ny // 2, :], "y mid-plane (x-z)"),
                            (axes[2], arr[:, :, nx // 2], "x mid-plane (y-z)")):
            im = ax.imshow(sl, origin="lower", cmap=cmap, vmin=vmin, vmax=vmax, aspect="auto")
            ax.set_title(lab)
        fig.colorbar(im, ax=list(axes))
    if title:
        fig.suptitle(title)
    fig.savefig(path, dpi=110)
    plt.close(fig)
    return path


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="plot a float32 result.bin")
    ap.add_argument("file")
    ap.add_argument("shape", nargs="+", type=int, help="Nx Ny [Nz]")
    ap.add_argument("-o", "--out", default=None)
    ap.add_argument("--title", default="")
    a = ap.parse_args(argv)
    shape = tuple(reversed(a.shape))
    arr = np.fromfile(a.file, dtype=np.float32).reshape(shape)
    out = a.out or a.file.rsplit(".", 1)[0] + ".png"
    plot_slices(arr, out, a.title)
    print(out)


if __name__ == "__main__":
    main()
