"""Solution output and checkpoint/restart.

* ``save_binary`` / ``load_binary``: the reference's raw float32, x-fastest, header-less
  ``result.bin`` / ``initial.bin`` (`MultiGPU/Diffusion3d_Baseline/Tools.c:91-119`,
  `SingleGPU/Diffusion2d/tools.cpp:48-73`), optionally including the ghost planes like
  the MultiGPU apps do (`main.c:341`).
* ``save_checkpoint`` / ``load_checkpoint``: lossless fp64 restart files (absent in the
  reference).  Every rank writes ONE shard holding its owned planes and a
  JSON header (global grid, time, iteration, model, the global plane range of the
  shard).  Any decomposition can restart from any set of shards: a rank memory-maps
  each shard and copies the planes it owns — so a run checkpointed on 8 GPUs restarts on
  1, 2 or 4.  The format executes nothing on load (magic + JSON + raw little-endian
  array), unlike pickle-based checkpoints.
"""
from __future__ import annotations

import json
import os
import struct
from pathlib import Path

import numpy as np

MAGIC = b"ADVDIFF1"


def save_binary(path, arr: np.ndarray) -> None:
    """Raw float32, x fastest (C-order of an array indexed [z][y][x])."""
    np.ascontiguousarray(arr, dtype=np.float32).tofile(path)


def load_binary(path, shape) -> np.ndarray:
    """Inverse of save_binary; shape = (nz, ny, nx) or (ny, nx)."""
    return np.fromfile(path, dtype=np.float32).reshape(shape)


def save_ascii(path, arr: np.ndarray) -> None:
    """One value per line ("%g"), x fastest — the reference's ASCII `Save3D`/`Save2D`
    dump (`MultiGPU/Diffusion3d_Baseline/Tools.c:66-86`)."""
    np.savetxt(path, np.ascontiguousarray(arr).reshape(-1), fmt="%g")


def format_field(arr: np.ndarray, fmt: str = "%8.2f") -> str:
    """Text block of a 2-D/3-D field, rows of x, blank line between planes — the
    reference's `Print3D`/`Print2D` debug printers (`Tools.c:32-61`)."""
    a = np.asarray(arr)
    planes = a.reshape((-1,) + a.shape[-2:]) if a.ndim >= 2 else a.reshape(1, 1, -1)
    out = []
    for p in planes:
        for row in p:
            out.append("".join(fmt % v for v in row))
        out.append("")
    return "\n".join(out) + "\n"


def _shard_name(prefix: Path, rank: int) -> Path:
    return prefix.parent / f"{prefix.name}.rank{rank:05d}.ckpt"


def save_checkpoint(prefix, rank: int, local: np.ndarray, plane0: int, meta: dict,
                    box0=None) -> Path:
    """Write this rank's shard. `local` holds global planes plane0 .. plane0+len-1 along
    axis 0 (no ghosts); for a Cartesian block ``box0`` gives its global offset on every
    axis.  `meta` must contain JSON-serialisable run metadata."""
    prefix = Path(prefix)
    prefix.parent.mkdir(parents=True, exist_ok=True)
    local = np.ascontiguousarray(local)
    header = dict(meta)
    header.update({"plane0": int(plane0), "nplanes": int(local.shape[0]),
                   "shape": list(local.shape), "dtype": str(local.dtype), "rank": rank,
                   "box0": [int(v) for v in (box0 if box0 is not None
                                              else [plane0] + [0] * (local.ndim - 1))]})
    hb = json.dumps(header, sort_keys=True).encode()
    path = _shard_name(prefix, rank)
    tmp = path.with_suffix(".tmp")
    with open(tmp, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<Q", len(hb)))
        f.write(hb)
        pad = (-(len(MAGIC) + 8 + len(hb))) % 64  # 64-B align the payload for mmap
        f.write(b"\0" * pad)
        f.write(local.astype(local.dtype.newbyteorder("<"), copy=False).tobytes())
    os.replace(tmp, path)
    return path


def remove_stale_shards(prefix, world: int) -> list:
    """Delete PREFIX.rankNNNNN.ckpt for every N >= world: shards of an earlier run on more
    ranks under the same prefix would otherwise be read back with this run's (call on one
    rank, after every rank's shard is written).  Returns the removed paths."""
    prefix = Path(prefix)
    gone = []
    for p in prefix.parent.glob(f"{prefix.name}.rank*.ckpt"):
        tail = p.name[len(prefix.name) + len(".rank"):-len(".ckpt")]
        if tail.isdigit() and int(tail) >= world:
            p.unlink()
            gone.append(p)
    return gone


def read_header(path):
    with open(path, "rb") as f:
        if f.read(len(MAGIC)) != MAGIC:
            raise ValueError(f"{path}: not an advdiff checkpoint")
        (n,) = struct.unpack("<Q", f.read(8))
        header = json.loads(f.read(n))
        off = len(MAGIC) + 8 + n
        off += (-off) % 64
    return header, off


def list_shards(prefix):
    prefix = Path(prefix)
    shards = sorted(prefix.parent.glob(f"{prefix.name}.rank*.ckpt"))
    if not shards:
        raise FileNotFoundError(f"no checkpoint shards for {prefix}")
    return shards


def load_checkpoint_box(prefix, box0, extents):
    """Assemble the global box [box0, box0+extents) (array axis order) from whatever
    shards exist (slab or Cartesian, any process count).  Returns (array, meta)."""
    out = None
    meta = None
    covered = 0
    for path in list_shards(prefix):
        h, off = read_header(path)
        if meta is None:
            meta = h
        elif (h.get("it"), h.get("t")) != (meta.get("it"), meta.get("t")):
            # e.g. stale shards of an earlier run on more ranks under the same prefix
            raise ValueError(f"{path}: shard of another checkpoint (it {h.get('it')} vs "
                             f"{meta.get('it')}) under the prefix {prefix}")
        if "world" in h and int(h.get("rank", 0)) >= int(h["world"]):
            raise ValueError(f"{path}: shard of rank {h.get('rank')} in a {h['world']}-rank "
                             f"checkpoint")
        dt = np.dtype(h["dtype"]).newbyteorder("<")
        shape = tuple(h["shape"])
        sb = h.get("box0", [h["plane0"]] + [0] * (len(shape) - 1))
        lo = [max(s, b) for s, b in zip(sb, box0)]
        hi = [min(s + n, b + e) for s, n, b, e in zip(sb, shape, box0, extents)]
        if any(b <= a for a, b in zip(lo, hi)):
            continue
        mm = np.memmap(path, dtype=dt, mode="r", offset=off, shape=shape)
        if out is None:
            out = np.empty(tuple(extents), dtype=np.dtype(h["dtype"]))
        dst = tuple(slice(a - b, c - b) for a, c, b in zip(lo, hi, box0))
        src = tuple(slice(a - s, c - s) for a, c, s in zip(lo, hi, sb))
        out[dst] = mm[src]
        n = 1
        for a, b in zip(lo, hi):
            n *= b - a
        covered += n
        del mm
    total = 1
    for e in extents:
        total *= e
    if covered > total:
        raise ValueError(f"checkpoint {prefix}: overlapping shards cover box {box0} + "
                         f"{extents} {covered / total:.2f} times (shards of two runs?)")
    if out is None or covered != total:
        raise ValueError(f"checkpoint {prefix} does not cover box {box0} + {extents}")
    return out, meta


def load_checkpoint(prefix, plane0: int, nplanes: int):
    """Assemble global planes [plane0, plane0+nplanes) (full extent of the other axes)
    from whatever shards exist.  Returns (array, meta of the first shard)."""
    h, _ = read_header(list_shards(prefix)[0])
    grid = list(h["grid"])[::-1]  # array order
    return load_checkpoint_box(prefix, [plane0] + [0] * (len(grid) - 1),
                               [nplanes] + grid[1:])
