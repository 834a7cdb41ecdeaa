"""Host-side unit test of the native C++ runtime (slab partition invariants, TCP star
collectives across forked ranks, summary block), compiled with AddressSanitizer and
UBSan (`make -C csrc check`).  GPU sanitizers are unavailable on the pool, so the host
code is where ASan runs (race detection / sanitizers)."""
import shutil
import subprocess
from pathlib import Path

import numpy as np
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


def _tree_hash(paths):
    import hashlib
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update((CSRC / p).read_bytes())
    return h.hexdigest()[:16]


def runtime_tree_hash():
    """Hash of the native runtime + app sources (csrc/Makefile RT_HASH)."""
    rel = [f"runtime/{p.name}" for p in (CSRC / "runtime").iterdir() if p.suffix in (".cpp", ".hpp")]
    rel += [f"apps/{p.name}" for p in (CSRC / "apps").iterdir() if p.suffix == ".cpp"]
    return _tree_hash(rel)


def test_native_binaries_match_tree():
    """bin/* embed the hash of the runtime/app sources they were built from
    (advdiff_runtime_hash); it must equal the tree's, so a stale bin/ fails here (and its
    banner is checked again by the GPU tests)."""
    r = subprocess.run(["make", "-s", "-C", str(CSRC), "rthash"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == runtime_tree_hash()
    bins = [CSRC.parent / "bin" / a for a in ("diffusion2d", "diffusion3d", "burgers2d", "burgers3d")]
    if not all(b.exists() for b in bins):
        pytest.skip("bin/ not built")
    for b in bins:
        assert runtime_tree_hash().encode() in b.read_bytes(), f"{b} is stale (make -C csrc apps)"


GEOMETRY_CASES = [
    # app, positional args, world, decomp, extra
    ("diffusion3d", [1, 1, 1, 1, 50, 44, 46, 9], 8, "2x2x2", []),
    ("diffusion3d", [1, 1, 1, 1, 66, 40, 45, 12], 4, "1x2x2", []),
    ("diffusion3d", [1, 1, 1, 1, 66, 40, 45, 12], 4, "2x2x1", ["--no-fused"]),
    ("diffusion3d", [1, 1, 1, 1, 66, 40, 45, 12], 3, "slab", []),
    ("burgers3d", [0.03, 0.3, 2, 2, 2, 40, 36, 41], 4, "2x1x2", []),
    ("diffusion2d", [1, 1, 1, 130, 90, 30], 4, "2x2", []),
    ("burgers2d", [0.1, 0.4, 2, 2, 140, 100], 2, "1x2", ["--weno", "js"]),
]


@pytest.mark.parametrize("corners", ["direct", "phased"])
@pytest.mark.parametrize("app,args,world,decomp,extra", GEOMETRY_CASES)
def test_native_geometry_matches_python(app, args, world, decomp, extra, corners):
    """Every rank's launch boxes, fused-step views and halo messages of the native runtime
    (bin/<app> --geometry, csrc/runtime/cart.cpp) equal the Python decomposition's
    (CartesianDecomposition, CartesianHalo.boxes, decomposition.fused_view)."""
    _check_native_geometry(app, args, world, decomp, extra, corners)


def _native_layouts():
    from hypothesis import strategies as st

    @st.composite
    def draw_layout(draw):
        app = draw(st.sampled_from(["diffusion3d", "diffusion2d", "burgers3d"]))
        dims = 2 if app.endswith("2d") else 3
        pgrid = [draw(st.integers(1, 3)) for _ in range(dims)]
        if all(p == 1 for p in pgrid):
            pgrid[0] = 2
        # array-order extents: >= R cells per block; thin blocks fall back to per-stage
        shape = [p * 3 + draw(st.integers(1, 24)) for p in pgrid]
        if app == "burgers3d":
            shape = [max(n, 7) for n in shape]
        ext = list(reversed(shape))  # Nx Ny [Nz]
        if app == "diffusion3d":
            args = [1, 1, 1, 1] + ext + [2]
        elif app == "diffusion2d":
            args = [1, 1, 1] + ext + [2]
        else:
            args = [0.01, 0.3, 2, 2, 2] + ext
        extra = draw(st.sampled_from([[], ["--no-fused"]])) if app.startswith("diff") else []
        corners = draw(st.sampled_from(["direct", "phased"]))
        decomp = "x".join(str(p) for p in pgrid)
        return app, args, int(np.prod(pgrid)), decomp, extra, corners
    return draw_layout()


def test_native_geometry_matches_python_random():
    """The same comparison over random layouts (hypothesis): process grids up to 3 per
    axis, uneven blocks, thin blocks that fall back to per-stage launches, both corner
    modes."""
    hyp = pytest.importorskip("hypothesis")
    if not (CSRC.parent / "bin" / "diffusion3d").exists():
        pytest.skip("bin/ not built")

    @hyp.settings(max_examples=60, deadline=None, derandomize=True)
    @hyp.given(_native_layouts())
    def run(layout):
        _check_native_geometry(*layout)
    run()


def _check_native_geometry(app, args, world, decomp, extra, corners):
    import json
    import os

    from multigpu_advectiondiffusion_amd.models import Burgers, Diffusion
    from multigpu_advectiondiffusion_amd.parallel.decomposition import (
        CartesianDecomposition, fused_view, parse_proc_grid)
    from multigpu_advectiondiffusion_amd.parallel.halo import CartesianHalo
    exe = CSRC.parent / "bin" / app
    if not exe.exists():
        pytest.skip("bin/ not built")
    env = dict(os.environ, RANK="0", WORLD_SIZE=str(world), ADVDIFF_CORNERS=corners)
    cmd = [str(exe)] + [str(a) for a in args] + ["--decomp", decomp, "--geometry"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=60, env=env)
    three = app.endswith("3d")
    if app.startswith("diffusion"):
        model = Diffusion(K=1.0, order=4)
        shape = tuple(reversed(args[4:7] if three else args[3:5]))
    else:
        model = Burgers(viscosity=1e-5, weno="js" if "js" in extra else "z", cfl=0.3)
        shape = tuple(reversed(args[5:8] if three else args[4:6]))
    R, B = model.radius, model.border
    pgrid = parse_proc_grid(None if decomp == "slab" else decomp, world, shape, R)
    fused = model.supports_fused and "--no-fused" not in extra and not any(
        n // p < 3 * R for n, p in zip(shape, pgrid) if p > 1)
    G = 3 * R if fused else R
    if r.returncode != 0 and "thinner than the ghost width" in r.stderr:
        # a layout both sides refuse (a block, or an unsplit axis 0, thinner than G)
        with pytest.raises(ValueError):
            CartesianDecomposition(shape, pgrid, 0, G)
        return
    assert r.returncode == 0, r.stderr
    native = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert len(native) == world
    lst = lambda box: [list(x) for x in box]  # noqa: E731
    for rank in range(world):
        cd = CartesianDecomposition(shape, pgrid, rank, G)
        nat = native[rank]
        assert nat["fused"] == fused and nat["ghost"] == G
        assert nat["coords"] == list(cd.coords)
        assert nat["alloc"] == list(cd.alloc)
        assert nat["own"] == lst(cd.owned_box())
        assert nat["full"] == lst(cd.compute_box(B))
        interior, boundary = cd.split_boxes(B, G)
        assert nat["interior"] == lst(interior)
        assert nat["boundary"] == [lst(b) for b in boundary]
        if fused:
            boxes = [cd.compute_box(B), interior] + list(boundary)
            boxes = [b for b in boxes if all(hi > lo for lo, hi in b)]
            assert len(nat["views"]) == len(boxes)
            for v, box in zip(nat["views"], boxes):
                assert v["box"] == lst(box)
                for a in range(1, len(shape)):
                    want = [list(x) for x in fused_view(cd, R, B, a, *box[a])]
                    assert v["axes"][a - 1] == want, (rank, box, a)
        if cd.size > 1 and not cd.is_slab:
            halo = CartesianHalo(None, cd, corners=fused, direct=corners == "direct")
            py = [[{"peer": p, "off": list(k), "send": lst(s), "recv": lst(rr)}
                   for p, s, rr, k in halo.boxes(axes)] for axes in halo._phases()]
            assert nat["halo"] == py, rank


def test_native_config_file_host(tmp_path):
    """bin/* --config FILE.json on the CPU (the file is applied before any device work):
    a config that carries the positional args and the decomposition gives the same
    --geometry output as the command line; malformed files fail with a message."""
    import json
    import os
    exe = CSRC.parent / "bin" / "diffusion3d"
    if not exe.exists():
        pytest.skip("bin/ not built")
    env = dict(os.environ, RANK="0", WORLD_SIZE="4")
    args = ["1", "1", "1", "1", "40", "36", "32", "5"]
    a = subprocess.run([str(exe), *args, "--decomp", "2x2x1", "--geometry"], env=env,
                       capture_output=True, text=True, timeout=60)
    cfg = tmp_path / "c.json"
    cfg.write_text(json.dumps({"args": [1, 1, 1, 1, 40, 36, 32, 5], "decomp": "2x2x1",
                               "geometry": True}))
    b = subprocess.run([str(exe), "--config", str(cfg)], env=env, capture_output=True,
                       text=True, timeout=60)
    assert a.returncode == 0 and b.returncode == 0, (a.stdout + a.stderr, b.stdout + b.stderr)
    assert a.stdout == b.stdout and a.stdout.count("\n") == 4
    for bad, msg in (('{"args": [1, 2}', 'bad "args" list'), ('{"ic": }', "bad value of ic"),
                     ('[1, 2]', "not a JSON object"), ('{1: 2}', "expected a key")):
        cfg.write_text(bad)
        r = subprocess.run([str(exe), "--config", str(cfg)], env=env, capture_output=True,
                           text=True, timeout=30)
        assert r.returncode != 0 and msg in r.stderr, (bad, r.stderr)
