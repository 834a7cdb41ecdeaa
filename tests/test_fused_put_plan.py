"""Host-side logic of the fused halo puts (transport "ipc+fused", round 6): the bench's
candidate list, the solver switch, and the peer-address plan SlabHalo.put_targets hands
the step kernel (the kernel itself: tests/test_ipc_gpu.py::test_ipc_fused_put_bitwise)."""
import sys
from pathlib import Path

import pytest
import torch

from multigpu_advectiondiffusion_amd import Diffusion, Grid, Solver
from multigpu_advectiondiffusion_amd.parallel import halo as halo_mod
from multigpu_advectiondiffusion_amd.parallel.decomposition import SlabDecomposition
from multigpu_advectiondiffusion_amd.parallel.preflight import transport_kwargs

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def test_candidates_and_kwargs(monkeypatch):
    import bench
    monkeypatch.delenv("ADVDIFF_SHARE_GPU", raising=False)
    monkeypatch.delenv("ADVDIFF_BACKEND", raising=False)
    assert "ipc+fused" in bench.planned_transports(4, True, "tune")
    assert bench.planned_transports(4, False, "tune") == ["host"]
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    assert bench.planned_transports(2, True, "tune") == ["host", "ipc", "ipc+fused"]
    assert transport_kwargs("ipc+fused") == {"transport": "ipc", "fused_put": True}


def test_solver_ignores_fused_put_off_device():
    """CPU (and any non-ipc / non-slab setting): the switch is ignored, the step is the
    ordinary one."""
    g = Grid((20, 18, 16), (1.0, 1.0, 1.0))
    s = Solver(Diffusion(K=1.0, order=4), g, dtype=torch.float64, device="cpu",
               fused_put=True)
    assert not s.fput
    s.run(iters=2)


class _FakeIpc:
    def __init__(self, strides):
        self.strides = strides
        self.seen = None

    def targets(self, msgs):
        self.seen = msgs
        # the peer's receive box address: an arbitrary distinct value per peer
        return [(1000 * (peer + 1), self.strides[0], self.strides[1]) for peer, _, _ in msgs]


class _FakeComm:
    def __init__(self, rank, size, ipc):
        self.rank, self.size, self._ipc = rank, size, ipc
        self.transport = "ipc"

    def ipc(self):
        return self._ipc


@pytest.mark.parametrize("rank,size", [(0, 3), (1, 3), (2, 3), (1, 2)])
def test_put_targets_plan(rank, size, monkeypatch):
    """Each neighbour gets (its receive-box address, my send planes): lower <- planes
    [o0, o0 + G), upper <- [o1 - G, o1); no neighbour: (0, 0, 0); a peer field with other
    strides is refused (the kernel addresses the peer with the own in-plane offset)."""
    monkeypatch.setattr(halo_mod, "_ipc_on", lambda h, f: True)
    d = SlabDecomposition(41, size, rank, 6)
    f = torch.zeros((d.alloc, 9, 12), dtype=torch.float64)
    ipc = _FakeIpc((f.stride(1), f.stride(0)))
    h = halo_mod.SlabHalo(_FakeComm(rank, size, ipc), d, transport="ipc")
    lo, hi = h.put_targets(f)
    if d.lower is None:
        assert lo == (0, 0, 0)
    else:
        assert lo == (1000 * (d.lower + 1),) + tuple(d.send_lower())
    if d.upper is None:
        assert hi == (0, 0, 0)
    else:
        assert hi == (1000 * (d.upper + 1),) + tuple(d.send_upper())
    if d.lower is not None or d.upper is not None:
        bad = halo_mod.SlabHalo(_FakeComm(rank, size, _FakeIpc((f.stride(1) + 1, f.stride(0)))),
                                d, transport="ipc")
        with pytest.raises(ValueError):
            bad.put_targets(f)


@pytest.mark.parametrize("rank", [0, 1, 2, 3])
def test_put_parts_striped_plan(rank, monkeypatch):
    """Striped fused puts: every channel-1 send box of the rank becomes one part — its
    planes, its row range, the receive address shifted back by its first row (so the own
    in-plane offset lands on row y - y0 of a helper's buffer), the receiver's plane size;
    per face, the parts' rows partition the plane's rows."""
    from multigpu_advectiondiffusion_amd.parallel.ipc import stripe_plan
    monkeypatch.setattr(halo_mod, "_ipc_on", lambda h, f: True)
    monkeypatch.setattr(halo_mod.SlabHalo, "_use_stripes", lambda h, f: h._plan is not None)
    monkeypatch.setenv("ADVDIFF_STRIPE_SHARED", "1")
    size = 4
    d = SlabDecomposition(41, size, rank, 6)
    f = torch.zeros((d.alloc, 20, 12), dtype=torch.float64)

    class _Ipc:
        epoch = 3

        def _resolve_pairs(self, ch, pairs, tag=None):
            assert ch == 1
            out = {}
            for peer, (send, recv) in pairs.items():
                if send is not None:  # a helper's buffer for a slice, else the ghost rows
                    rsz = send.shape[1] * f.stride(1) if send.shape[1] != f.shape[1] else \
                        f.stride(0)
                    out[peer] = (10**6 * (peer + 1), f.stride(1), rsz)
                else:
                    out[peer] = None
            return out
    h = halo_mod.SlabHalo(_FakeComm(rank, size, _Ipc()), d, transport="ipc", stripe=2)
    assert h._plan is not None and any(stripe_plan(size, 2, exclusive_links=False).values())
    parts = h.put_parts(f)
    e = f.element_size()
    faces = {}
    for dst, k0, k1, y0, y1, pb in parts:
        assert (k0, k1) in (tuple(d.send_lower()), tuple(d.send_upper()))
        assert (dst + y0 * f.stride(1) * e) % 10**6 == 0  # the receive address, shifted
        faces.setdefault((k0, k1), []).append((y0, y1))
    for rows in faces.values():
        rows.sort()
        assert rows[0][0] == 0 and rows[-1][1] == f.shape[1]
        assert all(a[1] == b[0] for a, b in zip(rows, rows[1:]))
    assert len(parts) <= 6


def test_striped_tags_unique_per_solver(monkeypatch):
    """Two striped solvers alive at once (the bench tunes ipc+stripe and ipc+fused+stripe
    side by side) must not share a handshake tag: the tag carries the ipc epoch each was
    made in (round-6 N = 8 rehearsal: "halo pattern (0, 0) with peer 1 changed its
    boxes")."""
    monkeypatch.setenv("ADVDIFF_STRIPE_SHARED", "1")

    class _Ipc:
        epoch = 0

    ipc = _Ipc()
    comm = _FakeComm(1, 4, ipc)
    d = SlabDecomposition(41, 4, 1, 6)
    f = torch.zeros((d.alloc, 20, 12), dtype=torch.float64)
    ipc.epoch = 5
    a = halo_mod.SlabHalo(comm, d, transport="ipc", stripe=2)
    ipc.epoch = 6
    b = halo_mod.SlabHalo(comm, d, transport="ipc", stripe=2)
    assert a.striped and b.striped
    assert a._tag(f, 0) != b._tag(f, 0) and a._tag(f, 0) == a._tag(f, 0)
