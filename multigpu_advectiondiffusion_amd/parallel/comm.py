"""Process-group bootstrap and collectives: one process per GPU over torch.distributed.

Replaces the reference's MPI layer (`MultiGPU/Diffusion3d_Baseline/Tools.c:228-242`
InitializeMPI/FinalizeMPI, `Util.cu:66-93` AssignDevices/ECCCheck, and the hand-rolled
Isend/Recv gather at `main.c:327-335`).

* Backend ``nccl`` (= RCCL on ROCm, point-to-point over xGMI) for device tensors,
  ``gloo`` for CPU runs and the CPU multi-process tests.
* Rendezvous from the standard torchrun environment (RANK, WORLD_SIZE, LOCAL_RANK,
  MASTER_ADDR, MASTER_PORT).  A single process needs no rendezvous at all.
* Device binding: ``cuda:LOCAL_RANK`` (the reference's ``rank % ndev``; here more ranks
  than GPUs is refused rather than silently oversubscribed — RCCL forbids two ranks on
  one GPU anyway).
* Halo transport (``transport``): "rccl" (grouped ncclSend/Recv on the comm stream, the
  default with the nccl backend), "ipc" (peer-mapped device puts + device flags,
  parallel/ipc.py; also runs several ranks on ONE GPU with ADVDIFF_SHARE_GPU=1) or "host"
  (host-staged through gloo — the reference's scheme, the default with gloo).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def pg_kwargs(backend: str, dev: torch.device) -> dict:
    """Extra init_process_group arguments for RCCL:
    * device_id: eager communicator creation (no lazy setup inside the first halo);
    * a HIGH-PRIORITY internal RCCL stream: the fused interior kernel fills every CU
      (VGPR/LDS), so RCCL's copy workgroups can only start as interior workgroups retire —
      at high priority they are dispatched first, which keeps the halo transfer inside
      the interior compute window (ADVDIFF_RCCL_HIGH_PRIORITY=0 disables)."""
    kw = {}
    if dev.type == "cuda" and backend == "nccl":
        kw["device_id"] = dev
        if os.environ.get("ADVDIFF_RCCL_HIGH_PRIORITY", "1") != "0":
            try:
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
                kw["pg_options"] = opts
            except (AttributeError, RuntimeError):  # pragma: no cover - older torch
                pass
    return kw


class Comm:
    def __init__(self, rank=0, size=1, local_rank=0, device=None, backend=None, group=None,
                 transport=None):
        self.rank = rank
        self.size = size
        self.local_rank = local_rank
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.backend = backend
        self.group = group
        self._owns_pg = False
        self._transport = transport
        self._ipc = None

    @property
    def transport(self) -> str:
        """Halo transport of device fields: "ipc", "rccl" or "host" (see module doc)."""
        if self._transport:
            return self._transport
        return "rccl" if self.backend == "nccl" else "host"

    @transport.setter
    def transport(self, v):
        if v not in (None, "ipc", "rccl", "host"):
            raise ValueError("transport must be ipc, rccl or host")
        self._transport = v

    @property
    def rccl_world(self) -> int:
        """Ranks of the RCCL communicator (0 when the process group is not nccl)."""
        return self.size if (self.size > 1 and self.backend == "nccl") else 0

    def transports(self) -> list:
        """Halo transports of device fields available on this Comm, the default first."""
        if self.size == 1 or self.device.type != "cuda":
            return [self.transport]
        alt = ["rccl", "ipc"] if self.backend == "nccl" else ["host", "ipc"]
        return [self.transport] + [t for t in alt if t != self.transport]

    def ipc(self):
        """The process's IPC peer context (created on first use, collectively)."""
        if self._ipc is None:
            from .ipc import IpcPeers
            self._ipc = IpcPeers(self)
        return self._ipc

    # ------------------------------------------------------------------------------
    @classmethod
    def from_env(cls, device: str | None = None, backend: str | None = None,
                 timeout_s: float | None = None, transport: str | None = None) -> "Comm":
        """Create (or attach to) the default process group from torchrun env vars.

        device: "cuda", "cpu" or None (= cuda if available).  backend defaults to
        nccl for cuda, gloo for cpu.
        """
        if timeout_s is None:  # collective timeout (a dead peer surfaces as an error)
            timeout_s = float(os.environ.get("ADVDIFF_COMM_TIMEOUT", "600"))
        # ADVDIFF_BACKEND=gloo: host-staged device halos (rehearsing multi-rank runs with
        # several ranks on one GPU together with ADVDIFF_SHARE_GPU=1; RCCL refuses that)
        backend = backend or os.environ.get("ADVDIFF_BACKEND") or None
        transport = transport or os.environ.get("ADVDIFF_TRANSPORT") or None
        size = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        if device.startswith("cuda"):
            ndev = torch.cuda.device_count()
            if ndev == 0:
                raise RuntimeError("device=cuda requested but no GPU is visible")
            share = os.environ.get("ADVDIFF_SHARE_GPU", "0") == "1"
            if share and size > 1:
                backend = backend or "gloo"  # RCCL refuses two ranks per GPU
            if size > 1 and local_rank >= ndev and not (share and backend == "gloo"):
                raise RuntimeError(f"local rank {local_rank} >= {ndev} visible GPUs "
                                   "(one process per GPU; oversubscription is refused — "
                                   "only gloo / ipc test runs may share with ADVDIFF_SHARE_GPU=1)")
            torch.cuda.set_device(local_rank % ndev)
            dev = torch.device("cuda", local_rank % ndev)
        else:
            dev = torch.device("cpu")
        c = cls(rank, size, local_rank, dev, transport=transport)
        if size > 1:
            c.backend = backend or ("nccl" if dev.type == "cuda" else "gloo")
            if not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                kw = dict(backend=c.backend, rank=rank, world_size=size,
                          timeout=datetime.timedelta(seconds=timeout_s))
                kw.update(pg_kwargs(c.backend, dev))
                dist.init_process_group(**kw)
                c._owns_pg = True
            c.group = dist.group.WORLD
        return c

    @property
    def distributed(self) -> bool:
        return self.size > 1

    def device_ids(self) -> list:
        """Device index of every rank (rank order), e.g. [0..7] on an 8-GPU node; proves
        that each rank drove its own GPU.  CPU ranks report -1."""
        mine = self.device.index if self.device.type == "cuda" else -1
        if self.size == 1:
            return [mine]
        t = torch.tensor([mine], dtype=torch.int64, device=self._coll_device())
        out = [torch.zeros_like(t) for _ in range(self.size)]
        dist.all_gather(out, t)
        return [int(x.item()) for x in out]

    # ---- collectives ---------------------------------------------------------------
    def barrier(self):
        if self.size > 1:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def _scalar(self, v: float, op):
        if self.size == 1:
            return float(v)
        t = torch.tensor([float(v)], dtype=torch.float64, device=self._coll_device())
        dist.all_reduce(t, op=op)
        return float(t.item())

    def _coll_device(self):
        return self.device if self.backend == "nccl" else torch.device("cpu")

    def allreduce_max(self, v: float) -> float:
        return self._scalar(v, dist.ReduceOp.MAX)

    def allreduce_min(self, v: float) -> float:
        return self._scalar(v, dist.ReduceOp.MIN)

    def allreduce_sum(self, v: float) -> float:
        return self._scalar(v, dist.ReduceOp.SUM)

    def allreduce_tensor(self, t: torch.Tensor, op="sum") -> torch.Tensor:
        if self.size == 1:
            return t
        ops = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}
        x = t.to(self._coll_device())
        dist.all_reduce(x, op=ops[op])
        return x.to(t.device)

    def gather_planes(self, local: torch.Tensor, counts: list[int]) -> torch.Tensor | None:
        """Gather per-rank slabs (axis 0) to rank 0 (returned on CPU; None elsewhere).
        Point-to-point so uneven slabs need no padding."""
        if self.size == 1:
            return local.detach().cpu()
        dev = self._coll_device()
        if self.rank == 0:
            parts = [local.detach().cpu()]
            for r in range(1, self.size):
                buf = torch.empty((counts[r],) + tuple(local.shape[1:]), dtype=local.dtype,
                                  device=dev)
                dist.recv(buf, src=r)
                parts.append(buf.cpu())
            return torch.cat(parts, 0)
        dist.send(local.detach().contiguous().to(dev), dst=0)
        return None

    def gather_boxes(self, local: torch.Tensor, boxes, global_shape) -> torch.Tensor | None:
        """Assemble per-rank blocks of a Cartesian decomposition on rank 0 (CPU tensor;
        None elsewhere).  boxes[r] = ((start, count) per array axis) of rank r."""
        if self.size == 1:
            return local.detach().cpu()
        dev = self._coll_device()
        if self.rank != 0:
            dist.send(local.detach().contiguous().to(dev), dst=0)
            return None
        out = torch.empty(tuple(global_shape), dtype=local.dtype)
        for r in range(self.size):
            box = boxes[r]
            if r == 0:
                part = local.detach().cpu()
            else:
                buf = torch.empty(tuple(c for _, c in box), dtype=local.dtype, device=dev)
                dist.recv(buf, src=r)
                part = buf.cpu()
            out[tuple(slice(s, s + c) for s, c in box)] = part
        return out

    def broadcast_object(self, obj):
        if self.size == 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=0)
        return lst[0]

    def finalize(self):
        if self._ipc is not None:
            self._ipc.close()
            self._ipc = None
        if self._owns_pg and dist.is_initialized():
            dist.destroy_process_group()
            self._owns_pg = False
