"""Distributed runtime: one process per GPU over torch.distributed (RCCL / gloo), slab
decomposition and halo exchange."""
from .comm import Comm
from .decomposition import SlabDecomposition, weak_scaling_grid
from .halo import SlabHalo

__all__ = ["Comm", "SlabDecomposition", "SlabHalo", "weak_scaling_grid"]
