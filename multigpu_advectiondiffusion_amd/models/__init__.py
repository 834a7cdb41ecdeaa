"""PDE models (the reference's applications): heat and WENO5 Burgers, 2-D and 3-D,
plus the serial MATLAB-prototype ports in :mod:`.prototypes`."""
from .base import Grid, Model, RunStats
from .burgers import Burgers
from .diffusion import Diffusion

MODELS = {"diffusion": Diffusion, "burgers": Burgers}

__all__ = ["Grid", "Model", "RunStats", "Diffusion", "Burgers", "MODELS"]
