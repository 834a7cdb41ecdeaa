"""Host utilities: initial conditions, I/O and checkpoints, metrics, tracing."""
