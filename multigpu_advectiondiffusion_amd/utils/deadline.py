"""A wall-clock deadline for a whole multi-rank job (bench.py).

The driver kills a bench run at its own limit and then has nothing: no JSON line, no
stack, no record of where the run was.  The reference's answer to a failing
communication call is to return the error and exit (`MPI_ERRORS_RETURN` + `MPI_CHECK`,
`MultiGPU/Diffusion3d_Baseline/Tools.c:228-234`); a hang returns nothing, so here every
rank arms a deadline below the driver's:

* `deadline - dump_s`: faulthandler prints every thread's stack (C-level timer thread,
  works while the main thread is blocked inside a device wait or a collective);
* `deadline`: a Python timer thread runs `on_expire` (rank 0 prints the partial result)
  and ends the process with `exit_code` via os._exit — no teardown that could block;
* SIGUSR1 also dumps the stacks (`launch.launch_cmd` sends it to ranks that are still
  alive when it gives up on a run);
* heartbeat (optional, rank 0): one stderr line every `heartbeat_s` naming the phase, so
  a long phase (the Burgers torch self-check: minutes with 8 ranks on one GPU) is not
  mistaken for a hang by a supervisor that watches the output.

The clock starts when the launcher started, not this process: under torchrun (or
bench.py's own self-launch) the parent's creation time, so the deadline is measured the
way the driver measures its limit.
"""
from __future__ import annotations

import faulthandler
import os
import signal
import sys
import threading
import time


def launch_start_time() -> float:
    """time.time() at which this job's launcher started: the parent process's creation
    time when the parent is a launcher (torch.distributed.run / torchrun / bench.py's
    self-launch), else this process's."""
    try:
        import psutil
        me = psutil.Process()
        t = me.create_time()
        parent = me.parent()
        if parent is not None:
            cmd = " ".join(parent.cmdline())
            if any(s in cmd for s in ("torch.distributed.run", "torchrun", "bench.py")):
                t = min(t, parent.create_time())
        return t
    except Exception:  # noqa: BLE001 - psutil missing / no /proc: this process's start
        return time.time() - time.process_time()


class Deadline:
    """Arm with `arm()`; `remaining()` in seconds; `phase` names what runs now."""

    def __init__(self, seconds: float, start: float | None = None, on_expire=None,
                 exit_code: int = 124, dump_s: float = 15.0, heartbeat_s: float = 0.0):
        self.seconds = float(seconds)
        self.start = launch_start_time() if start is None else float(start)
        self.on_expire = on_expire
        self.exit_code = int(exit_code)
        self.dump_s = float(dump_s)
        self.phase = "start"
        self.heartbeat_s = float(heartbeat_s)
        self._timer = None
        self._stop = threading.Event()

    @property
    def at(self) -> float:
        return self.start + self.seconds

    def remaining(self) -> float:
        return self.at - time.time()

    def arm(self) -> "Deadline":
        faulthandler.enable()
        try:
            faulthandler.register(signal.SIGUSR1, all_threads=True)
        except (AttributeError, ValueError, RuntimeError):  # pragma: no cover - no SIGUSR1
            pass
        left = self.remaining()
        faulthandler.dump_traceback_later(max(left - self.dump_s, 0.5), exit=False)
        self._timer = threading.Timer(max(left, 1.0), self._fire)
        self._timer.daemon = True
        self._timer.start()
        if self.heartbeat_s > 0:
            threading.Thread(target=self._beat, daemon=True).start()
        return self

    def _beat(self):
        while not self._stop.wait(self.heartbeat_s):
            print(f"[deadline] {time.time() - self.start:6.0f} s since launch, phase "
                  f"'{self.phase}', {self.remaining():.0f} s left", file=sys.stderr, flush=True)

    def cancel(self):
        self._stop.set()
        faulthandler.cancel_dump_traceback_later()
        if self._timer is not None:
            self._timer.cancel()

    def _fire(self):
        print(f"[deadline] {self.seconds:g} s since launch reached in phase "
              f"'{self.phase}': ending the run", file=sys.stderr, flush=True)
        try:
            if self.on_expire is not None:
                self.on_expire(self)
        except Exception as e:  # noqa: BLE001 - the exit below must happen
            print(f"[deadline] on_expire failed: {e!r}", file=sys.stderr, flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(self.exit_code)
