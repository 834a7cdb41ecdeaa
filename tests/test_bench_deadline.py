"""bench.py fails fast and still reports (CPU, gloo ranks).

* A (grid, transport) candidate that hangs in the preflight (ADVDIFF_FAULT=hang:<key>:
  the last rank's child sleeps, its peers block in the exchange) is dropped with a
  recorded reason and the run completes on the remaining candidates — within the
  preflight's per-candidate limit, not the process group's timeout.
* A run that hangs after the headline window (ADVDIFF_FAULT=hang:phase:heat: bitwise, the
  N-rank vs one-GPU check) ends at the bench deadline: rank 0 prints the JSON line with
  the timed heat result and the phase it stopped in, every rank dumps its stacks, and the
  exit code is non-zero.  (Optional phases that the time left cannot cover are skipped:
  the 45 s deadline of the test skips FD2 and Burgers.)
* The preflight itself: verdicts agree on every rank and a candidate whose ranks compute
  a wrong solution is rejected against the one-rank hash.
"""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SMALL = ["--device", "cpu", "--base", "20", "--burgers-base", "14", "--steps", "2",
         "--warmup", "1", "--sustained-steps", "0", "--check-steps", "2", "--settle-ms", "0"]


def _bench(args, env_extra=None, timeout=400):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "ADVDIFF_FAULT")}
    env.update(env_extra or {})
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    return r, time.monotonic() - t0


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_hanging_candidate_is_dropped_and_reported():
    key = "heat:2x2x1/host"
    r, secs = _bench(["--gpus", "4", "--no-fd2", "--no-burgers", "--preflight-cand-s", "12"]
                     + SMALL, {"ADVDIFF_FAULT": f"hang:{key}"})
    assert r.returncode == 0, r.stderr[-4000:]
    (res,) = _json_lines(r.stdout)
    assert res["status"] == "ok" and res["value"] > 0
    assert res["preflight"][key].startswith("hang or crash"), res["preflight"]
    assert res["preflight"]["heat:4x1x1/host"] == "ok"
    assert "2x2x1" not in json.dumps(res["transport_trials_ms_per_step"])
    assert res["config"]["parallelism"].startswith("z-slab4")
    # the hung child was asked for its stacks before it was killed
    assert "Current thread" in r.stderr or "Thread 0x" in r.stderr
    assert secs < 200, secs


def test_deadline_prints_partial_result_and_fails():
    r, secs = _bench(["--gpus", "2", "--no-burgers", "--deadline", "45"] + SMALL,
                     {"ADVDIFF_FAULT": "hang:phase:heat: bitwise"}, timeout=200)
    assert r.returncode != 0
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    res = lines[0]
    assert res["status"].startswith("incomplete") and "'heat: bitwise" in res["status"], \
        res["status"]
    assert res["value"] > 0 and res["n_gpus"] == 2          # the timed window had finished
    assert res["linf_vs_exact"] <= res["linf_bound"]
    assert "fd2_7pt" not in res
    # every rank dumped its stacks before the end (faulthandler)
    assert r.stderr.count("Most recent call first") >= 2 or r.stderr.count("Thread 0x") >= 2, \
        r.stderr[-3000:]
    assert secs < 45 + 40, secs


def _preflight_run(comm, cands, models, fault):
    # spawn_local rank: the preflight spawns its own children (fresh process groups)
    from multigpu_advectiondiffusion_amd.parallel.preflight import run_preflight
    if fault:
        os.environ["ADVDIFF_FAULT"] = fault
    try:
        return run_preflight(cands, models, device="cpu", backend="gloo", cand_s=10,
                             init_s=60, total_s=120, log=lambda m: None)
    finally:
        os.environ.pop("ADVDIFF_FAULT", None)


@pytest.mark.parametrize("fault", [None, "hang:heat:slab/host", "corrupt:heat:1x2x1/host"])
def test_preflight_verdicts_agree(fault):
    from multigpu_advectiondiffusion_amd.launch import spawn_local
    models = {"heat": {"model": ("diffusion", {"K": 1.0, "order": 4}), "shape": [16, 14, 24],
                       "spacing": [1.0, 1.0, 1.0], "ic": "sine", "dtype": "float64"}}
    cands = [("heat", None, "host"), ("heat", (1, 2, 1), "host")]
    out = spawn_local(2, _preflight_run, cands, models, fault, timeout=200)
    assert out[0] == out[1]
    if fault and fault.startswith("hang"):
        assert out[0]["heat:slab/host"].startswith("hang or crash")
        assert out[0]["heat:1x2x1/host"] == "ok"
    elif fault:
        assert out[0]["heat:slab/host"] == "ok"
        assert "differs from the one-rank solution" in out[0]["heat:1x2x1/host"] \
            or "disagree" in out[0]["heat:1x2x1/host"], out[0]
    else:
        assert out[0] == {"heat:slab/host": "ok", "heat:1x2x1/host": "ok"}


def test_preflight_under_torchrun():
    """Under torch.distributed.run (the driver's launcher) the workers inherit the elastic
    agent's store settings; the preflight children must still form their own group."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "ADVDIFF_FAULT")}
    from multigpu_advectiondiffusion_amd.launch import free_port
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(free_port()), str(ROOT / "bench.py"), "--gpus", "2",
                        "--no-fd2", "--no-burgers", "--preflight-cand-s", "20"] + SMALL,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    (res,) = _json_lines(r.stdout)
    assert res["preflight"] == {"heat:2x1x1/host": "ok"}, res["preflight"]


def _dead_at_init(comm, models):
    from multigpu_advectiondiffusion_amd.parallel.preflight import run_preflight
    import time as _t
    if comm.rank == 1:  # this rank's child cannot start (a bad backend name)
        os.environ["ADVDIFF_BACKEND"] = "no-such-backend"
    t0 = _t.monotonic()
    v = run_preflight([("heat", None, "host")], models, device="cpu", backend="gloo"
                      if comm.rank != 1 else "no-such-backend", cand_s=10, init_s=120,
                      total_s=200, log=lambda m: None)
    return v, _t.monotonic() - t0


def test_preflight_child_dying_at_init_ends_every_rank_fast():
    """One rank's child dies starting its process group: the other ranks' children, blocked
    in the rendezvous, are ended through the marker file well before init_s."""
    from multigpu_advectiondiffusion_amd.launch import spawn_local
    models = {"heat": {"model": ("diffusion", {"K": 1.0, "order": 4}), "shape": [16, 14, 24],
                       "spacing": [1.0, 1.0, 1.0], "ic": "sine", "dtype": "float64"}}
    out = spawn_local(2, _dead_at_init, models, timeout=200)
    for v, secs in out:
        assert v["heat:slab/host"].startswith("not run"), v
        assert secs < 60, secs
