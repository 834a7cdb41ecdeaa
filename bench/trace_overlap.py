#!/usr/bin/env python3
"""Overlap of the halo puts with the stencil launches, per rank, from rocprofv3 kernel
traces (`--kernel-trace --output-format csv`) of a multi-rank run: for every put kernel
(`ipc_put_kernel` / `advdiff_copy_box` into a neighbour's ghost box) of a rank, how much of
it ran while the SAME rank's step (or stage) kernel was running.  The wait kernels are
left out: their duration is the time spent waiting for the peer.

Ranks are told apart by their per-rank trace directory (`launch.py --profile DIR` writes
DIR/rank<r>/..., like the reference's `nvprof -o X.%q{OMPI_COMM_WORLD_RANK}.nvprof`,
`MultiGPU/Diffusion3d_Baseline/run.sh:2`), or — one trace of the whole launcher — by the
launching thread.

    python bench/trace_overlap.py <dir with */*kernel_trace.csv> [--md out.md]
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def _rank_of(path, row):
    m = re.search(r"[/\\]rank(\d+)[/\\]", path)
    return f"rank {m.group(1)}" if m else f"thread {row['Thread_Id']}"


def _is_put(name):
    return "ipc_put" in name or "copy_box" in name


def _is_step(name):
    """A stencil launch: the fused heat step, a per-stage kernel or a WENO stage
    (burgers*_w5*_kernel / burgers*_stage_kernel)."""
    return (("step_kernel" in name or "stage" in name or "_step" in name or "burgers" in name)
            and not _is_put(name))


def _union(iv):
    """Sorted, merged intervals (a put beside two concurrent step launches counts once)."""
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _overlap(a, b):
    """Total length of (union a) ∩ (union b)."""
    a, b = _union(a), _union(b)
    i = j = tot = 0
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        tot += max(0, hi - lo)
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    by_rank = defaultdict(list)
    for f in glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            by_rank[_rank_of(f, r)].append(
                (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    out = ["| rank | step launches | mean step µs | put kernels | put µs | of which beside the rank's own step launch |",
           "|---|---|---|---|---|---|"]
    for tid, ks in sorted(by_rank.items()):
        steps = [(s, e) for s, e, n in ks if _is_step(n)]
        puts = [(s, e) for s, e, n in ks if _is_put(n)]
        if not steps or not puts:
            continue
        tot = sum(e - s for s, e in _union(puts))
        hid = _overlap(puts, steps)
        mean_step = sum(e - s for s, e in steps) / len(steps) / 1e3
        out.append(f"| {tid} | {len(steps)} | {mean_step:.1f} | {len(puts)} | {tot / 1e3:.1f} | "
                   f"{hid / 1e3:.1f} ({hid / max(tot, 1):.0%}) |")
    text = "\n".join(out)
    print(text)
    if a.md:
        open(a.md, "w").write(text + "\n")


if __name__ == "__main__":
    main()
