#!/usr/bin/env python3
"""Overlap of the halo puts with the stencil launches, per rank, from a rocprofv3 kernel
trace (`--kernel-trace --output-format csv`) of a multi-rank native run (ranks told apart
by the launching thread): for every put kernel (`advdiff_copy_box` into a neighbour's
ghost box) of a rank, how much of it ran while the SAME rank's step kernel was running.
The wait kernels are left out: their duration is the time spent waiting for the peer.

    python bench/trace_overlap.py <dir with *kernel_trace.csv> [--md out.md]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    by_rank = defaultdict(list)
    for r in rows:
        by_rank[r["Thread_Id"]].append(
            (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    out = ["| rank (thread) | step launches | mean step µs | put kernels | put µs | of which beside the rank's own step launch |",
           "|---|---|---|---|---|---|"]
    for tid, ks in sorted(by_rank.items()):
        steps = [(s, e) for s, e, n in ks if "step_kernel" in n]
        puts = [(s, e) for s, e, n in ks if "copy_box" in n]
        if not steps or not puts:
            continue
        tot = sum(e - s for s, e in puts)
        hid = sum(max(0, min(ce, se) - max(cs, ss)) for cs, ce in puts for ss, se in steps)
        mean_step = sum(e - s for s, e in steps) / len(steps) / 1e3
        out.append(f"| {tid} | {len(steps)} | {mean_step:.1f} | {len(puts)} | {tot / 1e3:.1f} | "
                   f"{hid / 1e3:.1f} ({hid / max(tot, 1):.0%}) |")
    text = "\n".join(out)
    print(text)
    if a.md:
        open(a.md, "w").write(text + "\n")


if __name__ == "__main__":
    main()
