#!/usr/bin/env python3
"""Stall breakdown of rocprofv3 --pmc runs (scripts/pmc_r3.sh layout: <root>/<target>_<set>/
p_counter_collection.csv) for several roots side by side: per target and root, the wave-
cycle split (SQ_WAVE_CYCLES = SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY), LDS
issue stalls, VALU busy and the dispatch time (median over dispatches of the advdiff
kernel).

    python bench/pmc_compare.py label=root [label=root ...]
"""
import collections
import csv
import glob
import statistics
import sys


def load(root, tgt):
    agg, dur = collections.defaultdict(list), []
    for f in sorted(glob.glob(f"{root}/{tgt}_*/p_counter_collection.csv")):
        if not f.split("/")[-2][len(tgt) + 1:].isdigit():
            continue
        seen = set()
        for r in csv.DictReader(open(f)):
            if "advdiff" not in r["Kernel_Name"] or "step" not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Dispatch_Id"] not in seen:
                seen.add(r["Dispatch_Id"])
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: statistics.median(v) for k, v in agg.items()}, (statistics.median(dur) if dur else 0)


def main():
    roots = [a.split("=", 1) for a in sys.argv[1:]]
    tgts = sorted({p.split("/")[-2].rsplit("_", 1)[0] for _, r in roots
                   for p in glob.glob(f"{r}/*_*/p_counter_collection.csv")})
    print("| target | build | µs (median, counter runs) | VALU busy | wave-cycles: issuing | waiting (s_waitcnt / barrier) | issue-stalled | of which LDS issue | VALU instr | LDS instr | SALU instr |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for t in tgts:
        for label, root in roots:
            c, us = load(root, t)
            if not c:
                continue
            wc = c.get("SQ_WAVE_CYCLES", 0) or 1
            gui = c.get("GRBM_GUI_ACTIVE", 0) / 8  # per XCD
            busy = c.get("SQ_INSTS_VALU", 0) * 4 / (1024 * gui) if gui else 0
            print(f"| {t} | {label} | {us:.1f} | {busy:.0%} | {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.0%} "
                  f"| {c.get('SQ_WAIT_ANY', 0) / wc:.0%} | {c.get('SQ_WAIT_INST_ANY', 0) / wc:.0%} "
                  f"| {c.get('SQ_WAIT_INST_LDS', 0) / wc:.0%} | {c.get('SQ_INSTS_VALU', 0):.3g} "
                  f"| {c.get('SQ_INSTS_LDS', 0):.3g} | {c.get('SQ_INSTS_SALU', 0):.3g} |")


if __name__ == "__main__":
    main()
