#!/usr/bin/env python3
"""profiles/roofline.md from scripts/roofline.sh output (gpurun_out/roofline):
per kernel the analytic compulsory bytes, the TCC counter bytes, time, TB/s, % of the
measured HBM copy rate, VALU instructions per cell and an estimated VALU-busy share."""
import csv
import glob
import json
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/roofline"
KEYS = {"copy_box": "copy_box_kernel", "stage1": "diffusion3d_stage_kernel<double, 4, 64, 16, 0>",
        "stage2": "diffusion3d_stage_kernel<double, 4, 64, 16, 1>",
        "fused_fd4": "diffusion3d_step_cring_kernel<double, 4,",
        "fused_fd2": "diffusion3d_step_cring_kernel<double, 2,",
        "weno5_stage": "burgers3d_w5s_kernel<double, true, true, 1"}
meta = json.loads([l for l in open(f"{root}/trace.log") if l.startswith("{")][-1])


def which(name):
    for k, s in KEYS.items():
        if s in name:
            return k
    return None


dur = {}
for f in glob.glob(f"{root}/trace/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = which(r["Kernel_Name"])
        if k:
            dur.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
cnt = {}
for f in glob.glob(f"{root}/pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = which(r["Kernel_Name"])
        if k:
            cnt.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
rows = []
copy_tbps = None
for k in KEYS:
    if k not in meta or k not in dur:
        continue
    us = statistics.median(dur[k])
    c = {n: statistics.median(v) for n, v in cnt.get(k, {}).items()}
    cells, bpc = meta[k]["cells"], meta[k]["bytes_per_cell"]
    analytic = cells * bpc
    fetch = c.get("FETCH_SIZE", float("nan")) * 1024
    write = c.get("WRITE_SIZE", float("nan")) * 1024
    tbps = analytic / (us * 1e-6) / 1e12
    if k == "copy_box":
        copy_tbps = tbps
    valu = c.get("SQ_INSTS_VALU", float("nan"))
    grbm = c.get("GRBM_GUI_ACTIVE", float("nan")) / 8  # summed over the 8 XCDs
    clk = grbm / (us * 1e-6) / 1e9 if grbm == grbm else float("nan")
    busy = valu * 4 / (1024 * grbm) if grbm else float("nan")  # fp64-dominated: 4 cyc/instr
    rows.append((k, bpc, analytic / 1e9, (fetch + write) / 1e9, fetch / 1e9, write / 1e9,
                 us, tbps, valu * 64 / cells, busy, clk, c))
print("| kernel | analytic B/cell | analytic GB | TCC FETCH+WRITE GB (raw) | fetch GB | write GB |"
      " µs | TB/s (analytic) | % of copy rate | VALU lane-ops / cell | VALU busy (est.) | clock GHz |")
print("|---|---|---|---|---|---|---|---|---|---|---|---|")
for k, bpc, an, fw, fe, wr, us, tb, lpc, busy, clk, c in rows:
    pct = 100 * tb / copy_tbps if copy_tbps else float("nan")
    print(f"| {k} | {bpc} | {an:.3f} | {fw:.3f} | {fe:.3f} | {wr:.3f} | {us:.1f} | {tb:.2f} |"
          f" {pct:.0f} % | {lpc:.0f} | {100 * busy:.0f} % | {clk:.2f} |")
print()
print("raw counters (median per dispatch):")
for k, *_, c in rows:
    print(f"- {k}: " + ", ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
