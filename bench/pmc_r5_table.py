#!/usr/bin/env python3
"""Round-5 counter table (scripts/pmc_r5.sh layout: <root>/<target>_trace/p_kernel_trace.csv
and <root>/<target>_<set>/p_counter_collection.csv): per hot kernel its dispatch time
(kernel trace, min and median of the back-to-back launches), clock (GRBM_GUI_ACTIVE per
XCD over the counted dispatch's own duration), VALU busy, the
wave-cycle split (issuing / parked on s_waitcnt or the barrier / ready but not issued),
instruction counts and the fabric read bytes against the compulsory read.

    python bench/pmc_r5_table.py gpurun_out/pmc_r5 > profiles/r5/pmc_r5/table.md
"""
import collections
import csv
import glob
import statistics
import sys

# compulsory bytes read per dispatch by profile_target.py (n^3 fp64 fields)
COMPULSORY = {"copy": 512 ** 3 * 8, "fused": 512 ** 3 * 8, "fused2": 512 ** 3 * 8,
              "step2x": 512 ** 3 * 8, "burgers": 2 * 256 ** 3 * 8,
              "burgers512": 2 * 512 ** 3 * 8,
              # round 6, per-rank shapes of the 8-GPU run (profile_target.py): the planes
              # each launch reads (its outputs +- 3R)
              "slab8_int": 128 * 1024 * 1024 * 8, "slab8_bnd": 36 * 1024 * 1024 * 8,
              "r4x2_int": 256 * 518 * 1024 * 8, "cube1024": 1024 ** 3 * 8}
WHAT = {"copy": "copy_box 512³ (calibration)", "fused": "fused FD4 step 512³",
        "fused2": "fused FD2 step 512³", "step2x": "FD2 two steps per launch 512³",
        "burgers": "WENO5-Z + viscous stage 256³",
        "burgers512": "WENO5-Z + viscous stage 512³",
        "slab8_int": "FD4, 8-GPU slab rank 1024²×(128+12), interior launch (116 planes)",
        "slab8_bnd": "FD4, 8-GPU slab rank, both 6-plane boundary slabs (one launch)",
        "r4x2_int": "FD4, 4×2×1 rank 1024×518×268, interior launch (244 planes)",
        "cube1024": "FD4, 1024³ (one launch)"}
# output cells per dispatch (for instructions per cell)
CELLS = {"copy": 512 ** 3, "fused": 508 ** 3, "fused2": 510 ** 3, "step2x": 510 ** 3,
         "burgers": 250 ** 3, "burgers512": 506 ** 3,
         "slab8_int": 116 * 1020 * 1020, "slab8_bnd": 12 * 1020 * 1020,
         "r4x2_int": 244 * 514 * 1020, "cube1024": 1020 ** 3}


def counters(root, tgt):
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{root}/{tgt}_*/p_counter_collection.csv")):
        if not f.split("/")[-2][len(tgt) + 1:].isdigit():
            continue
        for r in csv.DictReader(open(f)):
            if "advdiff" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in agg.items()}


def clock_ghz(root, tgt):
    """Median over the dispatches of the counter run holding GRBM_GUI_ACTIVE of
    (GRBM_GUI_ACTIVE / 8 XCDs) / that dispatch's own duration."""
    out = []
    for f in sorted(glob.glob(f"{root}/{tgt}_*/p_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "advdiff" in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                out.append(float(r["Counter_Value"]) / 8 / ns)
    return statistics.median(out) if out else 0.0


def times(root, tgt):
    d = []
    for f in glob.glob(f"{root}/{tgt}_trace/p_kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            if "advdiff" in r["Kernel_Name"]:
                d.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return (min(d), statistics.median(d)) if d else (0.0, 0.0)


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_r5"
    print("| kernel | µs min / median (trace) | clock GHz | VALU busy | issuing | parked (waitcnt / barrier) "
          "| ready, not issued | VALU instr | LDS instr | SALU instr | read B / compulsory "
          "| VALU lane-ops / cell | µs per M cells |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for tgt in WHAT:
        c = counters(root, tgt)
        if not c:
            continue
        tmin, tmed = times(root, tgt)
        gui = c.get("GRBM_GUI_ACTIVE", 0) / 8  # cycles per XCD
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        busy = c.get("SQ_INSTS_VALU", 0) * 4 / (1024 * gui) if gui else 0
        rd = c.get("TCC_EA0_RDREQ_sum", 0) * 128
        print(f"| {WHAT[tgt]} | {tmin:.1f} / {tmed:.1f} | "
              f"{clock_ghz(root, tgt):.2f} | {busy:.0%} | {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.0%} | "
              f"{c.get('SQ_WAIT_ANY', 0) / wc:.0%} | {c.get('SQ_WAIT_INST_ANY', 0) / wc:.0%} | "
              f"{c.get('SQ_INSTS_VALU', 0):.3g} | {c.get('SQ_INSTS_LDS', 0):.3g} | "
              f"{c.get('SQ_INSTS_SALU', 0):.3g} | {rd / COMPULSORY[tgt]:.2f} | "
              f"{c.get('SQ_INSTS_VALU', 0) * 64 / CELLS[tgt]:.0f} | {tmin / CELLS[tgt] * 1e6:.2f} |")


if __name__ == "__main__":
    main()
