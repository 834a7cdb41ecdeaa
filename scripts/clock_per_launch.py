#!/usr/bin/env python3
"""Per-launch duration and effective shader clock of selected kernels from a rocprofv3
run with `--pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv`:
clock = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) / kernel duration.

    python scripts/clock_per_launch.py gpurun_out/clk/c_counter_collection.csv step_cring w5s
"""
import csv
import sys
from collections import defaultdict


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    rows = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = rows[int(r["Dispatch_Id"])]
        d["name"] = r["Kernel_Name"]
        d["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    for pat in pats:
        print(f"## {pat}: launch, us, GHz")
        n = 0
        for did in sorted(rows):
            d = rows[did]
            if pat not in d["name"] or "GRBM_GUI_ACTIVE" not in d:
                continue
            n += 1
            ghz = d["GRBM_GUI_ACTIVE"] / 8 / (d["us"] * 1e-6) / 1e9
            print(f"{n:3d} {d['us']:8.1f} {ghz:5.2f}")


if __name__ == "__main__":
    main()
