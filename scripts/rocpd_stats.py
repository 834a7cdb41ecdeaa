#!/usr/bin/env python3
"""Per-kernel time summary from a rocprofv3 rocpd database (the ROCm 7 default output):
    python scripts/rocpd_stats.py gpurun_out/prof/bench_results.db [--csv out.csv]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--instances", default=None,
                    help="substring of a kernel name: print that kernel's per-launch times "
                         "in launch order (µs) instead of the summary")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    if a.instances:
        rows = c.execute("select duration/1000.0 from kernels where name like ? order by start",
                         (f"%{a.instances}%",)).fetchall()
        print(" ".join(f"{r[0]:.1f}" for r in rows))
        return
    rows = c.execute("select name, count(*), avg(duration)/1000.0, sum(duration)/1e6, "
                     "min(duration)/1000.0, max(duration)/1000.0, max(vgpr_count), "
                     "max(lds_size), grid_x, grid_y, grid_z, workgroup_x, workgroup_y "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[3] for r in rows) or 1.0
    lines = ["name,calls,avg_us,total_ms,pct,min_us,max_us,vgpr,lds,grid,wg"]
    for r in rows:
        lines.append(f"\"{r[0]}\",{r[1]},{r[2]:.1f},{r[3]:.3f},{100 * r[3] / tot:.1f},"
                     f"{r[4]:.1f},{r[5]:.1f},{r[6]},{r[7]},{r[8]}x{r[9]}x{r[10]},{r[11]}x{r[12]}")
    for ln in lines[:a.top + 1]:
        print(ln)
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
