#!/usr/bin/env python3
"""Static instruction mix of a kernel's hot loop from gfx950 assembly (no GPU needed).

    hipcc -O3 --offload-arch=gfx950 -std=c++20 -Icsrc/include -Icsrc/kernels \
        --cuda-device-only -S csrc/kernels/burgers.hip -o /tmp/burgers.s
    python bench/isa_stats.py /tmp/burgers.s 'burgers3d_w5_kernelIdLb1ELb1ELi1ELi8ELb1'

For every kernel symbol matching the regex: VGPR/SGPR/LDS/scratch use, and for each
backward branch (a loop) the instruction counts between the loop head and the branch,
by class (VALU, SALU, LDS, VMEM) and the commonest VALU opcodes — the quantity to cut
when a kernel is VALU-issue bound (SQ_INSTS_VALU)."""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "other"


def analyse(lines, start):
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    loops = []
    for i, l in enumerate(body):
        m = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and labels.get(m.group(1), 1 << 30) < i:
            loops.append((labels[m.group(1)], i))
    meta = {}
    for l in lines[end:end + 400]:
        m = re.match(r"\s+\.(vgpr_count|sgpr_count|group_segment_fixed_size|private_segment_fixed_size):\s+(\d+)", l)
        if m and m.group(1) not in meta:
            meta[m.group(1)] = int(m.group(2))
    out = []
    for a, b in loops:
        c = Counter()
        ops = Counter()
        for l in body[a:b + 1]:
            t = l.strip().split()
            if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
                continue
            c[classify(t[0])] += 1
            if t[0].startswith("v_"):
                ops[t[0]] += 1
        out.append((a, b, c, ops))
    return meta, out


def main():
    path, pat = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if not m or not re.search(pat, m.group(1)):
            continue
        meta, loops = analyse(lines, i)
        print(m.group(1)[:110])
        print("  ", meta)
        for a, b, c, ops in loops:
            print(f"   loop [{a},{b}] valu={c['valu']} salu={c['salu']} lds={c['lds']} "
                  f"vmem={c['vmem']}")
            print("     ", ", ".join(f"{k}:{v}" for k, v in ops.most_common(14)))


if __name__ == "__main__":
    main()
