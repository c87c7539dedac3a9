#!/usr/bin/env python3
"""Per-launch durations of the cone kernel from a rocprofv3 --kernel-trace
run (kernel_trace.csv): the cone dispatches in start order, grouped into
steps of N launches (a bench step issues the same launch sequence every
step), and the median duration of each launch position over the steps.

usage: tools/prof_dispatch.py <dir with *kernel_trace.csv> N_LAUNCHES_PER_STEP [SKIP_STEPS [STEPS]]
(bench.py: SKIP_STEPS = its warmup steps, STEPS = its timed steps; the
self-check's default-schedule run that follows them is not counted)
"""
import csv
import glob
import statistics
import sys


def main():
    root, n = sys.argv[1], int(sys.argv[2])
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    want = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    rows = []
    for f in glob.glob(root + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "cone_kernel" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    rows = rows[skip * n:]
    steps = len(rows) // n if not want else min(want, len(rows) // n)
    rows = rows[:steps * n]
    print(f"{steps} steps x {n} cone launches")
    total = 0.0
    for i in range(n):
        d = [(rows[s * n + i][1] - rows[s * n + i][0]) / 1e6 for s in range(steps)]
        m = statistics.median(d)
        total += m
        name = rows[i][2].split("(")[0].replace("void rt::", "")
        print(f"{i:3d} {name:32s} {m:9.3f} ms")
    print(f"sum of medians {total:.3f} ms per step")


if __name__ == "__main__":
    main()
