#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd sqlite .db or the
csv kernel_stats file) into a short per-kernel table for profiles/.

usage: tools/prof_summary.py <run_results.db | *_kernel_stats.csv> [out.csv]
"""
import csv
import sqlite3
import sys


def short(n):
    return n.split("(")[0] if n.startswith("rt::") else n[:80]


def rows_from_db(path):
    c = sqlite3.connect(path)
    cur = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels")
    return [(short(n), int(k), float(t), float(a), float(p)) for n, k, t, a, p in cur]


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                        float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


def main():
    src = sys.argv[1]
    rows = rows_from_db(src) if src.endswith(".db") else rows_from_csv(src)
    out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
    for r in rows:
        w.writerow([r[0], r[1], f"{r[2]:.3f}", f"{r[3]:.3f}", f"{r[4]:.2f}"])


if __name__ == "__main__":
    main()
