#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace --stats run of bench.py
(tools/gpu_run.sh prof) as JSON for profiles/, stamped with the csrc_sha of
the kernel sources it was measured on (bench.source_digest) and the bench
line it came from, with the per-step prep time (every non-cone rt:: kernel).

usage: tools/prof_json.py <run_kernel_stats.csv> <bench.log> <out.json>
"""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from bench import source_digest
    stats, log, out = sys.argv[1:4]
    bench = None
    for line in open(log):
        if line.startswith('{"metric"'):
            bench = json.loads(line)
    rows = []
    for r in csv.DictReader(open(stats)):
        name = r["Name"]
        rows.append({"kernel": name.split("(")[0] if name.startswith(("rt::", "void rt::")) else name[:80],
                     "calls": int(r["Calls"]), "total_us": round(float(r["TotalDurationNs"]) / 1e3, 3),
                     "avg_us": round(float(r["AverageNs"]) / 1e3, 3), "percent": round(float(r["Percentage"]), 3)})
    # bench.py runs warmup + steps timed steps (+ one untimed self-check run)
    # of the prep kernels: their calls per kernel give the number of steps
    prep = [r for r in rows if "rt::" in r["kernel"] and "cone_kernel" not in r["kernel"]]
    steps = max((r["calls"] for r in prep if "downsample" in r["kernel"]), default=0)
    cone_calls = sum(r["calls"] for r in rows if "cone_kernel" in r["kernel"])
    res = {"csrc_sha": source_digest(), "source": os.path.relpath(stats, REPO),
           "bench": {k: bench[k] for k in ("value", "ms_per_step", "steps", "warmup")} if bench else None,
           "prep_runs": steps,
           "prep_ms_per_run": round(sum(r["total_us"] for r in prep) / 1e3 / steps, 4) if steps else None,
           "prep_kernels_ms_per_run": {r["kernel"]: round(r["total_us"] / 1e3 / max(steps, 1), 4) for r in prep},
           "cone_launches": cone_calls,
           "cone_ms_total": round(sum(r["total_us"] for r in rows if "cone_kernel" in r["kernel"]) / 1e3, 3),
           "kernels": rows}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))


if __name__ == "__main__":
    main()
