"""GPU idle time of a traced run: rocprofv3 --kernel-trace [--memory-copy-trace]
--output-format csv, every kernel and copy interval merged into busy spans,
the gaps between them reported (total, the largest ones, and which
kernel/copy ends before and starts after each).

    python tools/trace_gaps.py DIR [--from-ms T0] [--to-ms T1] [--top K]

DIR is searched for *kernel_trace.csv and *memory_copy_trace.csv.  Times are
relative to the first interval in the trace; --from-ms / --to-ms select a
window (e.g. the timed region of a bench run)."""
import argparse
import csv
import glob
import os


def _rows(path, kind):
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("Direction") or kind
            yield int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"{kind}:{name[:60]}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--from-ms", type=float, default=None)
    ap.add_argument("--to-ms", type=float, default=None)
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--min-gap-us", type=float, default=20.0)
    a = ap.parse_args()
    iv = []
    for p in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        iv += list(_rows(p, "K"))
    for p in glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), recursive=True):
        iv += list(_rows(p, "C"))
    if not iv:
        raise SystemExit("no trace csv under " + a.dir)
    iv.sort()
    t0 = iv[0][0]
    lo = t0 + int(a.from_ms * 1e6) if a.from_ms is not None else t0
    hi = t0 + int(a.to_ms * 1e6) if a.to_ms is not None else max(e for _, e, _ in iv)
    iv = [x for x in iv if x[1] > lo and x[0] < hi]
    gaps = []
    busy = 0
    cur_s, cur_e, cur_n = iv[0]
    for s, e, n in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, (cur_e - t0) / 1e6, cur_n, n))
            cur_s, cur_e, cur_n = s, e, n
        elif e > cur_e:
            cur_e, cur_n = e, n
    busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0]
    big = [g for g in gaps if g[0] >= a.min_gap_us * 1e3]
    print(f"window {(iv[0][0] - t0) / 1e6:.1f}..{(iv[-1][1] - t0) / 1e6:.1f} ms: span {span / 1e6:.1f} ms, "
          f"busy {busy / 1e6:.1f} ms ({busy / span:.1%}), {len(gaps)} gaps, "
          f"{len(big)} >= {a.min_gap_us:g} us totalling {sum(g[0] for g in big) / 1e6:.1f} ms")
    by_pair = {}
    for g in big:
        k = (g[2], g[3])
        c, t = by_pair.get(k, (0, 0))
        by_pair[k] = (c + 1, t + g[0])
    print("gap time by (before -> after):")
    for (b, n), (c, t) in sorted(by_pair.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {t / 1e6:8.2f} ms  x{c:<4d} {b}  ->  {n}")
    print("largest gaps:")
    for g in sorted(big, reverse=True)[:a.top]:
        print(f"  {g[0] / 1e3:9.1f} us at {g[1]:9.2f} ms  {g[2]}  ->  {g[3]}")


if __name__ == "__main__":
    main()
