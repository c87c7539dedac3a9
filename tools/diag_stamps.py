#!/usr/bin/env python3
"""Per-unit phase timeline of the cone kernel (diagnostic build).

Run on the GPU box after `make -C riptide_amd/csrc stamps`:
    RIPTIDE_AMD_LIB=riptide_amd/libriptide_amd_stamps.so python tools/diag_stamps.py [batch]
Every work unit writes one record (thread 0, s_memtime marks, no atomics):
start, setup done, fill issued, descriptor table built, fill landed, merge
done, end.  Reported: mean cycles per phase by unit kind (whole / tile,
final pass with the S/N epilogue or not), per-CU residency (how many units
a CU holds over time) and the idle gaps between units on a CU.
"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

MARKS = 16
REC = MARKS + 2
PHASES = ["wait", "begin_next", "merge", "tail"]


def main():
    import torch
    from riptide_amd import _lib, engine
    L = _lib.load()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from bench_configs import CONFIGS
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    c = {k["name"]: k for k in CONFIGS}[sys.argv[2] if len(sys.argv) > 2 else "cfg2"]
    n = c["n"]
    plan = engine.PeriodogramPlan.for_search(n, c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                             ducy_max=c["ducy_max"])
    buf = (ctypes.c_uint64 * 8)()
    _lib.check(L.rt_diag_stamps(buf, 1))     # allocates the device records
    x = torch.randn((B, n), device="cuda", dtype=torch.float32)
    out = plan.run(x)
    torch.cuda.synchronize()
    _lib.check(L.rt_diag_stamps(buf, 1))
    out = plan.run(x, out=out)
    torch.cuda.synchronize()
    cap = 1 << 23
    rec = np.zeros(cap * REC, dtype=np.uint64)
    cnt = ctypes.c_uint64(0)
    _lib.check(L.rt_diag_timeline(rec.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), cap, ctypes.byref(cnt)))
    nrec = int(cnt.value)
    e = rec[:nrec * REC].reshape(nrec, REC).astype(np.int64)
    starts = np.zeros(4096, dtype=np.uint64)
    _lib.check(L.rt_diag_launches(starts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), starts.size,
                                  ctypes.byref(cnt)))
    starts = starts[:int(cnt.value)].astype(np.int64)
    keep = e[:, 1] != 0                      # units that returned early write nothing
    launch = np.searchsorted(starts, np.nonzero(keep)[0], side="right") - 1
    e = e[keep]
    out = analyse(e)
    out["config"], out["batch"] = c["name"], B
    out["launch_tails"] = launch_tails(e, launch)
    print(json.dumps(out))


def launch_tails(e, launch, slots=512):
    """Per cone launch, on the device-wide 100 MHz clock (s_memrealtime at
    workgroup entry and exit): duration = last exit - first entry, tail =
    last exit - median exit, idle = 1 - busy workgroup time / (slots x
    duration) with slots = 2 workgroups x 256 CUs, drain = last exit - last
    entry (no unit left to start: the launch's tail proper).  Sums over
    launches, so the fractions weight long launches; times in microseconds."""
    t_in, t_out = e[:, 1 + 14], e[:, 1 + 15]
    dur = tail = busy = drain = 0.0
    per = []
    for li in np.unique(launch):
        m = launch == li
        d = float(t_out[m].max() - t_in[m].min())
        drain += float(t_out[m].max() - t_in[m].max())
        tl = float(t_out[m].max() - np.median(t_out[m]))
        dur += d
        tail += tl
        busy += float((t_out[m] - t_in[m]).sum()) / slots
        per.append((int(m.sum()), d, tl))
    per.sort(key=lambda r: -r[1])
    us = 0.01
    return {"launches": len(per), "sum_duration_us": round(dur * us, 1), "tail_frac": round(tail / dur, 4),
            "drain_frac": round(drain / dur, 4), "idle_slot_frac": round(1 - busy / dur, 4),
            "longest": [{"units": u, "us": round(d * us, 1), "tail_us": round(t * us, 1)} for u, d, t in per[:5]],
            "shortest": [{"units": u, "us": round(d * us, 1), "tail_us": round(t * us, 1)} for u, d, t in per[-3:]]}


def analyse(e):
    hw = e[:, 0] & 0xFFFFFFFF
    xcc = (e[:, 0] >> 32) & 0xF
    cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 0x7) << 5) | (xcc << 8)
    t = e[:, 1:1 + MARKS]
    tend = t[:, len(PHASES)]
    shape = e[:, 1 + MARKS]
    snr = (shape >> 48) & 1
    mode = (shape >> 24) & 0xFF
    lv = (shape >> 16) & 0xFF
    n0 = (shape >> 32) & 0xFFFF
    ph = np.diff(t[:, :len(PHASES) + 1], axis=1)
    out = {"units": int(e.shape[0]), "distinct_cus": int(np.unique(cu).size),
           "mean_cycles": dict(zip(PHASES, ph.mean(axis=0).round(0).tolist())),
           "mean_total": float((tend - t[:, 0]).mean())}
    # workgroup entry (mark 5) .. unit start (mark 0): prologue, view, blob
    # header and DMA issue; mark 4 .. mark 6: the end-of-unit wait, if any
    has_entry = bool(np.all(t[:, 5] > 0))
    if has_entry:
        out["mean_cycles"]["startup"] = float((t[:, 0] - t[:, 5]).mean())
        out["mean_cycles"]["exit"] = float((t[:, 6] - tend).mean())
        out["mean_total_entry_to_exit"] = float((t[:, 6] - t[:, 5]).mean())
        if np.all(t[:, 11:14] > 0):
            out["startup_split"] = {"view": float((t[:, 11] - t[:, 5]).mean()),
                                    "header": float((t[:, 12] - t[:, 11]).mean()),
                                    "dma_issue": float((t[:, 13] - t[:, 12]).mean()),
                                    "rest": float((t[:, 0] - t[:, 13]).mean())}
    groups = {}
    for km in (0, 1):
        for ks in (0, 1):
            m = (mode == km) & (snr == ks)
            if m.any():
                g = {"units": int(m.sum()), "levels": round(float(lv[m].mean()), 2),
                     "rows": round(float(n0[m].mean()), 1)}
                g.update(dict(zip(PHASES, ph[m].mean(axis=0).round(0).tolist())))
                if np.all(t[:, 11:14] > 0):
                    g["startup_split"] = {"view": round(float((t[m, 11] - t[m, 5]).mean())),
                                          "header": round(float((t[m, 12] - t[m, 11]).mean())),
                                          "dma_issue": round(float((t[m, 13] - t[m, 12]).mean()))}
                groups[("whole" if km == 0 else "tile") + ("_snr" if ks else "")] = g
    out["groups"] = groups
    m = (snr == 1) & np.all(t[:, 7:11] > 0, axis=1)
    if m.any():
        sn = t[m]
        out["snr_pass0"] = {"prefix": float((sn[:, 7] - sn[:, 3]).mean()), "barrier": float((sn[:, 8] - sn[:, 7]).mean()),
                            "window": float((sn[:, 9] - sn[:, 8]).mean()), "widths": float((sn[:, 10] - sn[:, 9]).mean()),
                            "rest": float((tend[m] - sn[:, 10]).mean())}
    # per-CU residency and idle gaps (s_memtime is per XCD: compare within a CU only)
    occ = np.zeros(4)
    gaps = []
    t_in = t[:, 5] if has_entry else t[:, 0]
    t_out = t[:, 6] if has_entry else tend
    for c in np.unique(cu):
        m = cu == c
        ev = np.concatenate([np.stack([t_in[m], np.ones(m.sum())], 1), np.stack([t_out[m], -np.ones(m.sum())], 1)])
        ev = ev[np.lexsort((-ev[:, 1], ev[:, 0]))]
        level, last, idle_from = 0, ev[0, 0], None
        for tt, d in ev:
            occ[min(int(level), 3)] += tt - last
            if level == 0 and d > 0 and idle_from is not None:
                gaps.append(tt - idle_from)
            level += d
            last = tt
            if level == 0:
                idle_from = tt
    tot = occ.sum()
    out["cu_residency_frac"] = {k: round(float(v / tot), 4) for k, v in zip(("0", "1", "2", "3+"), occ)}
    gaps = np.array(gaps)
    if gaps.size:
        edges = [0, 2e3, 8e3, 32e3, 128e3, 1e12]
        out["idle_gaps_count_cycles"] = {
            f"<{edges[i + 1]:.0e}": [int(((gaps >= edges[i]) & (gaps < edges[i + 1])).sum()),
                                      float(gaps[(gaps >= edges[i]) & (gaps < edges[i + 1])].sum())]
            for i in range(len(edges) - 1)}
    return out


if __name__ == "__main__":
    main()
