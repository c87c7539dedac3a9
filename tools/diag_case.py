#!/usr/bin/env python3
"""Diagnostic (GPU box): ffa2 of given shapes under several cone feature-flag
values, compared with the oracle; prints the first mismatching rows.

usage: python tools/diag_case.py 37x17,129x260 5,1,4,0
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from oracle import oracle as O
    from riptide_amd import libcpp as rt
    shapes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[1].split(",")]
    flags = sys.argv[2].split(",") if len(sys.argv) > 2 else ["5", "1"]
    for m, p in shapes:
        x = np.random.RandomState(m * 31 + p).normal(size=(m, p)).astype(np.float32)
        ref = O.ffa2(x)
        for f in flags:
            os.environ["RIPTIDE_AMD_CONE_FLAGS"] = f
            y = rt.ffa2(x)
            bad = np.where(~np.all(y == ref, axis=1))[0]
            print(f"{m}x{p} flags={f}: {bad.size} bad rows {bad[:12].tolist()}", flush=True)
            if bad.size:
                r = bad[0]
                cols = np.where(y[r] != ref[r])[0]
                print(f"   row {r}: bad cols {cols[:20].tolist()} got {y[r, cols[:4]].tolist()} "
                      f"want {ref[r, cols[:4]].tolist()}", flush=True)


if __name__ == "__main__":
    main()
