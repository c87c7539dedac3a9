"""CPU baseline for bench.py (TEST INFRASTRUCTURE, run in a subprocess).

Times one DM trial of the bench workload through the reference's CPU path:
the reference C++ periodogram (oracle/_ref/portable, built from the reference
sources with its own flags but a portable ISA) when present -> kind
"reference", otherwise the clean-room C restatement -> kind "port"; plus the
numpy dereddening/normalisation restated in oracle.py.  One process, one core
(threadpoolctl-style BLAS limits are irrelevant: no BLAS is used).

Prints one JSON object.
"""
import argparse
import glob
import importlib.util
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# run as a script: drop oracle/ itself from the path so `oracle` is the package
sys.path = [p for p in sys.path if os.path.abspath(p or '.') != HERE]
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 23)
    ap.add_argument("--tsamp", type=float, default=256e-6)
    ap.add_argument("--pmin", type=float, default=0.1)
    ap.add_argument("--pmax", type=float, default=10.0)
    ap.add_argument("--bmin", type=int, default=240)
    ap.add_argument("--bmax", type=int, default=260)
    ap.add_argument("--ducy-max", type=float, default=0.05)
    ap.add_argument("--trials", type=int, default=1)
    a = ap.parse_args()
    from oracle import oracle as O
    so = glob.glob(os.path.join(HERE, "_ref", "portable", "libcpp*.so"))
    kind = "port"
    pgram = None
    if so:
        try:
            spec = importlib.util.spec_from_file_location("libcpp", so[0])
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            pgram = mod.periodogram
            kind = "reference"
        except Exception:
            pgram = None
    if pgram is None:
        O.build()
        pgram = lambda d, ts, w, p0, p1, b0, b1: O.periodogram(d, ts, w, p0, p1, b0, b1)  # noqa: E731
    widths = O.generate_width_trials(a.bmin, a.ducy_max)
    rs = np.random.RandomState(1234)
    t_total = 0.0
    for _ in range(a.trials):
        raw = rs.normal(size=a.n).astype(np.float32)
        t0 = time.perf_counter()
        x = O.normalise(O.deredden(raw, a.tsamp, 4.0, 101))
        pgram(x, a.tsamp, widths, a.pmin, a.pmax, a.bmin, a.bmax)
        t_total += time.perf_counter() - t0
    print(json.dumps({"value": a.trials / t_total, "unit": "DM trials/s", "cores": 1, "kind": kind,
                      "sample": f"{a.trials} trial(s) of {a.n} samples: numpy deredden+normalise + "
                                f"{'reference C++ (-O3 -ffast-math -march=x86-64-v3)' if kind == 'reference' else 'oracle C'} "
                                f"periodogram, 1 process", "seconds": t_total}))


if __name__ == "__main__":
    main()
