"""Golden end-to-end peak lists from the REFERENCE (build container only;
/root/reference does not exist on the GPU box).  Writes
tests/golden/golden_e2e.json:

- ``rseek``: riptide/tests/test_rseek.py:31-54 -- the fake-pulsar PRESTO series
  of presto_generation.py:31-58 searched as rseek.run_program does
  (apps/rseek.py:104-146): ffa_search -> find_peaks -> cluster1d -> best peak
  per cluster, sorted by S/N.  Plus the pure-noise case (no peaks).
- ``pipeline``: riptide/tests/test_pipeline.py:39-74 with pipeline_config_A.yml:
  three DM trials searched as WorkerPool.process_fname does
  (pipeline/worker_pool.py:47-70), peaks sorted by period and clustered as
  Pipeline.cluster_peaks does (pipeline.py:177-215).
- ``cfg5``: the cfg5 beam of tests/golden/inputs.py (2^23-sample SIGPROC DM
  trials, example.yaml ranges), per file and per range find_peaks output.

The reference's own modules are loaded by path (make_golden.load_reference;
libffa.py in addition for generate_signal).  The orchestration lines of
TimeSeries / ffa_search / WorkerPool / rseek (which need astropy, absent
here) are restated with the same numpy expressions, as in make_golden.py.

Usage:  python tests/golden/make_golden_e2e.py   (needs `make -C oracle ref`)
"""
import hashlib
import importlib.util
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import inputs  # noqa: E402
import make_golden  # noqa: E402


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load_libffa(R):
    spec = importlib.util.spec_from_file_location("riptide.libffa", os.path.join(make_golden.REF, "libffa.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["riptide.libffa"] = mod
    spec.loader.exec_module(mod)
    R.libffa = mod
    return mod


def search_range(R, x, tsamp, tobs, dm, fs, fp):
    """ffa_search(deredden=False, already_normalised=True) + find_peaks
    (search.py:70-82, worker_pool.py:60-69)."""
    widths = R.ffautils.generate_width_trials(fs.get("bins_min", 240), ducy_max=fs.get("ducy_max", 0.2),
                                              wtsp=fs.get("wtsp", 1.5))
    periods, foldbins, snrs = R.libcpp.periodogram(x, tsamp, widths, fs["period_min"], fs["period_max"],
                                                   fs.get("bins_min", 240), fs.get("bins_max", 260))
    pg = make_golden._Pgram(widths, periods, foldbins, snrs, tobs, dm)
    peaks, _ = R.peak_detection.find_peaks(pg, **fp)
    return peaks


def peak_row(p):
    return [p.period, p.freq, int(p.width), p.ducy, p.dm, p.snr, int(p.ip), int(p.iw)]


def rseek_case(R, amplitude):
    c = inputs.RSEEK_CASE
    data = inputs.generated_series(c["tobs"], c["tsamp"], c["period"], amplitude, c["ducy"],
                                   R.libffa.generate_signal)
    tobs = data.size * c["tsamp"]
    x = make_golden.ref_deredden_normalise(R, data, c["tsamp"], c["rmed_width"], c["rmed_minpts"])
    fs = {"period_min": c["pmin"], "period_max": c["pmax"], "bins_min": c["bmin"], "bins_max": c["bmax"],
          "wtsp": c["wtsp"], "ducy_max": c["ducy_max"]}
    peaks = search_range(R, x, c["tsamp"], tobs, c["dm"], fs, {"smin": c["smin"], "clrad": c["clrad"]})
    raw = [peak_row(p) for p in peaks]
    best = []
    if peaks:
        freqs = np.asarray([p.freq for p in peaks])
        for ids in R.clustering.cluster1d(freqs, r=c["clrad"] / tobs):
            best.append(max([peaks[i] for i in ids], key=lambda p: p.snr))
        best = sorted(best, key=lambda p: p.snr, reverse=True)
    return {"input_sha": sha(data), "find_peaks": raw, "candidates": [peak_row(p) for p in best]}


def pipeline_case(R):
    c = inputs.PIPELINE_CASE
    peaks, shas = [], []
    for dm, amp, ducy in c["trials"]:
        data = inputs.generated_series(c["tobs"], c["tsamp"], c["period"], amp, ducy, R.libffa.generate_signal)
        shas.append(sha(data))
        tobs = data.size * c["tsamp"]
        d = c["dereddening"]
        x = make_golden.ref_deredden_normalise(R, data, c["tsamp"], d["rmed_width"], d["rmed_minpts"])
        for conf in c["ranges"]:
            peaks.extend(search_range(R, x, c["tsamp"], tobs, dm, conf["ffa_search"], conf["find_peaks"]))
    peaks = sorted(peaks, key=lambda p: p.period)                    # pipeline.py:187
    tmed = float(np.median([round(c["tobs"] / c["tsamp"]) * c["tsamp"]] * len(c["trials"])))
    freqs = np.asarray([p.freq for p in peaks])
    clusters = R.clustering.cluster1d(freqs, c["clustering_radius"] / tmed, already_sorted=True)
    centres = [max((peaks[i] for i in ids), key=lambda p: p.snr) for ids in clusters]
    top = max(centres, key=lambda p: p.snr)
    return {"input_sha": shas, "peaks": [peak_row(p) for p in peaks], "n_peaks": len(peaks),
            "n_clusters": len(clusters), "cluster_sizes": [len(ids) for ids in clusters], "top": peak_row(top)}


def cfg5_case(R):
    c = inputs.CFG5
    files = []
    for k in range(c["nfiles"]):
        t0 = time.time()
        stored, hdr = inputs.cfg5_trial(k)
        data = stored.astype(np.float32)
        tobs = data.size * hdr["tsamp"]
        d = c["dereddening"]
        x = make_golden.ref_deredden_normalise(R, data, hdr["tsamp"], d["rmed_width"], d["rmed_minpts"])
        ranges = []
        for conf in c["ranges"]:
            pk = search_range(R, x, hdr["tsamp"], tobs, hdr["refdm"], conf["ffa_search"], conf["find_peaks"])
            ranges.append([[int(p.ip), int(p.iw), p.snr] for p in pk])
        files.append({"k": k, "dm": hdr["refdm"], "dtype": str(stored.dtype), "input_sha": sha(stored),
                      "ranges": ranges})
        print(f"cfg5 file {k}: dm {hdr['refdm']} peaks {[len(r) for r in ranges]} ({time.time() - t0:.1f} s)")
    return {"files": files}


def main():
    R = make_golden.load_reference()
    load_libffa(R)
    out = {"meta": {"generated_by": "tests/golden/make_golden_e2e.py",
                    "reference_build": "g++ -O3 -ffast-math -march=native (setup.py:18)",
                    "numpy": np.__version__}}
    out["rseek"] = rseek_case(R, inputs.RSEEK_CASE["amplitude"])
    out["rseek_noise"] = rseek_case(R, 0.0)
    print("rseek top 3:", [(r[0], r[2], r[5]) for r in out["rseek"]["candidates"][:3]],
          "noise peaks:", len(out["rseek_noise"]["find_peaks"]))
    out["pipeline"] = pipeline_case(R)
    p = out["pipeline"]
    print("pipeline:", p["n_peaks"], "peaks", p["n_clusters"], "clusters, top", p["top"])
    out["cfg5"] = cfg5_case(R)
    with open(os.path.join(HERE, "golden_e2e.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
