"""End-to-end parity of the GPU path with the reference's own known answers and
reference-generated peak lists (tests/golden/golden_e2e.json, written by
tests/golden/make_golden_e2e.py from the reference build and the reference's
Python modules):

- rseek (riptide/tests/test_rseek.py:31-54): top candidates of the fake pulsar;
- rffa pipeline (riptide/tests/test_pipeline.py:39-74, pipeline_config_A.yml):
  the peak list of three DM trials, its clustering and the top candidate;
- cfg5 (BASELINE configs[4]): 2^23-sample SIGPROC files (float32 and 8-bit)
  searched by GpuWorkerPool in DMIterator chunks over the example.yaml ranges;
- the multi-rank dispatcher (2 gloo ranks sharing cuda:0) against the same
  golden list;
- the C ABI's device error flag and one host thread per stream.

Candidate lists must be identical (ip, iw, dm); S/N within 1e-4 relative
(BASELINE.json).
"""
import hashlib
import json
import os
import socket
import sys
import threading

import numpy as np
import pytest

import inputs

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_e2e.json")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def e2e():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    with open(GOLDEN) as f:
        return json.load(f)


def assert_peaks_equal(got, ref):
    """got: Peak tuples; ref: golden rows [period, freq, width, ducy, dm, snr, ip, iw]."""
    assert len(got) == len(ref)
    assert [(p.ip, p.iw, p.dm, p.width) for p in got] == [(r[6], r[7], r[4], r[2]) for r in ref]
    assert [p.period for p in got] == [r[0] for r in ref]          # bit-exact trial grid
    s = np.array([p.snr for p in got])
    r = np.array([row[5] for row in ref])
    assert np.all(np.abs(s - r) <= 1e-4 * np.maximum(np.abs(r), 1.0))


def _rseek(rt, tmp_path, amplitude):
    """rseek.run_program (apps/rseek.py:104-146) on a PRESTO file written like
    presto_generation.py:31-58."""
    from riptide_amd.clustering import cluster1d
    from riptide_amd.reading import write_presto
    c = inputs.RSEEK_CASE
    data = inputs.generated_series(c["tobs"], c["tsamp"], c["period"], amplitude, c["ducy"], rt.libffa.generate_signal)
    fn = write_presto(str(tmp_path / f"data_{amplitude}"), data, c["tsamp"], dm=c["dm"])
    ts = rt.TimeSeries.from_presto_inf(fn)
    _, pg = rt.ffa_search(ts, period_min=c["pmin"], period_max=c["pmax"], bins_min=c["bmin"], bins_max=c["bmax"],
                          rmed_width=c["rmed_width"], rmed_minpts=c["rmed_minpts"], wtsp=c["wtsp"], fpmin=1,
                          ducy_max=c["ducy_max"])
    peaks, _ = rt.find_peaks(pg, smin=c["smin"], clrad=c["clrad"])
    best = []
    if peaks:
        freqs = np.asarray([p.freq for p in peaks])
        best = [max([peaks[i] for i in ids], key=lambda p: p.snr) for ids in cluster1d(freqs, r=c["clrad"] / ts.length)]
        best = sorted(best, key=lambda p: p.snr, reverse=True)
    return data, peaks, best


def test_rseek_known_answer(e2e, tmp_path):
    import riptide_amd as rt
    g = e2e["rseek"]
    data, peaks, best = _rseek(rt, tmp_path, inputs.RSEEK_CASE["amplitude"])
    assert sha(data) == g["input_sha"]
    assert_peaks_equal(peaks, g["find_peaks"])
    assert_peaks_equal(best, g["candidates"])
    # the reference test's own assertions (test_rseek.py:48-54)
    top = best[0]
    assert abs(top.freq - 1.0) < 0.1 / 128.0 and abs(top.snr - 18.5) < 0.15
    assert top.dm == 0 and top.width == 13
    # the oracle's top three
    assert [(p.period, p.width) for p in best[:3]] == [(1.0000742364089852, 13), (0.5000246075102122, 28),
                                                       (1.9999992937570006, 6)]


def test_rseek_pure_noise(e2e, tmp_path):
    import riptide_amd as rt
    data, peaks, best = _rseek(rt, tmp_path, 0.0)
    assert sha(data) == e2e["rseek_noise"]["input_sha"]
    assert peaks == [] and best == [] and e2e["rseek_noise"]["find_peaks"] == []


def _pipeline_files(rt, tmp_path):
    from riptide_amd.reading import write_presto
    c = inputs.PIPELINE_CASE
    fns, shas = [], []
    for dm, amp, ducy in c["trials"]:
        data = inputs.generated_series(c["tobs"], c["tsamp"], c["period"], amp, ducy, rt.libffa.generate_signal)
        shas.append(sha(data))
        fns.append(write_presto(str(tmp_path / f"fake_DM{dm:.3f}"), data, c["tsamp"], dm=dm))
    return fns, shas


def test_pipeline_known_answer(e2e, tmp_path):
    """Pipeline.search + cluster_peaks (pipeline.py:177-215) with the GPU
    worker pool in place of the CPU pool (processes: 2 -> chunks of 2)."""
    import riptide_amd as rt
    from riptide_amd.clustering import cluster1d
    from riptide_amd.worker_pool import GpuWorkerPool, iterate_chunks
    c = inputs.PIPELINE_CASE
    g = e2e["pipeline"]
    fns, shas = _pipeline_files(rt, tmp_path)
    assert shas == g["input_sha"]
    pool = GpuWorkerPool(c["dereddening"], c["ranges"], processes=2, fmt="presto", batch=2)
    peaks = []
    for chunk in iterate_chunks(fns, chunksize=2):
        peaks.extend(pool.process_fname_list(chunk))
    peaks = sorted(peaks, key=lambda p: p.period)
    assert_peaks_equal(peaks, g["peaks"])
    tmed = float(np.median([rt.TimeSeries.from_presto_inf(f).length for f in fns]))
    clusters = cluster1d(np.asarray([p.freq for p in peaks]), c["clustering_radius"] / tmed, already_sorted=True)
    assert len(peaks) == g["n_peaks"] == 99 and len(clusters) == g["n_clusters"] == 15
    assert [len(ids) for ids in clusters] == g["cluster_sizes"]
    top = max((max((peaks[i] for i in ids), key=lambda p: p.snr) for ids in clusters), key=lambda p: p.snr)
    assert_peaks_equal([top], [g["top"]])
    # test_pipeline.py:71-74
    assert abs(top.period - 1.0) < 1e-4 and top.dm == 10.0 and top.width == 13 and abs(top.snr - 18.5) < 0.15


def _cfg5_files(tmp_path, e2e):
    from riptide_amd.reading import write_sigproc
    fns = []
    for f in e2e["cfg5"]["files"]:
        data, hdr = inputs.cfg5_trial(f["k"])
        if sha(data) != f["input_sha"]:
            pytest.fail(f"cfg5 input generator drifted on this host: input sha256 {sha(data)} != golden "
                        f"{f['input_sha']}; the cfg5 parity check cannot run")
        fn = str(tmp_path / f"cfg5_DM{hdr['refdm']:06.1f}.tim")
        write_sigproc(fn, data, hdr)
        fns.append(fn)
    return fns


def _cfg5_golden_rows(e2e):
    """Golden peaks in WorkerPool order: file, range, then find_peaks' S/N order."""
    rows = []
    for f in e2e["cfg5"]["files"]:
        for r in f["ranges"]:
            rows += [(f["dm"], ip, iw, snr) for ip, iw, snr in r]
    return rows


def test_cfg5_worker_pool_matches_reference(e2e, tmp_path):
    """BASELINE configs[4] at 8 trials: SIGPROC files (6 float32, 2 8-bit) ->
    GpuWorkerPool in DMIterator chunks (dmiter.py:231-243) -> peak lists
    identical to the reference's WorkerPool.process_fname on every file."""
    from riptide_amd.worker_pool import GpuWorkerPool, iterate_chunks
    c = inputs.CFG5
    fns = _cfg5_files(tmp_path, e2e)
    pool = GpuWorkerPool(c["dereddening"], c["ranges"], processes=c["chunksize"], fmt="sigproc", batch=c["chunksize"])
    got = []
    for chunk in iterate_chunks(fns, chunksize=c["chunksize"]):
        got.extend(pool.process_fname_list(chunk))
    ref = _cfg5_golden_rows(e2e)
    assert len(got) == len(ref) > 0
    assert [(p.dm, p.ip, p.iw) for p in got] == [r[:3] for r in ref]
    s = np.array([p.snr for p in got])
    r = np.array([x[3] for x in ref])
    assert np.all(np.abs(s - r) <= 1e-4 * np.maximum(np.abs(r), 1.0))


# ---------------------------------------------------------------- multi-rank dispatcher on the GPU
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dispatch_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import riptide_amd as rt
        from riptide_amd.dispatch import EngineSearcher, Trial, search_trials
        c = inputs.PIPELINE_CASE
        trials = []
        for dm, amp, ducy in c["trials"]:
            data = inputs.generated_series(c["tobs"], c["tsamp"], c["period"], amp, ducy, rt.libffa.generate_signal)
            trials.append(Trial(data=data, tsamp=c["tsamp"], metadata={"dm": dm}))
        peaks = search_trials(trials, EngineSearcher(c["dereddening"], c["ranges"], device=0, batch=2))
        q.put((rank, [tuple(p) for p in peaks]))
    except Exception as e:  # reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_dispatch_two_ranks_on_gpu(e2e):
    """search_trials over 2 gloo ranks that both drive cuda:0 with the GPU
    EngineSearcher: every rank gathers the full list, in trial order, equal
    to the reference's pipeline peaks (sorted by period as pipeline.py:187)."""
    import torch.multiprocessing as mp
    from riptide_amd.peak_detection import Peak
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dispatch_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert not isinstance(results[0], str), results[0]
    assert results[0] == results[1]
    dms = [p[7] for p in results[0]]
    assert dms == sorted(dms)                            # trial order
    peaks = sorted((Peak(*p) for p in results[0]), key=lambda p: p.period)
    assert_peaks_equal(peaks, e2e["pipeline"]["peaks"])


def _files_worker(rank, world, port, fns, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from riptide_amd.dispatch import search_files
        from riptide_amd.worker_pool import GpuWorkerPool
        c = inputs.CFG5
        pool = GpuWorkerPool(c["dereddening"], c["ranges"], fmt="sigproc", batch=2, device=0)
        peaks = search_files(fns, pool, chunksize=2)       # 4 files per rank: two chunks, prefetched
        q.put((rank, [tuple(p) for p in peaks]))
    except Exception as e:  # reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_search_files_two_ranks_cfg5(e2e, tmp_path):
    """The multi-rank file path (dispatch.search_files: round-robin shard,
    GpuWorkerPool.search_chunks with its prefetching page-locked ring, one
    gather) over 2 gloo ranks driving cuda:0: the cfg5 files' peak lists
    equal the reference's, in file order, on both ranks."""
    import torch.multiprocessing as mp
    fns = _cfg5_files(tmp_path, e2e)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_files_worker, args=(r, 2, port, fns, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=200) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert not isinstance(results[0], str), results[0]
    assert not isinstance(results[1], str), results[1]
    assert results[0] == results[1]
    ref = _cfg5_golden_rows(e2e)
    got = results[0]
    assert [(p[7], p[5], p[4]) for p in got] == [r[:3] for r in ref]     # (dm, ip, iw)
    s = np.array([p[6] for p in got])
    r = np.array([x[3] for x in ref])
    assert np.all(np.abs(s - r) <= 1e-4 * np.maximum(np.abs(r), 1.0))


def test_worker_pool_mixed_shapes_matches_per_file(e2e, tmp_path):
    """One chunk mixing two series lengths and an 8-bit file, with a device
    batch that divides neither group: GpuWorkerPool groups by (length,
    tsamp), splits into batches and returns the peaks in input order, equal
    to searching every file on its own."""
    from riptide_amd.reading import write_sigproc
    from riptide_amd.worker_pool import GpuWorkerPool
    c = inputs.CFG5
    fns = []
    for j, k in enumerate((0, 2, 7, 3, 4, 6, 1)):
        n = (1 << 20) if j % 3 == 1 else (3 << 19)     # two lengths: 1 Mi and 1.5 Mi samples
        data, hdr = inputs.cfg5_trial(k, n=n)
        fn = str(tmp_path / f"mix_{j}.tim")
        write_sigproc(fn, data, hdr)
        fns.append(fn)
    pool = GpuWorkerPool(c["dereddening"], c["ranges"][:2], fmt="sigproc", batch=3)
    got = pool.process_fname_list(fns)
    one = GpuWorkerPool(c["dereddening"], c["ranges"][:2], fmt="sigproc", batch=1)
    ref = [p for fn in fns for p in one.process_fname(fn)]
    assert len(got) == len(ref) > 0
    assert [(p.dm, p.ip, p.iw) for p in got] == [(p.dm, p.ip, p.iw) for p in ref]
    assert [p.snr for p in got] == [p.snr for p in ref]          # same kernels: identical


def test_search_chunks_pipelined_matches_per_file(e2e, tmp_path):
    """GpuWorkerPool.search_chunks with chunk k's periodograms queued before
    chunk k - 1's peak detection (three-part page-locked ring, detection on a
    side stream): chunks mixing two lengths and an 8-bit file, a batch that
    splits them (batches pipelined within a chunk too), a short last chunk --
    the per-chunk peak lists equal searching every file on its own."""
    from riptide_amd.reading import write_sigproc
    from riptide_amd.worker_pool import GpuWorkerPool
    c = inputs.CFG5
    fns = []
    for j, k in enumerate((5, 2, 7, 3, 4, 6, 1, 0, 2, 6, 5)):
        n = (1 << 20) if j % 3 == 1 else (3 << 19)
        data, hdr = inputs.cfg5_trial(k, n=n)
        fn = str(tmp_path / f"pipe_{j}.tim")
        write_sigproc(fn, data, hdr)
        fns.append(fn)
    pool = GpuWorkerPool(c["dereddening"], c["ranges"][:2], fmt="sigproc", batch=2)
    chunks = list(pool.search_chunks(fns, chunksize=3))
    assert [first for first, _ in chunks] == [0, 3, 6, 9]
    got = [p for _, per_file in chunks for plist in per_file for p in plist]
    one = GpuWorkerPool(c["dereddening"], c["ranges"][:2], fmt="sigproc", batch=1)
    ref = [p for fn in fns for p in one.process_fname(fn)]
    assert len(got) == len(ref) > 0
    assert [(p.dm, p.ip, p.iw) for p in got] == [(p.dm, p.ip, p.iw) for p in ref]
    assert [p.snr for p in got] == [p.snr for p in ref]


# ---------------------------------------------------------------- C ABI robustness
_ERROR_FLAG_BODY = r"""
import sys
import numpy as np
import pytest
import torch
sys.path[:0] = [REPO, GOLDEN]
import inputs
from riptide_amd import _lib, engine, libcpp
assert _lib.LIB_PATH.endswith("libriptide_amd_testhooks.so")
case = inputs.PGRAM_CASES[1]
x = torch.from_numpy(inputs.pgram_input(case)).cuda()
args = (case["n"], case["tsamp"], case["pmin"], case["pmax"], case["bmin"], case["bmax"])
good = engine.PeriodogramPlan.for_search(*args, ducy_max=case["ducy_max"])
good.run(x, check=True)                                # no error on a valid plan
lib = _lib.load()
lib.rt_test_corrupt_next_plans(1)                      # test-only C entry point
try:
    bad = engine.PeriodogramPlan.for_search(*args, ducy_max=case["ducy_max"])
    with pytest.raises(_lib.EngineError, match="LDS budget"):
        bad.run(x, check=True)
    bad.check()                                       # the flag was cleared by the failed check
    with pytest.raises(_lib.EngineError, match="LDS budget"):
        libcpp.periodogram(inputs.pgram_input(case), case["tsamp"], good.widths, case["pmin"], case["pmax"],
                           case["bmin"], case["bmax"])
finally:
    lib.rt_test_corrupt_next_plans(0)
good.check()
print("error-flag OK")
"""


def test_plan_device_error_flag():
    """A unit that breaks its budget is refused by the kernel, which raises
    the plan's sticky flag; PeriodogramPlan.check / run(check=True) and the
    host-buffer periodogram raise instead of returning unwritten rows.  The
    corrupting hook exists only in the test build of the library
    (libriptide_amd_testhooks.so), so the body runs in a child process that
    loads that build (RIPTIDE_AMD_LIB)."""
    import subprocess
    from riptide_amd import _lib
    assert os.path.exists(_lib.TESTHOOKS_PATH), "build the test library: make -C riptide_amd/csrc"
    env = dict(os.environ, RIPTIDE_AMD_LIB=_lib.TESTHOOKS_PATH)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"REPO = {repo!r}\nGOLDEN = {os.path.join(repo, 'tests', 'golden')!r}\n" + _ERROR_FLAG_BODY
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "error-flag OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_two_host_threads_one_device():
    """One host thread per stream on one device (the supported threading
    model): concurrent rt_periodogram_device calls with
    profiling on give the same S/N as sequential ones."""
    import torch
    from riptide_amd import engine
    case = inputs.PGRAM_CASES[1]
    plan = engine.PeriodogramPlan.for_search(case["n"], case["tsamp"], case["pmin"], case["pmax"], case["bmin"],
                                             case["bmax"], ducy_max=case["ducy_max"])
    xs = [torch.from_numpy(np.stack([inputs.with_signal(case["n"], case["tsamp"], 40 + 3 * t + b, 0.41, 12.0)
                                     for b in range(3)])).cuda() for t in range(2)]
    ref = [plan.run(x).cpu().numpy() for x in xs]
    torch.cuda.synchronize()
    # profiling records per run: one per cone launch, or one for the whole
    # sequence when the plan's slot-width chains run on two streams
    engine.profile_reset()
    engine.profile_enable(True)
    plan.run(xs[0])
    torch.cuda.synchronize()
    engine.profile_enable(False)
    per_run = engine.profile_read(0)["launches"]
    assert per_run in (1, plan.stats()["launches"])
    out = [None, None]
    errs = []

    def work(t):
        try:
            s = torch.cuda.Stream()
            for _ in range(3):
                y = plan.run(xs[t], stream=s)
            s.synchronize()
            out[t] = y.cpu().numpy()
        except Exception as e:
            errs.append(e)

    engine.profile_reset()
    engine.profile_enable(True)
    th = [threading.Thread(target=work, args=(t,)) for t in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    engine.profile_enable(False)
    assert not errs, errs
    for t in range(2):
        assert np.array_equal(out[t], ref[t])
    prof = engine.profile_read(0)
    assert prof["launches"] == 2 * 3 * per_run
    plan.check()


def test_engine_imported_before_torch():
    """`import riptide_amd` before `import torch` (a fresh process): the engine
    library binds torch's HIP runtime (riptide_amd/_lib.py load imports torch
    first); loaded alone it bound /opt/rocm's and its launches failed with "no
    ROCm-capable device is detected" once torch initialised its own."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "tools", "import_order_check.py")],
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "import order ok" in r.stdout, r.stdout + r.stderr
