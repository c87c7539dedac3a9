"""The multi-GPU dispatcher's distributed logic (sharding + peak gather) on
CPU with the gloo backend, world_size 2.  The per-trial search is the oracle
(test infrastructure) so the test runs without a GPU; the GPU searcher itself
is covered by tests/test_gpu_parity.py."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import inputs

CASE = dict(n=1 << 14, tsamp=256e-6, pmin=0.1, pmax=2.0, bmin=64, bmax=72, ducy_max=0.1)


def make_trials():
    from riptide_amd.dispatch import Trial
    out = []
    for k in range(7):
        x = inputs.with_signal(CASE["n"], CASE["tsamp"], 100 + k, 0.17 + 0.05 * k, 25.0 if k % 2 == 0 else 0.0)
        out.append(Trial(data=x, tsamp=CASE["tsamp"], metadata={"dm": float(k)}))
    return out


def oracle_searcher(trials):
    """Searcher contract: one peak list per trial, in the order given."""
    from oracle import oracle as O
    from riptide_amd import Periodogram, find_peaks
    out = []
    for t in trials:
        widths = O.generate_width_trials(CASE["bmin"], CASE["ducy_max"])
        periods, foldbins, snrs = O.periodogram(O.normalise(t.data), t.tsamp, widths, CASE["pmin"], CASE["pmax"],
                                                CASE["bmin"], CASE["bmax"])
        meta = dict(t.metadata, tobs=t.data.size * t.tsamp)
        found, _ = find_peaks(Periodogram(widths, periods, foldbins, snrs, metadata=meta), smin=5.0)
        out.append(found)
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from riptide_amd.dispatch import search_trials
        peaks = search_trials(make_trials(), oracle_searcher)
        q.put((rank, [tuple(p) for p in peaks]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_partition():
    from riptide_amd.dispatch import shard
    for n in (0, 1, 7, 64):
        for world in (1, 2, 3, 8):
            got = sorted(i for r in range(world) for i in shard(n, r, world))
            assert got == list(range(n))
            sizes = [len(shard(n, r, world)) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1


def test_gather_world2_matches_single():
    from riptide_amd.dispatch import search_trials
    single = search_trials(make_trials(), oracle_searcher)
    assert len(single) > 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank holds the full, identical list, equal to the single-process
    # run element by element: trial order, then range order (WorkerPool contract)
    assert results[0] == results[1]
    assert results[0] == [tuple(p) for p in single]
    dms = [p.dm for p in single]
    assert dms == sorted(dms)            # trials were given in DM order


def test_search_trials_restores_trial_order():
    """A searcher that groups trials (as EngineSearcher groups by shape) still
    yields the peaks in trial order."""
    from riptide_amd.dispatch import search_trials
    from riptide_amd.peak_detection import Peak
    trials = make_trials()

    def fake(ts):
        return [[Peak(1.0, 1.0, 1, 0.1, 0, k, 7.0, t.metadata["dm"])] for k, t in enumerate(ts)]
    out = search_trials(trials, fake)
    assert [p.dm for p in out] == [t.metadata["dm"] for t in trials]


class _FakePool:
    """GpuWorkerPool.search_chunks contract without a GPU: one peak per file
    whose dm is parsed from the file name; records the chunk sizes."""

    def __init__(self):
        self.chunks = []

    def search_chunks(self, fnames, chunksize=None):
        from riptide_amd.peak_detection import Peak
        cs = chunksize or 3
        for i in range(0, len(fnames), cs):
            part = fnames[i:i + cs]
            self.chunks.append(len(part))
            yield i, [[Peak(1.0, 1.0, 1, 0.1, 0, 0, 7.0, float(fn.split("_")[1]))] for fn in part]


def _files_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from riptide_amd.dispatch import search_files, search_trials
        pool = _FakePool()
        fn = [f"f_{k}" for k in range(11)]
        peaks = search_files(fn, pool, chunksize=2)
        # loader form: each rank loads only its own shard
        loaded = []
        trials = make_trials()

        def loader(i):
            loaded.append(i)
            return trials[i]
        tp = search_trials(len(trials), oracle_searcher, loader=loader, chunksize=2)
        q.put((rank, [p.dm for p in peaks], pool.chunks, sorted(loaded), [tuple(p) for p in tp]))
    finally:
        dist.destroy_process_group()


def test_search_files_and_loader_world2():
    """search_files shards the file list round-robin, feeds each rank's share
    to the pool in chunks, and gathers the per-file lists back in file order;
    search_trials with a loader loads only the rank's own trials."""
    from riptide_amd.dispatch import search_trials
    single = [tuple(p) for p in search_trials(make_trials(), oracle_searcher)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_files_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r = q.get(timeout=300)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in (0, 1):
        dms, chunks, loaded, tp = res[rank]
        assert dms == [float(k) for k in range(11)]                 # file order on every rank
        assert chunks == ([2, 2, 2] if rank == 0 else [2, 2, 1])     # 6 / 5 files in chunks of 2
        assert loaded == list(range(rank, 7, 2))                     # only the rank's own trials
        assert tp == single
