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
