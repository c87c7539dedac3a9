"""Multi-GPU DM-trial dispatcher: the replacement of rffa's CPU worker pool
(riptide/pipeline/worker_pool.py:10-70) with the same contract: a list of DM
trials in, the flat List[Peak] of every trial and search range out, in trial
order and, within a trial, in range order (WorkerPool.process_fname_list,
worker_pool.py:35-45, flattens its Pool.map results the same way).

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm, or
"gloo" for CPU tests).  Trials are independent, so they are partitioned
statically (round-robin by index) with no data-path collective; each rank
batches its trials through the device-resident engine (dereddening +
normalisation once per trial, then one periodogram per search range, exactly
as WorkerPool.process_fname does) and device peak detection, and the
per-rank peak lists -- tagged with their trial index -- are gathered once at
the end (KB-scale, latency-bound) and put back in trial order.
"""
import logging
import os
import typing

import numpy as np

from .peak_detection import Peak

log = logging.getLogger("riptide.dispatch")


class Trial(typing.NamedTuple):
    """One dedispersed time series to search."""
    data: np.ndarray          # samples as stored (float32, or uint8 / int8 8-bit data)
    tsamp: float
    metadata: dict            # must hold 'dm' (None allowed), like riptide Metadata


def shard(n_items, rank, world):
    """Indices of the trials owned by `rank`: round-robin, so every rank gets
    a near-equal share and consecutive DMs spread over the GPUs."""
    return list(range(rank, n_items, world))


def _group_by_shape(samples, tsamps):
    """{(length, tsamp): [indices]} in first-seen order (device batches need
    one series length and one sampling time)."""
    groups = {}
    for i, (x, ts) in enumerate(zip(samples, tsamps)):
        groups.setdefault((int(np.asarray(x).size), float(ts)), []).append(i)
    return groups


class EngineSearcher:
    """Batched GPU search of DM trials: the hot path.  For every search range:
    one compiled periodogram plan per (length, tsamp, range) and device peak
    detection (riptide_amd.peaks.PeakFinder); only the peaks leave the device.

    Calling it on a list of Trial returns one peak list per trial, in the
    order given (each in range order, as WorkerPool.process_fname)."""

    def __init__(self, deredden_params, range_confs, device=None, batch=8, check=True):
        self.deredden_params = dict(deredden_params)
        self.range_confs = list(range_confs)
        self.device = device
        self.batch = int(batch)
        self.check = bool(check)
        self._plans = {}
        self._finders = {}
        self._ws = {}
        self._side = {}

    def _plan(self, n, tsamp, conf):
        from . import engine
        kw = conf["ffa_search"]
        key = (n, tsamp, tuple(sorted(kw.items())))
        if key not in self._plans:
            self._plans[key] = engine.PeriodogramPlan.for_search(
                n, tsamp, kw["period_min"], kw["period_max"], kw.get("bins_min", 240), kw.get("bins_max", 260),
                ducy_max=kw.get("ducy_max", 0.2), wtsp=kw.get("wtsp", 1.5), device=self.device)
        return self._plans[key]

    def _finder(self, plan, tobs, conf):
        from .peaks import PeakFinder
        kw = conf.get("find_peaks", {}) or {}
        key = (id(plan), tobs, tuple(sorted(kw.items())))
        if key not in self._finders:
            self._finders[key] = PeakFinder(plan, tobs, **kw)
        return self._finders[key]

    def _workspace(self, plan, B):
        import torch
        need = plan.workspace_bytes(B)
        ws = self._ws.get(id(plan))
        if ws is None or ws.numel() < need:
            ws = torch.empty(need, dtype=torch.uint8, device=plan.device)
            self._ws[id(plan)] = ws
        return ws

    def _side_stream(self, dev):
        import torch
        if dev not in self._side:
            self._side[dev] = torch.cuda.Stream(device=dev)
        return self._side[dev]

    def search_device(self, raw, tsamp, metadatas):
        """Peaks of every trial of a device batch raw [B, N] (float32): one
        list per trial, in range order (WorkerPool.process_fname)."""
        return self._detect(self._enqueue(raw, tsamp, metadatas))

    def _enqueue(self, raw, tsamp, metadatas):
        """Queue a device batch's deredden + normalise and every range's
        periodogram on the current stream; returns the pending batch for
        _detect.  Nothing here waits for the device."""
        import torch
        from . import engine
        B, n = raw.shape
        ws = int(round(self.deredden_params["rmed_width"] / tsamp))
        x = engine.deredden_normalise(raw, ws, self.deredden_params["rmed_minpts"])
        dms = [m.get("dm") for m in metadatas]
        main = torch.cuda.current_stream(x.device)
        if os.environ.get("RIPTIDE_AMD_PEAKS_SERIAL"):
            return {"serial": True, "x": x, "n": n, "tsamp": tsamp, "dms": dms}
        runs = []
        for conf in self.range_confs:
            plan = self._plan(n, tsamp, conf)
            snr = plan.run(x, workspace=self._workspace(plan, B))
            ev = torch.cuda.Event()
            ev.record(main)
            runs.append((conf, plan, snr, ev))
        return {"serial": False, "runs": runs, "n": n, "tsamp": tsamp, "dms": dms, "B": B, "device": x.device}

    def _detect(self, pend):
        """Peak detection of a pending batch, range by range, on a side
        stream: each range's detection starts once its periodogram is done
        (an event), so its host stages (the order statistics' polyfits, the
        selected rows' clustering) overlap the periodograms queued after it
        -- the later ranges', and with submit_samples the next batch's --
        instead of leaving the GPU idle.  Same kernels on the same data:
        same peaks."""
        n, tsamp, dms = pend["n"], pend["tsamp"], pend["dms"]
        if pend["serial"]:
            # A/B (RIPTIDE_AMD_PEAKS_SERIAL): each range's detection right
            # after its periodogram, on the same stream, nothing queued ahead
            x = pend["x"]
            out = [[] for _ in range(x.shape[0])]
            for conf in self.range_confs:
                plan = self._plan(n, tsamp, conf)
                snr = plan.run(x, workspace=self._workspace(plan, x.shape[0]))
                if self.check:
                    plan.check()
                for b, (peaks, _) in enumerate(self._finder(plan, n * tsamp, conf)(snr, dms=dms)):
                    out[b].extend(peaks)
            return out
        out = [[] for _ in range(pend["B"])]
        side = self._side_stream(pend["device"])
        for conf, plan, snr, ev in pend["runs"]:
            side.wait_event(ev)
            snr.record_stream(side)
            for b, (peaks, _) in enumerate(self._finder(plan, n * tsamp, conf)(snr, dms=dms, stream=side)):
                out[b].extend(peaks)
        if self.check:
            for _, plan, _, _ in pend["runs"]:
                # device error flag, read on the side stream: ordered after
                # this batch's periodograms (the events), not waiting for
                # what is queued behind them; RuntimeError if a unit broke
                # its budget
                plan.check(side)
        return out

    def submit_samples(self, samples, tsamps, metadatas, uploaded=None):
        """search_samples in two halves: uploads and periodograms of every
        device batch queued now, peak detection when the returned callable is
        called (-> per-trial peak lists in input order).  A caller that
        submits chunk k + 1 before collecting chunk k keeps the device busy
        through chunk k's host stages (GpuWorkerPool.search_chunks); device
        batches within one call are pipelined the same way.  `uploaded()`, if
        given, is called once the last batch's upload is queued: the host
        samples may be reused after the device work queued at that moment (an
        event)."""
        from .reading import upload_samples
        batches = []
        for (n, tsamp), idx in _group_by_shape(samples, tsamps).items():
            for b0 in range(0, len(idx), self.batch):
                batches.append((tsamp, idx[b0:b0 + self.batch]))
        per = [None] * len(samples)
        state = {"next": 0, "pending": []}

        def enqueue_one():
            k = state["next"]
            if k < len(batches):
                tsamp, chunk = batches[k]
                x = upload_samples([samples[i] for i in chunk], device=self.device)
                if k + 1 == len(batches) and uploaded is not None:
                    uploaded()
                state["pending"].append((chunk, self._enqueue(x, tsamp, [metadatas[i] for i in chunk])))
                state["next"] = k + 1

        def collect():
            while state["pending"]:
                enqueue_one()           # batch j + 1 queued before batch j's detection
                chunk, pend = state["pending"].pop(0)
                for i, peaks in zip(chunk, self._detect(pend)):
                    per[i] = peaks
            return per

        enqueue_one()
        if not batches and uploaded is not None:
            uploaded()
        return collect

    def search_samples(self, samples, tsamps, metadatas):
        """Per-trial peak lists of host sample arrays (float32 or 8-bit, as
        stored): grouped by (length, tsamp), uploaded in device batches
        (8-bit data converted on the device), results in input order."""
        return self.submit_samples(samples, tsamps, metadatas)()

    def __call__(self, trials):
        return self.search_samples([t.data for t in trials], [t.tsamp for t in trials],
                                   [t.metadata for t in trials])


def _rank_world(group):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def _gather_tagged(tagged, group, world):
    """All ranks' (trial index, peak tuples) lists, gathered once (KB-scale),
    in trial order, flattened to the WorkerPool contract."""
    if world > 1:
        import torch.distributed as dist
        gathered = [None] * world
        dist.all_gather_object(gathered, tagged, group=group)
        tagged = [t for part in gathered for t in part]
    tagged.sort(key=lambda t: t[0])
    return [Peak(*p) for _, plist in tagged for p in plist]


def search_trials(trials, searcher, group=None, loader=None, chunksize=None):
    """Search this rank's share of the DM trials with `searcher` (a callable
    taking a list of Trial and returning one peak list per trial, in order)
    and gather every rank's lists.  Returns the full peak list on every
    rank, in trial order (then range order within a trial): the WorkerPool
    contract (worker_pool.py:35-45).

    `trials` is a sequence of Trial, or -- with `loader` -- the number of
    trials, `loader(i)` returning Trial i: each rank then loads only its own
    shard, `chunksize` trials at a time (default: the searcher's batch), so no
    rank ever holds the whole list."""
    rank, world = _rank_world(group)
    n = int(trials) if loader is not None else len(trials)
    get = loader if loader is not None else (lambda i: trials[i])
    mine = shard(n, rank, world)
    cs = int(chunksize or getattr(searcher, "batch", 0) or max(1, len(mine)))
    tagged = []
    for c0 in range(0, len(mine), cs):
        idx = mine[c0:c0 + cs]
        local = searcher([get(i) for i in idx])
        if len(local) != len(idx):
            raise RuntimeError("searcher must return one peak list per trial")
        tagged += [(i, [tuple(p) for p in plist]) for i, plist in zip(idx, local)]
    return _gather_tagged(tagged, group, world)


def search_files(fnames, pool, group=None, chunksize=None):
    """rffa's search stage over the ranks of one node (pipeline.py:177-189 with
    dmiter.py:231-243): each rank searches its round-robin share of the
    DM-ordered file list through `pool` (a GpuWorkerPool) in chunks of
    `chunksize` files (default: the pool's batch), the next chunk read into
    a bounded page-locked ring while the current one is on the device
    (GpuWorkerPool.search_chunks); one gather of the tagged peak lists.
    Returns the full peak list on every rank, in file order."""
    rank, world = _rank_world(group)
    fnames = list(fnames)
    mine = shard(len(fnames), rank, world)
    tagged = []
    for first, per_file in pool.search_chunks([fnames[i] for i in mine], chunksize=chunksize):
        tagged += [(mine[first + j], [tuple(p) for p in plist]) for j, plist in enumerate(per_file)]
    return _gather_tagged(tagged, group, world)
