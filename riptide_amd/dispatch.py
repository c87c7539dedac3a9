"""Multi-GPU DM-trial dispatcher: the replacement of rffa's CPU worker pool
(riptide/pipeline/worker_pool.py:10-70) with the same contract: a list of DM
trials in, the flat List[Peak] of every trial and search range out.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm, or
"gloo" for CPU tests).  Trials are independent, so they are partitioned
statically (round-robin by index) with no data-path collective; each rank
batches its trials through the device-resident engine (dereddening +
normalisation once per trial, then one periodogram per search range, exactly
as WorkerPool.process_fname does), runs peak detection on the host, and the
per-rank peak lists are gathered once at the end (KB-scale, latency-bound).
"""
import logging
import typing

import numpy as np

from .peak_detection import Peak

log = logging.getLogger("riptide.dispatch")


class Trial(typing.NamedTuple):
    """One dedispersed time series to search."""
    data: np.ndarray          # float32 samples
    tsamp: float
    metadata: dict            # must hold 'dm' (None allowed), like riptide Metadata


def shard(n_items, rank, world):
    """Indices of the trials owned by `rank`: round-robin, so every rank gets
    a near-equal share and consecutive DMs spread over the GPUs."""
    return list(range(rank, n_items, world))


class EngineSearcher:
    """Batched GPU search of trials of one length: the hot path.  For every
    search range: one compiled periodogram plan per (length, tsamp, range)
    and device peak detection (riptide_amd.peaks.PeakFinder); only the peaks
    leave the device."""

    def __init__(self, deredden_params, range_confs, device=None, batch=8):
        self.deredden_params = dict(deredden_params)
        self.range_confs = list(range_confs)
        self.device = device
        self.batch = int(batch)
        self._plans = {}
        self._finders = {}

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

    def search_device(self, raw, tsamp, metadatas):
        """Peaks of every trial of a device batch raw [B, N] (float32): one
        list per trial, in range order (WorkerPool.process_fname)."""
        from . import engine
        B, n = raw.shape
        ws = int(round(self.deredden_params["rmed_width"] / tsamp))
        x = engine.deredden_normalise(raw, ws, self.deredden_params["rmed_minpts"])
        out = [[] for _ in range(B)]
        dms = [m.get("dm") for m in metadatas]
        for conf in self.range_confs:
            plan = self._plan(n, tsamp, conf)
            snr = plan.run(x)
            for b, (peaks, _) in enumerate(self._finder(plan, n * tsamp, conf)(snr, dms=dms)):
                out[b].extend(peaks)
        return out

    def __call__(self, trials):
        import torch
        dev = torch.device("cuda", torch.cuda.current_device() if self.device is None else self.device)
        peaks = []
        groups = {}
        for t in trials:
            groups.setdefault((t.data.size, float(t.tsamp)), []).append(t)
        for (n, tsamp), group in groups.items():
            for b0 in range(0, len(group), self.batch):
                chunk = group[b0:b0 + self.batch]
                raw = torch.from_numpy(np.stack([np.asarray(t.data, np.float32) for t in chunk])).to(dev)
                for found in self.search_device(raw, tsamp, [t.metadata for t in chunk]):
                    peaks.extend(found)
        return peaks


def search_trials(trials, searcher, group=None):
    """Search this rank's share of `trials` with `searcher` (a callable taking
    a list of Trial and returning List[Peak]); gather every rank's peaks.
    Returns the full peak list on every rank, in trial order per rank."""
    import torch.distributed as dist
    distributed = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank(group) if distributed else 0
    world = dist.get_world_size(group) if distributed else 1
    mine = [trials[i] for i in shard(len(trials), rank, world)]
    local = searcher(mine) if mine else []
    if world == 1:
        return list(local)
    gathered = [None] * world
    dist.all_gather_object(gathered, [tuple(p) for p in local], group=group)
    return [Peak(*p) for part in gathered for p in part]
