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
            snr = plan.run(x, workspace=self._workspace(plan, B))
            if self.check:
                plan.check()          # device error flag: RuntimeError if a unit broke its budget
            for b, (peaks, _) in enumerate(self._finder(plan, n * tsamp, conf)(snr, dms=dms)):
                out[b].extend(peaks)
        return out

    def search_samples(self, samples, tsamps, metadatas):
        """Per-trial peak lists of host sample arrays (float32 or 8-bit, as
        stored): grouped by (length, tsamp), uploaded in device batches
        (8-bit data converted on the device), results in input order."""
        from .reading import upload_samples
        per = [None] * len(samples)
        for (n, tsamp), idx in _group_by_shape(samples, tsamps).items():
            for b0 in range(0, len(idx), self.batch):
                chunk = idx[b0:b0 + self.batch]
                x = upload_samples([samples[i] for i in chunk], device=self.device)
                for i, peaks in zip(chunk, self.search_device(x, tsamp, [metadatas[i] for i in chunk])):
                    per[i] = peaks
        return per

    def __call__(self, trials):
        return self.search_samples([t.data for t in trials], [t.tsamp for t in trials],
                                   [t.metadata for t in trials])


def search_trials(trials, searcher, group=None):
    """Search this rank's share of `trials` with `searcher` (a callable taking
    a list of Trial and returning one peak list per trial, in order); gather
    every rank's lists.  Returns the full peak list on every rank, in trial
    order (then range order within a trial): the WorkerPool contract."""
    import torch.distributed as dist
    distributed = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank(group) if distributed else 0
    world = dist.get_world_size(group) if distributed else 1
    mine = shard(len(trials), rank, world)
    local = searcher([trials[i] for i in mine]) if mine else []
    if len(local) != len(mine):
        raise RuntimeError("searcher must return one peak list per trial")
    tagged = [(i, [tuple(p) for p in plist]) for i, plist in zip(mine, local)]
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, tagged, group=group)
        tagged = [t for part in gathered for t in part]
    tagged.sort(key=lambda t: t[0])
    return [Peak(*p) for _, plist in tagged for p in plist]
