"""GPU replacement of rffa's WorkerPool (riptide/pipeline/worker_pool.py:10-70,
SURVEY.md §8 f2): same constructor arguments and the same
`process_fname_list(fnames) -> List[Peak]` contract, so Pipeline.search
(pipeline.py:177-189) can use it unchanged.

Instead of one CPU process per DM trial, the files of a chunk are read once
on the host (headers parsed, samples kept as stored), grouped by (length,
sampling time) and searched in device batches: raw samples go to the GPU
(8-bit data converted there), are dereddened and normalised once per trial
(worker_pool.py:53-58), then every search range runs the FFA periodogram (one
compiled plan per range and series shape) and device peak detection
(riptide_amd.peaks).  Peaks come back per file in input order and, within a
file, in range order -- the order WorkerPool.process_fname_list returns them
in.
"""
import logging

from .dispatch import EngineSearcher
from .reading import _raw_samples

log = logging.getLogger("riptide.worker_pool")

# host threads reading a chunk's files
_READ_THREADS = 8


def iterate_chunks(fnames, chunksize=1):
    """DMIterator.iterate_filenames (pipeline/dmiter.py:231-243) over an
    already selected, DM-ordered file list: chunks of `chunksize`, the last
    one possibly shorter."""
    chunk = []
    for fn in fnames:
        chunk.append(fn)
        if len(chunk) == chunksize:
            yield chunk
            chunk = []
    if chunk:
        yield chunk


class GpuWorkerPool:
    """deredden_params : dict (rmed_width, rmed_minpts)
    range_confs : list of dicts with 'ffa_search' and 'find_peaks' sections
    processes : accepted for interface compatibility (the device batch size
        is `batch`)
    fmt : 'sigproc' or 'presto'
    """

    def __init__(self, deredden_params, range_confs, processes=1, fmt="presto", batch=8, device=None):
        self.deredden_params = dict(deredden_params)
        self.range_confs = list(range_confs)
        self.processes = int(processes)
        self.fmt = fmt
        self.batch = int(batch)
        self.searcher = EngineSearcher(self.deredden_params, self.range_confs, device=device, batch=self.batch)

    def _stager(self, slot):
        """staging(nbytes) for file slot `slot` of a chunk: a page-locked
        uint8 buffer, grown when a file needs more (None without a GPU)."""
        import torch
        if not torch.cuda.is_available():
            return None
        if not hasattr(self, "_pinned"):
            self._pinned = {}

        def staging(nbytes):
            buf = self._pinned.get(slot)
            if buf is None or buf.numel() < nbytes:
                buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=True)
                self._pinned[slot] = buf
            return buf.numpy()
        return staging

    def process_fname(self, fname):
        return self.process_fname_list([fname])

    def process_fname_list(self, fnames):
        # the chunk's files are read concurrently (np.fromfile releases the
        # GIL), as rffa's pool reads one file per process
        fnames = list(fnames)
        # SIGPROC samples land in page-locked slots reused across chunks (one
        # per file of a chunk), so the uploads are asynchronous DMAs; every
        # device use of a chunk's samples has completed when search_samples
        # returns (its peak lists are on the host), before the slots are
        # refilled by the next call
        stagers = [self._stager(i) for i in range(len(fnames))] if self.fmt == "sigproc" else [None] * len(fnames)
        if len(fnames) > 1:
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(max_workers=min(len(fnames), _READ_THREADS)) as ex:
                loaded = list(ex.map(lambda a: _raw_samples(a[0], self.fmt, staging=a[1]), zip(fnames, stagers)))
        else:
            loaded = [_raw_samples(fn, self.fmt, staging=st) for fn, st in zip(fnames, stagers)]
        raws = [t[0] for t in loaded]
        metas = [t[1] for t in loaded]
        tsamps = [t[2] for t in loaded]
        per_file = self.searcher.search_samples(raws, tsamps, metas)
        for meta, peaks in zip(metas, per_file):
            log.debug(f"Done searching DM = {meta.get('dm')}, peaks found: {len(peaks)}")
        return [p for plist in per_file for p in plist]
