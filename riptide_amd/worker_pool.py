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

Long file lists (a rank's share of a beam, dmiter.py:231-243 chunks) go
through `search_chunks`: a reader thread reads chunk k + 1 into one part of a
fixed three-part ring of page-locked slots while chunk k is on the device and
chunk k - 1's peaks are detected, so host memory stays at 3 x chunk files
whatever the list length, and file reads and host detection stages overlap
the device work.
"""
import logging
import threading

from .dispatch import EngineSearcher
from .reading import _raw_samples

log = logging.getLogger("riptide.worker_pool")

# host threads reading a chunk's files
_READ_THREADS = 8

# page-locked ring parts of search_chunks: chunk k - 1 detecting, chunk k on
# the device, chunk k + 1 being read
_RING_PARTS = 3


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
        self.device = device
        self.searcher = EngineSearcher(self.deredden_params, self.range_confs, device=device, batch=self.batch)
        self._pinned = {}
        # per ring part: a device event recorded after the part's samples were
        # last uploaded; a part is refilled only after its event completed
        self._part_done = {}

    def _stager(self, slot):
        """staging(nbytes) for ring slot `slot` = (part, file index): a page-locked uint8 buffer,
        grown when a file needs more (None without a GPU or for PRESTO)."""
        import torch
        if self.fmt != "sigproc" or not torch.cuda.is_available():
            return None

        def staging(nbytes):
            buf = self._pinned.get(slot)
            if buf is None or buf.numel() < nbytes:
                buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=True)
                self._pinned[slot] = buf
            return buf.numpy()
        return staging

    def _wait_part(self, part):
        ev = self._part_done.pop(part, None)
        if ev is not None:
            ev.synchronize()

    def _release_part(self, part):
        """Record that the device work reading ring part `part` is queued:
        the next fill of the part waits for it (search_samples happens to
        synchronise when its peaks reach the host; this does not rely on it)."""
        import torch
        if not torch.cuda.is_available():
            return
        dev = torch.device("cuda", torch.cuda.current_device() if self.device is None else self.device)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        self._part_done[part] = ev

    def _read(self, fnames, part):
        """Read a chunk's files (concurrently: np.fromfile / readinto release
        the GIL) into ring part `part`.  Returns (raws, metas, tsamps)."""
        self._wait_part(part)
        stagers = [self._stager((part, i)) for i in range(len(fnames))]
        if len(fnames) > 1:
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(max_workers=min(len(fnames), _READ_THREADS)) as ex:
                loaded = list(ex.map(lambda a: _raw_samples(a[0], self.fmt, staging=a[1]), zip(fnames, stagers)))
        else:
            loaded = [_raw_samples(fn, self.fmt, staging=st) for fn, st in zip(fnames, stagers)]
        return [t[0] for t in loaded], [t[1] for t in loaded], [t[2] for t in loaded]

    def _search(self, loaded, part):
        return self._submit(loaded, part)()

    def _submit(self, loaded, part):
        """Queue a chunk's uploads and periodograms; returns the callable that
        runs its peak detection (-> per-file peak lists).  The ring part is
        released (its event) once the chunk's last upload is queued."""
        raws, metas, tsamps = loaded
        released = []

        def uploaded():
            self._release_part(part)
            released.append(True)
        collect = None
        try:
            collect = self.searcher.submit_samples(raws, tsamps, metas, uploaded=uploaded)
        finally:
            if collect is None and not released:
                self._release_part(part)

        def finish():
            try:
                per_file = collect()
            finally:
                if not released:
                    self._release_part(part)
            for meta, peaks in zip(metas, per_file):
                log.debug(f"Done searching DM = {meta.get('dm')}, peaks found: {len(peaks)}")
            return per_file
        return finish

    def process_fname(self, fname):
        return self.process_fname_list([fname])

    def process_fname_list(self, fnames):
        """WorkerPool.process_fname_list: one chunk, read then searched."""
        fnames = list(fnames)
        per_file = self._search(self._read(fnames, 0), 0)
        return [p for plist in per_file for p in plist]

    def search_chunks(self, fnames, chunksize=None):
        """Search a long file list chunk by chunk (DMIterator chunks of
        `chunksize`, default `batch`), yielding (first index, per-file peak
        lists) per chunk in order.  Chunk k + 1 is read by a background
        thread into a free part of the page-locked ring while chunk k's
        periodograms are queued and chunk k - 1's peak detection runs, so
        the device works through the detection's host stages
        (EngineSearcher.submit_samples): three ring parts (k - 1 detecting,
        k on the device, k + 1 being read), at most three chunks of samples
        held whatever the list length."""
        fnames = list(fnames)
        cs = int(chunksize or self.batch)
        chunks = [(i, fnames[i:i + cs]) for i in range(0, len(fnames), cs)]
        if not chunks:
            return
        box = {}

        def reader(k):
            try:
                box[k] = self._read(chunks[k][1], k % _RING_PARTS)
            except BaseException as e:   # re-raised in the searching thread
                box[k] = e

        th = threading.Thread(target=reader, args=(0,), daemon=True)
        th.start()
        prev = None
        try:
            for k, (first, _) in enumerate(chunks):
                th.join()
                loaded = box.pop(k)
                if isinstance(loaded, BaseException):
                    raise loaded
                if k + 1 < len(chunks):
                    # the next chunk's part was last read by chunk k - 2,
                    # collected in the previous iteration: its uploads are
                    # queued, and _read waits for their event before refilling
                    th = threading.Thread(target=reader, args=(k + 1,), daemon=True)
                    th.start()
                cur = (first, self._submit(loaded, k % _RING_PARTS))
                if prev is not None:
                    yield prev[0], prev[1]()      # chunk k - 1's detection while chunk k is on the device
                prev = cur
            if prev is not None:
                yield prev[0], prev[1]()
        finally:
            th.join()      # no reader left writing into the ring
