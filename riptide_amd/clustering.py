"""1-D friends-of-friends clustering (riptide/clustering.py:4-50) and the
pipeline's peak-clustering stage (riptide/pipeline/pipeline.py:177-215)."""
import numpy as np


def cluster1d(x, r, already_sorted=False):
    """Split points into clusters where consecutive sorted points are <= r apart.
    Returns a list of index arrays into x."""
    x = np.asarray(x)
    if not len(x):
        return []
    order = np.arange(len(x)) if already_sorted else x.argsort()
    gaps = np.abs(np.diff(x[order])) > r
    cuts = np.flatnonzero(gaps) + 1
    if not cuts.size:
        return [order]
    return np.split(order, cuts)


def cluster_peaks(peaks, radius, tobs_median):
    """Pipeline.search's final sort and Pipeline.cluster_peaks
    (pipeline.py:186, 192-215): the peaks sorted by increasing period
    (Python's stable sort, as `sorted(peaks, key=lambda p: p.period)`), then
    friends-of-friends in frequency with radius `radius` / tobs_median Hz
    (`clustering.radius` of the pipeline config, in units of 1 / Tobs).
    `peaks` are Peak objects or their tuples.  Returns (sorted peaks, list of
    clusters), each cluster the list of its peaks in sorted order -- the
    members of one reference PeakCluster."""
    from .peak_detection import Peak
    ps = sorted((p if isinstance(p, Peak) else Peak(*p) for p in peaks), key=lambda p: p.period)
    if not ps:
        return ps, []
    freqs = np.asarray([p.freq for p in ps])
    ids = cluster1d(freqs, radius / tobs_median, already_sorted=True)
    return ps, [[ps[i] for i in cl] for cl in ids]
