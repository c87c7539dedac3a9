"""ffa_search (riptide/search.py:10-82) on the MI355X engine."""
from . import libcpp
from .ffautils import generate_width_trials
from .periodogram import Periodogram
from .timing import timing


@timing
def ffa_search(tseries, period_min=1.0, period_max=30.0, fpmin=8, bins_min=240, bins_max=260,
               ducy_max=0.20, wtsp=1.5, deredden=True, rmed_width=4.0, rmed_minpts=101,
               already_normalised=False):
    """Deredden, normalise, then compute the FFA periodogram of a TimeSeries.

    Returns (searched TimeSeries, Periodogram).  With deredden=False and
    already_normalised=True the input TimeSeries object itself is returned.
    `fpmin` is accepted and unused, as in the reference (search.py:11).
    """
    if deredden and not already_normalised:
        tseries = tseries.deredden_normalise(rmed_width, minpts=rmed_minpts)
    else:
        if deredden:
            tseries = tseries.deredden(rmed_width, minpts=rmed_minpts)
        if not already_normalised:
            tseries = tseries.normalise()
    widths = generate_width_trials(bins_min, ducy_max=ducy_max, wtsp=wtsp)
    periods, foldbins, snrs = libcpp.periodogram(
        tseries.data, tseries.tsamp, widths, period_min, period_max, bins_min, bins_max)
    return tseries, Periodogram(widths, periods, foldbins, snrs, metadata=tseries.metadata)
