"""Periodogram result object (riptide/periodogram.py:9-97)."""
from .metadata import Metadata


class Periodogram:
    """Raw output of the FFA search of one time series.

    widths   : boxcar width trials (phase bins)
    periods  : trial periods in seconds, float64[L]
    foldbins : phase bins used for each trial period, uint32[L]
    snrs     : S/N, float32[L, num_widths]
    """

    def __init__(self, widths, periods, foldbins, snrs, metadata=None):
        self.widths = widths
        self.periods = periods
        self.foldbins = foldbins
        self.snrs = snrs
        self.metadata = metadata if metadata is not None else Metadata({})

    @property
    def freqs(self):
        """Trial frequencies in Hz, in decreasing order."""
        return 1.0 / self.periods

    @property
    def tobs(self):
        return self.metadata["tobs"]

    def to_dict(self):
        return {"widths": self.widths, "periods": self.periods, "foldbins": self.foldbins,
                "snrs": self.snrs, "metadata": self.metadata}

    @classmethod
    def from_dict(cls, items):
        return cls(items["widths"], items["periods"], items["foldbins"], items["snrs"],
                   metadata=items["metadata"])

    def plot(self, iwidth=None):
        """S/N versus trial period in the current matplotlib figure (best width if iwidth is None)."""
        import matplotlib.pyplot as plt
        snr = self.snrs.max(axis=1) if iwidth is None else self.snrs[:, iwidth]
        plt.plot(self.periods, snr, marker="o", markersize=2, alpha=0.5)
        plt.xlim(self.periods.min(), self.periods.max())
        plt.xlabel("Trial Period (s)", fontsize=16)
        plt.ylabel("S/N", fontsize=16)
        if iwidth is None:
            plt.title("Best S/N at any trial width", fontsize=18)
        else:
            plt.title("S/N at trial width = %d" % self.widths[iwidth], fontsize=18)
        plt.grid(linestyle=":")
        plt.tight_layout()

    def display(self, iwidth=None, figsize=(20, 5), dpi=100):
        import matplotlib.pyplot as plt
        plt.figure(figsize=figsize, dpi=dpi)
        self.plot(iwidth=iwidth)
        plt.show()
