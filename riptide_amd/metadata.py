"""Observation metadata carried by TimeSeries and Periodogram (riptide/metadata.py:26-119).

A dict with the reserved keys source_name, skycoord, dm, mjd, tobs, fname set
to None when absent.  Schema validation and the SIGPROC/PRESTO constructors are
outside the hot path and not reproduced.
"""
import pprint

RESERVED_KEYS = ("source_name", "skycoord", "dm", "mjd", "tobs", "fname")


class Metadata(dict):
    def __init__(self, items=None):
        super().__init__(items or {})
        for k in RESERVED_KEYS:
            self.setdefault(k, None)

    def to_dict(self):
        return dict(self)

    @classmethod
    def from_dict(cls, items):
        return cls(items)

    def __str__(self):
        return "Metadata %s" % pprint.pformat(dict(self))

    __repr__ = __str__
