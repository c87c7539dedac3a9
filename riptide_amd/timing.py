"""Wall-time logging decorator, logger ``riptide.timing`` (riptide/timing.py:6-15)."""
import logging
import time
from functools import wraps


def timing(func):
    @wraps(func)
    def wrapped(*args, **kwargs):
        t0 = time.time()
        out = func(*args, **kwargs)
        logging.getLogger("riptide.timing").debug(
            "{!r} runtime: {:.2f} ms".format(func.__name__, (time.time() - t0) * 1000.0))
        return out
    return wrapped
