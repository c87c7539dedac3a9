"""Readers of dedispersed time series files: SIGPROC .tim and PRESTO .inf/.dat
(riptide/reading/sigproc.py:1-197, riptide/reading/presto.py:1-149,
riptide/metadata.py:54-106, riptide/time_series.py:283-362).

Header parsing stays on the host; the bulk samples are read as raw bytes and,
for the device path (`load_device_batch`), converted to float32 on the GPU by
rt_convert_samples_device after one host-to-device copy of the raw bytes
(8-bit data moves 4x fewer bytes over PCIe than its float32 expansion).

astropy is not available here: sky coordinates are kept as `Coord`
(right ascension in hours, declination in degrees), parsed exactly as the
reference parses them before building its SkyCoord.
"""
import os
import struct
import typing

import numpy as np

from .metadata import Metadata


class Coord(typing.NamedTuple):
    """ICRS position: right ascension (hours), declination (degrees)."""
    ra_hours: float
    dec_deg: float


# ---------------------------------------------------------------------------
# SIGPROC (riptide/reading/sigproc.py)
# ---------------------------------------------------------------------------
# Header keys and their stored types: int = int32, float = float64,
# bool = unsigned char, str = int32 length + bytes (sigproc.py:18-62).
SIGPROC_KEYS = {
    "filename": str, "telescope_id": int, "telescope": str, "machine_id": int, "data_type": int,
    "rawdatafile": str, "source_name": str, "barycentric": int, "pulsarcentric": int, "az_start": float,
    "za_start": float, "src_raj": float, "src_dej": float, "tstart": float, "tsamp": float, "nbits": int,
    "nsamples": int, "fch1": float, "foff": float, "fchannel": float, "nchans": int, "nifs": int,
    "refdm": float, "flux": float, "period": float, "nbeams": int, "ibeam": int, "hdrlen": int, "pb": float,
    "ecc": float, "asini": float, "orig_hdrlen": int, "new_hdrlen": int, "sampsize": int, "bandwidth": float,
    "fbottom": float, "ftop": float, "obs_date": str, "obs_time": str, "accel": float, "signed": bool,
}
HEADER_START = "HEADER_START"
HEADER_END = "HEADER_END"


def _read_str(f):
    (size,) = struct.unpack("i", f.read(4))
    return f.read(size).decode()


def read_sigproc_header(f, extra_keys=None):
    """({key: value}, header byte size) of an open SIGPROC file (sigproc.py:109-147)."""
    keys = dict(SIGPROC_KEYS)
    if extra_keys:
        keys.update(extra_keys)
    f.seek(0)
    flag = _read_str(f)
    assert flag == HEADER_START, f"File starts with {flag!r} flag instead of the expected {HEADER_START!r}"
    attrs = {}
    while True:
        key = _read_str(f)
        if key == HEADER_END:
            break
        atype = keys.get(key)
        if atype is None:
            raise KeyError(f"Type of SIGPROC header attribute {key!r} is unknown, please specify it")
        if atype is str:
            val = _read_str(f)
        elif atype is int:
            (val,) = struct.unpack("i", f.read(4))
        elif atype is float:
            (val,) = struct.unpack("d", f.read(8))
        elif atype is bool:
            (val,) = struct.unpack("B", f.read(1))
            val = bool(val)
        else:
            raise ValueError(f"Key {key!r} has unsupported type {atype!r}")
        attrs[key] = val
    return attrs, f.tell()


def parse_float_coord(x):
    """SIGPROC's ddmmss.s / hhmmss.s float coordinate -> hours or degrees (sigproc.py:150-159)."""
    sign = np.sign(x)
    x = abs(x)
    hh, x = divmod(x, 10000.0)
    mm, ss = divmod(x, 100.0)
    return sign * (hh + mm / 60.0 + ss / 3600.0)


class SigprocHeader(dict):
    """Header of a SIGPROC file (sigproc.py:159-197)."""

    def __init__(self, fname, extra_keys=None):
        self._fname = os.path.abspath(fname)
        with open(self._fname, "rb") as f:
            attrs, self._bytesize = read_sigproc_header(f, extra_keys)
        super().__init__(attrs)

    @property
    def fname(self):
        return self._fname

    @property
    def bytesize(self):
        return self._bytesize

    @property
    def bytes_per_sample(self):
        return self["nchans"] * self["nbits"] // 8

    @property
    def nsamp(self):
        return (os.path.getsize(self.fname) - self.bytesize) // self.bytes_per_sample

    @property
    def tobs(self):
        return self.nsamp * self["tsamp"]

    @property
    def skycoord(self):
        return Coord(float(parse_float_coord(self["src_raj"])), float(parse_float_coord(self["src_dej"])))


def sigproc_metadata(sh):
    """Metadata.from_sigproc (metadata.py:74-106): checks and derived keys."""
    if sh["nchans"] > 1:
        raise ValueError(f"File {sh.fname!r} contains multi-channel data (nchans = {sh['nchans']}), "
                         "instead of a dedispersed time series")
    nbits = sh["nbits"]
    if nbits not in {8, 32}:
        raise ValueError(f"Only 8-bit and 32-bit SIGPROC data are supported. File {sh.fname!r} contains "
                         f"{nbits}-bit data")
    if nbits == 8 and "signed" not in sh:
        raise ValueError("SIGPROC Header says this is 8-bit data, but does not specify its signedness via the "
                         "'signed' key")
    attrs = dict(sh)
    attrs["dm"] = attrs.get("refdm", None)
    attrs["skycoord"] = sh.skycoord
    attrs["source_name"] = attrs.get("source_name", None)
    attrs["mjd"] = attrs.get("tstart", None)
    attrs["fname"] = os.path.realpath(sh.fname)
    attrs["tobs"] = sh.tobs
    return Metadata(attrs)


def sigproc_sample_dtype(meta):
    if meta["nbits"] == 8:
        return np.int8 if meta["signed"] else np.uint8
    return np.float32


def read_sigproc(fname, extra_keys=None):
    """(float32 samples, Metadata, tsamp) as TimeSeries.from_sigproc (time_series.py:320-362)."""
    sh = SigprocHeader(fname, extra_keys=extra_keys)
    meta = sigproc_metadata(sh)
    with open(sh.fname, "rb") as f:
        f.seek(sh.bytesize)
        data = np.fromfile(f, dtype=sigproc_sample_dtype(meta)).astype(np.float32)
    return data, meta, sh["tsamp"]


def write_sigproc(fname, data, header):
    """Write a SIGPROC time series file (used by tests and tools; the header
    keys must be in SIGPROC_KEYS)."""
    def wstr(f, s):
        b = s.encode()
        f.write(struct.pack("i", len(b)))
        f.write(b)

    with open(fname, "wb") as f:
        wstr(f, HEADER_START)
        for key, val in header.items():
            wstr(f, key)
            t = SIGPROC_KEYS[key]
            if t is str:
                wstr(f, val)
            elif t is int:
                f.write(struct.pack("i", int(val)))
            elif t is float:
                f.write(struct.pack("d", float(val)))
            elif t is bool:
                f.write(struct.pack("B", int(bool(val))))
        wstr(f, HEADER_END)
        np.ascontiguousarray(data).tofile(f)


# ---------------------------------------------------------------------------
# PRESTO (riptide/reading/presto.py)
# ---------------------------------------------------------------------------
SEP_COLUMN = 40
FAKE_TELESCOPE = "None (Artificial Data Set)"


def _inf_value(line, vtype):
    if not (len(line) > SEP_COLUMN and line[SEP_COLUMN] == "="):
        raise ValueError(f"Expected '=' character at column {SEP_COLUMN}")
    return vtype(line[SEP_COLUMN + 1:].strip())


def _bool01(s):
    return int(s) != 0


def _int_pair(s):
    a, b = s.split(",")
    return int(a), int(b)


def inf2dict(text):
    """Parse the text of a PRESTO .inf file (presto.py:55-125)."""
    lines = text.strip("\n").splitlines()

    def p(n, vtype):
        return _inf_value(lines[n], vtype)

    basename, telescope = p(0, str), p(1, str)
    if telescope == FAKE_TELESCOPE:
        raise ValueError("Reading data generated with PRESTO's makedata is not supported")
    items = {"basename": basename, "telescope": telescope, "instrument": p(2, str), "source_name": p(3, str),
             "raj": p(4, str), "decj": p(5, str), "observer": p(6, str), "mjd": p(7, float),
             "barycentered": p(8, _bool01), "nsamp": p(9, int), "tsamp": p(10, float), "breaks": p(11, _bool01),
             "onoff_pairs": []}
    lines = lines[12:]
    if items["breaks"]:
        for line in lines:
            try:
                items["onoff_pairs"].append(_inf_value(line, _int_pair))
            except Exception:
                break
    lines = lines[len(items["onoff_pairs"]):]
    em_band = p(0, str)
    items["em_band"] = em_band
    if em_band == "Radio":
        for k, (key, t) in enumerate([("fov_arcsec", float), ("dm", float), ("fbot", float), ("bandwidth", float),
                                      ("nchan", int), ("cbw", float), ("analyst", str)], start=1):
            items[key] = p(k, t)
    elif em_band in ("X-ray", "Gamma"):
        for k, (key, t) in enumerate([("fov_arcsec", float), ("central_energy_kev", float),
                                      ("energy_bandpass_kev", float), ("analyst", str)], start=1):
            items[key] = p(k, t)
    else:
        raise ValueError(f"EM Band {em_band!r} not supported")
    return items


def _sexagesimal(s):
    sign = -1.0 if s.strip().startswith("-") else 1.0
    parts = [abs(float(x)) for x in s.strip().lstrip("+-").split(":")]
    while len(parts) < 3:
        parts.append(0.0)
    return sign * (parts[0] + parts[1] / 60.0 + parts[2] / 3600.0)


class PrestoInf(dict):
    """PRESTO .inf metadata (presto.py:124-149)."""

    def __init__(self, fname):
        self._fname = os.path.realpath(fname)
        with open(fname, "r") as f:
            items = inf2dict(f.read())
        super().__init__(items)

    @property
    def fname(self):
        return self._fname

    @property
    def data_fname(self):
        return self.fname.rsplit(".", maxsplit=1)[0] + ".dat"

    @property
    def skycoord(self):
        return Coord(_sexagesimal(self["raj"]), _sexagesimal(self["decj"]))

    def load_data(self):
        return np.fromfile(self.data_fname, dtype=np.float32)


def presto_metadata(inf):
    """Metadata.from_presto_inf (metadata.py:54-71)."""
    attrs = dict(inf)
    attrs["skycoord"] = inf.skycoord
    attrs["fname"] = os.path.realpath(inf.fname)
    attrs["tobs"] = attrs["tsamp"] * attrs["nsamp"]
    return Metadata(attrs)


def read_presto(fname):
    """(float32 samples, Metadata, tsamp) as TimeSeries.from_presto_inf (time_series.py:283-318)."""
    inf = PrestoInf(fname)
    meta = presto_metadata(inf)
    if meta["em_band"] in ("X-ray", "Gamma"):
        import warnings
        warnings.warn(f" You have loaded file {fname!r}, which contains data observed at a high-energy band "
                      f"{meta['em_band']!r}. riptide is NOT designed to process low photon count time series, "
                      "i.e. where the background noise statistics are non-Gaussian. Be VERY careful when "
                      "interpreting any search outputs.", category=UserWarning)
    return inf.load_data(), meta, inf["tsamp"]


# ---------------------------------------------------------------------------
# Device batch loading
# ---------------------------------------------------------------------------
def _raw_samples(fname, fmt, extra_keys=None, staging=None):
    """(raw numpy samples as stored, Metadata, tsamp) without the float cast.
    `staging(nbytes)`, if given, returns a writable uint8 numpy array of at
    least nbytes (page-locked host memory) that SIGPROC samples are read into
    directly; the samples returned are then a view of it."""
    if fmt == "sigproc":
        sh = SigprocHeader(fname, extra_keys=extra_keys)
        meta = sigproc_metadata(sh)
        dt = np.dtype(sigproc_sample_dtype(meta))
        with open(sh.fname, "rb") as f:
            f.seek(sh.bytesize)
            if staging is None:
                raw = np.fromfile(f, dtype=dt)
            else:
                nbytes = (os.path.getsize(sh.fname) - sh.bytesize) // dt.itemsize * dt.itemsize
                buf = staging(nbytes)[:nbytes]
                got = f.readinto(memoryview(buf))
                if got != nbytes:
                    raise OSError(f"short read from {sh.fname}: {got} of {nbytes} bytes")
                raw = buf.view(dt)
        return raw, meta, sh["tsamp"]
    if fmt == "presto":
        data, meta, tsamp = read_presto(fname)
        return data, meta, tsamp
    raise ValueError(f"unknown time series format {fmt!r}")


def upload_samples(raws, device=None, stream=None):
    """Host sample arrays of equal length (float32, or uint8 / int8 8-bit data
    as stored) -> one float32 [B, N] device tensor.  8-bit samples are copied
    to the device as bytes (4x fewer bytes over PCIe than their float32
    expansion) and converted there by rt_convert_samples_device, bit-exact
    with numpy's astype(float32)."""
    import torch
    from . import _lib
    from .engine import _stream_handle
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    n = int(raws[0].size)
    if any(int(r.size) != n for r in raws):
        raise ValueError("upload_samples needs series of equal length")
    L = _lib.load()
    kinds = {np.dtype(np.uint8): 0, np.dtype(np.int8): 1}
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    with torch.cuda.stream(s):
        out = torch.empty((len(raws), n), dtype=torch.float32, device=dev)
        for b, raw in enumerate(raws):
            raw = np.asarray(raw)
            if raw.dtype != np.float32 and raw.dtype not in kinds:
                raw = raw.astype(np.float32)      # e.g. float64 series (EngineSearcher's old cast)
            raw = np.ascontiguousarray(raw)
            src = torch.from_numpy(raw if raw.dtype == np.float32 else raw.view(np.uint8))
            # asynchronous only from page-locked memory (_raw_samples' staging
            # slots, whose owner waits for the stream before refilling them);
            # pageable sources (and temporaries made here) are copied
            # synchronously, so nothing dropped below is still being read
            pinned = src.is_pinned()
            if raw.dtype == np.float32:
                out[b].copy_(src, non_blocking=pinned)
                continue
            staged = src.to(dev, non_blocking=pinned)
            _lib.check(L.rt_convert_samples_device(_lib.ptr(staged), n, kinds[raw.dtype], _lib.ptr(out[b]),
                                                   _stream_handle(s)))
    return out


def load_device_batch(fnames, fmt="sigproc", device=None, extra_keys=None, stream=None):
    """Load time series files of equal length into one float32 [B, N] device
    tensor (upload_samples).  Returns (tensor, [Metadata], tsamp)."""
    raws, metas, tsamps = [], [], []
    for fn in fnames:
        raw, meta, tsamp = _raw_samples(fn, fmt, extra_keys)
        raws.append(raw)
        metas.append(meta)
        tsamps.append(tsamp)
    if any(t != tsamps[0] for t in tsamps):
        raise ValueError("load_device_batch needs files of equal length and sampling time")
    return upload_samples(raws, device=device, stream=stream), metas, tsamps[0]


def write_presto(basename, data, tsamp, dm=0.0, mjd=60000.0, em_band="Radio"):
    """Write a PRESTO .inf/.dat pair (float32 samples; used by tests, tools and
    the cfg5 bench leg).  The .inf carries the keys inf2dict reads, one per
    line, value after '=' at column 40, as PRESTO's own writer lays them out."""
    data = np.ascontiguousarray(data, dtype=np.float32)
    name = os.path.basename(basename)

    def line(label, value):
        return f" {label:<39s}=  {value}"

    rows = [line("Data file name without suffix", name),
            line("Telescope used", "Parkes"),
            line("Instrument used", "Multibeam"),
            line("Object being observed", "Fake"),
            line("J2000 Right Ascension (hh:mm:ss.ssss)", "00:00:01.0000"),
            line("J2000 Declination     (dd:mm:ss.ssss)", "-00:00:01.0000"),
            line("Data observed by", "riptide_amd"),
            line("Epoch of observation (MJD)", f"{mjd:.6f}"),
            line("Barycentered?           (1=yes, 0=no)", "1"),
            line("Number of bins in the time series", f"{data.size:d}"),
            line("Width of each time series bin (sec)", f"{tsamp:.12e}"),
            line("Any breaks in the data? (1=yes, 0=no)", "0"),
            line("Type of observation (EM band)", em_band)]
    if em_band == "Radio":
        rows += [line("Beam diameter (arcsec)", "981"),
                 line("Dispersion measure (cm-3 pc)", f"{dm:.12f}"),
                 line("Central freq of low channel (Mhz)", "1182.1953125"),
                 line("Total bandwidth (Mhz)", "400"),
                 line("Number of channels", "1024"),
                 line("Channel bandwidth (Mhz)", "0.390625"),
                 line("Data analyzed by", "riptide_amd")]
    else:
        rows += [line("Field-of-view diameter (arcsec)", "100"),
                 line("Central energy (kev)", "1.0"),
                 line("Energy bandpass (kev)", "1.0"),
                 line("Data analyzed by", "riptide_amd")]
    with open(basename + ".inf", "w") as f:
        f.write("\n".join(rows) + "\n")
    data.tofile(basename + ".dat")
    return basename + ".inf"
