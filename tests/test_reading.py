"""SIGPROC / PRESTO readers (riptide/reading/*.py, time_series.py:283-362) on
files written here; device conversion of 8-bit samples in test_gpu_parity."""
import os

import numpy as np
import pytest

from riptide_amd.reading import (PrestoInf, SigprocHeader, inf2dict, parse_float_coord, read_presto,
                                 read_sigproc, write_sigproc)

HDR = {"source_name": "J0000+0000", "telescope_id": 4, "machine_id": 10, "data_type": 2, "src_raj": 123456.7,
       "src_dej": -301234.5, "tstart": 58000.25, "tsamp": 6.4e-5, "nbits": 32, "nchans": 1, "refdm": 123.4,
       "nifs": 1, "fch1": 1500.0, "foff": -0.5}


@pytest.mark.parametrize("nbits,signed,dtype", [(32, None, np.float32), (8, True, np.int8), (8, False, np.uint8)])
def test_sigproc_round_trip(tmp_path, nbits, signed, dtype):
    rng = np.random.RandomState(nbits)
    if dtype == np.float32:
        data = rng.normal(size=1000).astype(np.float32)
    else:
        info = np.iinfo(dtype)
        data = rng.randint(info.min, info.max + 1, size=1001).astype(dtype)
    hdr = dict(HDR, nbits=nbits)
    if signed is not None:
        hdr["signed"] = signed
    fn = str(tmp_path / "x.tim")
    write_sigproc(fn, data, hdr)
    x, meta, tsamp = read_sigproc(fn)
    assert x.dtype == np.float32 and np.array_equal(x, data.astype(np.float32))
    assert tsamp == HDR["tsamp"]
    assert meta["dm"] == HDR["refdm"] and meta["mjd"] == HDR["tstart"] and meta["source_name"] == "J0000+0000"
    assert meta["tobs"] == data.size * HDR["tsamp"]
    assert meta["fname"] == os.path.realpath(fn)
    sh = SigprocHeader(fn)
    assert sh.nsamp == data.size and sh.bytes_per_sample == nbits // 8
    assert np.isclose(sh.skycoord.ra_hours, 12 + 34 / 60 + 56.7 / 3600)
    assert np.isclose(sh.skycoord.dec_deg, -(30 + 12 / 60 + 34.5 / 3600))


@pytest.mark.parametrize("nbits,signed,dtype", [(32, None, np.float32), (8, True, np.int8), (8, False, np.uint8)])
def test_raw_samples_into_staging(tmp_path, nbits, signed, dtype):
    """_raw_samples reading straight into a caller's staging buffer (the
    worker pool's page-locked slots): the same samples as np.fromfile, a view
    of that buffer, and a slot larger than the file is fine."""
    from riptide_amd.reading import _raw_samples
    rng = np.random.RandomState(7 + nbits)
    if dtype == np.float32:
        data = rng.normal(size=777).astype(np.float32)
    else:
        info = np.iinfo(dtype)
        data = rng.randint(info.min, info.max + 1, size=779).astype(dtype)
    hdr = dict(HDR, nbits=nbits)
    if signed is not None:
        hdr["signed"] = signed
    fn = str(tmp_path / "s.tim")
    write_sigproc(fn, data, hdr)
    slot = np.zeros(4 * 1024, dtype=np.uint8)
    asked = []

    def staging(nbytes):
        asked.append(nbytes)
        return slot

    raw, meta, tsamp = _raw_samples(fn, "sigproc", staging=staging)
    ref, _, _ = _raw_samples(fn, "sigproc")
    assert asked == [data.nbytes]
    assert raw.dtype == ref.dtype == dtype and np.array_equal(raw, ref) and np.array_equal(raw, data)
    assert np.shares_memory(raw, slot)
    assert tsamp == HDR["tsamp"] and meta["dm"] == HDR["refdm"]


def test_sigproc_errors(tmp_path):
    fn = str(tmp_path / "bad.tim")
    write_sigproc(fn, np.zeros(10, np.float32), dict(HDR, nchans=4))
    with pytest.raises(ValueError):
        read_sigproc(fn)
    write_sigproc(fn, np.zeros(10, np.int16), dict(HDR, nbits=16))
    with pytest.raises(ValueError):
        read_sigproc(fn)
    write_sigproc(fn, np.zeros(10, np.uint8), dict(HDR, nbits=8))      # no 'signed' key
    with pytest.raises(ValueError):
        read_sigproc(fn)
    with open(fn, "wb") as f:
        f.write(b"\x04\x00\x00\x00JUNK")
    with pytest.raises(AssertionError):
        read_sigproc(fn)


def test_parse_float_coord():
    assert np.isclose(parse_float_coord(123456.7), 12 + 34 / 60.0 + 56.7 / 3600.0, rtol=0, atol=1e-12)
    assert parse_float_coord(-10000.0) == -1.0


INF = """ Data file name without suffix          =  fake_DM10.00
 Telescope used                         =  Parkes
 Instrument used                        =  Multibeam
 Object being observed                  =  J1234+5678
 J2000 Right Ascension (hh:mm:ss.ssss)  =  12:34:56.7000
 J2000 Declination     (dd:mm:ss.ssss)  =  -56:07:08.9000
 Data observed by                       =  Someone
 Epoch of observation (MJD)             =  55000.123456789
 Barycentered?           (1 yes, 0 no)  =  1
 Number of bins in the time series      =  2000
 Width of each time series bin (sec)    =  0.000256
 Any breaks in the data? (1 yes, 0 no)  =  0
 Type of observation (EM band)          =  Radio
 Beam diameter (arcsec)                 =  840
 Dispersion measure (cm-3 pc)           =  10
 Central freq of low channel (Mhz)      =  1182.1953125
 Total bandwidth (Mhz)                  =  400
 Number of channels                     =  1024
 Channel bandwidth (Mhz)                =  0.390625
 Data analyzed by                       =  Someone else
 Any additional notes:
    none
"""


def test_presto_round_trip(tmp_path):
    inf = tmp_path / "fake_DM10.00.inf"
    inf.write_text(INF)
    data = np.random.RandomState(2).normal(size=2000).astype(np.float32)
    data.tofile(str(tmp_path / "fake_DM10.00.dat"))
    x, meta, tsamp = read_presto(str(inf))
    assert np.array_equal(x, data) and tsamp == 0.000256
    assert meta["dm"] == 10.0 and meta["nsamp"] == 2000 and meta["em_band"] == "Radio"
    assert meta["tobs"] == 0.000256 * 2000 and meta["nchan"] == 1024
    assert np.isclose(PrestoInf(str(inf)).skycoord.dec_deg, -(56 + 7 / 60 + 8.9 / 3600))
    d = inf2dict(INF)
    assert d["barycentered"] is True and d["onoff_pairs"] == []
    with pytest.raises(ValueError):
        inf2dict(INF.replace("Parkes", "None (Artificial Data Set)"))


# ---------------------------------------------------------------- the reference's own fixtures
# riptide/tests/test_time_series.py:15-62 on riptide/tests/data/* (copied as
# data under tests/golden/ref_data/): 16 samples 0..15 at 64 us in every file.
REF_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_data")


def _check_fixture(ts):
    assert ts.nsamp == 16
    assert ts.tsamp == 64e-6
    assert ts.data.dtype == np.float32
    assert np.allclose(ts.data, np.arange(16))


def test_reference_presto_fixtures():
    from riptide_amd import TimeSeries
    for name in ("fake_presto_radio.inf", "fake_presto_radio_breaks.inf"):
        _check_fixture(TimeSeries.from_presto_inf(os.path.join(REF_DATA, name)))
    with pytest.warns(UserWarning):
        _check_fixture(TimeSeries.from_presto_inf(os.path.join(REF_DATA, "fake_presto_xray.inf")))
    inf = PrestoInf(os.path.join(REF_DATA, "fake_presto_radio_breaks.inf"))
    assert inf["breaks"] and len(inf["onoff_pairs"]) > 0


def test_reference_sigproc_fixtures():
    from riptide_amd import TimeSeries
    for name in ("fake_sigproc_float32.tim", "fake_sigproc_uint8.tim", "fake_sigproc_int8.tim"):
        _check_fixture(TimeSeries.from_sigproc(os.path.join(REF_DATA, name)))
    with pytest.raises(ValueError):
        TimeSeries.from_sigproc(os.path.join(REF_DATA, "fake_sigproc_uint8_nosignedkey.tim"))


def test_presto_writer_round_trip(tmp_path):
    from riptide_amd.reading import write_presto
    x = np.random.RandomState(3).normal(size=777).astype(np.float32)
    fn = write_presto(str(tmp_path / "p"), x, 2.56e-4, dm=12.5)
    data, meta, tsamp = read_presto(fn)
    assert np.array_equal(data, x) and tsamp == 2.56e-4 and meta["dm"] == 12.5
    assert meta["tobs"] == 777 * 2.56e-4
