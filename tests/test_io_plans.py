"""SIGPROC I/O, DM list, delay table and acceleration plan parity (CPU)."""
import os

import numpy as np
import pytest

from conftest import TUTORIAL, DATA
from peasoup_amd.utils import sigproc


def test_tutorial_header_native_and_python(C):
    h = C.read_header(TUTORIAL)
    p = sigproc.read_header(TUTORIAL)
    assert h["nchans"] == 64 and h["nbits"] == 2 and h["nsamples"] == 187520
    assert h["tsamp"] == pytest.approx(0.00032) and h["fch1"] == 1510.0 and h["foff"] == pytest.approx(-1.09)
    assert h["size"] == 244 == p["size"]
    for k in ("nchans", "nbits", "nsamples", "tsamp", "fch1", "foff", "tstart", "source_name", "signed"):
        assert h[k] == p[k], k
    fb = C.Filterbank.from_file(TUTORIAL)
    assert fb.nsamps == 187520 and fb.data_bytes == 187520 * 16
    assert fb.cfreq() == pytest.approx(1475.12, abs=1e-3)


def test_filterbank_threaded_pread_equals_mapping(C):
    """The device upload's staging reads (pread on threads) return the mapped
    data block byte for byte, at any offset and thread count."""
    fb = C.Filterbank.from_file(TUTORIAL)
    ref_ = np.array(fb.data())
    for off, n, nt in ((0, fb.data_bytes, 4), (0, fb.data_bytes, 1), (12345, 2_100_001, 3), (fb.data_bytes - 7, 7, 4)):
        out = np.zeros(n, dtype=np.uint8)
        fb.read_into(off, n, out.ctypes.data, nt)
        assert np.array_equal(out, ref_[off:off + n]), (off, n, nt)
    with pytest.raises(Exception):
        fb.read_into(fb.data_bytes - 2, 4, np.zeros(4, np.uint8).ctypes.data)


def test_filterbank_roundtrip(C, tmp_path):
    rng = np.random.default_rng(0)
    for nbits in (1, 2, 4, 8):
        vals = rng.integers(0, 1 << nbits, size=(300, 16), dtype=np.uint8)
        hdr = {"nchans": 16, "nbits": nbits, "tsamp": 1e-4, "fch1": 1400.0, "foff": -0.5, "nifs": 1,
               "source_name": "rt", "tstart": 55000.5}
        p = str(tmp_path / f"x{nbits}.fil")
        sigproc.write_filterbank(p, hdr, vals)
        back = sigproc.read_filterbank(p)
        assert np.array_equal(back.data, vals)
        nh = C.read_header(p)
        assert nh["nsamples"] == 300 and nh["nbits"] == nbits and nh["source_name"] == "rt"
        # native writer -> python reader
        p2 = str(tmp_path / f"y{nbits}.fil")
        C.write_filterbank(p2, hdr, sigproc.pack_samples(vals, nbits))
        assert np.array_equal(sigproc.read_filterbank(p2).data, vals)


def test_tim_roundtrip(C, tmp_path):
    x = np.linspace(-3, 3, 1000).astype(np.float32)
    p = str(tmp_path / "a.tim")
    C.write_tim(p, {"tsamp": 6.4e-5, "fch1": 1400.0, "source_name": "t"}, list(x))
    h, d = C.read_tim(p)
    assert h["nsamples"] == 1000 and np.allclose(d, x)
    h2, d2 = sigproc.read_tim(p)
    assert np.array_equal(d2, x)


def test_killfile_zapfile(C, tmp_path):
    k = tmp_path / "kill.txt"
    k.write_text("\n".join(["1"] * 60 + ["0"] * 4) + "\n")
    mask, ok = C.read_killfile(str(k), 64)
    assert ok and mask[:60] == [1] * 60 and mask[60:] == [0] * 4
    mask, ok = C.read_killfile(str(k), 128)  # wrong size: warning + all ones
    assert not ok and mask == [1] * 128
    f, w = C.read_zapfile(os.path.join(DATA, "default_zaplist.txt"))
    assert f == pytest.approx([50, 100, 150, 200, 250]) and w == pytest.approx([0.1, 0.15, 0.15, 0.15, 0.15])


def test_dm_list_matches_golden_bit_for_bit(C, golden):
    dms = C.generate_dm_list(0.0, 250.0, 0.00032, 64.0, 1510.0, -1.09, 64, 1.1)
    ref = golden.dm_list
    assert len(dms) == len(ref) == 59
    # golden values are float32 printed with 15 significant digits
    assert [C.xml_fmt_float(d) for d in dms] == [
        t.text for t in golden.root.find("dedispersion_trials").findall("trial")]


def test_delay_table_and_max_delay(C):
    from peasoup_amd.utils import reference as ref

    d = C.generate_delay_table(64, 0.00032, 1510.0, -1.09)
    assert np.allclose(d, ref.delay_table(64, 0.00032, 1510.0, -1.09))
    dms = C.generate_dm_list(0.0, 250.0, 0.00032, 64.0, 1510.0, -1.09, 64, 1.1)
    assert C.compute_max_delay(dms, d) == 140
    g = C.DedispGeometry.make(C.read_header(TUTORIAL), 187520, dms, [])
    assert g.out_nsamps == 187380 and g.out_scale == 1.0 and g.nactive == 64


def test_accel_plan_conventions(C):
    cf = C.Filterbank.from_file(TUTORIAL).cfreq()
    legacy = C.AccelPlan(-5, 5, 1.1, 64.0, 131072, 0.00032, cf, -1.09)
    assert legacy.generate(0.0) == [0.0, -5.0, 5.0]  # golden overview.xml:124-128
    assert legacy.step(0.0) == pytest.approx(239.9, rel=1e-3)
    cur = C.AccelPlan(-5, 5, 1.1, 64.0, 131072, 0.00032, cf, -1.09, C.AccelConvention.Reference)
    lst = cur.generate(0.0)
    assert len(lst) == 44 and lst[0] == 0.0 and lst[1] == -5.0 and lst[-1] == 5.0
    assert cur.step(0.0) == pytest.approx(0.2399, rel=1e-3)
    # 2^23 x 64 us, +-500
    big = C.AccelPlan(-500, 500, 1.1, 64.0, 1 << 23, 64e-6, 1400.0, -0.39)
    assert big.step(0.0) == pytest.approx(1.464, rel=2e-3)
    assert 680 <= len(big.generate(0.0)) <= 690
    assert C.AccelPlan(0, 0, 1.1, 64.0, 1024, 1e-4, 1400.0, -1).generate(3.0) == [0.0]


def test_prev_power_of_two_strictly_less(C):
    assert C.prev_power_of_two(187520) == 131072
    assert C.prev_power_of_two(1 << 23) == 1 << 22  # exact power -> half (utils.hpp:12-18)
    assert C.prev_power_of_two((1 << 23) + 1) == 1 << 23


def test_dada_header_and_channel_extraction(C, tmp_path):
    """PSRDADA header parse (DadaHeader semantics: BW as integer, nsamples
    from the payload size) and channel extraction for the correlator."""
    import numpy as np

    from peasoup_amd.utils import dada

    nant, nchan, npol, n = 3, 4, 2, 500
    rng = np.random.default_rng(1)
    payload = rng.integers(-20, 20, size=(n, nant, nchan, npol, 2), dtype=np.int8)
    hdr = {"HDR_VERSION": 1.0, "HDR_SIZE": 4096, "BW": 16.75, "FREQ": 1400.5, "NANT": nant, "NCHAN": nchan,
           "NDIM": 2, "NPOL": npol, "NBIT": 8, "TSAMP": 0.064, "SOURCE": "J0000+0000", "UTC_START": "2026-10-16-00:00:00",
           "ANT_ID": 7, "FILE_NUMBER": 2}
    path = str(tmp_path / "x.dada")
    dada.write(path, hdr, payload)
    h = C.read_dada_header(path)
    assert h["nant"] == nant and h["nchan"] == nchan and h["npol"] == npol and h["nbit"] == 8
    assert h["bw"] == 16.0 and h["freq"] == 1400.5 and h["tsamp"] == 0.064
    assert h["source_name"] == "J0000+0000" and h["ant_id"] == 7 and h["file_no"] == 2
    assert h["filesize"] == payload.nbytes and h["nsamples"] == n
    arr = dada.extract_channel(path, channel=2, size=100, offset=10, pol=1)
    assert arr.shape == (nant, 200)
    assert np.array_equal(arr[1].reshape(100, 2), payload[10:110, 1, 2, 1, :])


def test_fft4_geometries_for_every_series_length(C):
    """Host-side FFT plan choice (no device needed): the fused four-step
    geometry up to 2^25 points (rows and columns of at most 4096), the
    external-row geometry from 2^26 (columns of 4096 through the fused pass
    A, rows of 8192 / 16384 for rocFFT, natural Y rows with an off-power-of-two
    pitch), neither for lengths that are not powers of two."""
    K = C.kernels
    for log2n in range(15, 26):
        g = K.fft4_geometry(1 << (log2n - 1))
        assert g.ok and not g.rows_ext and g.n1 * g.n2 == 1 << (log2n - 1) and max(g.n1, g.n2) <= 4096
        assert not K.fft4_geometry_rows(1 << (log2n - 1)).ok
    for log2n, n1 in ((26, 8192), (27, 16384)):
        M = 1 << (log2n - 1)
        assert not K.fft4_geometry(M).ok
        g = K.fft4_geometry_rows(M)
        assert g.ok and g.rows_ext and (g.n1, g.n2) == (n1, 4096)
        assert g.ypitch == n1 + 8 and g.ystride == g.ypitch * 4096 and g.insize >= 2 * M
    assert not K.fft4_geometry(3 << 20).ok and not K.fft4_geometry_rows(3 << 24).ok


def test_static_chunk_sizes():
    """Long static shards take 64-DM blocks (fewer engine calls, each of which
    waits for its last batch), short ones and the override keep the 32-DM tile."""
    import os

    from peasoup_amd.models.search import DYNAMIC_CHUNK, static_chunk

    old = os.environ.pop("PSOUP_STATIC_CHUNK", None)
    try:
        assert static_chunk(2026) == 2 * DYNAMIC_CHUNK
        assert static_chunk(8 * DYNAMIC_CHUNK - 1) == DYNAMIC_CHUNK
        os.environ["PSOUP_STATIC_CHUNK"] = "100"
        assert static_chunk(2026) == 96
        os.environ["PSOUP_STATIC_CHUNK"] = "8"
        assert static_chunk(2026) == DYNAMIC_CHUNK
    finally:
        os.environ.pop("PSOUP_STATIC_CHUNK", None)
        if old is not None:
            os.environ["PSOUP_STATIC_CHUNK"] = old
