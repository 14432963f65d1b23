"""overview.xml / candidates.peasoup writers + readers and CLI parity (CPU)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN_CANDS, GOLDEN_XML, TUTORIAL
from peasoup_amd.utils.outputs import CandidateFileParser, OverviewFile, PeasoupOutput, radec_to_str


def test_golden_binary_layout_matches_overview(golden):
    """Record size = 4+8+64*16*4 + 4 + 24*ndets; offsets chain; ndets = nassoc+1."""
    out = PeasoupOutput(GOLDEN_XML, GOLDEN_CANDS)
    recs = CandidateFileParser(GOLDEN_CANDS).records()
    assert len(recs) == len(out) == 10
    for i, (off, fold, hits) in enumerate(recs):
        d = out.overview.get_candidate(i)
        assert d["byte_offset"] == off
        assert fold.shape == (16, 64)
        assert len(hits) == d["nassoc"] + 1
        assert hits[0]["dm"] == pytest.approx(d["dm"], rel=1e-6)
        assert 1.0 / hits[0]["freq"] == pytest.approx(d["period"], rel=1e-6)
    assert os.path.getsize(GOLDEN_CANDS) == 65888


def _cand(C, i):
    c = C.Candidate(10.0 + i, i, -1.5 * i, i % 5, 50.0 - i, 4.0 + i)
    c.folded_snr = 20.0 + i
    c.opt_period = 0.25
    if i % 2 == 0:
        c.fold = list(np.arange(1024, dtype=np.float32) * (i + 1))
        c.nbins, c.nints = 64, 16
    c.assoc = [C.Candidate(11.0, i + 1, 0.0, 1, 30.0, 8.0 + i)]
    return c


def test_binary_and_xml_writer_roundtrip(C, tmp_path):
    cands = [_cand(C, i) for i in range(5)]
    args = C.parse_cmdline(["peasoup", "-i", TUTORIAL, "-o", str(tmp_path), "--dm_end", "250",
                            "--acc_start", "-5", "--acc_end", "5", "--npdmp", "10", "-p"])[2]
    bm = C.write_candidates_binary(str(tmp_path), cands, "candidates.peasoup")
    C.write_overview(str(tmp_path / "overview.xml"), args, TUTORIAL, [0.0, 1.5], [0.0, -5.0, 5.0], [], cands, bm,
                     {"reading": 0.1, "total": 1.0, "searching": 0.5, "dedispersion": 0.2, "folding": 0.2},
                     {"dm_accel_trials_per_sec": 123.0})
    out = PeasoupOutput(str(tmp_path / "overview.xml"), str(tmp_path / "candidates.peasoup"))
    assert len(out) == 5
    for i in range(5):
        c = out.get_candidate(i)
        assert c.info["nassoc"] == 1 and len(c.hits) == 2
        assert c.info["period"] == pytest.approx(1 / (4.0 + i))
        if i % 2 == 0:
            assert np.array_equal(c.fold.reshape(-1), np.arange(1024, dtype=np.float32) * (i + 1))
        else:
            assert c.fold is None
    ov = OverviewFile(str(tmp_path / "overview.xml"))
    assert list(ov.execution_times) == ["dedispersion", "folding", "reading", "searching", "total"]
    assert ov.acc_list == [0.0, -5.0, 5.0]
    sp = ov.section("search_parameters")
    assert sp["dm_tol"] == "1.10000002384186" and sp["freq_tol"] == "9.99999974737875e-05"
    assert sp["max_harm"] == "16" and sp["progress_bar"] == "1" and sp["min_freq"] == "0.100000001490116"
    hp = ov.section("header_parameters")
    assert hp["source_name"] == "P: 250.000000000000 ms, DM: 30.000" and hp["nsamples"] == "187520"
    text = open(tmp_path / "overview.xml").read()
    assert text.startswith("<?xml version='1.0' encoding='ISO-8859-1'?>\n<peasoup_search>\n  <misc_info>\n")
    assert "<acceleration_trials DM='0' count='3'>" in text
    assert "    <trial id='1'>-5</trial>\n" in text


def test_xml_float_format_matches_reference(C, golden):
    # float32 values printed with %.15g, as std::setprecision(15) does
    assert C.xml_fmt_float(np.float32(86.9626083374023)) == "86.9626083374023"
    f = np.float32(1.0 / 0.249939903165736)  # golden candidate 0 frequency (float32)
    assert C.xml_fmt_double(1.0 / float(f)) == "0.249939903165736"


def test_cli_defaults_and_flags(C):
    ok, ex, a = C.parse_cmdline(["peasoup", "-i", "x.fil"])
    assert ok and not ex
    assert (a.max_num_threads, a.limit, a.size, a.dm_start, a.dm_end) == (14, 1000, 0, 0.0, 100.0)
    assert a.dm_tol == pytest.approx(1.1) and a.dm_pulse_width == 64.0 and a.acc_tol == pytest.approx(1.1)
    assert (a.nharmonics, a.npdmp, a.min_snr, a.max_harm) == (4, 0, 9.0, 16)
    assert a.min_freq == pytest.approx(0.1) and a.max_freq == 1100.0 and a.freq_tol == pytest.approx(1e-4)
    assert a.boundary_5_freq == pytest.approx(0.05) and a.boundary_25_freq == 0.5
    assert a.outdir.endswith("_peasoup/") and a.accel_convention == "legacy"
    ok, _, a = C.parse_cmdline(["peasoup", "--inputfile=y.fil", "-t", "2", "--fft_size", "1024", "-vp",
                                "--acc_start", "-5", "--max_harm_match", "8", "-k", "kill", "-z", "zap",
                                "--dm_end", "250", "-n", "3", "-m", "7.5", "--npdmp", "10", "--limit", "20"])
    assert ok and a.infilename == "y.fil" and a.max_num_threads == 2 and a.size == 1024
    assert a.verbose and a.progress_bar and a.acc_start == -5.0 and a.max_harm == 8
    assert (a.killfilename, a.zapfilename, a.nharmonics, a.min_snr, a.npdmp, a.limit) == ("kill", "zap", 3, 7.5, 10, 20)
    assert not C.parse_cmdline(["peasoup"])[0]  # -i is required
    assert not C.parse_cmdline(["peasoup", "-i", "a", "--bogus", "1"])[0]
    ok, ex, _ = C.parse_cmdline(["peasoup", "--help"])
    assert ok and ex
    ok, ex, _ = C.parse_cmdline(["peasoup", "--version"])
    assert ok and ex


def test_coincidencer_cli(C):
    ok, ex, a = C.parse_coincidencer_cmdline(["coinc", "a.fil", "b.fil", "--thresh", "5", "--beam_thresh", "2",
                                              "--o", "m.txt", "--o2", "b.txt"])
    assert ok and a.filterbanks == ["a.fil", "b.fil"] and a.threshold == 5.0 and a.beam_threshold == 2
    assert a.samp_outfilename == "m.txt" and a.spec_outfilename == "b.txt"
    assert not C.parse_coincidencer_cmdline(["coinc"])[0]


def test_radec_to_str():
    assert radec_to_str(123456.78) == "12:34:56.7800"
    assert radec_to_str(-12345.5) == "-1:23:45.5000"  # "%02d" of -1, as peasoup_tools.py


def test_per_candidate_binaries_and_text_files(C, tmp_path):
    """write_binaries (output_stats.hpp:272-307): one cand_%04d_P_DM_acc.peasoup
    per candidate with the same record format; text dumps (candidates.hpp:120-150)."""
    cands = [_cand(C, i) for i in range(3)]
    names = C.write_candidates_binaries(str(tmp_path / "bins"), cands)
    assert sorted(names) == [0, 1, 2]
    for i, c in enumerate(cands):
        base = "cand_%04d_%.5f_%.1f_%.1f.peasoup" % (i, 1.0 / np.float32(4.0 + i), np.float32(10.0 + i),
                                                   np.float32(-1.5 * i))
        assert os.path.basename(names[i]) == base and os.path.isabs(names[i])
        recs = CandidateFileParser(names[i]).records()
        assert len(recs) == 1
        off, fold, hits = recs[0]
        assert off == 0 and len(hits) == 2
        assert (fold is not None) == (i % 2 == 0)
        assert hits[0]["snr"] == pytest.approx(50.0 - i) and hits[1]["dm_idx"] == i + 1
    assert C.write_candidate_text_files(cands, str(tmp_path / "txt"))
    txt = sorted(os.listdir(tmp_path / "txt"))
    assert len(txt) == 3
    first = open(tmp_path / "txt" / txt[0]).read().splitlines()
    assert len(first) == 2 and len(first[0].split("\t")) == 13
    assert C.write_candidate_file(cands, str(tmp_path / "candidates.txt"))
    lines = open(tmp_path / "candidates.txt").read().splitlines()
    assert lines[0].startswith("#Period...Optimal period") and lines[1] == "#Candidate 0"
    assert sum(1 for ln in lines if ln.startswith("#Candidate")) == 3
