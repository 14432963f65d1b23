"""Checkpoint spill files are bound to the run that wrote them (CPU).

The reference has no checkpointing; these pin the resume
contract both drivers share: a spill is reused only under the same run
identity (input, header, result-affecting options, killfile/zapfile
contents), truncated or corrupt spills are detected, and writes are atomic.
"""
import os
import shutil

import pytest

from conftest import DATA, TUTORIAL


def _args(C, *extra):
    ok, _, args = C.parse_cmdline(["peasoup", "-i", TUTORIAL, "--dm_end", "250", "-n", "4", *extra])
    assert ok
    return args


def _header(C):
    return dict(C.Filterbank.from_file(TUTORIAL).header)


def _cands(C):
    a = C.Candidate(19.76, 7, 0.0, 4, 86.9, 4.0)
    a.assoc = [C.Candidate(23.0, 8, 5.0, 3, 70.0, 4.0001)]
    return [a, C.Candidate(30.0, 9, -5.0, 1, 12.5, 8.0)]


def test_identity_depends_on_result_affecting_options(C):
    hdr = _header(C)
    k0, text = C.checkpoint_identity(_args(C), hdr)
    assert "tutorial.fil" in text and "nharmonics=4" in text
    assert C.checkpoint_identity(_args(C), hdr)[0] == k0  # deterministic
    for extra in (["-m", "8"], ["--dm_end", "200"], ["--acc_start", "-5", "--acc_end", "5"], ["--fft_size", "65536"],
                  ["--accel_convention", "reference"], ["--max_freq", "500"], ["--freq_tol", "0.001"],
                  ["-z", os.path.join(DATA, "default_zaplist.txt")]):
        assert C.checkpoint_identity(_args(C, *extra), hdr)[0] != k0, extra
    # options that do not change the per-DM candidates keep the key
    for extra in (["--npdmp", "10"], ["--limit", "5"], ["--dedisp_kernel", "direct"], ["--accel_batch", "16"],
                  ["-t", "2"], ["-o", "/tmp/elsewhere"]):
        assert C.checkpoint_identity(_args(C, *extra), hdr)[0] == k0, extra
    hdr2 = dict(hdr, tsamp=hdr["tsamp"] * 2)
    assert C.checkpoint_identity(_args(C), hdr2)[0] != k0


def test_identity_tracks_input_and_zapfile_content(C, tmp_path):
    fil = tmp_path / "t.fil"
    shutil.copy(TUTORIAL, fil)
    zap = tmp_path / "zap.txt"
    zap.write_text("50.0 0.1\n")
    ok, _, args = C.parse_cmdline(["peasoup", "-i", str(fil), "-z", str(zap)])
    hdr = _header(C)
    k0 = C.checkpoint_identity(args, hdr)[0]
    zap.write_text("50.0 0.2\n")  # edited in place
    k1 = C.checkpoint_identity(args, hdr)[0]
    assert k1 != k0
    b = bytearray(fil.read_bytes())
    b[-1] ^= 0xFF  # the last sampled block of the data changes
    fil.write_bytes(bytes(b))
    assert C.checkpoint_identity(args, hdr)[0] != k1


def test_spill_roundtrip_mismatch_and_corruption(C, tmp_path):
    p = str(tmp_path / "dm_0_8.psoc")
    assert C.load_spill(p, 1)[0] == "missing"
    cands = _cands(C)
    C.save_spill(p, 1234, cands)
    st, got = C.load_spill(p, 1234)
    assert st == "loaded"
    assert [(c.dm_idx, c.snr, len(c.assoc)) for c in got] == [(7, pytest.approx(86.9), 1), (9, pytest.approx(12.5), 0)]
    st, got = C.load_spill(p, 999)
    assert st == "mismatch" and got == []
    raw = open(p, "rb").read()
    open(p, "wb").write(raw[: len(raw) - 7])  # truncated
    assert C.load_spill(p, 1234)[0] == "corrupt"
    flipped = bytearray(raw)
    flipped[-3] ^= 0x40  # payload bit flip
    open(p, "wb").write(bytes(flipped))
    assert C.load_spill(p, 1234)[0] == "corrupt"
    open(p, "wb").write(b"PSOC")  # round-1 format / garbage
    assert C.load_spill(p, 1234)[0] == "corrupt"
    # no temporary files are left behind
    assert sorted(os.listdir(tmp_path)) == ["dm_0_8.psoc"]


def test_failed_spill_write_raises(C, tmp_path):
    with pytest.raises(Exception):
        C.save_spill(str(tmp_path / "no_such_dir" / "dm_0_8.psoc"), 1, _cands(C))


def test_manifest_records_identity(C, tmp_path):
    d = tmp_path / "ck"
    hdr = _header(C)
    key = C.prepare_checkpoint_dir(str(d), _args(C), hdr)
    text = (d / "manifest.txt").read_text()
    assert text.splitlines()[0] == f"key {key:016x}"
    key2 = C.prepare_checkpoint_dir(str(d), _args(C, "-m", "7"), hdr)
    assert key2 != key
    assert (d / "manifest.txt").read_text().splitlines()[0] == f"key {key2:016x}"
    assert C.spill_path(str(d), 3, 9) == f"{d}/dm_3_9.psoc"
