"""`peasoup_tools` subcommands (the reference's stand-alone drivers:
harmonic_sum_test, resampling_test, hcfft, dedisp_test, folder_test,
rednoise_test, filterbank_test)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, TUTORIAL

EXE = os.path.join(REPO, "bin", "peasoup_tools")


def run(*args, timeout=300):
    return subprocess.run([EXE, *map(str, args)], capture_output=True, text=True, timeout=timeout)


def test_filterbank_roundtrip_cpu(tmp_path):
    r = run("filterbank", "--o", tmp_path / "x.fil", "--i", TUTORIAL)
    assert r.returncode == 0, r.stderr
    assert "round trip: OK" in r.stdout and "nchans 64" in r.stdout


def test_usage_error():
    r = run("nonsense")
    assert r.returncode == 2 and "usage" in r.stderr


def _write_tim(C, path, n=1 << 16, period=0.0123, tsamp=256e-6):
    t = np.arange(n) * tsamp
    rng = np.random.default_rng(0)
    x = rng.standard_normal(n).astype(np.float32) + 3.0 * (np.modf(t / period)[0] < 0.05)
    hdr = {"source_name": "tools", "tsamp": tsamp, "fch1": 1400.0, "foff": -1.0, "nchans": 1, "nbits": 32,
           "nifs": 1, "data_type": 2, "tstart": 60000.0, "refdm": 10.0}
    C.write_tim(str(path), hdr, x.tolist())
    return period


@pytest.mark.gpu
def test_tools_on_gpu(C, tmp_path):
    r = run("harmsum", "--nbins", 1000003, "--nlevels", 4, "--reps", 3)
    assert r.returncode == 0 and "mismatches 0/" in r.stdout, r.stdout + r.stderr
    r = run("resample", "--n", 1 << 18)
    assert r.returncode == 0 and "samples differ" in r.stdout, r.stderr
    r = run("fft", "--n", 1 << 20, "--loops", 3, "--batch", 4)
    assert r.returncode == 0 and "fused resample + four-step FFT" in r.stdout, r.stderr
    dump = tmp_path / "dd.bin"
    r = run("dedisp", "--i", TUTORIAL, "--dm_end", 50, "--dump", dump)
    assert r.returncode == 0, r.stderr
    ndm = int(r.stdout.split(" DM trials")[0].split()[-1])
    assert ndm > 5 and dump.stat().st_size % ndm == 0
    tim = tmp_path / "p.tim"
    period = _write_tim(C, tim)
    r = run("fold", tim, "--period", period, "--dump", tmp_path / "fold.bin")
    assert r.returncode == 0, r.stderr
    snr = float(r.stdout.split("folded S/N ")[1].split(",")[0])
    assert snr > 10 and (tmp_path / "fold.bin").stat().st_size == 64 * 16 * 4
    r = run("rednoise", tim, "--acc", 0, "--nharmonics", 2, "--outdir", tmp_path)
    assert r.returncode == 0, r.stderr
    for f in ("tim_r.bin", "non_interp_spec.bin", "interp_spec.bin", "pspec_post.bin", "harm1.bin", "harm2.bin"):
        assert (tmp_path / f).exists(), f
