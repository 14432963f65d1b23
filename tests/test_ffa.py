"""FFA periodicity search (the pipeline behind the reference's FFA options,
include/utils/cmdline.hpp:35-50, 211-292; Makefile:41-42 `ffaster`).

CPU: option parsing parity, octave planning, clustering.  GPU: FFA planes and
boxcar S/N vs a float64 numpy FFA oracle, downsampling, and an end-to-end
search that recovers an injected long-period pulsar (parity unpinned: the
reference's FFA source is not in its tree)."""
import os
import subprocess

import numpy as np
import pytest
import torch

from peasoup_amd import _C as C
from peasoup_amd.utils import reference as ref
from peasoup_amd.utils import synthetic

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ffa_cmdline_defaults_match_reference():
    ok, exit_now, a = C.parse_ffa_cmdline(["ffaster", "-i", "x.fil"])
    assert ok and not exit_now
    assert (a.max_num_threads, a.nstreams) == (14, 16)
    assert (a.dm_start, a.dm_end) == (0.0, 100.0)
    assert a.dm_tol == pytest.approx(1.10) and a.dm_pulse_width == 64.0
    assert a.p_start == pytest.approx(0.8) and a.p_end == 20.0 and a.min_dc == pytest.approx(0.001)
    assert not a.verbose and not a.progress_bar and a.killfilename == ""
    assert a.outfilename.endswith("_ffaster.output") and len(a.outfilename) == len("2026-01-01-00:00_ffaster.output")
    ok, _, a = C.parse_ffa_cmdline(["ffaster", "-i", "y.fil", "-o", "out.txt", "-k", "kill.txt", "-t", "2",
                                    "--nstreams", "4", "--dm_start", "5", "--dm_end", "50", "--p_start", "1.5",
                                    "--p_end", "9", "--min_dc", "0.01", "-vp", "--min_snr", "8", "--bins", "300"])
    assert ok and a.outfilename == "out.txt" and a.killfilename == "kill.txt" and a.max_num_threads == 2
    assert a.nstreams == 4 and a.p_start == 1.5 and a.p_end == 9.0 and a.verbose and a.progress_bar
    assert a.min_snr == 8.0 and a.nbins == 300
    ok, _, _ = C.parse_ffa_cmdline(["ffaster"])  # -i is required
    assert not ok


def test_ffa_plan_covers_period_range():
    p = C.FfaParams()
    p.tsamp, p.p_start, p.p_end, p.min_dc = 64e-6, 0.5, 7.0, 0.002
    p.arena_floats = 1 << 22
    n = 1 << 22
    plan = C.ffa_plan(p, n)
    nb0 = C.ffa_base_bins(p)
    assert nb0 == 250
    lo = hi = None
    for o in plan:
        bin_s = o["factor"] * p.tsamp
        assert o["factor"] >= 1.0 and o["nds"] == int(n // o["factor"])
        assert o["pb"] <= 2 * o["pa"]
        ps = [per[0] for c in o["chunks"] for per in c["periods"]]
        assert ps == list(range(o["pa"], o["pa"] + len(ps)))  # contiguous base periods
        for c in o["chunks"]:
            assert c["arena"] <= p.arena_floats
            for (P, m, m2, lg, off) in c["periods"]:
                assert m == o["nds"] // P and m2 == 1 << lg and m2 >= m > m2 // 2
        o_lo, o_hi = o["pa"] * bin_s, (o["pa"] + len(ps)) * bin_s
        assert lo is None or o_lo == pytest.approx(hi, rel=5e-3)
        lo = o_lo if lo is None else lo
        hi = o_hi
    assert lo == pytest.approx(0.5, rel=1e-3) and hi >= 7.0 * 0.999
    w = C.ffa_widths(nb0)
    assert w[0] == 1 and w == sorted(set(w)) and w[-1] <= nb0 // 2


def test_ffa_cluster_keeps_strongest_per_frequency_window():
    cands = []
    for period, snr in [(1.0, 10.0), (1.0001, 12.0), (1.5, 9.0), (0.99995, 8.0), (3.0, 20.0)]:
        c = C.FfaCandidate()
        c.period, c.snr = period, snr
        cands.append(c)
    out = C.ffa_cluster(cands, 1e-3)
    assert [round(c.period, 4) for c in out] == [3.0, 1.0001, 1.5]


@pytest.mark.gpu
@pytest.mark.parametrize("periods,nds", [([37, 38, 50, 64], 5000), ([300, 301, 511], 70000), ([1500, 1999], 40000)])
def test_ffa_planes_match_numpy(periods, nds):
    rng = np.random.default_rng(len(periods) + nds)
    ds = rng.standard_normal(nds).astype(np.float32)
    planes, widths = C.ffa_fold_planes(ds, periods, 1.0)
    for (P, m, m2, plane, best) in planes:
        exp = ref.ffa_transform(ref.ffa_fold_matrix(ds, P))
        assert plane.shape == exp.shape == (m2, P)
        np.testing.assert_allclose(plane, exp, rtol=1e-4, atol=2e-4 * np.sqrt(m))
        snr = np.array([ref.boxcar_best_snr(exp[s], widths, m * 1.0) for s in range(m2)])
        np.testing.assert_allclose(best, snr, rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
def test_ffa_downsample_matches_numpy():
    rng = np.random.default_rng(3)
    x = rng.standard_normal(100003).astype(np.float32)
    xt = torch.from_numpy(x).cuda()
    s = torch.cuda.current_stream().cuda_stream
    for f in (1.0, 2.0, 3.7, 17.25):
        nout = int(len(x) // f)
        out = torch.empty(nout, device="cuda")
        C.kernels.ffa_downsample(xt.data_ptr(), len(x), f, out.data_ptr(), nout, s)
        exp = ref.ffa_downsample(x, f)
        np.testing.assert_allclose(out.cpu().numpy(), exp[:nout], rtol=1e-4, atol=1e-4 * np.sqrt(f))


@pytest.mark.gpu
def test_ffa_pipeline_finds_long_period_pulsar(tmp_path):
    hdr = synthetic.make_header(nchans=64, nbits=2, tsamp=1e-3, fch1=1510.0, foff=-1.09)
    psr = synthetic.PulsarSpec(period=1.2345, dm=25.0, duty=0.02, amplitude=0.35)
    path = str(tmp_path / "ffa.fil")
    synthetic.write(path, 1 << 18, hdr, [psr], seed=11)
    out = str(tmp_path / "ffa.txt")
    ok, _, a = C.parse_ffa_cmdline(["ffaster", "-i", path, "-o", out, "--dm_start", "0", "--dm_end", "50",
                                    "--p_start", "0.5", "--p_end", "3.0", "--min_dc", "0.01", "-t", "1"])
    assert ok
    res = C.run_ffa_pipeline(a)
    assert res.candidates, "no FFA candidates"
    best = res.candidates[0]
    assert best.period == pytest.approx(psr.period, rel=2e-3) or best.period == pytest.approx(2 * psr.period, rel=2e-3)
    assert abs(best.dm - psr.dm) < 10.0 and best.snr > 15.0
    C.write_ffa_output(out, a, res)
    lines = [ln for ln in open(out) if not ln.startswith("#")]
    assert len(lines) == len(res.candidates)
    assert float(lines[0].split()[1]) == pytest.approx(best.period, rel=1e-9)


@pytest.mark.gpu
def test_ffaster_cli(tmp_path):
    hdr = synthetic.make_header(nchans=32, nbits=2, tsamp=1e-3)
    path = str(tmp_path / "c.fil")
    synthetic.write(path, 1 << 16, hdr, [synthetic.PulsarSpec(period=0.777, dm=10.0, duty=0.03, amplitude=0.5)],
                    seed=2)
    out = str(tmp_path / "c.txt")
    r = subprocess.run([os.path.join(REPO, "bin", "ffaster"), "-i", path, "-o", out, "--dm_end", "20",
                        "--p_start", "0.3", "--p_end", "2.0", "--min_dc", "0.02", "-t", "1"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rows = [ln.split() for ln in open(out) if not ln.startswith("#")]
    assert rows and float(rows[0][1]) == pytest.approx(0.777, rel=3e-3)


@pytest.mark.gpu
def test_ffa_detrend_removes_linear_trend():
    n, w = 50000, 4096
    t = np.arange(n)
    u8 = np.clip(np.rint(60 + 40 * t / n + np.random.default_rng(1).normal(0, 3, n)), 0, 255).astype(np.uint8)
    xt = torch.from_numpy(u8).cuda()
    out = torch.empty(n, device="cuda")
    means = torch.empty((n + w - 1) // w, device="cuda")
    sums = torch.empty((n + w - 1) // w, dtype=torch.int64, device="cuda")
    C.kernels.ffa_detrend(xt.data_ptr(), n, w, sums.data_ptr(), means.data_ptr(), out.data_ptr(),
                          torch.cuda.current_stream().cuda_stream)
    exp_means = np.array([u8[i:i + w].mean() for i in range(0, n, w)])
    np.testing.assert_allclose(means.cpu().numpy(), exp_means, rtol=1e-5)
    y = out.cpu().numpy()
    mid = slice(w, n - w)
    assert abs(np.polyfit(t[mid], y[mid], 1)[0]) < 1e-5 and abs(y[mid].mean()) < 0.2


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_ffa_two_rank_search_equals_native_pipeline(tmp_path):
    """DM-sharded FFA (2 ranks, gloo transport, one GPU) + gather + cross-DM
    clustering == the native thread-per-GPU pipeline's candidates."""
    import sys

    hdr = synthetic.make_header(nchans=32, nbits=2, tsamp=1e-3)
    path = str(tmp_path / "d.fil")
    synthetic.write(path, 1 << 16, hdr, [synthetic.PulsarSpec(period=0.6321, dm=15.0, duty=0.03, amplitude=0.5)],
                    seed=4)
    flags = ["-i", path, "--dm_end", "40", "--p_start", "0.3", "--p_end", "2.0", "--min_dc", "0.02", "-t", "1"]
    script = (
        "import os,sys; sys.path.insert(0, %r)\n"
        "from peasoup_amd.parallel import dist as pdist\n"
        "pdist.init(backend='gloo')\n"
        "from peasoup_amd import __main__ as m\n"
        "raise SystemExit(m.main(['x', 'ffa'] + sys.argv[1:]))\n" % REPO)
    f = tmp_path / "run.py"
    f.write_text(script)
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    out = str(tmp_path / "dist.txt")
    procs = [subprocess.Popen([sys.executable, str(f)] + flags + ["-o", out], env=dict(env, RANK=str(r), LOCAL_RANK="0"),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    for p in procs:
        _, err = p.communicate(timeout=300)
        assert p.returncode == 0, err[-3000:]
    ok, _, a = C.parse_ffa_cmdline(["ffaster"] + flags + ["-o", str(tmp_path / "native.txt")])
    res = C.run_ffa_pipeline(a)
    rows = [ln.split() for ln in open(out) if not ln.startswith("#")]
    assert len(rows) == len(res.candidates) > 0
    for row, c in zip(rows, res.candidates):
        assert float(row[1]) == pytest.approx(c.period, rel=1e-9) and int(row[4]) == c.dm_idx
        assert float(row[5]) == pytest.approx(c.snr, abs=1e-3)
