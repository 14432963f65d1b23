"""Coincidencer, correlator, python -m entry point and a 2-rank distributed
search (gloo transport, both ranks on the one visible GPU)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import REPO, TUTORIAL
from peasoup_amd.utils import reference as ref
from peasoup_amd.utils import synthetic

pytestmark = pytest.mark.gpu


def _beams(tmp_path, nbeam=4, nsamps=40000):
    hdr = synthetic.make_header(nchans=16, nbits=8, tsamp=256e-6, fch1=1400.0, foff=-4.0)
    rng = np.random.default_rng(0)
    paths = []
    for b in range(nbeam):
        vals = synthetic.generate(nsamps, dict(hdr, nsamples=nsamps), seed=b + 10)
        # common impulsive RFI in all beams + a periodic tone in 3 beams
        vals[12000:12010] = 255
        if b < 3:
            t = np.arange(nsamps)
            # weak in the time domain (keeps the burst > 4 sigma), a strong Fourier spike
            vals = np.clip(vals.astype(np.float32) + 8 * np.sin(2 * np.pi * 50.0 * t * 256e-6)[:, None], 0, 255)
            vals = vals.astype(np.uint8)
        p = str(tmp_path / f"beam{b}.fil")
        from peasoup_amd.utils.sigproc import write_filterbank

        write_filterbank(p, dict(hdr, nsamples=nsamps), vals)
        paths.append(p)
    return paths


def test_coincidencer_python_and_cli_agree(tmp_path):
    from peasoup_amd.models.coincidencer import run_coincidencer

    paths = _beams(tmp_path)
    out = run_coincidencer(paths, str(tmp_path / "m_py.txt"), str(tmp_path / "b_py.txt"), thresh=4.0, beam_thresh=3)
    assert out["masked_samples"] >= 10 and out["masked_bins"] >= 1
    exe = os.path.join(REPO, "bin", "peasoup_coincidencer")
    r = subprocess.run([exe] + paths + ["--o", str(tmp_path / "m_cli.txt"), "--o2", str(tmp_path / "b_cli.txt"),
                                        "--thresh", "4", "--beam_thresh", "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert open(tmp_path / "m_py.txt").read() == open(tmp_path / "m_cli.txt").read()
    assert open(tmp_path / "b_py.txt").read() == open(tmp_path / "b_cli.txt").read()
    mask = [int(x) for x in open(tmp_path / "m_py.txt").read().split("\n")[1:] if x]
    assert all(m == 0 for m in mask[12000:12010])  # the common RFI burst is masked
    birdies = [tuple(map(float, l.split())) for l in open(tmp_path / "b_py.txt") if l.strip()]
    assert any(abs(f - 50.0) < 0.5 for f, w in birdies)  # the 50 Hz tone in 3 beams


def test_correlator_finds_delays():
    from peasoup_amd.models.correlator import find_delays

    rng = np.random.default_rng(1)
    size = 1 << 14
    base = rng.integers(-60, 60, size=(2 * size + 400,)).astype(np.int8)
    arrays = []
    lags = [0, 7, -13]
    for lag in lags:
        s = 200 + 2 * lag
        arrays.append(base[s: s + 2 * size])
    d = find_delays(np.stack(arrays), 64)
    assert d[(0, 1)] == lags[1] - lags[0] or d[(0, 1)] == -(lags[1] - lags[0])
    assert abs(d[(0, 2)]) == 13 and abs(d[(1, 2)]) == 20


def test_python_module_entry_point(tmp_path):
    r = subprocess.run([sys.executable, "-m", "peasoup_amd", "-i", TUTORIAL, "-o", str(tmp_path), "--dm_start", "15",
                        "--dm_end", "35", "-n", "4", "--npdmp", "2", "-v"], capture_output=True, text=True,
                       timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stderr
    from peasoup_amd.utils.outputs import PeasoupOutput

    out = PeasoupOutput(str(tmp_path / "overview.xml"), str(tmp_path / "candidates.peasoup"))
    c = out.get_candidate(0)
    assert abs(c.info["period"] - 0.25) < 1e-3 and c.fold is not None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,schedule", [(2, "static"), (4, "static"), (2, "dynamic"), (3, "dynamic")])
def test_multi_rank_search_equals_single_rank(tmp_path, world, schedule):
    """DM distribution (static trial-weighted shards, or first-come chunks from
    the shared pdist.WorkQueue) + RCCL-style gather + distributed folding
    reproduce the single-process result (gloo transport, all ranks on one GPU)."""
    port = _free_port()
    dm_end = "120" if schedule == "static" else "250"  # dynamic: 59 DMs = two 32-DM chunks, 3 ranks (one idle)
    script = (
        "import os,sys; sys.path.insert(0, %r)\n"
        "from peasoup_amd.parallel import dist as pdist\n"
        "pdist.init(backend='gloo')\n"
        "from peasoup_amd import _C\n"
        "from peasoup_amd.models.search import run_search\n"
        "ok,_,a=_C.parse_cmdline(['peasoup','-i',%r,'-o',sys.argv[1],'--dm_end',%r,'-n','4','--npdmp','4',"
        "'--dm_schedule',%r,'--trace_json',sys.argv[1]+'.json'])\n"
        "run_search(a)\n"
        "pdist.shutdown()\n" % (REPO, TUTORIAL, dm_end, schedule))
    f = tmp_path / "run.py"
    f.write_text(script)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world))
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK="0")
        procs.append(subprocess.Popen([sys.executable, str(f), str(tmp_path / "dist")], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    for p in procs:
        out, err = p.communicate(timeout=600)
        assert p.returncode == 0, err[-3000:]
    e1 = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(f), str(tmp_path / "single")], env=e1, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    a = open(tmp_path / "dist" / "candidates.peasoup", "rb").read()
    b = open(tmp_path / "single" / "candidates.peasoup", "rb").read()
    assert a == b
    import json

    devs = json.load(open(str(tmp_path / "dist") + ".json"))["devices"]
    assert [d["dm_schedule"] for d in devs] == [schedule] * world
    if schedule == "dynamic":  # every 32-DM chunk searched exactly once, by some rank
        assert sum(d["dm_blocks"] for d in devs) == 2


def _run_ranks(tmp_path, script, world, out, extra_env=None):
    port = _free_port()
    f = tmp_path / "run.py"
    f.write_text(script)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), **(extra_env or {}))
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK="0")
        procs.append(subprocess.Popen([sys.executable, str(f), str(out)], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    for p in procs:
        _, err = p.communicate(timeout=600)
        assert p.returncode == 0, err[-3000:]


@pytest.mark.parametrize("world,schedule,slices", [(2, "static", "0"), (4, "static", "0"), (2, "dynamic", "3"),
                                                    (4, "dynamic", "0")])
def test_one_dm_job_acceleration_sliced_over_ranks(tmp_path, world, schedule, slices):
    """A 1-DM job (one 32-DM chunk) on 2 and 4 ranks: the DM's acceleration
    trials are cut into slices that the ranks search (static shards or the
    shared queue); the per-trial harmonic-distilled slice lists are joined in
    plan order on rank 0 and acceleration-distilled there, so the candidate
    file is byte-identical to one rank's unsliced search."""
    common = ("'-i',%r,'--dm_start','30','--dm_end','30','--acc_start','-20','--acc_end','20',"
              "'--accel_convention','reference','-n','3','--npdmp','3'" % (TUTORIAL,))
    script = (
        "import os,sys; sys.path.insert(0, %r)\n"
        "from peasoup_amd.parallel import dist as pdist\n"
        "pdist.init(backend='gloo')\n"
        "from peasoup_amd import _C\n"
        "from peasoup_amd.models import search as S\n"
        "S.MIN_SLICE_TRIALS = 4\n"
        "ok,_,a=_C.parse_cmdline(['peasoup',%s,'-o',sys.argv[1],'--dm_schedule',%r,'--accel_slices',%r,"
        "'--trace_json',sys.argv[1]+'.json'])\n"
        "S.run_search(a)\n"
        "pdist.shutdown()\n" % (REPO, common, schedule, slices))
    _run_ranks(tmp_path, script, world, tmp_path / "dist")
    single = (
        "import sys; sys.path.insert(0, %r)\n"
        "from peasoup_amd import _C\n"
        "from peasoup_amd.models.search import run_search\n"
        "ok,_,a=_C.parse_cmdline(['peasoup',%s,'-o',sys.argv[1]])\n"
        "res = run_search(a)\n"
        "print('NTRIALS', res.accel_trials)\n" % (REPO, common))
    f1 = tmp_path / "single.py"
    f1.write_text(single)
    r = subprocess.run([sys.executable, str(f1), str(tmp_path / "single")],
                       env=dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    ntrials = int(r.stdout.split("NTRIALS")[1].split()[0])
    assert ntrials >= 16
    a = open(tmp_path / "dist" / "candidates.peasoup", "rb").read()
    b = open(tmp_path / "single" / "candidates.peasoup", "rb").read()
    assert len(b) > 0 and a == b
    import json

    devs = json.load(open(str(tmp_path / "dist") + ".json"))["devices"]
    nsl = devs[0]["accel_slices"]
    assert nsl == (int(slices) if slices != "0" else 4 * world) and all(d["accel_slices"] == nsl for d in devs)
    # every trial searched exactly once over the ranks; more than one rank did work
    assert sum(d["accel_trials_planned"] for d in devs) == ntrials
    assert sum(1 for d in devs if d["accel_trials_planned"] > 0) >= 2


def test_dynamic_schedule_four_ranks_many_chunks(tmp_path):
    """The mode 8-GPU config 4 uses: four ranks claim first-come 32-DM chunks
    from the shared queue, with 18 chunks (>= 4 per rank) on a 572-DM list;
    the merged output is byte-identical to one rank's."""
    port = _free_port()
    script = (
        "import os,sys; sys.path.insert(0, %r)\n"
        "from peasoup_amd.parallel import dist as pdist\n"
        "pdist.init(backend='gloo')\n"
        "from peasoup_amd import _C\n"
        "from peasoup_amd.models.search import run_search\n"
        "ok,_,a=_C.parse_cmdline(['peasoup','-i',%r,'-o',sys.argv[1],'--dm_end','2000','--dm_tol','1.01',"
        "'-n','3','--npdmp','4','--dm_schedule','dynamic','--trace_json',sys.argv[1]+'.json'])\n"
        "run_search(a)\n"
        "pdist.shutdown()\n" % (REPO, TUTORIAL))
    f = tmp_path / "run.py"
    f.write_text(script)
    world = 4
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world))
    procs = [subprocess.Popen([sys.executable, str(f), str(tmp_path / "dist")], env=dict(env, RANK=str(r), LOCAL_RANK="0"),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    for p in procs:
        out, err = p.communicate(timeout=600)
        assert p.returncode == 0, err[-3000:]
    r = subprocess.run([sys.executable, str(f), str(tmp_path / "single")],
                       env=dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert open(tmp_path / "dist" / "candidates.peasoup", "rb").read() == \
        open(tmp_path / "single" / "candidates.peasoup", "rb").read()
    import json

    devs = json.load(open(str(tmp_path / "dist") + ".json"))["devices"]
    blocks = [d["dm_blocks"] for d in devs]
    assert sum(blocks) == 18 and [d["dm_schedule"] for d in devs] == ["dynamic"] * world
    assert min(blocks) >= 1, blocks


@pytest.mark.parametrize("world", [2, 3])
def test_time_sharded_run_search_equals_replicated(tmp_path, world):
    """--time_shards: every rank holds only its time slice of tutorial.fil,
    ring halo exchange + all-to-all corner turn to DM shards, search and fold
    of the rank's resident DM rows; the output files equal the
    replicated single-rank run's byte for byte."""
    port = _free_port()
    script = (
        "import os,sys; sys.path.insert(0, %r)\n"
        "from peasoup_amd.parallel import dist as pdist\n"
        "pdist.init(backend='gloo')\n"
        "from peasoup_amd import _C\n"
        "from peasoup_amd.models.search import run_search\n"
        "extra = ['--time_shards'] if sys.argv[2] == '1' else []\n"
        "ok,_,a=_C.parse_cmdline(['peasoup','-i',%r,'-o',sys.argv[1],'--dm_end','120','-n','4','--npdmp','6',"
        "'--acc_start','-5','--acc_end','5','--trace_json',sys.argv[1]+'.json'] + extra)\n"
        "assert a.time_shards == bool(extra)\n"
        "run_search(a)\n"
        "pdist.shutdown()\n" % (REPO, TUTORIAL))
    f = tmp_path / "run.py"
    f.write_text(script)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world))
    procs = [subprocess.Popen([sys.executable, str(f), str(tmp_path / "ts"), "1"],
                              env=dict(env, RANK=str(r), LOCAL_RANK="0"), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(world)]
    for p in procs:
        out, err = p.communicate(timeout=600)
        assert p.returncode == 0, err[-3000:]
    r = subprocess.run([sys.executable, str(f), str(tmp_path / "rep"), "0"],
                       env=dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    a = open(tmp_path / "ts" / "candidates.peasoup", "rb").read()
    b = open(tmp_path / "rep" / "candidates.peasoup", "rb").read()
    assert a == b and len(a) > 1000
    import json

    devs = json.load(open(str(tmp_path / "ts") + ".json"))["devices"]
    assert [d["dm_schedule"] for d in devs] == ["time_sharded"] * world


def test_forced_rccl_process_group_world1(tmp_path):
    """PSOUP_FORCE_PG=1: a world-1 RCCL process group, so every collective the
    pipeline uses (broadcast_bytes, broadcast_object_bytes, gather_bytes,
    all_reduce_sum, all_reduce_max_float, barrier, the store-backed work
    queue) executes on the GPU through RCCL; a search through it equals the
    plain single-process search byte for byte."""
    port = _free_port()
    script = (
        "import os,sys; sys.path.insert(0, %r)\n"
        "import torch\n"
        "from peasoup_amd.parallel import dist as pdist\n"
        "ctx = pdist.init()\n"
        "forced = os.environ.get('PSOUP_FORCE_PG') == '1'\n"
        "if forced:\n"
        "    import torch.distributed as dist\n"
        "    assert ctx.backend == 'nccl' and ctx.distributed and dist.get_backend() == 'nccl', ctx\n"
        "    b = torch.arange(1 << 20, dtype=torch.int64, device=ctx.device).to(torch.uint8)\n"
        "    out = pdist.broadcast_bytes(b, b.numel())\n"
        "    assert out.is_cuda and torch.equal(out, b)\n"
        "    assert pdist.broadcast_object_bytes(b'header') == b'header'\n"
        "    assert pdist.gather_bytes(b'abc', dst=None) == [b'abc']\n"
        "    t = torch.tensor([7, 9], dtype=torch.int64, device=ctx.device)\n"
        "    assert pdist.all_reduce_sum(t).tolist() == [7, 9]\n"
        "    assert pdist.all_reduce_max_float(2.5) == 2.5\n"
        "    pdist.barrier()\n"
        "    q = pdist.WorkQueue('forced', 3)\n"
        "    assert [q.claim() for _ in range(4)] == [0, 1, 2, None]\n"
        "from peasoup_amd import _C\n"
        "from peasoup_amd.models.search import run_search\n"
        "ok,_,a=_C.parse_cmdline(['peasoup','-i',%r,'-o',sys.argv[1],'--dm_end','250','--acc_start','-5',"
        "'--acc_end','5','-n','4','--npdmp','10','--dm_schedule','dynamic'])\n"
        "run_search(a)\n"
        "pdist.shutdown()\n"
        "print('OK forced' if forced else 'OK plain')\n" % (REPO, TUTORIAL))
    f = tmp_path / "run.py"
    f.write_text(script)
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    outs = {}
    for forced in ("1", "0"):
        r = subprocess.run([sys.executable, str(f), str(tmp_path / forced)], env=dict(base, PSOUP_FORCE_PG=forced),
                           capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        assert ("OK forced" if forced == "1" else "OK plain") in r.stdout
        outs[forced] = open(tmp_path / forced / "candidates.peasoup", "rb").read()
    assert outs["1"] == outs["0"] and len(outs["1"]) > 1000


def test_time_shard_native_windows_match_whole(C):
    """Each rank's haloed window dedispersed by the MFMA kernel equals the
    corresponding columns of the whole-observation dedispersion."""
    import numpy as np
    import torch

    from peasoup_amd.parallel import timeshard
    from peasoup_amd.utils import reference as ref
    from peasoup_amd.utils import sigproc, synthetic

    nchans, nbits, nsamps = 64, 2, 20000
    hdr = synthetic.make_header(nchans=nchans, nbits=nbits, tsamp=0.00032, fch1=1510.0, foff=-1.09, nsamples=nsamps)
    dms = C.generate_dm_list(0.0, 150.0, 0.00032, 64.0, 1510.0, -1.09, nchans, 1.1)
    vals = np.random.default_rng(9).integers(0, 4, size=(nsamps, nchans), dtype=np.uint8)
    packed = sigproc.pack_samples(vals, nbits)
    offs = ref.dm_offsets(dms, ref.delay_table(nchans, 0.00032, 1510.0, -1.09))
    world = 3
    plan = timeshard.make_plan(hdr, nsamps, dms, world)
    full = ref.dedisperse(vals, offs, nbits, None, plan.out_nsamps)
    fn = timeshard.native_dedisperser(hdr, dms)
    for r in range(world):
        w = plan.windows[r]
        lo = w.start * plan.bytes_per_sample
        hi = (w.stop + plan.max_delay) * plan.bytes_per_sample
        ext = torch.from_numpy(packed[lo:hi].copy()).cuda()
        got = fn(ext, w.stop + plan.max_delay - w.start, len(w)).cpu().numpy()
        assert np.array_equal(got, full[:, w.start:w.stop]), r


def test_python_entry_fault_then_resume(tmp_path):
    """python -m peasoup_amd: an injected fault exits non-zero with rank
    context; a re-run with the same --checkpoint_dir resumes from the spill
    files and matches a clean run byte for byte."""
    import subprocess
    import sys

    from conftest import REPO, TUTORIAL

    ck = tmp_path / "ck"
    base = [sys.executable, "-m", "peasoup_amd", "-i", TUTORIAL, "--dm_end", "120", "-n", "3"]
    env = dict(os.environ, PYTHONPATH=REPO)
    r = subprocess.run(base + ["-o", str(tmp_path / "a"), "--checkpoint_dir", str(ck), "--fault_after_dms", "33"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert r.returncode != 0 and "[rank 0] peasoup failed: fault injection" in r.stderr
    assert len(list(ck.glob("dm_*.psoc"))) >= 1
    r = subprocess.run(base + ["-o", str(tmp_path / "b"), "--checkpoint_dir", str(ck)], capture_output=True, text=True,
                       timeout=600, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr
    r = subprocess.run(base + ["-o", str(tmp_path / "c")], capture_output=True, text=True, timeout=600, env=env,
                       cwd=REPO)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "b" / "candidates.peasoup").read_bytes() == (tmp_path / "c" / "candidates.peasoup").read_bytes()


def test_python_resume_with_changed_options_recomputes(C, tmp_path):
    """The Python driver ignores spills of a different run (here: another
    --min_snr) and recomputes, matching a clean run."""
    from conftest import TUTORIAL
    from peasoup_amd.models.search import run_search

    ck = str(tmp_path / "ck")

    def search(out, *extra):
        ok, _, args = C.parse_cmdline(["peasoup", "-i", TUTORIAL, "--dm_end", "80", "-n", "3", "-o",
                                       str(tmp_path / out), *extra])
        assert ok
        return C.serialize_candidates(run_search(args).candidates)

    a = search("a", "--checkpoint_dir", ck)
    assert search("a2", "--checkpoint_dir", ck) == a  # same run: resumed
    import warnings
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        b = search("b", "-m", "7", "--checkpoint_dir", ck)
    assert any("mismatch" in str(x.message) for x in w)
    assert b == search("c", "-m", "7") and b != a


def test_accmap_tool_finds_injected_delay(tmp_path):
    """tools/peasoup_accmap.py on a synthetic DADA file with a known lag."""
    import json
    import subprocess
    import sys

    import numpy as np

    from conftest import REPO
    from peasoup_amd.utils import dada

    rng = np.random.default_rng(3)
    n, nant, nchan, lag = 1 << 14, 2, 2, 37
    base = rng.integers(-40, 40, size=(n + lag, 2), dtype=np.int8)
    payload = np.zeros((n, nant, nchan, 1, 2), dtype=np.int8)
    payload[:, 0, 1, 0, :] = base[lag:lag + n]
    payload[:, 1, 1, 0, :] = base[:n]
    path = str(tmp_path / "v.dada")
    dada.write(path, {"HDR_SIZE": 4096, "NANT": nant, "NCHAN": nchan, "NPOL": 1, "NDIM": 2, "NBIT": 8}, payload)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "peasoup_accmap.py"), path, "--channel", "1",
                        "--size", str(n), "--max-delay", "128"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert abs(d["delays"]["0-1"]) == lag


def test_rank_fault_aborts_group_then_resume(tmp_path):
    """Peer failure, gloo world 3 on the one GPU: rank 1 alone
    faults after its first DM chunk; every rank exits non-zero within 60 s,
    the survivors naming rank 1; a re-run with the same --checkpoint_dir
    resumes from the spills and writes the clean run's candidates byte for byte."""
    ck = tmp_path / "ck"
    base = [sys.executable, "-m", "peasoup_amd", "-i", TUTORIAL, "--dm_end", "250", "-n", "3", "--npdmp", "4"]
    env = dict(os.environ, PYTHONPATH=REPO, MASTER_ADDR="127.0.0.1", WORLD_SIZE="3", PSOUP_DIST_BACKEND="gloo",
               PSOUP_HEARTBEAT_S="0.5")

    def group(out, extra, extra_env=None):
        e = dict(env, MASTER_PORT=str(_free_port()), **(extra_env or {}))
        ps = [subprocess.Popen(base + ["-o", str(out)] + extra, env=dict(e, RANK=str(r), LOCAL_RANK="0"),
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=REPO)
              for r in range(3)]
        out_ = []
        for p in ps:
            _, err = p.communicate(timeout=600)
            out_.append((p.returncode, err))
        return out_

    import time as _time

    t0 = _time.monotonic()
    res = group(tmp_path / "a", ["--checkpoint_dir", str(ck), "--fault_after_dms", "1", "--dm_schedule", "static"],
                {"PSOUP_FAULT_RANK": "1"})
    dt = _time.monotonic() - t0
    assert dt < 120, dt  # includes three interpreter + GPU start-ups
    for r, (rc, err) in enumerate(res):
        assert rc != 0, (r, err[-2000:])
        assert "rank 1" in err, (r, err[-2000:])
    assert "[rank 1] peasoup failed: fault injection" in res[1][1]
    res = group(tmp_path / "b", ["--checkpoint_dir", str(ck), "--dm_schedule", "static"])
    assert all(rc == 0 for rc, _ in res), [e[-2000:] for _, e in res]
    res = group(tmp_path / "c", ["--dm_schedule", "static"])
    assert all(rc == 0 for rc, _ in res), [e[-2000:] for _, e in res]
    assert (tmp_path / "b" / "candidates.peasoup").read_bytes() == (tmp_path / "c" / "candidates.peasoup").read_bytes()
