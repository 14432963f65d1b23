"""Python output tools (CPU): the predictor, candidate-data access and the
candidate plotter on the reference's golden output (tests/data/golden_*,
copied from /root/reference/example_output).  Reference:
tools/peasoup_tools.py:149-412."""
import os
import shutil
import subprocess
import sys

import numpy as np

from conftest import GOLDEN_CANDS, GOLDEN_XML, REPO
from peasoup_amd.utils.outputs import OverviewFile
from peasoup_amd.utils.plotting import CandidatePlotter, candidate_panels


def _outdir(tmp_path):
    shutil.copy(GOLDEN_XML, tmp_path / "overview.xml")
    shutil.copy(GOLDEN_CANDS, tmp_path / "candidates.peasoup")
    return tmp_path


def test_make_predictor_matches_reference_format(tmp_path):
    """make_predictor formats float32 candidate fields exactly as the
    reference (peasoup_tools.py:153-164): PERIOD %.15f of the float32 period,
    DM / ACC %.3f, RA / DEC through radec_to_str."""
    ov = OverviewFile(str(_outdir(tmp_path) / "overview.xml"))
    assert ov.make_predictor(0).split("\n") == [
        "SOURCE: P: 250.000000000000 ms, DM: 30.000",
        "PERIOD: 0.249939903616905",
        "DM: 19.762",
        "ACC: 0.000",
        "RA: 00:00:00.0000",
        "DEC: 00:00:00.0000",
    ]
    for i in range(len(ov)):
        lines = ov.make_predictor(i).split("\n")
        assert [ln.split(":")[0] for ln in lines] == ["SOURCE", "PERIOD", "DM", "ACC", "RA", "DEC"]
        assert float(lines[1].split()[1]) == np.float32(ov.get_candidate(i)["period"])


def test_get_candidate_data_reads_the_record(tmp_path):
    ov = OverviewFile(str(_outdir(tmp_path) / "overview.xml"))
    for i in (0, 3, 9):
        d = ov.get_candidate(i)
        fold, hits = ov.get_candidate_data(i).cand_from_offset(d["byte_offset"])
        assert fold.shape == (16, 64) and len(hits) == d["nassoc"] + 1
        assert hits[0]["dm"] == np.float32(d["dm"])


def test_candidate_panels_and_png(tmp_path):
    out = _outdir(tmp_path)
    pl = CandidatePlotter(str(out))
    p = candidate_panels(pl.out, 0)
    assert p["subints"].shape == (16, 64) and p["subints"].min() == 0.0 and p["subints"].max() == 1.0
    assert p["profile"].shape == (64,)
    assert p["subint_stats"].shape == (6, 16)
    assert sum(len(g) for _, g in p["hit_groups"]) == 156  # nassoc 155 + the candidate itself
    assert p["all"].shape == (4, 10)
    assert [r[0] for r in p["table"]] == ["R.A.", "Decl.", "P0", "Opt P0", "DM", "Acc", "Harmonic", "Spec S/N",
                                         "Fold S/N", "Adjacent?", "Physical?", "DDM ratio 1", "DDM ratio 2", "Nassoc"]
    path = pl.plot_cand(0, str(tmp_path / "c0.png"))
    assert os.path.getsize(path) > 10000
    assert open(path, "rb").read(8) in (b"\x89PNG\r\n\x1a\n",) or path.endswith(".npz")


def test_plot_script_all_and_predictor(tmp_path):
    out = _outdir(tmp_path)
    script = os.path.join(REPO, "tools", "peasoup_plot_cand.py")
    r = subprocess.run([sys.executable, script, str(out), "2", "--predictor"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("SOURCE: ")
    r = subprocess.run([sys.executable, script, str(out), "--all", "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert sorted(os.listdir(out))[:3] == ["Cand0000.png", "Cand0001.png", "Cand0002.png"]
