"""Candidate diagnostic plots for peasoup outputs (Python 3).

The reference's ``CandidatePlotter`` (tools/peasoup_tools.py:167-383) draws,
per candidate of ``overview.xml`` + ``candidates.peasoup``: the folded
profile, the sub-integration image, per-sub-integration statistics, an info
table, DM / acceleration / S/N scatters of the candidate's associated hits
coloured by harmonic, a DM-acceleration map, and every candidate of the
search in period-DM space with a crosshair on the current one.

Here the panel data are computed first (:func:`candidate_panels`, NumPy
only) and then drawn (:class:`CandidatePlotter`, matplotlib's Agg backend).
Without matplotlib the panels are written as one ``.npz`` instead of a PNG,
so the data path is testable anywhere.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import numpy as np

from .outputs import OverviewFile, PeasoupOutput, radec_to_str

HARM_COLOURS = ["darkblue", "lightblue", "green", "orange", "darkred", "purple"]


def candidate_panels(out: PeasoupOutput, idx: int) -> Dict[str, object]:
    """Every panel's data for candidate ``idx`` (NumPy arrays / lists)."""
    cand = out.get_candidate(idx)
    info = cand.info
    hits = np.sort(cand.hits, order="snr")[::-1] if cand.hits.size else cand.hits
    p: Dict[str, object] = {"index": idx}
    fold = None if cand.fold is None else np.array(cand.fold, dtype=np.float64)
    if fold is not None:
        lo, hi = fold.min(), fold.max()
        fold = (fold - lo) / (hi - lo) if hi > lo else fold * 0.0
        p["subints"] = fold                                     # [nints, nbins], normalised to [0, 1]
        p["profile"] = fold.sum(axis=0)
        std = fold.std(axis=1)
        mean = fold.mean(axis=1)
        p["subint_stats"] = np.stack([mean, std, mean - 3 * std, mean + 3 * std, fold.min(axis=1), fold.max(axis=1)])
    # associated hits, grouped by harmonic number (the scatters and the DM-acc map)
    groups: List[Tuple[int, np.ndarray]] = []
    for nh in np.unique(hits["nh"]) if hits.size else []:
        groups.append((int(nh), hits[hits["nh"] == nh]))
    p["hits"] = hits
    p["hit_groups"] = groups
    if hits.size:
        p["dm_acc_limits"] = (float(hits["dm"].min()), float(hits["dm"].max()), float(hits["acc"].min()),
                              float(hits["acc"].max()))
    # every candidate of the search, period vs DM (crosshair on this one)
    allc = out.overview.as_array()
    p["all"] = np.stack([allc["period"], allc["dm"], allc["snr"], allc["nh"]]) if allc.size else np.zeros((4, 0))
    p["crosshair"] = (float(info["period"]), float(info["dm"]))
    hdr = out.overview.header
    ra = radec_to_str(float(hdr.get("src_raj", "0") or 0))
    dec = radec_to_str(float(hdr.get("src_dej", "0") or 0))
    p["table"] = [("R.A.", ra), ("Decl.", dec), ("P0", "%.9f" % info["period"]),
                  ("Opt P0", "%.9f" % info["opt_period"]), ("DM", "%.2f" % info["dm"]), ("Acc", "%.2f" % info["acc"]),
                  ("Harmonic", "%d" % info["nh"]), ("Spec S/N", "%.1f" % info["snr"]),
                  ("Fold S/N", "%.1f" % info["folded_snr"]), ("Adjacent?", str(bool(info["is_adjacent"]))),
                  ("Physical?", str(bool(info["is_physical"]))), ("DDM ratio 1", "%.4f" % info["ddm_count_ratio"]),
                  ("DDM ratio 2", "%.4f" % info["ddm_snr_ratio"]), ("Nassoc", "%d" % info["nassoc"])]
    p["title"] = hdr.get("source_name", "")
    return p


def _sizes(snr: np.ndarray) -> np.ndarray:
    s = np.asarray(snr, dtype=np.float64)
    if s.size == 0:
        return s
    rng = s.max() - s.min()
    return 5.0 + 250.0 * ((s - s.min()) / rng if rng > 0 else np.zeros_like(s))


class CandidatePlotter:
    """Draws :func:`candidate_panels` for any candidate of one search
    output.  ``plot_cand(idx, filename)`` writes ``filename`` (PNG, or
    ``.npz`` panels when matplotlib is missing) and returns its path."""

    def __init__(self, outdir: Optional[str] = None, overview: Optional[str] = None,
                 candidates: Optional[str] = None):
        overview = overview or os.path.join(outdir, "overview.xml")
        candidates = candidates or os.path.join(os.path.dirname(os.path.abspath(overview)), "candidates.peasoup")
        self.out = PeasoupOutput(overview, candidates)
        try:
            import matplotlib

            matplotlib.use("Agg")
            import matplotlib.pyplot as plt

            self._plt = plt
        except ImportError:  # pragma: no cover - matplotlib is in the image
            self._plt = None

    @property
    def overview(self) -> OverviewFile:
        return self.out.overview

    def __len__(self) -> int:
        return len(self.out)

    def plot_cand(self, idx: int, filename: Optional[str] = None) -> str:
        p = candidate_panels(self.out, idx)
        if self._plt is None:
            path = (filename or f"cand_{idx:04d}") + ("" if str(filename).endswith(".npz") else ".npz")
            arrays = {k: v for k, v in p.items() if isinstance(v, np.ndarray)}
            arrays["table"] = np.array(p["table"], dtype=object).astype(str)
            np.savez(path, **arrays)
            return path
        path = filename or f"cand_{idx:04d}.png"
        fig = self._draw(p)
        fig.savefig(path)
        self._plt.close(fig)
        return path

    # the reference's grid: 5 x 9 cells for the upper panels, the all-candidates strip below
    def _draw(self, p: Dict[str, object]):
        plt = self._plt
        fig = plt.figure(figsize=[14, 12])
        prof_ax = plt.subplot2grid([5, 9], [0, 1], colspan=2, fig=fig)
        fold_ax = plt.subplot2grid([5, 9], [1, 1], colspan=2, rowspan=2, sharex=prof_ax, fig=fig)
        subs_ax = plt.subplot2grid([5, 9], [1, 0], rowspan=2, sharey=fold_ax, fig=fig)
        table_ax = plt.subplot2grid([5, 9], [0, 3], colspan=3, rowspan=3, frameon=False, fig=fig)
        dm_ax = plt.subplot2grid([5, 9], [0, 6], colspan=2, fig=fig)
        acc_ax = plt.subplot2grid([5, 9], [1, 8], rowspan=2, fig=fig)
        dm_acc_ax = plt.subplot2grid([5, 9], [1, 6], colspan=2, rowspan=2, sharex=dm_ax, sharey=acc_ax, fig=fig)
        all_ax = plt.subplot2grid([6, 9], [4, 0], colspan=9, rowspan=2, fig=fig)
        if "subints" in p:
            sub = p["subints"]
            prof_ax.plot(p["profile"])
            prof_ax.set_title("Profile")
            prof_ax.set_ylabel("Flux")
            fold_ax.imshow(sub, aspect="auto", interpolation="nearest", origin="lower")
            fold_ax.set_xlim(-0.5, sub.shape[1] - 0.5)
            fold_ax.set_xlabel("Phase bin")
            mean, _, lo3, hi3, mn, mx = p["subint_stats"]
            y = np.arange(sub.shape[0])
            subs_ax.fill_betweenx(y, lo3, hi3, alpha=0.5, color="lightblue", label="+-3 sigma")
            subs_ax.plot(mean, y, lw=2, alpha=0.8, color="lightblue", label="mean")
            subs_ax.plot(mn, y, lw=2, color="darkblue", label="min")
            subs_ax.plot(mx, y, lw=2, color="darkred", label="max")
            subs_ax.legend(loc="lower left", bbox_to_anchor=(-0.2, 1.0), prop={"size": 8})
            subs_ax.invert_xaxis()
            subs_ax.set_ylim(-0.5, sub.shape[0] - 0.5)
            subs_ax.set_ylabel("Subintegration")
        else:
            fold_ax.text(0.5, 0.5, "not folded", ha="center", va="center", transform=fold_ax.transAxes)
        table_ax.xaxis.set_major_locator(plt.NullLocator())
        table_ax.yaxis.set_major_locator(plt.NullLocator())
        tab = table_ax.table(cellText=[list(r) for r in p["table"]], cellLoc="left", colLoc="left", loc="center")
        for cell in tab.get_celld().values():
            cell.set_linewidth(0)
        tab.scale(1.0, 1.6)
        for ii, (nh, g) in enumerate(p["hit_groups"]):
            col = HARM_COLOURS[ii % len(HARM_COLOURS)]
            dm_ax.scatter(g["dm"], g["snr"], facecolor=col, edgecolor="none", s=10, label="Harm. %d" % nh)
            acc_ax.scatter(g["snr"], g["acc"], facecolor=col, edgecolor="none", s=10)
            dm_acc_ax.scatter(g["dm"], g["acc"], facecolor=col, edgecolor="none", s=_sizes(g["snr"]))
        dm_ax.set_ylabel("S/N")
        dm_ax.yaxis.tick_right()
        if p["hit_groups"]:
            dm_ax.legend(loc="lower left", bbox_to_anchor=(0.0, 1.0), prop={"size": 8}, ncol=3)
        acc_ax.yaxis.tick_right()
        acc_ax.yaxis.set_label_position("right")
        acc_ax.set_ylabel("Acceleration (m/s/s)", rotation=-90, labelpad=12)
        acc_ax.set_xlabel("S/N")
        if "dm_acc_limits" in p:
            d0, d1, a0, a1 = p["dm_acc_limits"]
            dm_acc_ax.set_xlim(d0 - 0.5, d1 + 0.5)
            dm_acc_ax.set_ylim(a0 - 0.5, a1 + 0.5)
        dm_acc_ax.set_xlabel("DM (pc cm^-3)")
        per, dm, snr, nh = p["all"]
        if per.size:
            all_ax.scatter(per, dm, s=_sizes(snr), c=nh, cmap="viridis", edgecolor="none")
            all_ax.set_xscale("log")
            x, y = p["crosshair"]
            all_ax.axvline(x, color="k", lw=0.8)
            all_ax.axhline(y, color="k", lw=0.8)
        all_ax.set_xlabel("Period (s)")
        all_ax.set_ylabel("DM (pc cm^-3)")
        fig.suptitle(f"{p['title']}  candidate {p['index']}")
        return fig


def plot_all(outdir: str, limit: int = 100, dest: Optional[str] = None) -> List[str]:
    """``Cand%04d.png`` for the first ``limit`` candidates (the reference's
    ``main``, peasoup_tools.py:403-412)."""
    pl = CandidatePlotter(outdir)
    dest = dest or outdir
    return [pl.plot_cand(i, os.path.join(dest, "Cand%04d.png" % i)) for i in range(min(limit, len(pl)))]
