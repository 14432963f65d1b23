"""Distillers, scorer, peak clustering, serialisation vs pure-Python oracles."""
import math
import random

import numpy as np
import pytest

from peasoup_amd.utils import reference as ref


class Cand:
    def __init__(self, dm, dm_idx, acc, nh, snr, freq):
        self.dm, self.dm_idx, self.acc, self.nh, self.snr, self.freq = dm, dm_idx, acc, nh, snr, freq
        self.assoc = []


def py_distill(cands, cond):
    cands = sorted(cands, key=lambda c: -c.snr)
    uniq = [True] * len(cands)
    start = 0
    while True:
        idx = -1
        for ii in range(start, len(cands)):
            if uniq[ii]:
                start, idx = ii + 1, ii
                break
        if idx < 0:
            break
        cond(cands, idx, uniq)
    return [c for c, u in zip(cands, uniq) if u]


def f32(x):
    return float(np.float32(x))


def harm_cond(tol, max_harm, keep, frac):
    def cond(c, idx, uniq):
        f0 = c[idx].freq
        for ii in range(idx + 1, len(c)):
            maxd = 2.0 ** c[ii].nh if frac else 1
            for jj in range(1, int(max_harm) + 1):
                kk = 1
                while kk <= maxd:
                    r = kk * c[ii].freq / (jj * f0)
                    if 1 - f32(tol) < r < 1 + f32(tol):
                        if keep:
                            c[idx].assoc.append(c[ii])
                        uniq[ii] = False
                    kk += 1
    return cond


def acc_cond(tobs, tol, keep):
    toc = f32(tobs) / 299792458.0

    def cond(c, idx, uniq):
        f0, a0 = c[idx].freq, c[idx].acc
        edge = f0 * f32(tol)
        for ii in range(idx + 1, len(c)):
            af = f32(f0 + (a0 - c[ii].acc) * f0 * toc)
            f = c[ii].freq
            rel = (f0 - edge < f < af + edge) if af > f0 else (af - edge < f < f0 + edge)
            if rel:
                if keep:
                    c[idx].assoc.append(c[ii])
                uniq[ii] = False
    return cond


def dm_cond(tol, keep):
    def cond(c, idx, uniq):
        for ii in range(idx + 1, len(c)):
            r = c[ii].freq / c[idx].freq
            if 1 - f32(tol) < r < 1 + f32(tol):
                if keep:
                    c[idx].assoc.append(c[ii])
                uniq[ii] = False
    return cond


def random_cands(rng, n, base_freqs=(4.0, 7.3, 11.1)):
    out = []
    for _ in range(n):
        f0 = rng.choice(base_freqs)
        h = rng.choice([1, 2, 3, 0.5, 0.25, 1.5])
        f = f32(f0 * h * (1 + rng.uniform(-2e-5, 2e-5)))
        out.append((f32(rng.uniform(0, 100)), rng.randrange(0, 50), f32(rng.uniform(-50, 50)), rng.randrange(0, 5),
                    f32(rng.uniform(9, 60)), f))
    return out


def to_native(C, tuples):
    return [C.Candidate(*t) for t in tuples]


def sig(c):
    return (round(c.snr, 5), round(c.freq, 7), c.nh, c.dm_idx, round(c.acc, 4))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_harmonic_distiller_matches_python(C, seed):
    rng = random.Random(seed)
    tup = random_cands(rng, 120)
    for keep, frac in ((False, True), (True, False), (True, True)):
        nat = C.HarmonicDistiller(1e-4, 16, keep, frac).distill(to_native(C, tup))
        py = py_distill([Cand(*t) for t in tup], harm_cond(1e-4, 16, keep, frac))
        assert [sig(c) for c in nat] == [sig(c) for c in py]
        if keep:
            assert [c.count_assoc() for c in nat] == [len(c.assoc) for c in py]


@pytest.mark.parametrize("seed", [3, 4])
def test_acceleration_and_dm_distillers_match_python(C, seed):
    rng = random.Random(seed)
    tup = random_cands(rng, 150)
    nat = C.AccelerationDistiller(41.94304, 1e-4, True).distill(to_native(C, tup))
    py = py_distill([Cand(*t) for t in tup], acc_cond(41.94304, 1e-4, True))
    assert [sig(c) for c in nat] == [sig(c) for c in py]
    assert [c.count_assoc() for c in nat] == [len(c.assoc) for c in py]
    nat = C.DMDistiller(1e-4, True).distill(to_native(C, tup))
    py = py_distill([Cand(*t) for t in tup], dm_cond(1e-4, True))
    assert [sig(c) for c in nat] == [sig(c) for c in py]


@pytest.mark.parametrize("seed", [5, 6])
def test_indexed_distillers_equal_reference_scan(C, seed):
    # above 64 candidates the distillers look fundamentals' relation windows up
    # in a frequency index; the output (order, assoc trees, multiplicity) must
    # equal the reference's O(n^2) scan exactly
    rng = random.Random(seed)
    tup = random_cands(rng, 1500, base_freqs=(0.37, 1.9, 4.0, 7.3, 11.1, 53.2, 210.0))
    tup += [(t[0], t[1], t[2], t[3], f32(t[4] + 0.5), f32(t[5] * (1 + 3e-4))) for t in tup[:200]]
    dists = [C.HarmonicDistiller(1e-4, 16, k, fr) for k, fr in ((True, True), (False, True), (True, False))]
    dists += [C.HarmonicDistiller(3e-3, 8, True, True), C.AccelerationDistiller(41.94304, 1e-4, True),
              C.AccelerationDistiller(600.0, 2e-4, True), C.DMDistiller(1e-4, True), C.DMDistiller(5e-3, True)]
    for d in dists:
        fast = d.distill(to_native(C, tup))
        slow = d.distill_reference(to_native(C, tup))
        assert 0 < len(fast) < len(tup)
        assert [[tuple(p) for p in c.pods()] for c in fast] == [[tuple(p) for p in c.pods()] for c in slow]


def test_keep_related_appends_once_per_match(C):
    # candidate at 2x the fundamental matches jj=2,kk=1 and jj=4,kk=2 (nh=1 -> 2 denominators)
    c = [C.Candidate(10, 1, 0, 1, 50.0, 1.0), C.Candidate(10, 1, 0, 1, 20.0, 2.0)]
    out = C.HarmonicDistiller(1e-4, 16, True, True).distill(c)
    assert len(out) == 1 and out[0].count_assoc() == 2


def test_scorer(C):
    cands = [C.Candidate(20.0, 6, 0.0, 4, 80.0, 4.0)]
    a1 = C.Candidate(23.0, 7, 0.0, 3, 70.0, 4.0)
    a2 = C.Candidate(100.0, 30, 0.0, 3, 10.0, 4.0)
    cands[0].assoc = [a1, a2]
    s = C.CandidateScorer(0.00032, 1475.12, -1.09, 1.09 * 64).score_all(cands)[0]
    assert s.is_physical  # always true for foff < 0
    assert s.is_adjacent  # has dm_idx + 1
    ftop, fbot = 1475.12 + 1.09 * 32, 1475.12 - 1.09 * 32
    ddm = 1.0 / (4.0 * 4150.0 * (1 / fbot ** 2 - 1 / ftop ** 2))
    inside = 1 + (abs(20 - 23) <= ddm) + (abs(20 - 100) <= ddm)
    assert s.ddm_count_ratio == pytest.approx(inside / 3)
    lone = C.CandidateScorer(0.00032, 1475.12, -1.09, 69.76).score_all([C.Candidate(1, 3, 0, 0, 9, 2)])[0]
    assert lone.is_adjacent and lone.ddm_count_ratio == 1.0


def test_identify_unique_peaks(C):
    rng = np.random.default_rng(5)
    idx = np.sort(rng.choice(100000, 2000, replace=False)).astype(np.int32)
    snr = rng.uniform(9, 30, size=2000).astype(np.float32)
    pi, ps = C.identify_unique_peaks(list(idx), list(snr), 30)
    exp = ref.unique_peaks(idx, snr, 30)
    assert list(zip(pi, ps)) == [(a, pytest.approx(b)) for a, b in exp]
    # gap measured from the last MAXIMUM: 0(10) 20(5) 45(4) -> one cluster? 45-0 >= 30 -> split
    pi, ps = C.identify_unique_peaks([0, 20, 45], [10.0, 5.0, 4.0], 30)
    assert pi == [0, 45]


def test_peak_bounds_match_reference(C):
    for nb, bw, nh in ((65537, 0.0238, 0), (65537, 0.0238, 3), (4194305, 0.00186, 3)):
        s, e, f = C.peak_bounds(nb, bw, nh, 0.1, 1100.0)
        rs, re_, rf = ref.peak_bounds(nb, bw, nh, 0.1, 1100.0)
        assert (s, e) == (rs, re_) and f == pytest.approx(rf, rel=1e-12)


def test_serialisation_roundtrip(C):
    a = C.Candidate(1.5, 2, -3.0, 4, 55.5, 3.25)
    a.folded_snr = 12.5
    a.opt_period = 0.3077
    a.fold = [float(i) for i in range(64 * 16)]
    a.nbins, a.nints = 64, 16
    b = C.Candidate(2.5, 3, 1.0, 1, 22.0, 6.5)
    b.assoc = [C.Candidate(3.5, 4, 0.0, 0, 11.0, 13.0)]
    a.assoc = [b]
    blob = C.serialize_candidates([a, b])
    back = C.deserialize_candidates(blob)
    assert len(back) == 2 and back[0].count_assoc() == 2 and back[0].fold == a.fold
    assert back[0].opt_period == a.opt_period and back[0].assoc[0].assoc[0].freq == 13.0
    assert [p[5] for p in back[0].pods()] == [3.25, 6.5, 13.0]
    assert C.deserialize_candidates(C.serialize_candidates([])) == []


def test_merge_candidate_blobs_equals_python_merge(C):
    """The native multi-rank merge (deserialise every rank's blob, stable sort
    by DM index, global DM + harmonic distillation and scoring) equals the
    step-by-step Python path, tree for tree; serialize_candidates reads the
    Python objects in place."""
    from conftest import TUTORIAL

    rng = random.Random(5)
    ok, _, args = C.parse_cmdline(["peasoup", "-i", TUTORIAL, "--dm_end", "250", "-n", "4"])
    hdr = dict(C.Filterbank.from_file(TUTORIAL).header)
    ranks = []
    for r in range(3):
        lst = []
        for _ in range(60):
            f = rng.choice([rng.uniform(1, 300), 4.0, 8.0, 33.3]) * (1 + rng.uniform(-2e-5, 2e-5))
            c = C.Candidate(rng.uniform(0, 250), rng.randrange(0, 59), rng.uniform(-5, 5), rng.randrange(0, 5),
                            rng.uniform(9, 90), f)
            c.assoc = [C.Candidate(1.0, c.dm_idx, 0.0, 1, rng.uniform(9, 20), f * 1.00001)] * rng.randrange(0, 3)
            lst.append(c)
        ranks.append(lst)
    blobs = [C.serialize_candidates(lst) for lst in ranks]
    got = C.merge_candidate_blobs(blobs, args, hdr)
    cands = []
    for b in blobs:
        cands.extend(C.deserialize_candidates(b))
    cands.sort(key=lambda c: c.dm_idx)
    exp = C.global_distill_and_score(cands, args, hdr)
    assert len(got) > 5
    assert C.serialize_candidates(got) == C.serialize_candidates(exp)


def test_compact_serialisation_of_search_stage_lists(C):
    """Lists of unfolded, unscored candidates use the 28-byte compact record
    (magic PSOD) and round-trip field for field; any folded or scored node
    switches the whole stream to the full form.  Streams over 8 MB rebuild on
    several threads (both forms)."""
    rng = random.Random(11)

    def tree(depth):
        c = C.Candidate(rng.uniform(0, 500), rng.randrange(0, 3000), rng.uniform(-500, 500), rng.randrange(0, 5),
                        rng.uniform(6, 60), rng.uniform(0.1, 900))
        if depth < 2:
            c.assoc = [tree(depth + 1) for _ in range(rng.randrange(0, 4))]
        return c

    def nodes(c):
        return 1 + sum(nodes(a) for a in c.assoc)

    def fields(c):
        return ((c.dm, c.dm_idx, c.acc, c.nh, c.snr, c.freq, c.folded_snr, c.opt_period, c.is_adjacent,
                 c.is_physical, c.ddm_count_ratio, c.ddm_snr_ratio, c.nbins, c.nints, list(c.fold)),
                [fields(a) for a in c.assoc])

    for n in (50, 80000):  # the second one: a > 8 MB stream in both forms
        lst = [tree(0) for _ in range(n)]
        blob = C.serialize_candidates(lst)
        assert blob[:4] == b"DOSP" and len(blob) == 12 + 28 * sum(map(nodes, lst))
        back = C.deserialize_candidates(blob)
        assert [fields(c) for c in back] == [fields(c) for c in lst]
        lst[n // 2].assoc[0].folded_snr = 12.5 if lst[n // 2].assoc else 0.0
        lst[n // 3].is_physical = True
        full = C.serialize_candidates(lst)
        assert full[:4] == b"COSP" and len(full) > len(blob)
        back = C.deserialize_candidates(full)
        assert [fields(c) for c in back] == [fields(c) for c in lst]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_accel_distill_slices_equals_whole_dm_distillation(C, seed):
    """Acceleration trials split into slices searched by different ranks
    (search.accel_units): joined per DM in slice order and acceleration-
    distilled (C.accel_distill_slices), the result equals distilling each
    DM's whole trial-ordered list -- whatever order the ranks' lists arrive in."""
    import random

    rng = random.Random(seed)
    tobs, tol = 42.0, 1e-4
    per_dm = {}
    for d in (3, 7, 8):
        lst = []
        for trial in range(40):  # plan order; each trial a few harmonic-distilled candidates
            acc = -5.0 + 0.25 * trial
            for _ in range(rng.randrange(0, 4)):
                f = rng.choice([4.0, 8.0, 12.5]) * (1 + rng.uniform(-2e-4, 2e-4))
                lst.append(C.Candidate(10.0 + d, d, acc, rng.randrange(0, 4), rng.uniform(6, 60), f))
        per_dm[d] = lst
    expect = []
    for d in sorted(per_dm):
        expect += C.AccelerationDistiller(tobs, tol, True).distill(list(per_dm[d]))
    S = 5
    units = []  # (rank-claimed unit, its candidates, slice index)
    for d, lst in per_dm.items():
        n = len(lst)
        for s in range(S):
            units.append((lst[s * n // S:(s + 1) * n // S], s))
    rng.shuffle(units)  # ranks return their units in any order
    cands, slices = [], []
    for lst, s in units:
        cands += lst
        slices += [s] * len(lst)
    got = C.accel_distill_slices(cands, slices, tobs, tol, 3)
    key = lambda c: (c.dm_idx, c.acc, c.nh, c.snr, c.freq, len(c.assoc))  # noqa: E731
    assert [key(c) for c in got] == [key(c) for c in expect]
    assert [[key(a) for a in c.assoc] for c in got] == [[key(a) for a in c.assoc] for c in expect]
