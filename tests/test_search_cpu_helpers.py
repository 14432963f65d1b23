"""CPU checks of the search driver's host-side helpers."""
import pytest

from peasoup_amd.models.search import RankSearcher


@pytest.mark.parametrize("lo,hi,chunk", [(0, 100, 32), (5, 70, 32), (31, 33, 32), (64, 128, 64), (7, 8, 32)])
def test_chunk_ranges_cut_at_tile_multiples(lo, hi, chunk):
    blocks = RankSearcher.chunk_ranges(range(lo, hi), chunk)
    assert blocks[0][0] == lo and blocks[-1][1] == hi
    for (a0, a1), (b0, _) in zip(blocks, blocks[1:]):
        assert a1 == b0
    for d0, d1 in blocks[1:]:
        assert d0 % chunk == 0
    for d0, d1 in blocks:
        assert 0 < d1 - d0 <= chunk
        assert d1 == hi or d1 % chunk == 0


def test_chunk_ranges_empty_and_noncontiguous():
    assert RankSearcher.chunk_ranges([], 32) == []
    with pytest.raises(AssertionError):
        RankSearcher.chunk_ranges([0, 1, 3], 32)


def test_dm_schedule_option():
    """--dm_schedule: dynamic is the multi-rank default, auto on a single rank
    is static (in-order chunks), an explicit dynamic runs the queue even on
    one rank, bad values are rejected."""
    from peasoup_amd import _C
    from peasoup_amd.models.search import dm_schedule

    ok, _, a = _C.parse_cmdline(["peasoup", "-i", "x.fil"])
    assert ok and a.dm_schedule == "auto"
    assert dm_schedule(a, 1) == "static" and dm_schedule(a, 8) == "dynamic"
    assert dm_schedule(a, 8, 2026) == "dynamic"  # 64 chunks >= 4 per rank
    assert dm_schedule(a, 8, 113) == "static"    # 4 chunks for 8 ranks
    assert dm_schedule(a, 2, 225) == "dynamic" and dm_schedule(a, 2, 224) == "static"  # 8 vs 7 chunks
    ok, _, a = _C.parse_cmdline(["peasoup", "-i", "x.fil", "--dm_schedule", "static"])
    assert ok and dm_schedule(a, 8) == "static"
    ok, _, a = _C.parse_cmdline(["peasoup", "-i", "x.fil", "--dm_schedule", "dynamic"])
    assert ok and dm_schedule(a, 1) == "dynamic" and dm_schedule(a, 8, 64) == "dynamic"
    a.dm_schedule = "roundrobin"
    with pytest.raises(ValueError):
        dm_schedule(a, 2)


def test_dynamic_blocks_cover_the_dm_list_once():
    """The dynamic schedule's block grid (claimed first-come by the ranks)
    covers every DM exactly once, in 32-DM tile-aligned chunks."""
    from peasoup_amd.models.search import DYNAMIC_CHUNK

    for ndm in (1, 31, 32, 59, 2026):
        blocks = RankSearcher.chunk_ranges(range(ndm), DYNAMIC_CHUNK)
        assert [d for b in blocks for d in range(*b)] == list(range(ndm))
        assert all(b[0] % DYNAMIC_CHUNK == 0 for b in blocks)


def test_time_shards_option():
    """--time_shards (Python driver: halo exchange + all-to-all corner turn)."""
    from peasoup_amd import _C

    ok, _, a = _C.parse_cmdline(["peasoup", "-i", "x.fil"])
    assert ok and a.time_shards is False
    ok, _, a = _C.parse_cmdline(["peasoup", "-i", "x.fil", "--time_shards"])
    assert ok and a.time_shards is True


def test_sort_order_by_folded_snr_is_the_sort_permutation():
    """The fold merge reorders the Python candidate list by the permutation
    sort_by_folded_snr (std::sort, unstable) applies: equal keys included."""
    import numpy as np

    from peasoup_amd import _C

    rng = np.random.default_rng(4)
    for n in (1, 5, 17, 300, 2000):
        cands = []
        for i in range(n):
            c = _C.Candidate(1.0, i, 0.0, 0, float(rng.integers(9, 14)), float(i + 1))
            c.folded_snr = float(rng.integers(0, 16)) if rng.random() < 0.5 else 0.0
            cands.append(c)
        ref = [c.freq for c in _C.sort_by_folded_snr(cands)]
        order = _C.sort_order_by_folded_snr([c.snr for c in cands], [c.folded_snr for c in cands])
        assert [cands[i].freq for i in order] == ref


def test_resident_rows_lookup_and_fold_owners(monkeypatch):
    """keep_trials bookkeeping: row lookup inside kept blocks, the owner map of
    a single rank, and the PSOUP_KEEP_TRIALS override of the memory rule."""
    import types

    import torch

    from peasoup_amd.models import search as S

    rs = types.SimpleNamespace(row_stride=4, resident_rows={}, ctx=types.SimpleNamespace(device=torch.device("cpu")))
    rs.resident_rows[0] = (3, torch.arange(12, dtype=torch.uint8))
    rs.resident_rows[32] = (34, torch.arange(100, 108, dtype=torch.uint8))
    row = S.RankSearcher.resident_row(rs, 2)
    assert row.tolist() == [8, 9, 10, 11]
    assert S.RankSearcher.resident_row(rs, 33).tolist() == [104, 105, 106, 107]
    assert S.RankSearcher.resident_row(rs, 3) is None and S.RankSearcher.resident_row(rs, 31) is None
    assert S.RankSearcher.resident_dms(rs) == [0, 1, 2, 32, 33]
    ctx = types.SimpleNamespace(world_size=1, rank=0)
    assert S.fold_owners(rs, ctx) == {0: 0, 1: 0, 2: 0, 32: 0, 33: 0}
    assert S.keep_trials_fits(rs, 100, 1) is False  # no GPU: never kept
    monkeypatch.setenv("PSOUP_KEEP_TRIALS", "1")
    assert S.keep_trials_fits(rs, 100, 1) is True
    monkeypatch.setenv("PSOUP_KEEP_TRIALS", "0")
    assert S.keep_trials_fits(rs, 100, 1) is False
