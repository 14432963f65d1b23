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
