"""Host-side batching logic (CPU): pipeline splits cover every pair exactly once."""
import pytest
import torch

from fpm import synth
from fpm.batch import DeviceBatch


@pytest.mark.parametrize("k,tail", [(1, 0), (3, 0), (3, 1), (8, 1), (2, 2), (7, 3)])
def test_split_covers_all_pairs(k, tail):
    pairs = synth.make_batch(9, 7, [20, 18, 20, 19, 20, 17, 20])
    bt = DeviceBatch.from_pairs(pairs, torch.device("cpu"))
    parts = bt.split(k, tail)
    ranges = [getattr(p, "pair_range", (0, bt.B)) for p in parts]
    assert ranges[0][0] == 0 and ranges[-1][1] == bt.B
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    assert sum(p.B for p in parts) == bt.B
    for p, (b0, b1) in zip(parts, ranges):
        assert p.B == b1 - b0 and p.nmax == bt.nmax
        for side in range(2):
            assert p.E[side] == int(bt.edge_off[side][b1] - bt.edge_off[side][b0])
