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


def test_hilbert_block_order():
    """DeviceBatch.ord2 (the GNN layers' graph-2 block order for boxes over 256 keypoints): a
    permutation per pair, padding slots last in index order, spatially local (consecutive keypoints
    ~10x closer than in generation order); carried by sub-batches; absent at or below 256."""
    import numpy as np
    from fpm.batch import hilbert_order
    n2 = [300, 280, 300]
    pairs = synth.make_batch(5, 3, [40, 40, 40], n2=n2)
    bt = DeviceBatch.from_pairs(pairs, torch.device("cpu"))
    assert bt.ord2 is not None and tuple(bt.ord2.shape) == (3, 300) and bt.ord2.dtype == torch.int32
    for b, p in enumerate(pairs):
        o = bt.ord2[b].tolist()
        assert sorted(o) == list(range(300))
        n = p[1]["n"]
        assert o[n:] == list(range(n, 300))
        P = p[1]["P"]
        step = np.linalg.norm(np.diff(P[o[:n]], axis=0), axis=1).mean()
        base = np.linalg.norm(np.diff(P, axis=0), axis=1).mean()
        assert step < base / 5, (step, base)
    sub = bt.split_range(1, 3)
    assert torch.equal(sub.ord2, bt.ord2[1:3])
    small = DeviceBatch.from_pairs(synth.make_batch(5, 2, 64), torch.device("cpu"))
    assert small.ord2 is None
    # a 2 x 2 grid in Hilbert order (0,0) (0,1) (1,1) (1,0)
    P = torch.tensor([[[0.0, 0.0], [319.0, 0.0], [0.0, 239.0], [319.0, 239.0]]])
    assert hilbert_order(P, [4], 4)[0].tolist() == [0, 2, 3, 1]
