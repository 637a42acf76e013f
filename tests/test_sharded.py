"""Pair-sharded forward in the product API (``fpm.parallel.ShardedNet``): contiguous
pair ranges, one host thread + streams per device, one shared Hungarian pool, one gather.  On the
one-GPU box the device list repeats cuda:0 (shards run concurrently on it); the gathered outputs
must equal the single-device forward bit for bit."""
import numpy as np
import pytest
import torch

import fpm
from fpm import params, synth
from fpm.batch import DeviceBatch
from fpm.parallel import ShardedNet, shard_bounds

DEV = torch.device("cuda", 0)


def test_shard_bounds():
    assert shard_bounds(1024, 8) == [(i * 128, (i + 1) * 128) for i in range(8)]
    assert shard_bounds(10, 4) == [(0, 3), (3, 6), (6, 8), (8, 10)]
    assert shard_bounds(2, 4) == [(0, 1), (1, 2)]            # empty shards dropped
    b = shard_bounds(10001, 8)
    assert b[0][0] == 0 and b[-1][1] == 10001 and all(x[1] == y[0] for x, y in zip(b, b[1:]))
    assert max(e - s for s, e in b) - min(e - s for s, e in b) <= 1


def test_batch_split_range_keeps_padding():
    """A shard keeps the parent's padded sizes and renumbers its edges from 0 (host-only check on
    CPU tensors)."""
    pairs = synth.make_batch(3, 5, [20, 24, 18, 24, 22], n2=[24, 19, 24, 21, 24])
    bt = DeviceBatch.from_pairs(pairs, torch.device("cpu"))
    sub = bt.split_range(1, 4)
    assert sub.B == 3 and sub.nmax == bt.nmax and sub.pair_range == (1, 4)
    for side in range(2):
        e0 = int(bt.edge_off[side][1])
        e1 = int(bt.edge_off[side][4])
        nm = bt.nmax[side]
        assert torch.equal(sub.src[side], bt.src[side][e0:e1] - nm)
        assert torch.equal(sub.x[side], bt.x[side][nm:4 * nm])
    with pytest.raises(ValueError):
        bt.split_range(3, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,devices", [("bf16", [0, 0]), ("f32", [0, 0, 0])])
def test_sharded_equals_single_device(dtype, devices):
    sd = params.init_params(7)
    pairs = synth.make_batch(41, 7, [48, 40, 44, 48, 30, 48, 47], n2=[48, 48, 44, 41, 48, 36, 48])
    net = fpm.Net(regression=True, dtype=dtype, backbone=False)
    net.load_state_dict(sd)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    ref = net.run(bt)
    sh = ShardedNet(net, devices=devices)
    out = sh.run(bt)
    for k in ("s", "ss", "ds_mat", "perm_mat", "k_prob", "cls_prob"):
        assert out[k].device == DEV
        assert torch.equal(out[k], ref[k]), k
    assert float(out["ks_loss"]) == pytest.approx(float(ref["ks_loss"]), abs=1e-7)
    assert len(sh.last_timing["bounds"]) == len(devices)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [96, 300])
def test_sharded_equals_single_device_fp32_chain(n):
    """Boxes above the fp64 k chain's 64 keypoints: the fp32 GNN / Sinkhorn kernels under ShardedNet's
    HIP-graph replay equal the eager single-device forward bit for bit -- at n = 300 incl. the
    split streaming Sinkhorn (its workspace allocated and its counters zeroed inside the captured
    graphs) and the GNN layers' Hilbert block order."""
    sd = params.init_params(8)
    pairs = synth.make_batch(44, 5, [n, n - 7, n, n - 20, n], n2=[n, n, n - 11, n, n - 3])
    net = fpm.Net(regression=True, dtype="bf16", backbone=False)
    net.load_state_dict(sd)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    assert (bt.ord2 is not None) == (n > 256)
    ref = net.run(bt)
    sh = ShardedNet(net, devices=[0, 0])
    for _ in range(2):                              # capture, then replay
        out = sh.run(bt)
        for k in ("s", "ss", "ds_mat", "perm_mat", "k_prob", "cls_prob"):
            assert torch.equal(out[k], ref[k]), (k, n)


@pytest.mark.gpu
def test_sharded_forward_data_dict():
    """The reference call shape: ShardedNet(net)(data_dict) -> data_dict with the reference keys,
    equal to Net(data_dict) (gt_perm_mat / label sliced per shard, losses over the whole batch)."""
    sd = params.init_params(5)
    pairs = synth.make_batch(42, 5, 40, n2=[40, 33, 40, 38, 40])
    B = len(pairs)

    def dd():
        d = {"ns": [torch.tensor([p[s]["n"] for p in pairs]) for s in range(2)], "pyg_graphs": [],
             "node_features": [], "global_features": []}

        class G:
            pass
        for side in range(2):
            g = G()
            offs = np.cumsum([0] + [p[side]["n"] for p in pairs])
            g.edge_index = torch.from_numpy(np.concatenate([p[side]["edge_index"] + offs[b]
                                                            for b, p in enumerate(pairs)], 1))
            g.edge_attr = torch.from_numpy(np.concatenate([p[side]["pseudo"] for p in pairs]))
            g.ptr = torch.from_numpy(offs)
            d["pyg_graphs"].append(g)
            d["node_features"].append(torch.from_numpy(np.concatenate([p[side]["x"] for p in pairs])))
            d["global_features"].append(torch.from_numpy(np.stack([p[side]["w"] for p in pairs])))
        gt = torch.zeros(B, 40, 40)
        for b in range(B):
            m = min(pairs[b][0]["n"], pairs[b][1]["n"])
            gt[b, range(m), range(m)] = 1
        d["gt_perm_mat"] = gt
        d["label"] = torch.tensor([1.0, 0.0, 1.0, 1.0, 0.0])
        return d

    net = fpm.Net(regression=True, backbone=False)
    net.load_state_dict(sd)
    ref = net(dd())
    out = ShardedNet(net, devices=[0, 0])(dd())
    for k in ("ds_mat", "perm_mat", "k_prob", "cls_prob"):
        assert torch.equal(out[k], ref[k]), k
    for k in ("ks_loss", "ks_error", "cls_loss"):
        assert float(out[k]) == pytest.approx(float(ref[k]), rel=1e-6, abs=1e-7), k


@pytest.mark.gpu
def test_sharded_host_enqueue_flat():
    """ShardedNet's device threads replay per-shard HIP graphs (captured once per batch object): the
    host CPU time spent enqueueing (summed over the device threads: the GIL-serialised part) per
    1024 pairs stays far below the ~8 ms of eager launches at C3 as the shard count grows -- one
    shard of 1024 pairs vs four shards of 1024 pairs each -- and the outputs stay equal to the
    single-device forward."""
    sd = params.init_params(7)
    pairs = synth.make_batch(43, 4096, 32)
    net = fpm.Net(regression=True, dtype="bf16", backbone=False)
    net.load_state_dict(sd)
    bt4 = DeviceBatch.from_pairs(pairs, DEV)
    bt1 = bt4.split_range(0, 1024)
    ref = net.run(bt1)
    enq = {}
    for n, bt in ((1, bt1), (4, bt4)):
        sh = ShardedNet(net, devices=[0] * n)
        for rep in range(4):
            out = sh.run(bt)
            if rep == 0:
                for k in ("ds_mat", "perm_mat", "k_prob", "cls_prob"):
                    assert torch.equal(out[k][:1024], ref[k]), (n, k)
            else:
                enq[n] = min(enq.get(n, 1.0), sh.last_timing["enqueue_cpu_s"])
        assert all(t["graphs"] for t in sh.last_timing["shards"])
    per1, per4 = enq[1] * 1e3, enq[4] / 4 * 1e3
    print("enqueue CPU per 1024 pairs: 1 shard %.2f ms, 4 shards %.2f ms" % (per1, per4))
    assert per4 < max(3.0 * per1, 2.0), (per1, per4)


@pytest.mark.gpu
@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two or more GPUs (distinct devices)")
def test_sharded_distinct_devices_equal_single_device():
    """Real cross-device sharding (peer copies of the shards, per-device streams and graphs, the
    gather's peer copies into the output device): equal to the single-device forward bit for bit.
    Runs on the first multi-GPU box (the one-GPU pool skips it)."""
    sd = params.init_params(7)
    pairs = synth.make_batch(45, 10, [48, 40, 44, 48, 30, 48, 47, 41, 48, 36], n2=[48, 47, 40, 30, 48, 44, 48, 48, 39, 48])
    net = fpm.Net(regression=True, dtype="bf16", backbone=False)
    net.load_state_dict(sd)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    ref = net.run(bt)
    devices = list(range(min(4, torch.cuda.device_count())))
    sh = ShardedNet(net, devices=devices)
    for _ in range(2):
        out = sh.run(bt)
        for k in ("s", "ss", "ds_mat", "perm_mat", "k_prob", "cls_prob"):
            assert out[k].device == DEV
            assert torch.equal(out[k], ref[k]), k


@pytest.mark.gpu
def test_sharded_recaptures_after_weight_and_tau_change():
    """Replicas replay HIP graphs captured per batch object; a weight change (as an optimizer step
    makes) or a new tau between two forwards on the SAME batch must be seen: ShardedNet re-captures
    stale graphs on the calling thread before its device threads start, and the outputs equal an
    eager single-device forward with the new weights."""
    sd = params.init_params(7)
    pairs = synth.make_batch(44, 512, 32)
    net = fpm.Net(regression=True, dtype="bf16", backbone=False)
    net.load_state_dict(sd)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    sh = ShardedNet(net, devices=[0, 0])
    first = sh.run(bt)
    with torch.no_grad():
        net.classifier.weight.mul_(1.5)
    net.tau = 0.02
    out = sh.run(bt)
    assert all(t["graphs"] for t in sh.last_timing["shards"])
    ref = net.run(bt)
    assert not torch.equal(out["ds_mat"], first["ds_mat"])
    for k in ("ds_mat", "perm_mat", "k_prob", "cls_prob"):
        assert torch.equal(out[k], ref[k]), k
