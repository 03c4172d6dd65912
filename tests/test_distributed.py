"""The multi-GPU exchange protocol (facerecognition_amd/distributed.py) on CPU with
gloo, world_size 2: all-gather of embeddings → shard-local top-k with global indices → all-gather of
candidates → merge.  The merged result must equal the single-device exact top-k over the whole
gallery bit for bit, including ties that straddle shard boundaries.

Scores are made exact (entries are multiples of 1/8 with small magnitude, so every f32 dot product is
exact whatever the accumulation order), hence a bit-exact comparison is meaningful."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle.match import merge_topk, topk_dot

D, B, K, ROWS = 64, 6, 5, 203


def _data():
    rng = np.random.default_rng(5)
    G = (rng.integers(-4, 5, size=(ROWS, D)) / 8).astype(np.float32)
    G[150] = G[17]            # exact tie across the shard boundary (rank 0 row vs rank 1 row)
    G[101] = G[100]           # tie inside one shard... and at the boundary for world 2 (101 = split)
    P = (rng.integers(-4, 5, size=(2 * B, D)) / 8).astype(np.float32)
    P[3] = G[17]              # probe whose best match is the tied pair
    P[7] = G[100]
    return G, P


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from facerecognition_amd.distributed import ShardedMatcher, shard_range

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        G, P = _data()
        lo, hi = shard_range(ROWS, rank, world)
        shard = G[lo:hi]

        def local_search(probes, out_s, out_i):
            s, i = topk_dot(probes.numpy(), shard, K)
            i = np.where(i >= 0, i + lo, -1)
            out_s.copy_(torch.from_numpy(s))
            out_i.copy_(torch.from_numpy(i.astype(np.int32)))

        def merge(xchg, k, out_s, out_i):
            # the all-gathered exchange block [world, 2, P, k] decoded back into [P, world, k] lists
            x = xchg.numpy()
            cs = x[:, 0].view(np.float32).transpose(1, 0, 2)
            ci = x[:, 1].transpose(1, 0, 2)
            s, i = merge_topk(np.ascontiguousarray(cs), np.ascontiguousarray(ci), k)
            out_s.copy_(torch.from_numpy(s))
            out_i.copy_(torch.from_numpy(i.astype(np.int32)))

        m = ShardedMatcher(B, D, K, local_search, torch.device("cpu"), merge=merge)
        bufs = (m.send.data_ptr(), m.xchg.data_ptr(), m.out_s.data_ptr())
        s, i = m.search(torch.from_numpy(P[rank * B:(rank + 1) * B]))
        s2, i2 = m.search(torch.from_numpy(P[rank * B:(rank + 1) * B]))  # buffers reused, same answer
        assert (m.send.data_ptr(), m.xchg.data_ptr(), m.out_s.data_ptr()) == bufs
        assert torch.equal(s, s2) and torch.equal(i, i2)
        s, i = s.clone(), i.clone()
        # short last batches, a different count per rank: masked rows ride along
        n = B - 2 + rank
        ss, si = m.search(torch.from_numpy(P[rank * B:rank * B + n]))
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), s=s.numpy(), i=i.numpy(), ss=ss.numpy(), si=si.numpy(),
                 valid=m.valid.numpy())
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_partitions_rows():
    from facerecognition_amd.distributed import shard_range
    for rows in (0, 1, 7, 203, 10000):
        for world in (1, 2, 3, 8):
            r = [shard_range(rows, k, world) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == rows
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
            assert max(h - l for l, h in r) - min(h - l for l, h in r) <= 1


def test_merge_oracle_matches_global_topk():
    G, P = _data()
    lists = [topk_dot(P, G[lo:hi], K) for lo, hi in ((0, 90), (90, 91), (91, ROWS))]
    cs = np.stack([s for s, _ in lists], 1)
    ci = np.stack([np.where(i >= 0, i + lo, -1) for (_, i), lo in zip(lists, (0, 90, 91))], 1)
    s, i = merge_topk(cs, ci, K)
    gs, gi = topk_dot(P, G, K)
    assert np.array_equal(i, gi) and np.array_equal(s, gs)


@pytest.mark.timeout(180)
def test_sharded_match_world2_gloo_equals_single_device():
    G, P = _data()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        r0, r1 = (np.load(os.path.join(d, f"r{r}.npz")) for r in (0, 1))
        gs, gi = topk_dot(P, G, K)
        for r in (r0, r1):  # every rank holds the full, identical answer
            assert np.array_equal(r["i"], gi.astype(np.int32))
            assert np.array_equal(r["s"], gs)
        assert list(gi[3][:2]) == [17, 150] and list(gi[7][:2]) == [100, 101]
        # short batches: rank j sent B - 2 + j probes; its valid rows are the single-device answer, the rest
        # (-inf, -1)
        valid = np.zeros(2 * B, bool)
        for j in (0, 1):
            valid[j * B:j * B + B - 2 + j] = True
        for r in (r0, r1):
            assert np.array_equal(r["valid"], valid)
            assert np.array_equal(r["si"][valid], gi[valid].astype(np.int32))
            assert np.array_equal(r["ss"][valid], gs[valid])
            assert (r["si"][~valid] == -1).all() and np.isneginf(r["ss"][~valid]).all()


def test_world1_short_batch_and_one_argument_search():
    """World 1 (no process group): a batch shorter than the constructor's works, results are the matcher's views
    of that many rows, and the round-3 one-argument local_search(probes) -> (scores, idx) is still accepted."""
    from facerecognition_amd.distributed import ShardedMatcher
    G, P = _data()

    def three(probes, out_s, out_i):
        s, i = topk_dot(probes.numpy(), G, K)
        out_s.copy_(torch.from_numpy(s))
        out_i.copy_(torch.from_numpy(i.astype(np.int32)))

    def one(probes):
        s, i = topk_dot(probes.numpy(), G, K)
        return torch.from_numpy(s), torch.from_numpy(i.astype(np.int32))

    def defaulted(probes, out_s=None, out_i=None):  # three positional parameters: the three-argument form
        assert out_s is not None and out_i is not None
        three(probes, out_s, out_i)

    gs, gi = topk_dot(P, G, K)
    for fn in (three, one, defaulted):
        m = ShardedMatcher(B, D, K, fn, torch.device("cpu"))
        s, i = m.search(torch.from_numpy(P[:B]))
        assert np.array_equal(i.numpy(), gi[:B]) and np.array_equal(s.numpy(), gs[:B])
        s, i = m.search(torch.from_numpy(P[:B - 2]))  # a short last batch
        assert s.shape == (B - 2, K) and np.array_equal(i.numpy(), gi[:B - 2])
        with pytest.raises(ValueError):
            m.search(torch.from_numpy(P[:B + 1]))
