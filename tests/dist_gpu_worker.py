"""One rank of the world-2 sharded-match check (tests/test_gpu_distributed.py), run as its own process.

Both ranks share cuda:0 (the test box has one GPU), so the collectives run on gloo staged through host
memory; the data path is the product one: DeviceGallery.search_device (fr_match_topk with the rank's
index_base) for the shard-local top-k and native_merge_ranks (fr_topk_merge_ranks) for the merge."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ROWS, B, K, D = 250_000, 64, 5, 512


def data(dev):
    """Gallery [ROWS, D] and probes [2B, D] (rank r owns probes [rB, rB+B)), with ties that straddle
    the world-2 shard boundary (row 125000)."""
    from facerecognition_amd.synthetic import synthetic_gallery_rows
    G = synthetic_gallery_rows(0, ROWS, dev, seed=7)
    G[124_999] = G[7]        # rank 0 rows 7 and 124999, rank 1 row 125000: a three-way exact tie
    G[125_000] = G[7]
    G[200_001] = G[125_003]  # tie inside rank 1 against a rank-1 row
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    P = torch.randn((2 * B, D), generator=g, device=dev)
    P /= P.norm(dim=1, keepdim=True)
    P[0] = G[7]                                   # rank 0 probe → the three-way tie
    P[B + 1] = G[125_003]                         # rank 1 probe → tie (125003, 200001)
    P[B + 2] = G[124_999] * 0.75 + P[B + 2] * 0.25
    P[B + 2] /= P[B + 2].norm()
    return G, P


C4_ROWS, C4_B = 1_000_000, 256  # BASELINE config 4 per-rank probe count against its 1M-row gallery


def data_config4(dev, lo, hi):
    """Config-4 shape: rows [lo, hi) of the 1M-row synthetic gallery (generated per shard, identical
    whatever the sharding) and 2 x 256 probes, the first 64 of each rank planted near gallery rows spread
    over both shards."""
    from facerecognition_amd.synthetic import synthetic_gallery_rows
    G = synthetic_gallery_rows(lo, hi, dev, seed=11)
    g = torch.Generator(device=dev)
    g.manual_seed(123)
    P = torch.randn((2 * C4_B, D), generator=g, device=dev)
    planted = torch.arange(128, device=dev) * 7_777 + 3
    rows = synthetic_gallery_rows(0, C4_ROWS, dev, seed=11)[planted] if hi - lo < C4_ROWS else G[planted]
    for r in range(2):
        P[r * C4_B:r * C4_B + 64] = rows[r * 64:(r + 1) * 64] + 0.05 * P[r * C4_B:r * C4_B + 64] / D ** 0.5
    P /= P.norm(dim=1, keepdim=True)
    return G, P


def main():
    rank, world, out_dir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    mode = sys.argv[4] if len(sys.argv) > 4 else "ties"
    import torch.distributed as dist
    from facerecognition_amd.distributed import ShardedMatcher, shard_range
    from facerecognition_amd.gallery import DeviceGallery

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows, b = (C4_ROWS, C4_B) if mode == "config4" else (ROWS, B)
        lo, hi = shard_range(rows, rank, world)
        if mode == "config4":
            Gs, P = data_config4(dev, lo, hi)
        else:
            G, P = data(dev)
            Gs = G[lo:hi].contiguous()
        gal = DeviceGallery(device=0, index_base=lo)
        gal.set_device_rows(Gs)
        m = ShardedMatcher(b, D, K, lambda p, s, i: gal.search_device(p, K, s, i), dev)  # merge = native_merge_ranks
        s, i = m.search(P[rank * b:(rank + 1) * b].contiguous())
        torch.cuda.synchronize(dev)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), s=s.cpu().numpy(), i=i.cpu().numpy(),
                 fallbacks=gal.fallbacks())
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
