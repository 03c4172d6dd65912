"""World-2 sharded match on the GPU (facerecognition_amd/distributed.py).

Two rank processes share cuda:0, each holding half of a 250k-row gallery (the bf16x3 candidate path
with exact rescoring, fr_match_topk with index_base) and merging with fr_topk_merge.  Every rank's
merged answer must equal the single-device top-k over the whole gallery bit for bit, including exact
ties that straddle the shard boundary (lowest global index first)."""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_world2(mode):
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
        procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_gpu_worker.py"), str(r), "2", d, mode],
                                  env=env) for r in range(2)]
        try:
            codes = [p.wait(timeout=200) for p in procs]
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        assert codes == [0, 0], f"rank exit codes {codes}"
        return [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in (0, 1)]


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_world2_native_exchange_equals_single_device():
    import dist_gpu_worker as W
    from facerecognition_amd.gallery import DeviceGallery

    r0, r1 = _run_world2("ties")

    dev = torch.device("cuda", 0)
    G, P = W.data(dev)
    gal = DeviceGallery(device=0)
    gal.set_device_rows(G)
    s, i = gal.search_device(P, W.K)
    gs, gi = s.cpu().numpy(), i.cpu().numpy()
    for r in (r0, r1):  # every rank holds the full, identical answer
        assert np.array_equal(r["i"], gi)
        assert np.array_equal(r["s"].view(np.uint32), gs.view(np.uint32))
    assert list(gi[0][:3]) == [7, 124_999, 125_000]
    assert list(gi[W.B + 1][:2]) == [125_003, 200_001]
    # and the single-device answer itself agrees with a float64 host check of the ranking
    Gh, Ph = G.cpu().double().numpy(), P.cpu().double().numpy()
    S = Ph @ Gh.T
    top1 = np.argmax(S, axis=1)
    assert np.array_equal(gi[:, 0], top1)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_world2_config4_shape_equals_single_device():
    """BASELINE config 4's exchange at its per-rank shape on the one GPU of the test box: 256 probes per
    rank gathered to 512, against the 1M-row gallery split in two (500k rows per rank, bf16x3 candidates
    + exact rescoring per shard).  Every rank's merged top-5 equals the single-device top-5 over the
    whole 1M rows bit for bit, and top-1 equals a chunked float64 host argmax where the gap allows."""
    import dist_gpu_worker as W
    from facerecognition_amd.gallery import DeviceGallery

    r0, r1 = _run_world2("config4")
    dev = torch.device("cuda", 0)
    G, P = W.data_config4(dev, 0, W.C4_ROWS)
    gal = DeviceGallery(device=0)
    gal.set_device_rows(G)
    s, i = gal.search_device(P, W.K)
    gs, gi = s.cpu().numpy(), i.cpu().numpy()
    for r in (r0, r1):
        assert np.array_equal(r["i"], gi)
        assert np.array_equal(r["s"].view(np.uint32), gs.view(np.uint32))
    planted = np.arange(128) * 7_777 + 3
    assert np.array_equal(gi[np.r_[0:64, 256:320], 0], planted)
    Gh, Ph = G.cpu().double().numpy(), P.cpu().double().numpy()
    best, second = np.full(len(Ph), -np.inf), np.full(len(Ph), -np.inf)
    arg = np.zeros(len(Ph), np.int64)
    for c in range(0, len(Gh), 125_000):  # chunked float64 argmax with the lowest-index tie rule
        S = Ph @ Gh[c:c + 125_000].T
        a = np.argmax(S, axis=1)
        m = S[np.arange(len(S)), a]
        S[np.arange(len(S)), a] = -np.inf
        m2 = S.max(axis=1)
        upd = m > best
        second = np.where(upd, np.maximum(best, m2), np.maximum(second, m))
        arg, best = np.where(upd, a + c, arg), np.where(upd, m, best)
    clear = best - second > 1e-5
    assert clear.mean() > 0.9
    assert np.array_equal(gi[clear, 0], arg[clear])
    print(f"config4 world-2: {int(r0['fallbacks'])}+{int(r1['fallbacks'])} rank fallbacks, "
          f"{int((~clear).sum())} near-tie probes of {len(Ph)}")
