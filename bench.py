#!/usr/bin/env python3
"""Headline benchmark: aligned faces/sec, embed + match, IResNet100 @112, bs=256 per GPU.

BASELINE.json metric "aligned faces/sec (embed+match) ArcFace@112 bs=256, 1/2/4/8 MI355X",
workload = configs[1] (IResNet100 bf16 bs=256 on one MI355X, 10k x 512 gallery, top-k match).

One step = one pass of the hot path over one batch of HBM-resident synthetic u8 crops:
  fr_embed (preprocess → IResNet100 forward → folded head → L2 norm)  [libfrhip.so]
  N > 1: RCCL all-gather of the normalized embeddings
  fr_match_topk of all gathered probes against this rank's gallery shard (global indices)
  N > 1: RCCL all-gather of the per-shard top-k candidates + fr_topk_merge
Weak scaling: every rank embeds 256 faces; the gallery is row-sharded across ranks.
value = faces embedded by all ranks / max-over-ranks wall time of the timed steps.

Launch: python bench.py --gpus N --steps K --warmup W
  N > 1 either under torch.distributed.run (RANK/WORLD_SIZE set), or directly: the parent process then
  never touches the GPU and starts N fresh child processes, one per GPU, with RANK/LOCAL_RANK/
  WORLD_SIZE/MASTER_ADDR=127.0.0.1/MASTER_PORT set (launch_ranks).
  Gallery default: 10k rows at N = 1 (BASELINE config 2), 1M rows at N > 1 (config 4: bs 2048 over 8
  GPUs, 125k rows per rank).
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "aligned faces/sec (embed+match) ArcFace@112 bs=256, 1/2/4/8 MI355X"
GFLOP_PER_FACE = {"iresnet100": 24.179, "resnet50_arcface": 2.154, "irv1_facenet": 2.835}
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16/f16 MFMA
FP8_DENSE_PEAK_TFLOPS = 5000.0  # MI355X_MICROARCH.md: ~5 PF dense fp8 (block-scaled f8f6f4 MFMA)
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s spec (about 6.3 TB/s achievable)


def class_peak(name):
    """Dense MFMA peak of a kernel class: the e4m3 classes (the per-conv fp8 kernel and the fp8 layer3 stage,
    engine.cpp "stage8 layer3") run on the block-scaled f8f6f4 MFMA, everything else on bf16 / f16."""
    return FP8_DENSE_PEAK_TFLOPS if name.startswith(("conv_fp8", "stage8")) else BF16_DENSE_PEAK_TFLOPS
C4_ROWS = 1_000_000  # BASELINE config 4's gallery (the N > 1 default)
PROF_STRIDE = 8  # roofline: sample every 8th dominant-kernel launch (event overhead ~0.5 % instead of ~4 %)


# bench kernel class (fr_prof_get name prefix) -> rocprofv3 kernel-name fragment of its dispatches (only
# classes whose kernel instantiation serves no other class: the two conv_rows classes share one)
CLASS_KERNEL = [("stage layer3", ("::stage13_kernel", "::stage_kernel<")), ("stage layer2", ("SplitGeo<28,",)),
                ("stage layer1", ("SplitGeo<56,",)), ("conv_wring", ("conv_wring_kernel<",)),
                ("stem u8 fused", ("stem_u8_kernel<",)), ("conv_fp8", ("conv_fp8_kernel<",)),
                ("stage8 layer3", ("::stage8_kernel",))]


def pmc_passes(args):
    """HBM traffic of THIS build, measured live: two separate rocprofv3 --pmc passes (FETCH_SIZE, then
    WRITE_SIZE; never combined with a tracing domain) over a short child run of this same bench
    configuration, started before this process touches the GPU.  Returns ({rocprof kernel name:
    (fetch bytes, write bytes, dispatches)}, None) or (None, reason).  Corrections per
    MI355X_MICROARCH.md's HBM section: both counters are in KiB and FETCH_SIZE counts half the bytes
    of 16-B/lane streaming reads on gfx950 (doubled here)."""
    import shutil
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_traffic import per_kernel
    if not shutil.which("rocprofv3"):
        return None, "rocprofv3 not on PATH"
    child = [sys.executable, os.path.abspath(__file__), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
             "--no-prof", "--no-pmc", "--no-n1-1m", "--arch", args.arch, "--batch", str(args.batch), "--k", str(args.k)]
    if args.dtype:
        child += ["--dtype", args.dtype]
    if args.gallery_rows:
        child += ["--gallery-rows", str(args.gallery_rows)]
    out = {}
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            print(f"[bench] rocprofv3 --pmc {counter} pass", file=sys.stderr, flush=True)
            cmd = ["timeout", "-s", "KILL", "150", "rocprofv3", "--pmc", counter, "--output-format", "csv",
                   "-d", os.path.join(d, counter), "-o", "run", "--"] + child
            r = subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE, text=True)
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {counter} pass failed (rc {r.returncode}): {r.stderr[-300:]}"
            out[counter] = per_kernel(os.path.join(d, counter), counter)
    f, w = out["FETCH_SIZE"], out["WRITE_SIZE"]
    return {k: (2 * 1024 * f[k][0], 1024 * w[k][0], f[k][1]) for k in f if k in w and f[k][1] == w[k][1]}, None


def class_traffic(cls, pmc):
    """HBM bytes per launch of bench kernel class `cls` from pmc_passes' per-kernel totals."""
    frag = next((k for c, k in CLASS_KERNEL if cls.startswith(c)), None)
    if frag is None or not pmc:
        return None
    ks = [k for k in pmc if any(f in k for f in frag)]
    n = sum(pmc[k][2] for k in ks)
    return round(sum(pmc[k][0] + pmc[k][1] for k in ks) / n) if n else None


def dtype_label(args) -> str:
    """The arithmetic the path computes in: IRV1's bf16 plan keeps its high-resolution stem in f16
    (DESIGN.md §5), IResNet100's fp8 plan is e4m3 for the layer3 tail only (weights.FP8_PLAN)."""
    if args.arch == "irv1_facenet" and args.dtype == "bf16" and os.environ.get("FR_IRV1_BF16_STEM") != "1":
        return "bf16 (f16 stem)"
    if args.dtype == "fp8" and os.environ.get("FR_FP8_PLAN") != "all":
        return "fp8 e4m3 (layer3.16-29) + bf16" if args.arch == "iresnet100" else "fp8 e4m3 + bf16"
    return args.dtype


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)  # >= 50 iterations after 10 warm-up
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--gallery-rows", type=int, default=None,
                    help="default 10000 at --gpus 1 (config 2), 1000000 at --gpus > 1 (config 4)")
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--arch", default="iresnet100")
    ap.add_argument("--dtype", default=None,
                    help="bf16 | f16 | fp8 (default: the arch's parity dtype; fp8 = BASELINE config 5)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bound on the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-prof", action="store_true", help="skip the per-kernel event timing (roofline)")
    ap.add_argument("--eager-prof", action="store_true",
                    help="time every 8th launch of the dominant class in eager steps instead of graph slots")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the live rocprofv3 --pmc traffic passes (roofline.traffic = null)")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank uses cuda:0 and the collectives run on gloo "
                         "(staged through host memory); never a measurement")
    ap.add_argument("--no-n1-1m", action="store_true",
                    help="N = 1: skip the extra timed run at config 4's 1M-row gallery (the weak-scaling "
                         "curve's N = 1 point, reported beside the headline as same_workload_as_multi_gpu)")
    ap.add_argument("--host-input", action="store_true",
                    help="crops start in pinned host memory and are copied H2D inside each step "
                         "(PCIe-inclusive rate, DESIGN.md; never the headline value)")
    return ap.parse_args()


def _time_embed(model, arch, u8, M):
    t0 = time.perf_counter()
    e = M.embed(model, arch, u8)
    return e, time.perf_counter() - t0


def cpu_baseline(arch, seconds):
    """BASELINE configs[0] / SURVEY.md §8d config 1 on the host cores, through the oracle (PyTorch fp32
    CPU restatement of the path; kind='port').  Two legs, each one bs=256 batch of synthetic crops:

      * `arch` (the bench's model; IResNet100 by default, which has no reference code) fp32 forward +
        F.normalize + the notebook's batched np.dot top-5 against a 1k-row gallery -> `value`;
      * the reference's own model, ResNet-50 ArcFaceModel (oracle golden-checked against the
        reference import, tests/test_golden.py), at bs=256, matched both ways the reference does:
        the recognize_with_db per-row cosine_similarity loop + stable sort (recognition_engine.py:
        267-289) for every probe, and the batched np.dot + argmax/top-5 (evaluate_arcface_kaggle.ipynb).

    `seconds` bounds the IResNet100 leg: when one bs=256 forward would exceed it (estimated from a
    32-crop probe batch), the leg times the largest multiple of 32 crops that fits and says so."""
    from facerecognition_amd.synthetic import synthetic_crops
    from facerecognition_amd.weights import INPUT_SIZE, synth_state_dict
    from oracle import models as M
    from oracle.match import recognize_with_db, topk_dot

    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    gal = np.random.default_rng(1).standard_normal((1000, 512)).astype(np.float32)
    gal /= np.linalg.norm(gal, axis=1, keepdims=True)
    out = {"unit": "faces/s", "cores": threads, "kind": "port"}

    # leg 1: the bench's model at bs=256 (bounded)
    s = INPUT_SIZE[arch]
    model = M.build_model(arch, synth_state_dict(arch))
    u8 = synthetic_crops(256, s, seed=11)
    M.embed(model, arch, u8[:2])  # warm the allocator / kernels
    _, t32 = _time_embed(model, arch, u8[:32], M)
    n = 256 if t32 * 8 <= seconds else max(32, int(seconds / t32) * 32)
    e, t_emb = _time_embed(model, arch, u8[:n], M)
    t0 = time.perf_counter()
    topk_dot(e, gal, 5)
    t_dot = time.perf_counter() - t0
    out["value"] = round(n / (t_emb + t_dot), 3)
    out["sample"] = (f"{n} synthetic {s}x{s} crops in ONE batch of {n}: {arch} fp32 forward + F.normalize "
                     f"({t_emb:.2f}s) + np.dot top-5 vs 1000x512 gallery ({t_dot * 1e3:.1f} ms), "
                     f"torch {threads} threads")
    del model

    # leg 2: the reference's own path (ResNet-50 ArcFaceModel), bs=256, both match styles
    if arch != "resnet50_arcface":
        r50 = M.build_model("resnet50_arcface", synth_state_dict("resnet50_arcface"))
        u8 = synthetic_crops(256, 112, seed=11)
        M.embed(r50, "resnet50_arcface", u8[:2])
        e, t_emb = _time_embed(r50, "resnet50_arcface", u8, M)
        db = {f"id_{j}": gal[j] for j in range(len(gal))}
        t0 = time.perf_counter()
        for row in e:
            recognize_with_db(row, db, 0.5)
        t_loop = time.perf_counter() - t0
        t0 = time.perf_counter()
        topk_dot(e, gal, 5)
        t_dot = time.perf_counter() - t0
        out["reference_resnet50"] = {
            "embed_faces_per_s": round(256 / t_emb, 2),
            "embed_plus_recognize_with_db_loop_faces_per_s": round(256 / (t_emb + t_loop), 2),
            "embed_plus_batched_dot_faces_per_s": round(256 / (t_emb + t_dot), 2),
            "recognize_with_db_loop_s": round(t_loop, 3), "batched_dot_ms": round(t_dot * 1e3, 2),
            "sample": "256 synthetic 112x112 crops, one batch of 256: ResNet-50 ArcFaceModel fp32 forward + "
                      "F.normalize, then recognize_with_db's per-row cosine_similarity loop + sort over a "
                      f"1000-row dict db for every probe, and np.dot + top-5; torch {threads} threads"}
    return out


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`python bench.py --gpus N` without a launcher.  This process has not touched the GPU (importing
    torch does not initialise HIP) and never does: it starts N fresh child processes of this same
    command, one per GPU, with the torch.distributed.run environment, forwards their output and
    returns the worst exit code.  If one rank fails the others are stopped by their exact PIDs."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:
                    q.terminate()
        time.sleep(0.1)
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.gallery_rows is None:
        args.gallery_rows = 10000 if world == 1 else C4_ROWS
    pmc, pmc_why = None, "not collected (--no-pmc / --no-prof / N > 1)"
    if world == 1 and not args.no_pmc and not args.no_prof:  # before this process touches the GPU
        pmc, pmc_why = pmc_passes(args)
    if args.share_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.share_device:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from facerecognition_amd.distributed import ShardedMatcher, shard_range
    from facerecognition_amd.gallery import DeviceGallery
    from facerecognition_amd.model import FRModel
    from facerecognition_amd.synthetic import synthetic_crops, synthetic_gallery_rows
    from facerecognition_amd import _native as N

    B, K = args.batch, args.k
    model = FRModel.synthetic(args.arch, device=local, max_batch=B, dtype=args.dtype)
    args.dtype = model.dtype
    size = model.input_size
    u8 = torch.from_numpy(synthetic_crops(B, size, seed=100 + rank)).to(dev)  # HBM-resident input
    # gallery: rows [r*rows/N, (r+1)*rows/N) on rank r; global indices via index_base
    rows = args.gallery_rows
    lo, hi = shard_range(rows, rank, world)
    gallery = DeviceGallery(device=local, index_base=lo)
    gallery.set_device_rows(synthetic_gallery_rows(lo, hi, dev))
    emb = torch.empty((B, 512), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    matcher = ShardedMatcher(B, 512, K, lambda p, s, i: gallery.search_device(p, K, s, i), dev,
                             pad_short=False)  # full batches every step

    u8_host = u8.cpu().pin_memory() if args.host_input else None

    def step(i=None):
        if u8_host is not None:
            u8.copy_(u8_host, non_blocking=True)
        if i is not None:
            ev[i][0].record(stream)
        model.embed(u8, out=emb, sync=False)  # FR_EMBED_ASYNC: checked once after the timed steps
        if i is not None:
            ev[i][1].record(stream)
        return matcher.search(emb)  # N > 1: RCCL all-gather + shard top-k + all-gather + merge

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    kclasses_all = {}
    dominant = None
    slot_mode = False
    if not args.no_prof:
        # untimed pass with every launch bracketed (eager) -> per-class breakdown and the dominant class;
        # the timed steps then time only the dominant class's launches
        L = N.lib()
        N.check(L.fr_prof_enable(model.handle, 1), "fr_prof_enable")
        for _ in range(2):
            step()
        torch.cuda.synchronize(dev)
        kclasses_all = N.prof_read(model.handle)
        dominant = max(kclasses_all.items(), key=lambda kv: kv[1][0])[0]
        if kclasses_all[dominant][1] % 2 == 0 and not args.eager_prof:
            # the timed steps replay hipGraphs, as the product path does, each step its own captured graph
            # with an event pair around ONE launch of the dominant class (fr_prof_slots): step i times the
            # class's launch i mod L (L launches per forward; IResNet100: the layer3 stage, L = 1); two
            # untimed forwards per slot: first sighting, capture
            N.check(L.fr_prof_enable(model.handle, 0), "fr_prof_enable")
            N.check(L.fr_prof_slots(model.handle, dominant.encode(), args.steps), "fr_prof_slots")
            for i in range(args.steps):
                N.check(L.fr_prof_slot_select(model.handle, i), "fr_prof_slot_select")
                step()
                step()
            slot_mode = True
        else:
            # reset, then time every PROF_STRIDE-th launch of the dominant class during the timed steps
            # (eager launches)
            N.check(L.fr_prof_enable(model.handle, PROF_STRIDE), "fr_prof_enable")
            N.check(L.fr_prof_only(model.handle, dominant.encode()), "fr_prof_only")
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        if slot_mode:
            N.lib().fr_prof_slot_select(model.handle, i)
        out_s, out_i = step(i)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kclasses = {}
    if slot_mode:
        L = N.lib()
        ms_slots, fl_slots, by_slots = [], [], []
        for i in range(args.steps):
            v = ctypes.c_float(0.0)
            fl, by = ctypes.c_double(0.0), ctypes.c_double(0.0)
            N.check(L.fr_prof_slot_ms(model.handle, i, ctypes.byref(v)), "fr_prof_slot_ms")
            N.check(L.fr_prof_slot_work(model.handle, i, ctypes.byref(fl), ctypes.byref(by)), "fr_prof_slot_work")
            ms_slots.append(v.value)
            fl_slots.append(fl.value)
            by_slots.append(by.value)
        N.check(L.fr_prof_slot_select(model.handle, -1), "fr_prof_slot_select")
        N.check(L.fr_prof_slots(model.handle, None, 0), "fr_prof_slots")
        # the sampled launches (one per timed step) with their own algorithmic work
        kclasses = {dominant: (float(np.sum(ms_slots)), args.steps, float(np.sum(fl_slots)), float(np.sum(by_slots)))}
    elif not args.no_prof:
        kclasses = N.prof_read(model.handle)
        N.check(N.lib().fr_prof_enable(model.handle, 0), "fr_prof_enable")
        N.check(N.lib().fr_prof_only(model.handle, None), "fr_prof_only")
    embed_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))  # forward duration on its stream
    # a split-stage halo wait that ran out (FR_EMBED_ASYNC: NaN embeddings, latched) voids the run
    model.sync_check()
    timeouts = model.stage_timeouts()
    if timeouts:
        raise SystemExit(f"rank {rank}: {timeouts} split-stage halo waits ran out: embeddings invalid, no result")
    if dist:
        t = torch.tensor([elapsed, embed_ms], dtype=torch.float64, device="cpu" if args.share_device else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, embed_ms = float(t[0]), float(t[1])
    # sanity: top-1 indices are valid global gallery rows (FR_TIMING_ONLY=1: timing-only experiment
    # libraries, tools/variant.sh, whose results are wrong by construction)
    if os.environ.get("FR_TIMING_ONLY") != "1":
        assert int(out_i[:, 0].min()) >= 0 and int(out_i[:, 0].max()) < rows

    faces = world * B * args.steps
    value = faces / elapsed
    flop_fwd = GFLOP_PER_FACE[args.arch] * 1e9 * B
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "faces/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": dtype_label(args),
        "data": f"synthetic u8 {size}x{size}x3 aligned crops ({'pinned host, H2D per step' if args.host_input else 'HBM-resident'}), "
                "random-init BN-calibrated weights, random unit-norm gallery",
        "config": {"workload": f"{args.arch} {args.dtype} embed bs={B}/GPU + top-{K} match vs "
                               f"{rows}x512 f32 gallery (row-sharded over {world} GPU(s))",
                   "batch_per_gpu": B, "global_batch": world * B, "gallery_rows": rows, "k": K,
                   "parallelism": f"dp{world}" + (" (shared-device gloo rehearsal, not a measurement)"
                                                   if args.share_device else "")},
    }
    if flop_fwd:
        result["forward"] = {"embed_ms": round(embed_ms, 4),
                             "tflops": round(flop_fwd / (embed_ms * 1e-3) / 1e12, 2)}
    if kclasses:
        # dominant kernel = the class with the most GPU time; achieved = its algorithmic FLOPs per
        # launch (2*M*N*K of the conv it computes) / its mean launch duration (HIP events on the
        # stream it is launched on, over the timed steps)
        name = dominant
        ms, launches, flops, _ = kclasses[name]
        achieved = flops / (ms * 1e-3) / 1e12
        traffic = class_traffic(name, pmc)
        peak = class_peak(name)
        result["roofline"] = {
            "bound": "mfma", "kernel": name, "achieved": round(achieved, 2), "peak": peak,
            "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
            "traffic": traffic,
            "traffic_source": ("rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes (separate) of this build, run by "
                               "this bench as a 2-step child of the same configuration; bytes per dispatch = "
                               "2*FETCH_SIZE + WRITE_SIZE (KiB, gfx950 FETCH half-count correction)")
                              if traffic is not None else (pmc_why if pmc is None else f"no rocprof kernel mapping for {name!r}"),
            "sampled_launches": launches, "sample_stride": 1 if slot_mode else PROF_STRIDE,
            "timing": ("HIP event pair around one launch of the class in every timed step (step i: launch i mod "
                       f"{kclasses_all[name][1] // 2} of the forward), captured into that step's hipGraph "
                       "(the timed steps replay graphs, as the product path does)") if slot_mode else
                      ("HIP events stamped by every sample_stride-th dispatch (hipExtLaunchKernel), eager launches"),
            "us_per_launch": round(ms / launches * 1e3, 2), "gflop_per_launch": round(flops / launches / 1e9, 3),
            "share_of_forward": round(kclasses_all[name][0] / 2 / embed_ms, 4)}
        # per-class breakdown from the untimed all-launch pass (2 steps), each class against both
        # rooflines: MFMA (algorithmic FLOPs / time / dense peak) and HBM (algorithmic bytes -- every
        # input, weight and output byte once -- / time / 8 TB/s); "bound" is the nearer one
        def cls_entry(name, v):
            ms, launches, fl, by = v
            peak = class_peak(name)
            tf = fl / (ms * 1e-3) / 1e12 if fl else None
            gbs = by / (ms * 1e-3) / 1e9 if by else None
            mf = tf / peak if tf else 0.0
            hf = gbs / HBM_PEAK_GBPS if gbs else 0.0
            e = {"ms_per_step": round(ms / 2, 4), "launches": launches // 2,
                 "tflops": round(tf, 1) if tf else None, "mfma_frac": round(mf, 3),
                 "gbps": round(gbs, 1) if gbs else None, "hbm_frac": round(hf, 3),
                 "bound": "mfma" if mf >= hf else "hbm"}
            tb = class_traffic(name, pmc)
            if tb is not None:  # PMC memory-side bytes per launch vs the algorithmic bytes per launch
                e["pmc_bytes_per_launch"] = tb
                e["pmc_over_algorithmic"] = round(tb / (by / launches), 2) if by else None
            return e
        result["kernels"] = {k: cls_entry(k, v) for k, v in sorted(kclasses_all.items(), key=lambda kv: -kv[1][0])}
    if world == 1 and rows != C4_ROWS and not args.no_n1_1m and not args.host_input and \
            os.environ.get("FR_TIMING_ONLY") != "1":
        # the N > 1 runs use config 4's 1M-row gallery (per rank: N*256 probes x 1M/N rows, i.e. the match
        # work of 256 probes x 1M rows whatever N): time that workload at N = 1 too, so the 1 -> 8 curve
        # has a same-workload N = 1 point (the headline `value` stays config 2's 10k gallery)
        g1m = DeviceGallery(device=local, index_base=0)
        g1m.set_device_rows(synthetic_gallery_rows(0, C4_ROWS, dev))
        m1m = ShardedMatcher(B, 512, K, lambda p, s, i: g1m.search_device(p, K, s, i), dev, pad_short=False)

        def step1m():
            model.embed(u8, out=emb, sync=False)
            return m1m.search(emb)

        for _ in range(max(2, args.warmup)):
            step1m()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            _, o_i = step1m()
        torch.cuda.synchronize(dev)
        el1 = time.perf_counter() - t1
        model.sync_check()
        assert int(o_i[:, 0].min()) >= 0 and int(o_i[:, 0].max()) < C4_ROWS
        result["same_workload_as_multi_gpu"] = {
            "gallery_rows": C4_ROWS, "value": round(B * args.steps / el1, 2), "unit": "faces/s",
            "ms_per_step": round(el1 / args.steps * 1e3, 4), "steps": args.steps,
            "note": "N = 1 run of the per-rank workload of the N > 1 lines (bs 256 embed + top-k of 256 probes x 1M "
                    "rows, bf16x3 match): the weak-scaling curve's same-workload N = 1 point"}
        g1m.close()
        del g1m, m1m
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.arch, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
