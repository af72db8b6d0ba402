#!/usr/bin/env python3
"""Benchmark: Gatys iters/s at 512x512 (+ fast_st train images/s at 256x256).

BASELINE.json metric "Gatys iters/sec at 512x512 + fast_st images/sec at
256x256, 1/2/4/8 GPUs".  `value` = Gatys iterations/s of the whole job (config 2:
gatys_st 512x512 single image, Adam iterations = forward + backward + Adam update
of the image, one hipGraph replay each).  Gatys optimises one image serially, so
ranks run independent replicas and the job rate is the sum.
The fast_st leg (config 4 shape: 256x256, per-GPU batch 8, data-parallel with one
RCCL all-reduce of the flat ImageTransformNet gradient per step) is reported in
the same line under "fast_st".  Inputs are resident in HBM before timing.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...    (one rank per GPU)
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import platform
import subprocess
import sys
import time

import socket

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
os.environ.setdefault("STX_NO_LOGFILE", "1")

# libstx-facing modules are imported by _imports(), after the launcher decision: the
# parent of a `--gpus N` run must not touch the GPU before it starts its N ranks
ops = V = W = N = None


def _imports():
    global ops, V, W, N
    from styletransfer_amd import ops as _ops
    from styletransfer_amd import vgg as _V
    from styletransfer_amd import weights as _W
    from styletransfer_amd import _native as _N
    ops, V, W, N = _ops, _V, _W, _N

METRIC = ("Gatys iters/sec at 512×512 + fast_st images/sec at 256×256, "
          "1/2/4/8 GPUs")
# algorithmic FLOPs (2*MAC), SURVEY.md §8(d)
GATYS_GFLOP = {512: 139.25, 256: 34.81}
FAST_ST_GFLOP_PER_IMAGE = 107.59
PEAK_F32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: f32-input MFMA = f32 vector peak
PEAK_F16_MFMA_TFLOPS = 2500.0  # dense fp16/bf16 MFMA (no sparsity)
# the split conv spends 3 fp16 MFMA products per fp32 product (hi*hi + hi*lo + lo*hi):
# its fp32-equivalent ceiling is the fp16 dense peak / 3
PEAK_SPLIT_TFLOPS = PEAK_F16_MFMA_TFLOPS / 3
PEAK_HBM_GBS = 8000.0


# the roofline kernel instance and its per-launch HBM traffic (rocprofv3 FETCH_SIZE /
# WRITE_SIZE passes of tools/pmc_r3.sh over an eager Gatys iteration, calibrated on
# kernels of known byte count: tools/pmc_r3_summary.py -> profiles/r6_pmc.json, the
# passes over the current build)
DG_KERNEL = "conv3x3_f16x3_v2_kernel<64, 0, {}, 2, 1>"
ROOFLINE_KERNEL = "conv3x3_f16x3_v2_kernel<64, 1, 0, 2, 1>"
ROOFLINE_MATCH = ROOFLINE_KERNEL
PMC_FILE = os.path.join(REPO, "profiles", "r6_pmc.json")
# algorithmic bytes of conv1_2 fwd @512^2 as the iteration launches it: Z1 in, Z2 and the
# fused relu+pool output P2 out, weights + bias, and the fused Gram partials (1024 tiles
# x 64 x 64 fp32)
CONV1_2_BYTES = (2 * 64 * 512 * 512 * 4 + 64 * 256 * 256 * 4 + 64 * 64 * 9 * 4 + 64 * 4
                 + 1024 * 64 * 64 * 4)


def pmc_traffic():
    """(bytes per launch, source, record) of ROOFLINE_KERNEL at 512^2 (grid 1024 blocks of
    256 threads) from the committed PMC record: FETCH_SIZE calibrated with the 4-B/lane
    read factor (the halo loads that carry the bytes), WRITE_SIZE with the 4-B store
    factor."""
    try:
        with open(PMC_FILE) as f:
            rec = json.load(f)
    except OSError:
        return None, None, None
    for r in rec.get("kernels", []):
        if ROOFLINE_MATCH in r["kernel"] and r["grid"] == 1024 * 256 and \
                "fetch_bytes_cal4" in r and "write_bytes_cal4" in r:
            return (round(r["fetch_bytes_cal4"] + r["write_bytes_cal4"]),
                    os.path.relpath(PMC_FILE, REPO), r)
    return None, None, None


def conv_gflop(cin, cout, h, w, ks=3):
    return 2.0 * cin * cout * ks * ks * h * w / 1e9


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--fast-batch", type=int, default=8, help="fast_st images per GPU")
    ap.add_argument("--fast-steps", type=int, default=50, help="timed fast_st train steps")
    ap.add_argument("--fast-b64-steps", type=int, default=10,
                    help="timed steps of the B=64-on-one-GPU fast_st leg (world 1; 0 = skip)")
    ap.add_argument("--gatys-run-iters", type=int, default=500,
                    help="config 2 as written: one timed run of this many Gatys iterations")
    ap.add_argument("--lbfgs-steps", type=int, default=10,
                    help="timed outer L-BFGS steps of the train_gatys leg (0 = skip)")
    ap.add_argument("--lbfgs-fill", type=int, default=20,
                    help="untimed outer L-BFGS steps at most, to fill the 100-pair history")
    ap.add_argument("--loader-images", type=int, default=256,
                    help="synthetic 640x480 JPEGs of the COCO loader leg (0 = skip)")
    ap.add_argument("--loader-epochs", type=int, default=3)
    ap.add_argument("--skip-fast", action="store_true")
    ap.add_argument("--fast-only", action="store_true", help="profiling: fast_st leg only")
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--skip-infer", action="store_true", help="skip the video/convert legs")
    ap.add_argument("--cpu-iters", type=int, default=8, help="timed Gatys iterations (CPU leg)")
    ap.add_argument("--cpu-fast-batch", type=int, default=8,
                    help="fast_st CPU leg batch (the per-GPU batch of config 4)")
    ap.add_argument("--cpu-fast-steps", type=int, default=2, help="timed fast_st CPU steps")
    ap.add_argument("--cpu-convert-batch", type=int, default=32,
                    help="convert CPU leg batch (config 3)")
    ap.add_argument("--no-graph", action="store_true")
    return ap.parse_args()


def timed(fn, k, world, dev):
    """barrier + sync on both sides of exactly k calls; max over ranks (seconds)."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


# Untimed warm-up before every timed window: at least W calls, continued until WARM_MS of
# wall time has passed.  The GPU's clocks ramp after the host-side work that precedes a
# window (weights, capture): on one box the Gatys graph's per-replay time fell from 0.771 ms
# (first replay) through 0.709 (3rd) to 0.662 ms (median of 40) -- tools/replay_probe.py,
# DESIGN §5 -- so a 20-step window opened after 5 warm-ups read 6-7 % below the same
# process's 500-iteration run.  The timed window itself is unchanged (exactly K steps).
WARM_MS = 150.0


def warm(fn, w, dev, world=1):
    """W untimed calls, then more until WARM_MS of wall time; returns the number made.
    With world > 1 every rank makes the same number of calls (fn may hold a collective --
    the fast_st step's all-reduce -- so a rank that stopped early would leave the others
    waiting in it): after each round the ranks agree whether any still needs time."""
    t0 = time.perf_counter()
    n = 0
    while True:
        for _ in range(max(1, w)):
            fn()
            n += 1
        torch.cuda.synchronize(dev)
        more = (time.perf_counter() - t0) * 1e3 < WARM_MS
        if world > 1:
            t = torch.tensor([1.0 if more else 0.0], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            more = bool(t.item() > 0)
        if not more:
            return n


def event_avg_ms(fn, reps=10):
    """Average duration of `fn` (one kernel launch) by HIP events on the stream the
    kernel is launched on (torch's current stream)."""
    st = torch.cuda.current_stream()
    fn()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def box_calibration(dev):
    """Per-box calibration, timed in this process before the legs (box-to-box
    spread of ~7 % is larger than a round's kernel gains): a fixed fp16 GEMM on the MFMA
    pipes (8192^3 through torch.matmul = hipBLASLt, TF/s) and a 1 GiB device-to-device
    copy (read + write bytes, GB/s).  A driver number divided by these separates "the
    kernels got faster" from "the box is faster"."""
    n = 8192
    a = torch.randn(n, n, device=dev, dtype=torch.float16)
    b = torch.randn(n, n, device=dev, dtype=torch.float16)
    c = torch.empty(n, n, device=dev, dtype=torch.float16)
    mm_ms = min(event_avg_ms(lambda: torch.matmul(a, b, out=c), reps=10) for _ in range(3))
    del a, b, c
    src = torch.empty(1 << 28, device=dev, dtype=torch.float32)
    src.fill_(1.0)
    dst = torch.empty_like(src)
    cp_ms = min(event_avg_ms(lambda: dst.copy_(src), reps=10) for _ in range(3))
    nbytes = 2 * src.numel() * 4
    del src, dst
    return {"fp16_gemm_tflops": round(2.0 * n ** 3 / (mm_ms * 1e-3) / 1e12, 1),
            "hbm_copy_gbs": round(nbytes / (cp_ms * 1e-3) / 1e9, 1),
            "note": "fp16 8192^3 torch.matmul (hipBLASLt) and a 1 GiB torch copy_ (2 GiB "
                    "moved), HIP events, best of 3 x 10; same process, before the legs"}


def gatys_leg(args, world, rank, dev):
    H = args.size
    style = torch.from_numpy(W.synthetic_image(1000 + rank, (1, 3, H, H))).to(dev)
    content = torch.from_numpy(W.synthetic_image(2000 + rank, (1, 3, H, H))).to(dev)
    feat = V.VGGFeatures(V.load_vgg19_weights(), dev)
    eng = V.GatysEngine(feat, style, content)
    first_replay_ms = None
    if args.no_graph:
        for _ in range(args.warmup):
            eng.step()
    else:
        # one eager iteration (allocates every buffer), the capture, then the W warm-up steps
        # as graph replays: a graph's first replay pays its one-time upload (timed here, it
        # is reported), and the replays bring the clocks up before the timed window (round
        # 5's 20-step window opened on the first replay: 7 % below the 500-iteration run)
        eng.capture(warmup=1)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        eng.step()
        torch.cuda.synchronize(dev)
        first_replay_ms = (time.perf_counter() - t0) * 1e3
    nwarm = warm(eng.step, args.warmup, dev, world)
    dt = timed(eng.step, args.steps, world, dev)
    rate = world * args.steps / dt
    run = None
    if args.gatys_run_iters > 0:
        # BASELINE config 2 as written: one gatys_st run of 500 Adam iterations
        n = args.gatys_run_iters
        dtr = timed(eng.step, n, world, dev)
        run = dict(iters=n, s=dtr, rate=world * n / dtr)
    # dominant kernel: the 3x3 implicit-GEMM conv at 64 channels, 512x512 (conv1_2
    # forward, the single launch with this kernel instance in a Gatys iteration, so
    # the rocprof average of the same command is directly comparable)
    # exactly the launch the iteration makes: input scale from conv1_1's epilogue slot,
    # fused ReLU+MaxPool output for conv2_1, max|Z2| for conv2_1's input scale
    z1 = eng.st.z[0]
    out = torch.empty_like(z1)
    # max|Z1| as conv1_1's epilogue reports it (the iteration's slot itself was zeroed by
    # its Adam launch for the next iteration)
    am = ops.amax(z1)
    am_out = torch.zeros(N.STX_AMAX_SLOTS, device=dev)
    pool = torch.empty_like(eng.st.pools[1])
    gparts = eng.st.grams[1]
    grouped = isinstance(gparts, tuple)  # (per-tile scratch + group sums, group counters)
    if grouped:
        gp = (torch.empty_like(gparts[0]), torch.zeros_like(gparts[1]))
    else:
        gp = torch.empty_like(gparts) if gparts is not None else None

    def conv12(g):
        kw = {}
        if g is not None:
            kw = dict(gram_part=g[0], gram_cnt=g[1]) if grouped else dict(gram_part=g)
        return ops.conv2d(z1, feat.wt[1], 64, 64, 3, in_mode=N.STX_IN_RELU, bias=feat.b[1],
                          out=out, wt16=feat.wt16[1], in_amax=am, out_amax=am_out,
                          pool_out=pool, **kw)

    fwd_ms = event_avg_ms(lambda: conv12(gp), reps=20)
    gf_conv = conv_gflop(64, 64, H, H)
    gf_gram = 2.0 * 64 * 64 * H * H / 1e9
    gf = gf_conv + (gf_gram if gp is not None else 0.0)
    achieved = gf / (fwd_ms * 1e-3) / 1e3  # TFLOP/s
    # the style-loss Gram of conv1_2's output (C=64, HW=H^2): fused into the conv's
    # epilogue (cost = the launch with gram_part minus the launch without, plus the
    # finalize from the partials), or split partials + finalize when not fusable
    z2 = eng.st.z[1]
    if gp is not None:
        plain_ms = event_avg_ms(lambda: conv12(None), reps=20)
        conv12(gp)
        if grouped:  # the finalize reads the group sums only
            nt = gp[1].numel()
            parts = gp[0][gp[0].numel() - nt * 4096:]
        else:
            nt, parts = gp.numel() // 4096, gp
        wsb = torch.empty(N.lib().stx_gram_ws(1, 64, H * H), device=dev, dtype=torch.uint8)
        tgt = eng.targets[1]
        fin_ms = event_avg_ms(lambda: ops.style_loss_from_parts(parts, nt, 1, 64, H * H, tgt,
                                                                defer_ws=wsb), reps=20)
        gram = dict(ms=max(fwd_ms - plain_ms, 0.0) + fin_ms, fused=True, epi_ms=fwd_ms - plain_ms,
                    finalize_ms=fin_ms, conv_ms=plain_ms, partials=nt, grouped=grouped)
        # in the iteration the five taps' finalizes are ONE launch: this tap's share of it by
        # partial bytes (job 1 = conv1_2's tap), re-launched here on the iteration's jobs
        jobs = eng.st.fin_jobs or []
        if len(jobs) > 1 and jobs[1].c == 64:
            arr = (N.GramFinJob * len(jobs))(*jobs)

            def pbytes(j):
                nt_ = (j.c + 63) // 64
                return j.b * nt_ * (nt_ + 1) // 2 * j.nsplit * 16384
            batch_ms = event_avg_ms(lambda: N.check(N.lib().stx_gram_finalize_batch(
                arr, len(jobs), ops._stream()), "stx_gram_finalize_batch"), reps=20)
            share = pbytes(jobs[1]) / sum(pbytes(j) for j in jobs)
            gram.update(batch_finalize_ms=batch_ms, batch_share=share,
                        in_iteration_ms=max(fwd_ms - plain_ms, 0.0) + share * batch_ms)
    else:
        zam = V.slot(eng.st.amax, 2).clone()
        gram = dict(ms=event_avg_ms(lambda: ops.gram(z2, z_amax=zam), reps=20), fused=False)
    gram.update(gflop=gf_gram, bytes=64 * H * H * 4)
    # the iteration's largest launch: conv1_2's data gradient with the fused Gram-backward
    # phase (dZ1 = mask * conv1_2^T(dZ2) + A1 Z1, vgg.loss_backward), same buffers and scales
    st, sc = eng.st, eng.scratch
    dz1 = torch.empty_like(sc["dz1"])
    am_b = torch.zeros(N.STX_AMAX_SLOTS, device=dev)

    dz2_am, z1_am = ops.amax(sc["dz2"]), ops.amax(st.z[0])

    # (the split phase's A scale: the group the batched finalize wrote, when it did)
    ca = st.coef_amax[0] if st.coef_amax else None

    def dgrad12():
        return feat.dgrad(1, sc["dz2"], dz1, mask=st.z[0], p2_z=st.z[0], p2_coef=st.coef[0],
                          p2_scale=None, in_amax=dz2_am, out_amax=am_b, p2_amax=z1_am,
                          p2_wt_amax=ca)
    dg_ms = event_avg_ms(dgrad12, reps=20)
    dg_gf = gf_conv + 2.0 * 64 * 64 * H * H / 1e9
    loss = float(eng.total)
    # the kernel instance that launch takes (conv16.hip launch16v2): P2 = 3 the split
    # phase, 1 the fp32-MFMA phase
    p2 = 1 if ca is None or N.knob("STX_P2_SPLIT", "1") == "0" else 3
    return dict(rate=rate, dt=dt, loss=loss, run=run, first_replay_ms=first_replay_ms,
                warm_calls=nwarm,
                kernel=dict(fwd_ms=fwd_ms, gflop=gf,
                                                         dg_kernel=DG_KERNEL.format(p2),
                                                         gflop_conv=gf_conv, tflops=achieved,
                                                         gram_fused=gp is not None,
                                                         dg_ms=dg_ms, dg_gflop=dg_gf,
                                                         dg_tflops=dg_gf / (dg_ms * 1e-3) / 1e3),
                gram=gram)


def gatys_lbfgs_leg(args, world, rank, dev):
    """The gatys_st CLI's default optimiser (StyleNetwork.train_gatys: torch.optim.LBFGS,
    history 100, max_iter 20, stransfer/network.py:411-458) at 512^2 on the same
    synthetic images: vgg.GatysLBFGS (one hipGraph replay + one host read per L-BFGS
    iteration).  The optimisation starts from a noise image (the reference's commented
    alternative start, network.py:430-433): from the content image the synthetic VGG
    weights' small style gradients let torch's tolerance tests end the run within ~60
    iterations, before the history fills.  Outer steps run until the history holds its
    100 pairs (at most `lbfgs_fill` steps; that fill phase is timed too), then
    `lbfgs_steps` outer steps are timed.  Rates: closure evaluations as torch counts them
    (func_evals), outer steps."""
    H = args.size
    style = torch.from_numpy(W.synthetic_image(1000 + rank, (1, 3, H, H))).to(dev)
    content = torch.from_numpy(W.synthetic_image(2000 + rank, (1, 3, H, H))).to(dev)
    gen = torch.Generator().manual_seed(3000 + rank)
    noise = torch.rand((1, 3, H, H), generator=gen).to(dev)
    feat = V.VGGFeatures(V.load_vgg19_weights(), dev)
    eng = V.GatysLBFGS(feat, style, content, init=noise).capture()
    fill = 0
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    while fill < args.lbfgs_fill and eng.history()[0] < 100:
        eng.step()
        fill += 1
    torch.cuda.synchronize(dev)
    fill_dt, fill_evals = time.perf_counter() - t0, eng.func_evals
    pairs0 = eng.history()[0]
    ev0, runs0 = eng.func_evals, eng.closure_runs
    dt = timed(eng.step, args.lbfgs_steps, world, dev)
    evals, runs = eng.func_evals - ev0, eng.closure_runs - runs0
    pairs1, n_iter = eng.history()
    # the reference's own start (stransfer/network.py:429: input_image = content.clone()):
    # the same number of outer steps from the content image, timed from the first one
    # (the history grows from 0 as the run goes; torch's tolerance tests may end steps early)
    engc = V.GatysLBFGS(feat, style, content, init=content.clone()).capture()
    ev0c = engc.func_evals
    dtc = timed(engc.step, args.lbfgs_steps, world, dev)
    evc = engc.func_evals - ev0c
    pairs_c, n_iter_c = engc.history()
    from_content = dict(evals_per_s=world * evc / dtc, steps_per_s=world * args.lbfgs_steps / dtc,
                        dt=dtc, steps=args.lbfgs_steps, evals=evc, pairs_at_end=pairs_c,
                        n_iter=n_iter_c, loss=float(engc.total))
    return dict(evals_per_s=world * evals / dt, steps_per_s=world * args.lbfgs_steps / dt,
                dt=dt, steps=args.lbfgs_steps, evals=evals, closure_runs=runs,
                fill_steps=fill, pairs_at_start=pairs0, pairs_at_end=pairs1, n_iter=n_iter,
                fill_evals_per_s=fill_evals / fill_dt, loss=float(eng.total),
                from_content=from_content)


def coco_loader_leg(args, dev, fast_rate=None):
    """the fast_st input pipeline (dataset.get_coco_loader with GPU
    conditioning: worker processes decode + pack JPEG batches, the pinned batch is
    uploaded and centre-cropped / Pillow-exact-resized / normalised on a side stream,
    the consumer's stream waits on an event) over synthetic 640x480 JPEGs at the
    per-GPU batch of 8; images/s of conditioned [8, 3, 256, 256] batches in HBM."""
    import shutil
    import tempfile
    from styletransfer_amd import dataset
    tmp = tempfile.mkdtemp(prefix="stx_coco_")
    try:
        n = args.loader_images
        dataset.write_synthetic_jpegs(tmp, n, seed=7)
        _, train = dataset.get_coco_loader(batch_size=args.fast_batch, test_split=0.0, path=tmp,
                                           gpu_conditioning=True)
        workers = train.loader.num_workers
        for _ in train:  # warm-up epoch: workers started, pinned/host caches filled
            pass
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        count = 0
        for _ in range(args.loader_epochs):
            for b in train:
                count += b.shape[0]
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        return dict(rate=count / dt, images=count, s=dt, workers=workers, files=n,
                    usable_cpus=dataset.usable_cpus(),
                    jpeg_kb=round(sum(os.path.getsize(os.path.join(tmp, f))
                                      for f in os.listdir(tmp)) / n / 1024, 1))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def fast_st_leg(args, world, rank, dev, B=None, steps=None):
    """fast_st train steps (config 4 shape): per-rank batch B, one SUM all-reduce of the
    flat gradient per step at world > 1.  A failed hipGraph capture is an error (no
    silent fall-back to eager steps in a process whose stream may be left in a failed
    capture state); --no-graph times eager steps."""
    from styletransfer_amd import network
    from styletransfer_amd.train import FastStTrainer
    B = B or args.fast_batch
    style = torch.from_numpy(W.synthetic_image(3000, (1, 3, 256, 256))).to(dev)
    itn = network.ImageTransformNet(style, batch_size=B).to(dev)
    itn.load_state_dict({k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)})
    tr = FastStTrainer(itn, style, world_size=world)
    batch = torch.from_numpy(W.synthetic_image(4000 + rank, (B, 3, 256, 256))).to(dev)
    steps = steps or args.fast_steps
    graph = not args.no_graph and N.knob("STX_FAST_GRAPH", "1") != "0"
    if graph:  # hipGraph replays per training step (FastStTrainer.capture)
        replay, static, _ = tr.capture(batch, warmup=max(1, min(args.warmup, 2)))
        warm(replay, 1, dev, world)
        dt = timed(replay, steps, world, dev)
        return dict(rate=world * B * steps / dt, dt=dt, steps=steps, batch=B, graph=True)
    for _ in range(max(1, min(args.warmup, 2))):
        tr.step(batch)
    warm(lambda: tr.step(batch), 1, dev, world)
    dt = timed(lambda: tr.step(batch), steps, world, dev)
    ips = world * B * steps / dt
    return dict(rate=ips, dt=dt, steps=steps, batch=B, graph=False)


def video_leg(args, world, rank, dev):
    """BASELINE config 5 ("video_st convert-video 1080p@30fps"): per frame, a decoded
    1920x1080 uint8 frame is conditioned on the GPU (centre crop, Pillow-exact resize to
    IMSIZE, normalisation; stransfer/dataset.py:280-306) and stylised by the 6-channel
    ImageTransformNet on cat([frame, previous output]) with the temporal-loss norms --
    one hipGraph replay per frame (FrameEngine(raw_hw=...)).  Frames are resident in
    HBM as uint8 (video decode and the PNG write excluded); `pcie` re-times the same
    loop with every frame uploaded from pinned host memory, `conditioned` the network
    alone on pre-conditioned IMSIZE frames."""
    from styletransfer_amd import network, video
    H, FH, FW = 256, 1080, 1920
    sd = {k: torch.from_numpy(v) for k, v in W.itn_synthetic(4322, in_channels=6)}
    g = torch.Generator().manual_seed(5000 + rank)
    raw = torch.randint(0, 256, (8, FH, FW, 3), generator=g, dtype=torch.uint8)
    n = max(10, args.steps)
    out = {}
    for mode in ("hbm", "pcie", "conditioned"):
        net = network.VideoTransformNet(torch.rand([3, H, H])).to(dev)
        net.load_state_dict(sd)
        if mode == "conditioned":
            frames = torch.from_numpy(W.synthetic_image(5000 + rank, (8, 3, H, H))).to(dev)
            eng = video.FrameEngine(net, (1, 3, H, H), dev, graph=not args.no_graph)
            src = lambda i: frames[i % 8:i % 8 + 1]  # noqa: E731
            fn = eng.step
        else:
            frames = raw.to(dev) if mode == "hbm" else raw.pin_memory()
            eng = video.FrameEngine(net, (1, 3, H, H), dev, graph=not args.no_graph,
                                    raw_hw=(FH, FW))
            src = lambda i: frames[i % 8]  # noqa: E731
            fn = eng.step_raw
        i = [0]

        def step():
            fn(src(i[0]))
            i[0] += 1
        for _ in range(3):
            step()
        warm(step, 1, dev, world)
        dt = timed(step, n, world, dev)
        out[mode] = dict(rate=world * n / dt, dt=dt)
        if mode == "hbm":
            out["tl"] = eng.temporal_loss()
    return dict(rate=out["hbm"]["rate"], dt=out["hbm"]["dt"], steps=n, size=H, tl=out["tl"],
                pcie=out["pcie"], conditioned=out["conditioned"], frame_hw=(FH, FW))


def itn_forward_gflop(h, w):
    """ImageTransformNet forward FLOPs per image (2*MAC; stransfer/network.py:520-611):
    conv 3->32 9x9, 32->64 and 64->128 3x3 stride 2, 5 residual blocks of two 128->128 3x3
    convs at h/4, nearest x2 + 128->64 and x2 + 64->32 3x3, 32->3 9x9."""
    c = lambda ci, co, k, oh, ow: 2.0 * ci * co * k * k * oh * ow
    return (c(3, 32, 9, h, w) + c(32, 64, 3, h // 2, w // 2) + c(64, 128, 3, h // 4, w // 4)
            + 10 * c(128, 128, 3, h // 4, w // 4) + c(128, 64, 3, h // 2, w // 2)
            + c(64, 32, 3, h, w) + c(32, 3, 9, h, w)) / 1e9


def convert_leg(args, world, rank, dev):
    """BASELINE config 3: fast_st convert-image, batch 32 at 256^2 (ITN forward), as one
    hipGraph replay per batch (eager launches timed beside it)."""
    from styletransfer_amd import network
    B, H = 32, 256
    itn = network.ImageTransformNet(torch.rand([3, H, H]), batch_size=B).to(dev)
    itn.load_state_dict({k: torch.from_numpy(v) for k, v in W.itn_synthetic(4321)})
    x = torch.from_numpy(W.synthetic_image(6000 + rank, (B, 3, H, H))).to(dev)
    n = max(3, args.steps // 5)
    with torch.no_grad():
        for _ in range(2):
            itn(x)
        warm(lambda: itn(x), 1, dev, world)
        dt_eager = timed(lambda: itn(x), n, world, dev)
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                itn(x)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with ops.graph_capture(g):
                y = itn(x)
            warm(g.replay, 1, dev, world)
            dt = timed(g.replay, n, world, dev)
            ref = itn(x)
            torch.cuda.synchronize(dev)
            same = bool(torch.equal(y, ref))
        except RuntimeError as e:  # report the eager rate rather than lose the line
            print(f"convert leg: graph capture failed ({e}); eager rate reported", file=sys.stderr)
            dt, same = dt_eager, None
    gf = itn_forward_gflop(H, H) * B
    graph_rate = world * B * n / dt
    if same is False:  # a capture that changes the output is not a speed-up: eager rate
        print("convert leg: graph output != eager output; eager rate reported", file=sys.stderr)
        dt = dt_eager
    return dict(rate=world * B * n / dt, dt=dt, steps=n, batch=B, eager_rate=world * B * n / dt_eager,
                graph_rate=graph_rate, gflop=gf, tflops=gf * n / dt / 1e3, graph_equals_eager=same)


def _host_cpu():
    """(threads to use, description): the CPUs this process may run on (affinity /
    cgroup cpuset), which on a shared GPU box is the box's CPU share, not the
    whole machine's os.cpu_count()."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    threads = min(aff, quota) if quota else aff
    model = ""
    try:
        out = subprocess.check_output(["lscpu"], text=True)
        model = next((l.split(":", 1)[1].strip() for l in out.splitlines()
                      if l.startswith("Model name")), "")
    except Exception:  # noqa: BLE001
        model = platform.processor()
    return threads, (f"{model}; {threads} threads = usable CPUs (affinity {aff}, cgroup quota "
                     f"{quota}, os.cpu_count {os.cpu_count()})")


def cpu_baseline(args):
    """The oracle (torch-CPU restatement of the reference schedule) on the host cores:
    the Gatys Adam loop at 512^2 (the `value` metric), plus the fast_st train step and
    the convert-image forward at 256^2 (north_star: images/s next to the reference CPU
    path timed on the same box)."""
    from oracle import reference_cpu as O
    threads, host = _host_cpu()
    torch.set_num_threads(threads)
    H = args.size
    s = torch.from_numpy(W.synthetic_image(1000, (1, 3, H, H)))
    c = torch.from_numpy(W.synthetic_image(2000, (1, 3, H, H)))
    net = O.StyleNetwork(s, c)
    x = c.clone()
    opt = net.get_content_optimizer(x)
    O.gatys_adam_iter(net, x, c, opt)  # warm-up
    n = args.cpu_iters
    t0 = time.perf_counter()
    for _ in range(n):
        O.gatys_adam_iter(net, x, c, opt)
    dt = time.perf_counter() - t0
    # fast_st train step (static_train closure + Adam) and ITN forward at 256^2
    B = args.cpu_fast_batch
    itn = O.image_transform_net(4321)
    st = torch.from_numpy(W.synthetic_image(3000, (1, 3, 256, 256)))
    ln = O.StyleNetwork(st, torch.rand([1, 3, 256, 256]))
    batch = torch.from_numpy(W.synthetic_image(4000, (B, 3, 256, 256)))
    aopt = torch.optim.Adam(itn.parameters())

    def fast_step():
        aopt.zero_grad()
        O.fast_st_closure(itn, ln, batch)
        aopt.step()
    fast_step()  # warm-up
    nf = args.cpu_fast_steps
    t1 = time.perf_counter()
    for _ in range(nf):
        fast_step()
    dtf = time.perf_counter() - t1
    Bc = args.cpu_convert_batch
    cbatch = torch.from_numpy(W.synthetic_image(5000, (Bc, 3, 256, 256)))
    nc = 3
    with torch.no_grad():
        itn(cbatch)
        t2 = time.perf_counter()
        for _ in range(nc):
            itn(cbatch)
        dtc = time.perf_counter() - t2
    return dict(value=n / dt, unit="iters/s", cores=threads, kind="port",
                sample=f"oracle/reference_cpu.py Gatys Adam loop {H}x{H}, {n} timed iters "
                       f"after 1 warm-up ({dt:.1f} s), reference schedule incl. prefix "
                       f"re-runs and VGG wgrad; torch {torch.__version__} CPU, {host}",
                fast_st=dict(value=nf * B / dtf, unit="images/s", batch=B, s=round(dtf, 2),
                             sample=f"oracle fast_st_closure + torch.optim.Adam, B={B} 256^2 "
                                    f"(config 4's per-GPU batch), {nf} timed steps after 1 "
                                    "warm-up"),
                convert=dict(value=nc * Bc / dtc, unit="images/s", batch=Bc, s=round(dtc, 2),
                             sample=f"oracle ImageTransformNet forward, B={Bc} 256^2 (config 3), "
                                    f"no_grad, {nc} timed passes after 1 warm-up"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(n):
    """`python bench.py --gpus N` without a launcher: start N rank processes (the
    torchrun environment contract, one per GPU) and exit with the worst exit code.
    This parent process never touches the GPU."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    # a rank that fails leaves the others waiting in a rendezvous or collective: stop
    # them (the processes started here, by PID) and report the failure
    rc = 0
    while procs:
        for p in list(procs):
            r = p.poll()
            if r is None:
                continue
            procs.remove(p)
            if r != 0:
                rc = r
                for q in procs:
                    q.terminate()
                for q in procs:
                    try:
                        q.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                procs = []
                break
        time.sleep(0.2)
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args.gpus))
    _imports()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    # more ranks than visible GPUs (a same-device rehearsal on a 1-GPU box; or
    # STX_BENCH_SAME_DEVICE=1): ranks share cuda:0 and exchange over gloo, and the line
    # says so ("devices"); the driver's 8-GPU runs have one GPU per rank and use RCCL
    ndev = torch.cuda.device_count()
    same = os.environ.get("STX_BENCH_SAME_DEVICE", "0") != "0" or ndev < world
    if same:
        local = 0
        os.environ.setdefault("STX_BENCH_BACKEND", "gloo" if world > 1 else "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("STX_BENCH_BACKEND", "nccl")
        # (a bounded wait: a rank that never arrives fails the run instead of hanging it)
        pg_timeout = datetime.timedelta(seconds=300)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout)
        else:
            dist.init_process_group(backend, timeout=pg_timeout)
    N.lib()
    if args.fast_only:
        fs = fast_st_leg(args, world, rank, dev)
        if rank == 0:
            print(json.dumps({"fast_st_images_per_s": round(fs["rate"], 3),
                              "ms_per_step": round(1e3 * fs["dt"] / fs["steps"], 3)}))
        return
    box = box_calibration(dev)
    g = gatys_leg(args, world, rank, dev)
    lb = gatys_lbfgs_leg(args, world, rank, dev) if args.lbfgs_steps > 0 else None
    fs = None if args.skip_fast else fast_st_leg(args, world, rank, dev)
    fs64 = None
    if not args.skip_fast and world == 1 and args.fast_b64_steps > 0:
        # at 1 GPU the config-4 global batch of 64 on one device
        fs64 = fast_st_leg(args, world, rank, dev, B=64, steps=args.fast_b64_steps)
    vid = conv = None
    if not args.skip_infer:
        vid = video_leg(args, world, rank, dev)
        conv = convert_leg(args, world, rank, dev)
    ld = None
    if args.loader_images > 0 and not args.skip_infer:
        # every rank runs its own loader on its share of the node's CPUs (the worker count
        # follows LOCAL_WORLD_SIZE); the line reports the slowest rank
        ld = coco_loader_leg(args, dev)
        if world > 1:
            t = torch.tensor([ld["rate"]], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            ld["rate_min_rank"] = float(t.item())
    cpu = None
    if rank == 0 and world == 1 and not args.skip_cpu:
        cpu = cpu_baseline(args)
    if rank == 0:
        k = g["kernel"]
        traffic_bytes, traffic_src, traffic_rec = pmc_traffic()
        res = {
            "metric": METRIC,
            "value": round(g["rate"], 3),
            "unit": "iters/s",
            "n_gpus": world,
            "devices": 1 if same else world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * g["dt"] / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (hash-PRNG images and VGG-19 weights; no pretrained download)",
            "config": {"workload": f"gatys_st {args.size}x{args.size} single image, Adam "
                                   "iterations (BASELINE configs[1]); one independent image "
                                   "per GPU (replicas)",
                       "image": args.size, "batch": 1, "parallelism": f"replicas{world}",
                       "graph": not args.no_graph},
            "roofline": {
                "bound": "mfma",
                "kernel": f"{ROOFLINE_KERNEL} (conv1_2 forward, 64->64 3x3 @ "
                          f"{args.size}^2, fused ReLU loader + ReLU/MaxPool output"
                          + (" + the style-loss Gram partials of its output" if k["gram_fused"]
                             else "") + ", fp16 hi/lo split MFMA; the same launch as in the "
                          "iteration)",
                "achieved": round(k["tflops"], 3),
                "peak": round(PEAK_SPLIT_TFLOPS, 1),
                "unit": "TFLOP/s",
                "frac": round(k["tflops"] / PEAK_SPLIT_TFLOPS, 4),
                "peak_note": "fp32-equivalent FLOPs (algorithmic 2*MAC); peak = dense fp16 "
                             "MFMA 2500 TF / 3 products per fp32 product of the hi/lo split "
                             "(fp32-input MFMA peak is 157.3 TF)",
                "traffic": traffic_bytes,
                "per_launch_gflop": round(k["gflop"], 3),
                "per_launch_gflop_note": "3x3 conv 2*64*64*9*H*W"
                                         + (" + Gram 2*64*64*H*W" if k["gram_fused"] else ""),
                "fwd_ms": round(k["fwd_ms"], 4),
                "traffic_source": traffic_src,
                "traffic_raw": None if traffic_rec is None else {
                    "fetch": traffic_rec.get("FETCH_SIZE_bytes_raw"),
                    "write": traffic_rec.get("WRITE_SIZE_bytes_raw")},
                "algorithmic_bytes": CONV1_2_BYTES if args.size == 512 else None,
                "iteration_tflops": round(GATYS_GFLOP.get(args.size, float("nan")) * g["rate"]
                                          / world / 1e3, 3),
                "dominant_kernel": {
                    "kernel": k["dg_kernel"] + " (conv1_2 data gradient "
                              f"@ {args.size}^2 with the fused Gram-backward phase: dZ1 = "
                              "[Z1 > 0] conv1_2^T(dZ2) + A1 Z1; the iteration's longest launch)",
                    "achieved": round(k["dg_tflops"], 3),
                    "frac": round(k["dg_tflops"] / PEAK_SPLIT_TFLOPS, 4),
                    "per_launch_gflop": round(k["dg_gflop"], 3),
                    "ms": round(k["dg_ms"], 4),
                },
            },
            "gram_roofline": {
                "kernel": ("fused into conv1_2's epilogue (launch with gram_part minus launch "
                           "without; with gram_cnt the epilogue also sums each group of "
                           f"{N.STX_GRAM_GROUP} tiles' partials in-launch) + gram_finalize_kernel "
                           "from the partials it leaves"
                           if g["gram"]["fused"] else
                           "gram_partial_f16_kernel + gram_finalize_kernel")
                          + f" (StyleLoss.gram_matrix of conv1_2's output, C=64, HW={args.size}^2)",
                "ms": round(g["gram"]["ms"], 4),
                "parts_ms": {kk: round(v, 4) for kk, v in g["gram"].items()
                             if kk in ("epi_ms", "finalize_ms", "conv_ms")},
                "finalize_partials": g["gram"].get("partials"),
                "finalize_partial_mb": round(g["gram"].get("partials", 0) * 16384 / 1e6, 2),
                "achieved_tflops_fp32eq": round(g["gram"]["gflop"] / g["gram"]["ms"], 2),
                "mfma_bf16_peak_frac": round(3 * g["gram"]["gflop"] / g["gram"]["ms"]
                                             / PEAK_F16_MFMA_TFLOPS, 4),
                "in_iteration": None if "in_iteration_ms" not in g["gram"] else {
                    "ms": round(g["gram"]["in_iteration_ms"], 4),
                    "batch_finalize_ms": round(g["gram"]["batch_finalize_ms"], 4),
                    "tap_share_of_batch": round(g["gram"]["batch_share"], 4),
                    "mfma_bf16_peak_frac": round(3 * g["gram"]["gflop"]
                                                 / g["gram"]["in_iteration_ms"]
                                                 / PEAK_F16_MFMA_TFLOPS, 4),
                    "note": "as the iteration runs it: the epilogue delta + this tap's share "
                            "(by partial bytes) of the ONE batched finalize launch of all five "
                            "taps (timed on the iteration's own jobs)"},
                "epilogue_mfma_bf16_peak_frac": round(3 * g["gram"]["gflop"]
                                                      / max(g["gram"].get("epi_ms", 0.0), 1e-9)
                                                      / PEAK_F16_MFMA_TFLOPS, 4)
                if g["gram"]["fused"] else None,
                "hbm_gbs": round(g["gram"]["bytes"] / (g["gram"]["ms"] * 1e-3) / 1e9, 1),
                "hbm_frac": round(g["gram"]["bytes"] / (g["gram"]["ms"] * 1e-3) / 1e9
                                  / PEAK_HBM_GBS, 4),
                "note": "standalone it is HBM-bound (2*C^2*HW FLOPs over C*HW*4 bytes = 32 "
                        "FLOP/B); fused, Z is not re-read and the cost is the epilogue's extra "
                        "time + the partial reduction; hbm_* rate Z's bytes over that time; the "
                        "MFMA fraction counts the 3 fp16 products per fp32 product",
            },
            "cpu_baseline": cpu,
            "box": box,
            "gatys_loss": g["loss"],
        }
        if g.get("first_replay_ms") is not None:
            # (untimed: the captured graph's first replay, before the W - 1 other warm-ups)
            res["gatys_first_replay_ms"] = round(g["first_replay_ms"], 3)
        res["gatys_warmup_calls"] = g["warm_calls"]
        if g["run"]:
            r = g["run"]
            res["gatys_config2_run"] = {
                "iters": r["iters"], "seconds": round(r["s"], 4), "value": round(r["rate"], 3),
                "unit": "iters/s", "note": "BASELINE config 2 as written: one timed run of "
                "500 Adam iterations at 512^2 (hipGraph replays), after the K timed steps"}
        if lb:
            res["gatys_lbfgs"] = {
                "value": round(lb["evals_per_s"], 3), "unit": "closure evaluations/s",
                "outer_steps_per_s": round(lb["steps_per_s"], 4),
                "vs_adam_iteration_rate": round(lb["evals_per_s"] / g["rate"], 4),
                "evals": lb["evals"], "closure_runs": lb["closure_runs"],
                "steps": lb["steps"], "seconds": round(lb["dt"], 4),
                "history_pairs": [lb["pairs_at_start"], lb["pairs_at_end"]],
                "fill_steps": lb["fill_steps"], "torch_n_iter": lb["n_iter"],
                "fill_evals_per_s": round(lb["fill_evals_per_s"], 3),
                "note": "gatys_st's default optimiser (StyleNetwork.train_gatys: L-BFGS, "
                        "history 100, max_iter 20) at 512^2 from a noise image; timed after "
                        "the history filled (fill_evals_per_s: the filling steps, history "
                        "0..100); "
                        "per iteration one hipGraph replay (compact-form direction + x update + "
                        "closure + gradient statistics) and one host read of the scalars "
                        "torch's control flow tests; evaluations as torch counts them",
                "from_content": None if not lb.get("from_content") else {
                    "value": round(lb["from_content"]["evals_per_s"], 3),
                    "unit": "closure evaluations/s",
                    "vs_adam_iteration_rate": round(lb["from_content"]["evals_per_s"] / g["rate"], 4),
                    "evals": lb["from_content"]["evals"], "steps": lb["from_content"]["steps"],
                    "seconds": round(lb["from_content"]["dt"], 4),
                    "history_pairs_at_end": lb["from_content"]["pairs_at_end"],
                    "torch_n_iter": lb["from_content"]["n_iter"],
                    "note": "the reference's start (stransfer/network.py:429 input_image = "
                            "content.clone()): the same outer steps timed from the first, "
                            "the history growing from empty"}}
        if fs:
            res["fast_st"] = {
                "value": round(fs["rate"], 3), "unit": "images/s",
                "per_gpu_batch": fs["batch"], "global_batch": fs["batch"] * world,
                "steps": fs["steps"], "ms_per_step": round(1e3 * fs["dt"] / fs["steps"], 3),
                "parallelism": f"dp{world}", "scaling": "weak",
                "collective": (f"{os.environ.get('STX_BENCH_BACKEND', 'nccl').replace('nccl', 'RCCL')}"
                               " all_reduce(SUM) of 1,679,235 fp32 grads per step")
                              if world > 1 else None,
                "tflops_per_gpu": round(FAST_ST_GFLOP_PER_IMAGE * fs["rate"] / world / 1e3, 3),
                "graph": fs["graph"],
            }
        if fs64:
            res["fast_st_b64"] = {
                "value": round(fs64["rate"], 3), "unit": "images/s", "batch": 64,
                "steps": fs64["steps"], "ms_per_step": round(1e3 * fs64["dt"] / fs64["steps"], 3),
                "tflops": round(FAST_ST_GFLOP_PER_IMAGE * fs64["rate"] / 1e3, 3),
                "graph": fs64["graph"], "note": "config-4 global batch 64 on one GPU (the "
                "1-GPU point of the strong-scaling view; the weak-scaling legs keep 8/GPU)"}
        if ld:
            per_rank_step = fs["rate"] / world if fs else None
            per_worker = ld["rate"] / max(1, ld["workers"])
            res["coco_loader"] = {
                "value": round(ld.get("rate_min_rank", ld["rate"]), 1), "unit": "images/s",
                "per_rank": True, "batch": args.fast_batch,
                "workers": ld["workers"], "usable_cpus": ld["usable_cpus"],
                "images_per_s_per_worker": round(per_worker, 1),
                "images": ld["images"], "seconds": round(ld["s"], 3),
                "jpeg": f"{ld['files']} synthetic 640x480 JPEGs, {ld['jpeg_kb']} KB avg",
                "vs_fast_st_step_rate": round(ld.get("rate_min_rank", ld["rate"]) / per_rank_step, 3)
                if fs else None,
                "cpus_for_8_ranks": (round(8 * (per_rank_step / per_worker + 1), 1)
                                     if fs else None),
                "note": "dataset.get_coco_loader(gpu_conditioning=True): decode workers -> "
                        "pinned packed batch -> side-stream upload + GPU crop/resize/normalise "
                        "(bit-identical to the PIL path); per rank, fed by this rank's CPU share "
                        "(usable CPUs / LOCAL_WORLD_SIZE - 1 workers); value = the slowest rank; "
                        "cpus_for_8_ranks = 8 x (the per-rank fast_st step rate / images per "
                        "worker + 1 for the training loop)"}
        if vid:
            res["video_st"] = {
                "value": round(vid["rate"], 2), "unit": "frames/s",
                "input": f"{vid['frame_hw'][1]}x{vid['frame_hw'][0]} uint8", "frame": vid["size"],
                "ms_per_frame": round(1e3 * vid["dt"] / vid["steps"], 4),
                "steps": vid["steps"], "graph": not args.no_graph, "parallelism":
                f"replicas{world}",
                "pcie_value": round(vid["pcie"]["rate"], 2),
                "conditioned_value": round(vid["conditioned"]["rate"], 2),
                "note": "BASELINE config 5: per 1080p uint8 frame, GPU conditioning (crop, "
                "Pillow-exact resize to 256, normalise) + 6-channel ImageTransformNet + "
                "temporal-loss norms, one hipGraph replay; frames resident in HBM (decode and "
                "PNG write excluded). pcie_value: frames uploaded from pinned host memory each "
                "step; conditioned_value: the network alone on pre-conditioned 256^2 frames"}
        if conv:
            res["fast_st_convert"] = {
                "value": round(conv["rate"], 2), "unit": "images/s", "batch": conv["batch"],
                "ms_per_batch": round(1e3 * conv["dt"] / conv["steps"], 3),
                "steps": conv["steps"], "eager_value": round(conv["eager_rate"], 2),
                "graph_value": round(conv["graph_rate"], 2),
                "gflop_per_batch": round(conv["gflop"], 2),
                "tflops": round(conv["tflops"], 1),
                "split_peak_frac": round(conv["tflops"] / PEAK_SPLIT_TFLOPS, 4),
                "graph_equals_eager": conv["graph_equals_eager"],
                "note": "BASELINE config 3: ImageTransformNet forward, batch 32 at 256x256, "
                        "one hipGraph replay per batch (eager_value: the same launches issued "
                        "eagerly); FLOPs 2*MAC of the convs, fraction of the 833 TF split peak"}
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
