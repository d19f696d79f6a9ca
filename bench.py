#!/usr/bin/env python3
"""bench.py — Msamples/s of the per-pixel render path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scene 0] [--width 1920] [--height 1080]
                    [--spp 512] [--bounces 16] [--inflight 2] [--no-cpu-baseline]

A "step" is one frame: RNG seeding + longest-first schedule probe + render kernel + device tonemap
to PPM bytes (+ the RCCL gather of the u8 rows to rank 0 when N>1), with the scene already resident
in HBM.  Default workload = BASELINE
config 2: scene 0 (fv1) at 1920x1080, spp 512, depth 16 on one GPU.  With N ranks
(torch.distributed.run, one process per GPU, backend "nccl" = RCCL) the frame grows to ~N x the
pixels at the same aspect and camera (weak scaling) and rows are interleaved across ranks.  Up to
--inflight frames are queued at once on separate streams (frames are independent; the next frame
fills the SIMDs the previous frame's slowest pixels leave idle).  Rank 0 prints ONE JSON line.

The printed value is samples of all ranks x K frames / max-over-ranks wall time of the K timed steps.
roofline: VALU-bound kernel; achieved = algorithmic FP32 ops per render launch (op model of
SURVEY §8d evaluated on this workload's measured per-sample visit counts) / the render kernel's
HIP-event duration on an isolated frame (no overlap; profile with --inflight 1 to compare with
rocprofv3).  cpu_baseline: the C oracle on this host's cores over a bounded row sample, whose GPU
render is compared bit for bit.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

import torch  # first: one HIP runtime per process (cuda_raytracing_amd._abi._bind_single_hip_runtime)
import torch.distributed as dist

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))
import cuda_raytracing_amd as rt  # noqa: E402
from cuda_raytracing_amd import _abi  # noqa: E402
from cuda_raytracing_amd.multi_gpu import gather_rows, weak_scaled_resolution  # noqa: E402

# FP32 op weights per event (counted from the reference source, unfused, 1 op each)
OP_WEIGHTS = {
    "visit_sphere": 31, "visit_bvh": 24, "visit_triangle": 49, "visit_quad": 49,
    "visit_translate": 3, "visit_yrotate": 12, "visit_group": 0,
    "shades": 100, "perlin": 1500,
}
OPS_PER_SAMPLE_FIXED = 30                 # camera ray generation
# non-packed FP32 VALU peak: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md: 157.3 TFLOPS
# spec counts an FMA as 2; the path is compiled without contraction, so 1 op = 1 lane-instruction)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12


TRAV_NAMES = {0: "lane-dfs", 1: "wave-packet-dfs", 2: "scene-specialised", 3: "verified-sah"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def op_model(counters: dict, samples: int) -> float:
    ops = sum(OP_WEIGHTS[k] * counters[k] for k in OP_WEIGHTS) + OPS_PER_SAMPLE_FIXED * samples
    return ops / max(samples, 1)


def cpu_baseline(world, settings, W, H, spp, bounces, budget_s, ctx=None):
    """Oracle (C, OpenMP) on this host: the same scene/camera, a bounded row sample.

    The same sample is then rendered on the GPU through the product context and compared bit for bit
    (the PSNR half of the BASELINE metric: identical frames -> PSNR = inf, reported as "bit-exact")."""
    import ctypes as C
    import numpy as np
    L = _abi.oracle_lib()
    cam, W, H = rt.camera_from_settings(settings, W, H)

    def run(stride, s):
        rows = len(range(0, H, stride))
        p = rt.make_params(settings, W, H, spp=s, bounces=bounces, row_offset=0, row_stride=stride, row_count=rows)
        out = np.zeros((rows, W, 3), np.float32)
        st = _abi.Stats()
        t = time.perf_counter()
        rc = L.rt_render_cpu(C.byref(world.scene()), C.byref(cam), C.byref(p), out.ctypes.data_as(C.c_void_p),
                             C.byref(st))
        dt = time.perf_counter() - t
        assert rc == 0, rc
        return rows * W * s, dt, out

    # calibrate on a sparse row sample (twice: the first call also spins up the OpenMP pool), then
    # render every stride-th row of the frame at the FULL spp so the per-pixel work equals the GPU's
    # calibrate: t = a*pixels (RNG seeding by jumps) + b*samples, from two short runs on every 16th row
    run(16, 2)
    s1, s2 = min(spp, 8), min(spp, 32)
    n1, t1, _ = run(16, s1)
    n2, t2, _ = run(16, s2)
    px = n1 / s1
    b = max((t2 - t1) / max(n2 - n1, 1), 1e-12) if s2 > s1 else t1 / n1
    a = max((t1 - b * n1) / px, 0.0)
    full_s = a * W * H + b * W * H * spp
    stride = max(1, math.ceil(full_s / budget_s))
    rows = len(range(0, H, stride))
    s = spp
    n, dt, ref = run(stride, s)
    parity = None
    if ctx is not None:
        import torch
        p = rt.make_params(settings, W, H, spp=s, bounces=bounces, row_offset=0, row_stride=stride, row_count=rows)
        dev = torch.empty((rows, W, 3), dtype=torch.float32, device="cuda")
        ctx.render_into(cam, p, dev.data_ptr(), torch.cuda.current_stream().cuda_stream)
        ctx.timing()
        g = dev.cpu().numpy()
        mse = float(np.mean((np.clip(np.sqrt(g), 0, 1) - np.clip(np.sqrt(ref), 0, 1)) ** 2))
        parity = {"bit_exact": bool(np.array_equal(g.view(np.uint32), ref.view(np.uint32))),
                  "psnr_db": None if mse == 0 else round(10 * math.log10(1.0 / mse), 2),
                  "note": "GPU vs oracle on this sample; psnr_db null = identical frames (PSNR infinite)"}
    return {
        "value": n / dt / 1e6, "unit": "Msamples/s", "cores": int(L.rt_oracle_threads()), "kind": "port",
        "sample": f"frame rows 0::{stride} ({rows} rows x {W} px) at spp {s}, d{bounces}: {n:.3g} samples in {dt:.1f} s",
        "parity": parity,
    }


def load_traffic(workload: str):
    f = REPO / "profiles" / "hbm_traffic.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text()).get(workload)
        return int(d["bytes"]) if d else None
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", type=int, default=0)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=512)
    ap.add_argument("--bounces", type=int, default=16)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of oracle wall time (bounded sample)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inflight", type=int, default=2, help="frames queued at once (own context + stream each)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL, default) or gloo (plumbing rehearsal)")
    args = ap.parse_args()

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world_size}; using WORLD_SIZE")
    dev = local_rank % max(torch.cuda.device_count(), 1)   # == local_rank on a node with a GPU per rank
    torch.cuda.set_device(dev)
    if world_size > 1:
        if args.dist_backend == "nccl":   # RCCL over xGMI, one rank per GPU
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:                             # rehearsal of the multi-rank plumbing (CPU collectives)
            dist.init_process_group(args.dist_backend)

    # ---- host pre-pass (untimed, like the reference's make_bvh + camera) ----
    world, settings = rt.build_scene(args.scene)
    W, H = weak_scaled_resolution(args.width, args.height, world_size)
    cam, W, H = rt.camera_from_settings(settings, W, H)
    off, stride, rows = rt.shard_rows(H, rank, world_size)
    params = rt.make_params(settings, W, H, spp=args.spp, bounces=args.bounces,
                            row_offset=off, row_stride=stride, row_count=rows)
    nf = max(1, args.inflight)
    ctxs = [rt.RenderContext(world.scene(), device=dev) for _ in range(nf)]
    ctx = ctxs[0]
    streams = [torch.cuda.Stream() for _ in range(nf)]
    outs = [torch.empty((rows, W, 3), dtype=torch.float32, device="cuda") for _ in range(nf)]
    outs8 = [torch.empty((rows, W, 3), dtype=torch.uint8, device="cuda") for _ in range(nf)]
    stream, out = streams[0], outs[0]
    workload = f"scene{args.scene}_{rt.scene_name(args.scene)}_{W}x{H}_spp{args.spp}_d{args.bounces}"

    # ---- op model: per-sample event rates of THIS workload (counting variant, untimed) ----
    model_spp = min(args.spp, 8)
    pc = rt.make_params(settings, W, H, spp=model_spp, bounces=args.bounces,
                        row_offset=off, row_stride=stride, row_count=rows, flags=rt.RT_FLAG_COUNT)
    ctx.render_into(cam, pc, out.data_ptr(), stream.cuda_stream)
    cst = ctx.timing()
    counters = cst.counter_dict()
    ops_per_sample = op_model(counters, counters["samples"])

    # Frames are independent, so up to `inflight` frames are queued on their own streams (each with its
    # own context: RNG states, colour stack, schedule): the next frame's blocks fill the SIMDs that
    # the previous frame's last pixels leave idle, and the rank-0 gather of frame k overlaps frame k+1.
    # Every frame is rendered completely; the timed region ends when the last one is retired.
    pending = []
    stats = []

    def launch(k):
        i = k % nf
        # the render kernel writes each finished pixel's PPM bytes too (no separate tonemap pass
        # queued behind the next frame's render blocks)
        ctxs[i].render_into(cam, params, outs[i].data_ptr(), streams[i].cuda_stream, outs8[i].data_ptr())
        pending.append(i)

    def retire():
        i = pending.pop(0)
        st = ctxs[i].timing()                                  # waits on that frame's render events
        torch.cuda.current_stream().wait_stream(streams[i])    # ... and its tonemap
        if world_size > 1:
            if args.dist_backend == "nccl":
                gather_rows(outs8[i], H, W, rank, world_size)  # u8 rows: 3 B/pixel over xGMI
            else:
                gather_rows(outs8[i].cpu(), H, W, rank, world_size)
        stats.append(st)

    def run(frames):
        for k in range(frames):
            if len(pending) == nf:
                retire()
            launch(k)
        while pending:
            retire()

    run(max(args.warmup, 1) if nf > 1 else args.warmup)
    # isolated frames: the render kernel's own duration for the roofline (no overlap); the median
    # of three, since one frame's tail varies by a few percent from run to run
    isos = []
    for _ in range(3):
        launch(0)
        retire()
        isos.append(stats[-1])
    iso = sorted(isos, key=lambda st: st.render_ms)[1]
    stats.clear()
    if world_size > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    if world_size > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world_size > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        if args.dist_backend != "nccl":
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    render_ms = [st.render_ms for st in stats]
    init_ms = [st.init_ms for st in stats]
    sched_ms = [st.sched_ms for st in stats]

    samples_per_step = W * H * args.spp                  # all ranks together
    value = samples_per_step * args.steps / elapsed / 1e6
    mean_render_ms = iso.render_ms
    local_samples = rows * W * args.spp
    achieved = ops_per_sample * local_samples / (mean_render_ms / 1e3) / 1e12

    if rank == 0:
        line = {
            "metric": f"Msamples/sec (pixels x spp / s) at {args.width}x{args.height} spp={args.spp} d={args.bounces}"
                      + (f" scene {args.scene}" if args.scene != 0 else ""),
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: reference scene catalog rebuilt on the host (glibc-rand seed 1), XORWOW seed 1234",
            "config": {
                "workload": workload,
                "scene": args.scene, "width": W, "height": H, "spp": args.spp, "bounces": args.bounces,
                "parallelism": f"rows interleaved x{world_size}" + ((" + RCCL u8 gather" if args.dist_backend == "nccl" else f" + {args.dist_backend} u8 gather") if world_size > 1 else ""),
                "output": "PPM bytes written by the render kernel (rt_context_render_ppm)",
                "pixels_per_gpu": rows * W,
                "frames_in_flight": nf,
                "traversal": TRAV_NAMES.get(cst.traversal, str(cst.traversal)),
                "kernel": {rt.RT_TRAV_STATIC: "rt_static_render (hipRTC)", rt.RT_TRAV_ACCEL: "rt_accel_render (hipRTC)"}.get(
                    cst.traversal, "rt_lane_render (hipRTC)"),
            },
            "kernel_ms": {"render_isolated": round(iso.render_ms, 3), "seed_isolated": round(iso.init_ms, 3),
                          "schedule_isolated": round(iso.sched_ms, 3),
                          "single_frame_msamples_s": round(local_samples / ((iso.render_ms + iso.init_ms +
                                                                             iso.sched_ms) / 1e3) / 1e6, 1),
                          "render_mean_in_flight": round(sum(render_ms) / len(render_ms), 3)},
            "roofline": {
                "bound": "valu",
                "achieved": round(achieved, 3),
                "peak": round(VALU_PEAK_TOPS, 2),
                "unit": "Tops/s",
                "frac": round(achieved / VALU_PEAK_TOPS, 4),
                "traffic": load_traffic(workload),
                "ops_per_sample": round(ops_per_sample, 1),
                "measured_on": "median of three isolated frames: render-kernel HIP events on its stream",
                "counters_per_sample": {k: round(v / max(counters["samples"], 1), 4) for k, v in counters.items()
                                        if k not in ("samples", "max_stack", "stack_overflow", "rng_draws")},
            },
        }
        if world_size == 1 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(world, settings, W, H, args.spp, args.bounces, args.cpu_budget,
                                                    ctx)
            except Exception as e:  # the baseline must never hide the GPU number
                line["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(line), flush=True)
    for c in ctxs:
        c.close()
    if world_size > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
