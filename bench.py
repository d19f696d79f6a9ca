#!/usr/bin/env python3
"""bench.py — Msamples/s of the per-pixel render path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scene 0] [--width 1920] [--height 1080]
                    [--spp 512] [--bounces 16] [--frame weak|fixed] [--pipelined-steps K2]
                    [--no-cpu-baseline] [--no-e2e]

A "step" is one frame, rendered to completion before the next starts (the frames run one after the other
on one stream; the host enqueues the next frame while the GPU renders the current one, so no host
round trip sits between them) — the reference's metric is one
cuda_calc launch (raytracing.cu:1752-1768) with init_gpu_data's seeding (:1746): longest-first schedule probe +
render kernel (RNG seeding fused into its tile pickup) writing float RGB and PPM bytes (+ the RCCL gather of the u8 rows to rank 0 when N>1), with the scene
already resident in HBM.  Default workload = BASELINE config 2: scene 0 (fv1) at 1920x1080, spp 512,
depth 16 on one GPU.  With N ranks (torch.distributed.run, one process per GPU, backend "nccl" = RCCL)
rows are interleaved across ranks and
  --frame weak  (default) the frame grows to ~N x the pixels at the same aspect and camera;
  --frame fixed the stated W x H is split N ways (BASELINE configs 4 and 5: one frame over 8 GPUs).
Rank 0 prints ONE JSON line.  value = samples of all ranks x K / max-over-ranks wall time of the K
timed frames.  Secondary keys: `pipelined` (2 frames in flight on two streams: the next frame fills
the SIMDs the previous frame's last pixels leave idle), `e2e` (bin/raytracing wall time of the whole
reference render() region, cold and warm code-object cache), `cpu_baseline` (the C oracle built
-O3 -march=native on this host, all cores and 1 core, on a bounded row sample whose GPU render is
compared bit for bit).
roofline: VALU-bound kernel; achieved = algorithmic FP32 ops per render launch (op model of SURVEY §8d
on this workload's measured per-sample visit counts) / the render kernel's median duration over the timed
frames, measured by the kernel itself (first wave start to last wave end on the device's s_memrealtime wall
clock, rt_stats.render_kernel_ms — what rocprofv3 reports as the kernel's duration; the stream-event window
around the launch is reported beside it).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import torch  # first: one HIP runtime per process (cuda_raytracing_amd._abi._bind_single_hip_runtime)
import torch.distributed as dist

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))
import cuda_raytracing_amd as rt  # noqa: E402
from cuda_raytracing_amd import _abi  # noqa: E402
from cuda_raytracing_amd.multi_gpu import gather_rows, max_shard_rows, weak_scaled_resolution  # noqa: E402

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


TRAV_NAMES = {0: "lane-dfs", 1: "wave-packet-dfs", 2: "scene-specialised", 3: "verified-sah", 4: "verified-mixed"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def op_model(counters: dict, samples: int) -> float:
    ops = sum(OP_WEIGHTS[k] * counters[k] for k in OP_WEIGHTS) + OPS_PER_SAMPLE_FIXED * samples
    return ops / max(samples, 1)


# the verified SAH walk of all-sphere worlds (AccelTraceK): per executed node visit two child boxes of the
# reference's slab test (2 x visit_bvh), per leaf test one sphere test (visit_sphere)
EXEC_NODE_OPS = 2 * OP_WEIGHTS["visit_bvh"]
EXEC_PRIM_OPS = OP_WEIGHTS["visit_sphere"]


def executed_op_model(counters: dict, samples: int):
    """Ops per sample of the work the verified walk EXECUTES (its node visits and leaf tests, counted by the
    counting variant, exec_node / exec_prim) in place of the reference walk's BVH and sphere visits; None
    when the workload does not take that walk.  The headline frac keeps the reference's visits (the same
    op model in every round); this second frac says how busy the VALU is on the work actually done."""
    if not counters.get("exec_node"):
        return None
    ops = op_model(counters, samples) * max(samples, 1)
    ops -= OP_WEIGHTS["visit_bvh"] * counters["visit_bvh"] + OP_WEIGHTS["visit_sphere"] * counters["visit_sphere"]
    ops += EXEC_NODE_OPS * counters["exec_node"] + EXEC_PRIM_OPS * counters["exec_prim"]
    return ops / max(samples, 1)


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def baseline_oracle():
    """The oracle built for speed on THIS host (BASELINE.md CPU plan: -O3 -march=native -fopenmp), from
    the same source and with the same parity flags (no FP contraction, IEEE div/sqrt).  Built into a
    temporary directory at run time because -march=native must describe the box's own CPU; falls back
    to the prebuilt -O2 test build if no compiler is usable."""
    src = REPO / "oracle" / "oracle_rt.c"
    flags = ["-O3", "-march=native", "-std=c11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fopenmp"]
    d = Path(tempfile.mkdtemp(prefix="rt_cpu_baseline_"))
    lib = d / "liboracle_rt_native.so"
    try:
        r = subprocess.run([os.environ.get("CC", "cc"), *flags, "-I", str(REPO / "include"), "-shared", str(src),
                            "-o", str(lib), "-lm"], capture_output=True, text=True, timeout=120)
        if r.returncode == 0 and lib.exists():
            return _abi.oracle_lib(lib), " ".join(flags)
        log(f"cpu baseline: native build failed ({r.stderr.strip()[:200]}); using the -O2 test build")
    except (OSError, subprocess.TimeoutExpired) as e:
        log(f"cpu baseline: native build failed ({e}); using the -O2 test build")
    return _abi.oracle_lib(), "-O2 -std=c11 -ffp-contract=off -fno-fast-math -fopenmp (prebuilt test build)"


def cpu_quota():
    """CPUs' worth of time the cgroup grants this process (cpu.max quota / period), None if unlimited."""
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(world, settings, W, H, spp, bounces, budget_s, ctx=None):
    """Oracle (C, OpenMP) on this host: the same scene/camera, a bounded row sample, on EVERY core the
    process may run on (sched_getaffinity), on the cgroup's CPU quota, and on 1 core.

    BASELINE.md asks for all host cores.  The GPU box exposes 256 hardware threads to the process but its
    cgroup grants a 16-CPU time quota (cpu.max): a 256-thread run is throttled to that share, so both runs
    are made and the faster one is the headline (`cores` = its thread count; the other is reported beside
    it).  `projection_full_host` scales the measured 1-core rate to the machine's physical cores — a
    projection, not a measurement.  The same sample is then rendered on the GPU through the product context
    and compared bit for bit (the PSNR half of the BASELINE metric: identical frames -> PSNR = inf)."""
    import ctypes as C
    import numpy as np
    L, build = baseline_oracle()
    default_threads = int(L.rt_oracle_threads())
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or default_threads
    quota = cpu_quota()
    cam, W, H = rt.camera_from_settings(settings, W, H)

    def run(stride, s, offset=0):
        rows = len(range(offset, H, stride))
        p = rt.make_params(settings, W, H, spp=s, bounces=bounces, row_offset=offset, row_stride=stride, row_count=rows)
        out = np.zeros((rows, W, 3), np.float32)
        st = _abi.Stats()
        t = time.perf_counter()
        rc = L.rt_render_cpu(C.byref(world.scene()), C.byref(cam), C.byref(p), out.ctypes.data_as(C.c_void_p),
                             C.byref(st))
        dt = time.perf_counter() - t
        assert rc == 0, rc
        return rows * W * s, dt, out

    def sample_stride(budget):
        # calibrate: t = a*pixels (RNG seeding by jumps) + b*samples, from two short runs on every 16th row
        # (run twice at first: the first call also spins up the OpenMP pool)
        s1, s2 = min(spp, 8), min(spp, 32)
        n1, t1, _ = run(16, s1)
        n2, t2, _ = run(16, s2)
        px = n1 / s1
        b = max((t2 - t1) / max(n2 - n1, 1), 1e-12) if s2 > s1 else t1 / n1
        a = max((t1 - b * n1) / px, 0.0)
        return max(1, math.ceil((a * W * H + b * W * H * spp) / budget))

    def leg(threads, budget, offset=0):
        L.rt_oracle_set_threads(threads)
        run(16, 2)
        stride = sample_stride(budget)
        n, dt, out = run(stride, spp, offset)
        return {"threads": threads, "value": round(n / dt / 1e6, 3), "stride": stride, "samples": n, "seconds": dt,
                "out": out}

    legs = []
    try:
        legs.append(leg(affinity, budget_s))                       # every core of the affinity mask
        if quota is not None and int(quota) < affinity:
            legs.append(leg(max(1, int(quota)), budget_s))          # the cgroup's CPU share
        one = leg(1, budget_s / 4)
    finally:
        L.rt_oracle_set_threads(default_threads)
    best = max(legs, key=lambda d: d["value"])
    ref, stride, rows = best["out"], best["stride"], best["out"].shape[0]
    parity = None
    if ctx is not None:
        import torch
        p = rt.make_params(settings, W, H, spp=spp, bounces=bounces, row_offset=0, row_stride=stride, row_count=rows)
        dev = torch.empty((rows, W, 3), dtype=torch.float32, device="cuda")
        ctx.render_into(cam, p, dev.data_ptr(), torch.cuda.current_stream().cuda_stream)
        ctx.timing()
        g = dev.cpu().numpy()
        mse = float(np.mean((np.clip(np.sqrt(g), 0, 1) - np.clip(np.sqrt(ref), 0, 1)) ** 2))
        parity = {"bit_exact": bool(np.array_equal(g.view(np.uint32), ref.view(np.uint32))),
                  "psnr_db": None if mse == 0 else round(10 * math.log10(1.0 / mse), 2),
                  "note": "GPU vs oracle on this sample; psnr_db null = identical frames (PSNR infinite)"}
    phys = affinity // 2 if affinity >= 2 else 1   # 2 hardware threads per core on the EPYC hosts
    return {
        "value": best["value"], "unit": "Msamples/s", "cores": best["threads"], "kind": "port",
        "sample": f"frame rows 0::{stride} ({rows} rows x {W} px) at spp {spp}, d{bounces}: "
                  f"{best['samples']:.3g} samples in {best['seconds']:.1f} s on {best['threads']} threads",
        "legs": [{"threads": d["threads"], "value": d["value"], "sample_rows_stride": d["stride"],
                  "seconds": round(d["seconds"], 2)} for d in legs],
        "single_core": {"value": one["value"], "unit": "Msamples/s", "cores": 1,
                        "sample": f"frame rows 0::{one['stride']} at spp {spp}: {one['samples']:.3g} samples in "
                                  f"{one['seconds']:.1f} s"},
        "projection_full_host": {"value": round(one["value"] * phys, 1), "unit": "Msamples/s", "cores": phys,
                                 "note": "PROJECTION (not measured): 1-core rate x physical cores of the affinity mask"},
        "cpu_model": cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
        "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "build": build,
        "parity": parity,
    }


def e2e_cli(scene: int, W: int, H: int, spp: int, bounces: int):
    """End-to-end wall time of `bin/raytracing` (the reference's `./raytracing scene sN bN` plus the
    resolution flags): scene build, BVH, kernel compile or code-object cache load, upload, RNG seeding,
    render, D2H copy and PPM write (raytracing.cu:1649-1773).  Cold = empty code-object cache (hipRTC
    compiles), warm = a second process that loads the cached code object."""
    exe = REPO / "bin" / "raytracing"
    if not exe.exists():
        return {"error": "bin/raytracing not built"}
    d = Path(tempfile.mkdtemp(prefix="rt_e2e_"))
    env = dict(os.environ, RT_JIT_CACHE_DIR=str(d / "cache"))
    res = {"command": f"bin/raytracing {scene} s{spp} b{bounces} w{W} h{H}"}
    try:
        for leg in ("cold", "warm"):
            t = time.perf_counter()
            r = subprocess.run([str(exe), str(scene), f"s{spp}", f"b{bounces}", f"w{W}", f"h{H}"], cwd=d,
                               capture_output=True, text=True, timeout=600, env=env)
            wall = time.perf_counter() - t
            if r.returncode != 0:
                return {"error": (r.stdout + r.stderr)[-400:]}
            info = {"process_wall_ms": round(wall * 1e3, 1)}
            for line in r.stdout.splitlines():
                if line.startswith("End-to-end:"):
                    info["e2e_ms"] = round(float(line.split(":")[1].split("ms")[0]), 1)
                    info["kernels"] = line.split("[", 1)[1].split("]", 1)[0]
                elif line.startswith("Rendering time:") and line.rstrip().endswith("ms"):
                    info["render_ms"] = round(float(line.split(":")[1].split("ms")[0]), 3)
                elif line.startswith("RNG seeding time:"):
                    info["seed_ms"] = round(float(line.split(":")[1].split("ms")[0]), 3)
            res[leg] = info
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return res


def load_traffic(workload: str, key: str = "bytes"):
    """PMC HBM bytes per launch of the render kernel ("bytes") or of the whole step ("step_bytes": seeding,
    probe, tile order, render), from profiles/hbm_traffic.json (tools/traffic_from_pmc.py)."""
    f = REPO / "profiles" / "hbm_traffic.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text()).get(workload)
        return int(d[key]) if d and key in d else None
    except Exception:
        return None


def launch_plan(gpus: int, env, device_count: int, backend: str = "nccl"):
    """How `bench.py --gpus N` runs: ("run", None) in this process, ("spawn", n) = start n rank processes (no
    launcher set WORLD_SIZE and N > 1), or ("error", message).  Decided before the first GPU call: counting
    devices does not initialise the GPU.  The reference renders on one device (raytracing.cu:1649-1773); N ranks
    take interleaved rows (multi_gpu.py) and are one process per GPU, so N ranks need N devices — except the gloo
    rehearsal, which may share one device between ranks."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        if gpus <= 1:
            return "run", None
        if device_count < gpus:
            return "error", (f"--gpus {gpus} needs {gpus} GPUs (one rank per GPU) but {device_count} "
                             f"{'is' if device_count == 1 else 'are'} visible; refusing to report a smaller run")
        return "spawn", gpus
    world = int(ws)
    if world != gpus:
        return "error", f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks"
    if world > 1 and backend == "nccl" and device_count < world:
        return "error", f"WORLD_SIZE={world} ranks over RCCL need {world} GPUs, {device_count} visible"
    return "run", None


def spawn_ranks(n: int, argv, script=None, env=None) -> int:
    """--gpus N without a launcher: run this script as N ranks under torch.distributed.run (one process per GPU,
    rendezvous on 127.0.0.1), as a child process; returns its exit code.  This process has not touched the GPU.
    (script: another rank program under the same launcher — tests/dist_rank.py drives the gather path on CPU.)"""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(script or Path(__file__).resolve()), *argv]
    log("launching: " + " ".join(cmd))
    return subprocess.run(cmd, env=env).returncode


def gather_frame(local_u8: "torch.Tensor", H: int, W: int, rank: int, world: int, backend: str):
    """The frame's one collective: every rank's u8 PPM rows to rank 0 (RCCL over xGMI with "nccl"; host tensors with
    gloo), re-interleaved there (multi_gpu.gather_rows); None on the other ranks."""
    return gather_rows(local_u8 if backend == "nccl" else local_u8.cpu(), H, W, rank, world)


def gather_check_step(H: int, world: int) -> int:
    """Row stride of rank 0's check of the gathered frame: co-prime with the world size, so every rank's rows are among
    the checked ones, and ~17 rows at 1080p (a bounded oracle sample); small frames: about 5 rows or more."""
    step = 67 if H > 67 * 4 else max(1, H // 5)
    while math.gcd(step, world) != 1:
        step -= 1
    return max(step, 1)


def gather_check(img, H: int, W: int, world: int, reference_rows) -> dict:
    """Rank 0, untimed: rows 0::step of the assembled frame against reference_rows(step) (u8 [rows, W, 3], the CPU
    oracle's bytes of those rows — the checker).  The RNG subsequence is the global pixel index, so shards + gather +
    un-permute must reproduce the oracle's rows byte for byte."""
    import numpy as np
    step = gather_check_step(H, world)
    ref = np.asarray(reference_rows(step))
    got = img[0::step].cpu().numpy()
    return {"gather_bit_exact": bool(got.shape == ref.shape and np.array_equal(got, ref)),
            "checked_rows": f"0::{step} ({ref.shape[0]} rows x {W} px, ranks {sorted({r % world for r in range(0, H, step)})})",
            "checked_against": "CPU oracle (oracle/oracle_rt.c, the checker) bytes of those rows"}


def oracle_rows_u8(world_, settings, cam, W, H, spp, bounces, step):
    """The checker's bytes of rows 0::step: the CPU oracle's float rows (all host threads) through the host tonemap
    (pixels_to_ppm's conversion, rt_host)."""
    import ctypes as C
    import numpy as np
    rows = len(range(0, H, step))
    p = rt.make_params(settings, W, H, spp=spp, bounces=bounces, row_offset=0, row_stride=step, row_count=rows)
    out = np.zeros((rows, W, 3), np.float32)
    st = _abi.Stats()
    rc = _abi.oracle_lib().rt_render_cpu(C.byref(world_.scene()), C.byref(cam), C.byref(p),
                                         out.ctypes.data_as(C.c_void_p), C.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle rows failed: {rc}")
    return rt.tonemap(out)


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
    ap.add_argument("--frame", choices=("weak", "fixed"), default="weak",
                    help="N>1: weak = ~N x the pixels (fixed work per GPU), fixed = the stated frame split N ways")
    ap.add_argument("--pipelined-steps", type=int, default=-1,
                    help="frames of the secondary 2-in-flight measurement (default: --steps; 0 = skip)")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of oracle wall time (bounded sample)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the bin/raytracing end-to-end leg")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL, default) or gloo (plumbing rehearsal)")
    args = ap.parse_args()

    plan, what = launch_plan(args.gpus, os.environ, torch.cuda.device_count(), args.dist_backend)
    if plan == "error":
        log(f"bench.py: {what}")
        sys.exit(2)
    if plan == "spawn":
        sys.exit(spawn_ranks(what, sys.argv[1:]))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local_rank % max(torch.cuda.device_count(), 1)   # == local_rank on a node with a GPU per rank
    torch.cuda.set_device(dev)
    if world_size > 1:
        if args.dist_backend == "nccl":   # RCCL over xGMI, one rank per GPU
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:                             # rehearsal of the multi-rank plumbing (CPU collectives)
            dist.init_process_group(args.dist_backend)

    # ---- host pre-pass (untimed, like the reference's make_bvh + camera) ----
    world, settings = rt.build_scene(args.scene)
    if args.frame == "weak":
        W, H = weak_scaled_resolution(args.width, args.height, world_size)
    else:
        W, H = args.width, args.height
    cam, W, H = rt.camera_from_settings(settings, W, H)
    off, stride, rows = rt.shard_rows(H, rank, world_size)
    params = rt.make_params(settings, W, H, spp=args.spp, bounces=args.bounces,
                            row_offset=off, row_stride=stride, row_count=rows)
    ctxs = [rt.RenderContext(world.scene(), device=dev) for _ in range(2)]
    ctx = ctxs[0]
    streams = [torch.cuda.Stream() for _ in range(2)]
    outs = [torch.empty((rows, W, 3), dtype=torch.float32, device="cuda") for _ in range(2)]
    outs8 = [torch.empty((rows, W, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    workload = f"scene{args.scene}_{rt.scene_name(args.scene)}_{W}x{H}_spp{args.spp}_d{args.bounces}"

    # ---- op model: per-sample event rates of THIS workload (counting variant, untimed) ----
    model_spp = min(args.spp, 8)
    pc = rt.make_params(settings, W, H, spp=model_spp, bounces=args.bounces,
                        row_offset=off, row_stride=stride, row_count=rows, flags=rt.RT_FLAG_COUNT)
    # (on the second slot's context: its buffers are allocated here, untimed, as the first slot's are by the
    # warmup frame)
    ctxs[1].render_into(cam, pc, outs[1].data_ptr(), streams[0].cuda_stream)
    cst = ctxs[1].timing()
    counters = cst.counter_dict()
    ops_per_sample = op_model(counters, counters["samples"])

    pending = []
    stats = []
    gathered = {}   # rank 0: the last frame assembled from every rank's u8 rows

    def launch(k, nf):
        # two slots (context + output buffers); nf = 1: both slots on ONE stream, so frames run strictly one
        # after the other on the GPU while the host stays one frame ahead; nf = 2: a stream per slot, so a
        # frame's tail overlaps the next frame
        i = k % 2
        s = streams[i] if nf > 1 else streams[0]
        # the slot's buffers may still be read by the previous frame's gather on the current stream
        s.wait_stream(torch.cuda.current_stream())
        # the render kernel writes each finished pixel's PPM bytes too (no separate tonemap pass)
        ctxs[i].render_into(cam, params, outs[i].data_ptr(), s.cuda_stream, outs8[i].data_ptr())
        pending.append((i, s))

    def retire():
        i, s = pending.pop(0)
        st = ctxs[i].timing()                                  # waits on that frame's render events
        torch.cuda.current_stream().wait_stream(s)
        if world_size > 1:
            img = gather_frame(outs8[i], H, W, rank, world_size, args.dist_backend)   # u8 rows: 3 B/pixel over xGMI
            if img is not None:
                gathered["img"] = img
        stats.append(st)

    def run(frames, nf):
        for k in range(frames):
            if len(pending) == 2:
                retire()
            launch(k, nf)
        while pending:
            retire()

    def timed(frames, nf):
        stats.clear()
        if world_size > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(frames, nf)
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
        return elapsed, list(stats)

    samples_per_step = W * H * args.spp                  # all ranks together
    local_samples = rows * W * args.spp

    # ---- headline: one frame at a time (the reference's one-launch metric) ----
    run(args.warmup, 1)
    elapsed, fstats = timed(args.steps, 1)
    value = samples_per_step * args.steps / elapsed / 1e6
    med = lambda xs: sorted(xs)[len(xs) // 2]  # noqa: E731
    render_ms = med([st.render_kernel_ms if st.render_kernel_ms > 0 else st.render_ms for st in fstats])
    render_event_ms = med([st.render_ms for st in fstats])
    # frames run one after the other on one stream, so the timed frames' kernel spans cannot add up to more
    # than the timed wall time: mean span <= mean step (a span above it would be a timing defect)
    spans = [st.render_kernel_ms if st.render_kernel_ms > 0 else st.render_ms for st in fstats]
    render_mean_ms = sum(spans) / len(spans)
    step_mean_ms = elapsed / args.steps * 1e3
    timing_consistent = render_mean_ms <= step_mean_ms
    if not timing_consistent:
        log(f"bench.py: timing defect: mean render span {render_mean_ms:.3f} ms > mean step {step_mean_ms:.3f} ms")
    seed_ms = med([st.init_ms for st in fstats])
    sched_ms = med([st.sched_ms for st in fstats])
    achieved = ops_per_sample * local_samples / (render_ms / 1e3) / 1e12
    exec_ops = executed_op_model(counters, counters["samples"])

    # ---- secondary: two frames in flight (independent frames overlap their tails) ----
    psteps = args.steps if args.pipelined_steps < 0 else args.pipelined_steps
    pipelined = None
    if psteps > 0:
        run(2, 2)
        pel, pst = timed(psteps, 2)
        pipelined = {"value": round(samples_per_step * psteps / pel / 1e6, 2), "unit": "Msamples/s",
                     "frames_in_flight": 2, "steps": psteps, "ms_per_step": round(pel / psteps * 1e3, 3),
                     "render_ms_mean": round(sum(st.render_ms for st in pst) / len(pst), 3)}

    # ---- N>1: rank 0 checks the gathered frame (untimed) against the CPU oracle's bytes of a strided row sample
    # (rows of every rank): the RNG subsequence is the global pixel index, so the shards, the gather and the
    # un-permute must put every pixel in place byte for byte (the oracle is the checker here, never measured) ----
    dist_check = None
    if world_size > 1:
        dist_check = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
                      "gather_bytes_per_frame": max_shard_rows(H, world_size) * W * 3 * world_size,
                      "gather_bit_exact": None}
        if rank == 0 and "img" in gathered:
            dist_check.update(gather_check(gathered["img"], H, W, world_size,
                                           lambda step: oracle_rows_u8(world, settings, cam, W, H, args.spp,
                                                                       args.bounces, step)))
        dist.barrier()

    if rank == 0:
        line = {
            "metric": f"Msamples/sec (pixels x spp / s) at {W}x{H} spp={args.spp} d={args.bounces}"
                      + (f" scene {args.scene}" if args.scene != 0 else ""),
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak" if (args.frame == "weak" or world_size == 1) else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: reference scene catalog rebuilt on the host (glibc-rand seed 1), XORWOW seed 1234",
            "config": {
                "workload": workload,
                "scene": args.scene, "width": W, "height": H, "spp": args.spp, "bounces": args.bounces,
                "frame": args.frame,
                "parallelism": f"rows interleaved x{world_size}" + ((" + RCCL u8 gather" if args.dist_backend == "nccl" else f" + {args.dist_backend} u8 gather") if world_size > 1 else ""),
                "step": "one frame to completion: schedule probe + render (RNG seeding at tile pickup, float RGB + PPM bytes); "
                        "frames in order on one stream, the host one frame ahead"
                        + (" + gather to rank 0" if world_size > 1 else ""),
                "pixels_per_gpu": rows * W,
                "traversal": TRAV_NAMES.get(cst.traversal, str(cst.traversal)),
                # the launched render kernel as the register allocator built it (rt_stats.kernel, code-object metadata)
                "kernel_build": fstats[-1].kernel.as_dict(),
                "kernel": {rt.RT_TRAV_STATIC: "rt_static_render (hipRTC)", rt.RT_TRAV_ACCEL: "rt_accel_render (hipRTC)",
                           rt.RT_TRAV_MIXED: "rt_mixed_render (hipRTC)"}.get(
                    cst.traversal, "rt_lane_render (hipRTC)"),
            },
            "timing_consistent": timing_consistent,
            "kernel_ms": {"render_median": round(render_ms, 3), "render_mean": round(render_mean_ms, 3),
                          "render_event_median": round(render_event_ms, 3),
                          "seed_median": round(seed_ms, 3),
                          "schedule_median": round(sched_ms, 3),
                          "render_only_msamples_s": round(local_samples / (render_ms / 1e3) / 1e6, 1)},
            "pipelined": pipelined,
            "distributed": dist_check,
            "roofline": {
                "bound": "valu",
                "achieved": round(achieved, 3),
                "peak": round(VALU_PEAK_TOPS, 2),
                "unit": "Tops/s",
                "frac": round(achieved / VALU_PEAK_TOPS, 4),
                "traffic": load_traffic(workload),
                "step_traffic": load_traffic(workload, "step_bytes"),
                "ops_per_sample": round(ops_per_sample, 1),
                "executed": None if exec_ops is None else {
                    "ops_per_sample": round(exec_ops, 1),
                    "frac": round(exec_ops * local_samples / (render_ms / 1e3) / 1e12 / VALU_PEAK_TOPS, 4),
                    "note": "verified SAH walk's executed node visits (2 boxes each) and leaf tests instead of the "
                            "reference tree's visits"},
                "measured_on": "median render-kernel duration over the timed frames, from the kernel's own first-wave-start "
                               "to last-wave-end s_memrealtime stamps (rt_stats.render_kernel_ms)",
                "counters_per_sample": {k: round(v / max(counters["samples"], 1), 4) for k, v in counters.items()
                                        if k not in ("samples", "max_stack", "stack_overflow", "rng_draws")},
            },
        }
        if world_size == 1 and not args.no_e2e:
            try:
                line["e2e"] = {"config1": e2e_cli(0, 256, 144, 4, 4),
                               "this_config": e2e_cli(args.scene, W, H, args.spp, args.bounces)}
            except Exception as e:  # the secondary legs must never hide the GPU number
                line["e2e"] = {"error": str(e)}
        if world_size == 1 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(world, settings, W, H, args.spp, args.bounces, args.cpu_budget,
                                                    ctx)
            except Exception as e:
                line["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(line), flush=True)
    for c in ctxs:
        c.close()
    if world_size > 1:
        dist.destroy_process_group()
    if not timing_consistent:   # the line above carries the measurement; the run still fails
        sys.exit(3)


if __name__ == "__main__":
    main()
