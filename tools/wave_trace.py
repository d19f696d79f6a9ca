"""Per-wave start/end timeline of one render (RT_WAVE_TRACE diagnostics): tail and launch skew.

    python3 tools/wave_trace.py --scene 0 --spp 512 [--env RT_TILE_ORDER=1]
Prints lifetime statistics in % of the kernel span (s_memrealtime, 100 MHz).
"""
import argparse, os, sys, tempfile
from pathlib import Path
import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("--scene", type=int, default=0)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=512)
ap.add_argument("--bounces", type=int, default=16)
ap.add_argument("--env", action="append", default=[])
a = ap.parse_args()
path = Path(tempfile.mkdtemp()) / "trace.bin"
os.environ["RT_WAVE_TRACE"] = str(path)
for kv in a.env:
    k, v = kv.split("=")
    os.environ[k] = v
import torch  # noqa: F401,E402
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import cuda_raytracing_amd as rt  # noqa: E402

w, s = rt.build_scene(a.scene)
cam, W, H = rt.camera_from_settings(s, a.width, a.height)
fb, st = rt.render(w.scene(), cam, rt.make_params(s, W, H, spp=a.spp, bounces=a.bounces), with_stats=True)
rec = np.fromfile(path, dtype=np.uint64).reshape(-1, 23)
rec = rec[rec[:, 1] > 0]
t0 = rec[:, 0].min()
start = (rec[:, 0] - t0).astype(np.float64)
end = (rec[:, 1] - t0).astype(np.float64)
span = end.max()
life = (end - start) / span
print(f"render {st.render_ms:.2f} ms, waves {len(rec)}, span {span / 100:.0f} us (100 MHz ticks)")
print("start (pct of span): p50 %.1f p90 %.1f max %.1f" % tuple(100 * np.percentile(start / span, [50, 90, 100])))
print("end (pct of span): min %.1f p10 %.1f p50 %.1f p90 %.1f" % tuple(100 * np.percentile(end / span, [0, 10, 50, 90])))
print("lifetime mean %.1f pct of span; idle wave-time %.1f pct" % (100 * life.mean(), 100 * (1 - life.mean())))
tiles = rec[:, 2].astype(np.int64)
print("tiles/wave: min %d mean %.2f max %d" % (tiles.min(), tiles.mean(), tiles.max()))
rounds = rec[:, 4].astype(np.float64); busy = rec[:, 5].astype(np.float64)
print("busy lanes per round (wave mean): %.1f of 64; rounds/wave mean %.0f" % (busy.sum() / rounds.sum(), rounds.mean()))
ph = rec[:, 6:13].astype(np.float64).sum(axis=0)
print("phase cycles: refill %.1f%%  traverse %.1f%%  loop-back %.1f%%  material+scatter %.1f%%  rejection %.1f%%  unwind %.1f%%  "
      "sum+camera/write %.1f%%" % tuple(100 * ph / ph.sum()))
xcc = (rec[:, 3] >> np.uint64(32)).astype(np.int64)
for x in np.unique(xcc):
    m = xcc == x
    print(f"  xcc {x}: waves {m.sum()} end p50 {100 * np.median(end[m] / span):.1f}% max {100 * end[m].max() / span:.1f}%")
top = np.argsort(-end)[:5]
for w in top:
    r = rec[w]
    ph = r[6:13].astype(np.float64)
    print(f"straggler wave {w}: end {100 * end[w] / span:.1f}% rounds {int(r[4])} busy-lane-rounds {int(r[5])} "
          f"tiles {int(r[2])} us/round {(end[w] - start[w]) / 100 / max(int(r[4]), 1):.2f} phases (cycles/round): "
          + " ".join(f"{n} {v / max(int(r[4]), 1):.0f}" for n, v in
                     zip(("refill", "trace", "back", "mat", "rej", "unwind", "cam"), ph)))
# the rounds with at most 2 busy lanes (the tail: trapped pixels alone in their wave)
lr = rec[:, 13].astype(np.float64)
lph = rec[:, 14:21].astype(np.float64)
if lr.sum() > 0:
    tot = lph.sum(axis=0)
    print("tail rounds (<= 2 busy lanes): %d total, %.1f%% of all rounds; cycles/round: " % (lr.sum(), 100 * lr.sum() / rounds.sum())
          + " ".join(f"{n} {v / lr.sum():.0f}" for n, v in zip(("refill", "trace", "back", "mat", "rej", "unwind", "cam"), tot)))
    print("  of which cooperative noise (in mat): all rounds %.0f cycles/round, tail rounds %.0f"
          % (rec[:, 21].astype(np.float64).sum() / rounds.sum(), rec[:, 22].astype(np.float64).sum() / lr.sum()))
    for w in top[:3]:
        if rec[w, 13] > 0:
            print(f"  straggler wave {w}: tail rounds {int(rec[w, 13])} cycles/round: "
                  + " ".join(f"{n} {v / rec[w, 13]:.0f}" for n, v in
                             zip(("refill", "trace", "back", "mat", "rej", "unwind", "cam"), rec[w, 14:21].astype(np.float64))))
# per dispatch rank: block b reaches its CU in round b // n_cu of the dispatch (n_cu = 256 blocks
# per round on MI355X), so its waves are the (b // n_cu)-th oldest of their SIMDs
wid = np.arange(len(rec))
rank = (wid // 4) // 256
for rk in np.unique(rank):
    m = rank == rk
    upr = (end[m] - start[m]) / 100 / np.maximum(rec[m, 4].astype(np.float64), 1)
    print(f"  dispatch rank {rk}: waves {m.sum()} us/round mean {upr.mean():.2f} rounds mean {rec[m, 4].mean():.0f} "
          f"tiles mean {tiles[m].mean():.2f} end p50 {100 * np.median(end[m] / span):.1f}% max {100 * end[m].max() / span:.1f}%")
