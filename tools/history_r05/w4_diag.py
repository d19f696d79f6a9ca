#!/usr/bin/env python3
"""Round-5 diagnosis of the 4-wide verified walk's register-budget-dependent mismatch.

    python3 -u tools/r05/w4_diag.py [--seeds 0 3] [--out gpurun_out/w4]

For each random sphere world of tests/test_gpu_parity.py::_random_sphere_world (64x36, spp 4, d12) renders
the 4-wide walk built for 6 and for 5 waves per SIMD, lists the pixels that differ from the oracle, and then
re-renders both builds with RT_JIT_OPTS=-DRT_DBG_PX=<pixel> so that the render kernel prints that pixel's
path segments (rt_body.h, RT_DBG_PX): the first differing line of the two traces is where the builds part.
Code objects of the plain builds are dumped (RT_JIT_DUMP) for an ISA diff.  Test infrastructure: the oracle
is only the checker.
"""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="*", default=[0, 3])
    ap.add_argument("--out", default="gpurun_out/w4")
    ap.add_argument("--waves", type=int, nargs="*", default=[6, 5])
    ap.add_argument("--no-trace", action="store_true", help="only list the differing pixels (builds without RT_DBG_PX)")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    import torch  # noqa: F401  (one HIP runtime per process)
    import cuda_raytracing_amd as rt
    from conftest import oracle_render, bits
    from test_gpu_parity import _random_sphere_world

    os.environ["RT_ACCEL_WIDTH"] = "4"
    os.environ["RT_ACCEL_QUANT"] = "0"
    os.environ["RT_JIT_CACHE_DIR"] = "0"
    report = []
    for seed in a.seeds:
        w, s = _random_sphere_world(seed)
        cam, W, H = rt.camera_from_settings(s, 64, 36)
        p = rt.make_params(s, W, H, spp=4, bounces=12)
        rc, ref, _ = oracle_render(w.scene(), cam, p)
        assert rc == 0
        p.flags = rt.RT_FLAG_FORCE_ACCEL
        diffs = {}
        for wv in a.waves:
            os.environ["RT_ACCEL_WAVES"] = str(wv)
            os.environ.pop("RT_JIT_OPTS", None)
            os.environ["RT_JIT_DUMP"] = str(out)
            runs = []
            for rep in range(a.reps):
                fb, st = rt.render(w.scene(), cam, p, with_stats=True)
                bad = np.argwhere((bits(fb) != bits(ref)).any(axis=-1))
                runs.append([[int(r), int(c)] for r, c in bad])
            os.environ.pop("RT_JIT_DUMP", None)
            diffs[wv] = runs
            print(f"seed {seed} waves {wv}: {[len(x) for x in runs]} differing pixels, first {runs[0][:6]}", flush=True)
            report.append({"seed": seed, "waves": wv, "bad": runs, "traversal": st.traversal})
        first = next((d[0][0] for d in diffs.values() if d[0]), None)
        if first is None or a.no_trace:
            continue
        r, c = first
        px = (r << 16) | c
        gb = fb[r, c]
        print(f"seed {seed}: pixel ({r},{c}) oracle {bits(ref)[r, c].tolist()} last render {bits(fb)[r, c].tolist()}",
              flush=True)
        for wv in a.waves:
            os.environ["RT_ACCEL_WAVES"] = str(wv)
            os.environ["RT_JIT_OPTS"] = f"-DRT_DBG_PX={px}"
            print(f"=== trace seed {seed} waves {wv} pixel ({r},{c})", flush=True)
            fb, st = rt.render(w.scene(), cam, p, with_stats=True)
            ok = bool((bits(fb)[r, c] == bits(ref)[r, c]).all())
            print(f"=== end seed {seed} waves {wv}: pixel matches oracle: {ok}", flush=True)
        os.environ.pop("RT_JIT_OPTS", None)
        del gb
    (out / "report.json").write_text(json.dumps(report))


if __name__ == "__main__":
    main()
