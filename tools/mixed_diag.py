"""Mixed-world walk diagnostics on the GPU: final_scene (or another) frame time, macro fallbacks, occupancy,
under A/B environment settings (each in a child process, since the knobs are read at context creation).

    python3 tools/mixed_diag.py [--scene 3] [--size 800 | --width W --height H] [--spp 16] [--bounces 40] VAR=VAL,VAR=VAL ...
"""
import json, os, subprocess, sys

args = sys.argv[1:]
def opt(name, default):
    if name in args:
        i = args.index(name); v = args[i + 1]; del args[i:i + 2]; return v
    return default
scene, size, spp, b = int(opt("--scene", 3)), int(opt("--size", 800)), int(opt("--spp", 16)), int(opt("--bounces", 40))
width, height = int(opt("--width", size)), int(opt("--height", size))
child = r'''
import json, sys, time
sys.path.insert(0, "REPO")
import torch
import cuda_raytracing_amd as rt
w, s = rt.build_scene(SCENE)
cam, W, H = rt.camera_from_settings(s, WIDTH, HEIGHT)
p = rt.make_params(s, W, H, spp=SPP, bounces=B)
ctx = rt.RenderContext(w.scene(), 0)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
ms = []
for k in range(3):
    ctx.render_into(cam, p, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    st = ctx.timing()
    ms.append(st.render_ms)
import hashlib
frame = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:16]   # every schedule must give this frame
print(json.dumps({"render_ms": sorted(ms)[1], "traversal": st.traversal, "mix_fallbacks": st.mix_fallbacks,
                  "mix_macros": st.mix_macros, "msamples_s": W * H * SPP / sorted(ms)[1] / 1e3, "frame_sha1": frame}))
'''.replace("REPO", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))).replace("SCENE", str(scene)) \
   .replace("WIDTH", str(width)).replace("HEIGHT", str(height)).replace("SPP", str(spp)).replace("B)", str(b) + ")")
for cfg in (args or [""]):
    env = dict(os.environ, RT_DEBUG="1")
    for kv in filter(None, cfg.split(",")):
        k, v = kv.split("=", 1)
        env[k] = v
    r = subprocess.run([sys.executable, "-c", child], env=env, capture_output=True, text=True, timeout=600)
    occ = [l for l in r.stderr.splitlines() if "launch:" in l or "occupancy" in l or "fallbacks" in l or "diag" in l][-4:]
    print(json.dumps({"cfg": cfg, "result": r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-800:],
                      "debug": occ}), flush=True)
    if r.returncode != 0:
        sys.exit(r.returncode)
