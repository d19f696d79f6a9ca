"""First-contact GPU probe: GPU render vs CPU oracle on small cases, then a timing sample."""
import torch
import ctypes as C, sys, time, json
import numpy as np
sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import cuda_raytracing_amd as rt
from cuda_raytracing_amd import _abi

def oracle(sc, cam, p):
    out = np.zeros((p.row_count, p.width, 3), np.float32); st = _abi.Stats()
    rc = _abi.oracle_lib().rt_render_cpu(C.byref(sc), C.byref(cam), C.byref(p), out.ctypes.data_as(C.c_void_p), C.byref(st))
    assert rc == 0, rc
    return out, st

res = {}
for idx, W, H, spp, b in [(0, 64, 36, 4, 4), (0, 96, 54, 16, 16), (1, 48, 48, 8, 50), (17, 64, 36, 8, 50), (2, 64, 36, 4, 16), (3, 32, 32, 2, 40)]:
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=b)
    sc = w.scene()
    t = time.time(); g, gst = rt.render(sc, cam, p, with_stats=True); tg = time.time() - t
    t = time.time(); o, ost = oracle(sc, cam, p); to = time.time() - t
    eq = np.array_equal(g.view(np.uint32), o.view(np.uint32))
    nd = int((g.view(np.uint32) != o.view(np.uint32)).sum())
    md = float(np.abs(g - o).max())
    res[f"{idx}_{W}x{H}_s{spp}_b{b}"] = dict(bit_exact=eq, ndiff=nd, maxdiff=md, gpu_render_ms=gst.render_ms, gpu_init_ms=gst.init_ms, lds=gst.scene_in_lds, stack=gst.stack_needed, oracle_s=to)
    print(idx, W, H, spp, b, 'bit_exact', eq, 'ndiff', nd, 'maxdiff', md, 'gpu ms', gst.render_ms, gst.init_ms, 'lds', gst.scene_in_lds, flush=True)

# timing sample: scene 0 1920x1080 spp 64 d16 via context
w, s = rt.build_scene(0)
cam, W, H = rt.camera_from_settings(s, 1920, 1080)
import torch
for spp in (8, 64):
    p = rt.make_params(s, W, H, spp=spp, bounces=16)
    ctx = rt.RenderContext(w.scene(), 0)
    out = torch.empty((H, W, 3), dtype=torch.float32, device='cuda')
    for it in range(2):
        ctx.render_into(cam, p, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        st = ctx.timing()
    ms = st.render_ms
    print('scene0 1080p spp', spp, 'render ms', ms, 'init ms', st.init_ms, 'Msamples/s', W*H*spp/ms/1e3, flush=True)
    res[f"timing_spp{spp}"] = dict(render_ms=ms, init_ms=st.init_ms, msps=W*H*spp/ms/1e3)
json.dump(res, open('gpurun_out/probe.json', 'w'), indent=1)
