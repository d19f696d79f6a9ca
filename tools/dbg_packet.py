import os, sys
import torch
sys.path.insert(0, '/root/repo')
import numpy as np, cuda_raytracing_amd as rt
w, s = rt.build_scene(0)
for W,H,spp,b in ((1,1,1,1),(2,1,1,1),(4,1,1,1),(8,1,1,1),(8,8,1,1),(1,1,4,1),(2,1,4,1)):
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=b, flags=rt.RT_FLAG_COUNT)
    res = {}
    for mode in ('0','1'):
        os.environ['RT_TRAVERSAL'] = mode
        fb, st = rt.render(w.scene(), cam, p, with_stats=True)
        res[mode] = (fb, st.counter_dict())
    diffs = {k: (res['0'][1][k], res['1'][1][k]) for k in res['0'][1] if res['0'][1][k] != res['1'][1][k]}
    print(W, H, spp, b, 'fb equal', np.array_equal(res['0'][0], res['1'][0]), diffs, flush=True)
