"""One rank of the CPU rehearsal of bench.py's N>1 path (tests/test_distributed.py::test_bench_rank_path_gloo).

Started by bench.spawn_ranks (torch.distributed.run on 127.0.0.1) exactly as `bench.py --gpus N` starts its ranks.
Each rank takes its interleaved rows (rt.shard_rows), renders them — with the CPU oracle here, as this container has no
GPU (on the box bench.py renders them with librt_hip) — and hands its u8 rows to bench.gather_frame; rank 0 runs
bench.gather_check against the oracle's bytes of a strided row sample, as bench.py does, and also compares the whole
assembled frame with a single-process oracle frame.

    python -m torch.distributed.run --nproc-per-node 2 tests/dist_rank.py OUT.json W H SPP BOUNCES
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
import cuda_raytracing_amd as rt  # noqa: E402
from conftest import oracle_render  # noqa: E402


def main():
    out = Path(sys.argv[1])
    W, H, spp, bounces = (int(x) for x in sys.argv[2:6])
    world_size = int(os.environ["WORLD_SIZE"])
    plan = bench.launch_plan(world_size, os.environ, 0, "gloo")
    assert plan == ("run", None), plan
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, W, H)
    off, stride, rows = rt.shard_rows(H, rank, world_size)
    rc, shard, _ = oracle_render(w.scene(), cam, rt.make_params(s, W, H, spp=spp, bounces=bounces, row_offset=off,
                                                                 row_stride=stride, row_count=rows))
    assert rc == 0
    img = bench.gather_frame(torch.from_numpy(rt.tonemap(shard)), H, W, rank, world_size, "gloo")
    if rank == 0:
        chk = bench.gather_check(img, H, W, world_size,
                                 lambda step: bench.oracle_rows_u8(w, s, cam, W, H, spp, bounces, step))
        rc, full, _ = oracle_render(w.scene(), cam, rt.make_params(s, W, H, spp=spp, bounces=bounces))
        chk["whole_frame_equal"] = bool(np.array_equal(img.numpy(), rt.tonemap(full)))
        chk["world_size"] = world_size
        out.write_text(json.dumps(chk))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
