"""Multi-rank frame sharding + gather, world_size 2 over gloo on CPU.

The GPU bench runs the same cuda_raytracing_amd.multi_gpu.gather_rows over RCCL; here each rank renders
its row-interleaved shard with the CPU oracle (test infrastructure) and rank 0 checks the gathered
frame against a single-process render bit for bit.
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, bits, oracle_render


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, W, H, result):
    sys.path.insert(0, str(REPO))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cuda_raytracing_amd as rt
    from cuda_raytracing_amd.multi_gpu import gather_rows
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, W, H)
    off, stride, cnt = rt.shard_rows(H, rank, world)
    rc, shard, _ = oracle_render(w.scene(), cam, rt.make_params(s, W, H, spp=3, bounces=6, row_offset=off,
                                                                 row_stride=stride, row_count=cnt))
    assert rc == 0
    img = gather_rows(torch.from_numpy(shard), H, W, rank, world)
    # the u8 (PPM byte) gather the bench uses after the device tonemap: 4x smaller messages
    img8 = gather_rows(torch.from_numpy(rt.tonemap(shard)), H, W, rank, world)
    if rank == 0:
        rc, full, _ = oracle_render(w.scene(), cam, rt.make_params(s, W, H, spp=3, bounces=6))
        result["equal"] = bool(np.array_equal(bits(img.numpy()), bits(full)))
        result["equal_u8"] = bool(np.array_equal(img8.numpy(), rt.tonemap(full)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("H", [17, 18])
def test_gather_rows_world2(H):
    mgr = mp.Manager()
    result = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), 24, H, result), nprocs=2, join=True)
    assert result.get("equal") is True
    assert result.get("equal_u8") is True


@pytest.mark.parametrize("world,H", [(2, 22), (3, 31)])
def test_bench_rank_path_gloo(tmp_path, world, H):
    """bench.py's N>1 path end to end on CPU: launch_plan decides to spawn, spawn_ranks starts the ranks under
    torch.distributed.run (127.0.0.1), each rank's rows go through bench.gather_frame (gloo), and rank 0's
    bench.gather_check compares the assembled rows with the oracle's bytes (tests/dist_rank.py)."""
    sys.path.insert(0, str(REPO))
    import bench
    assert bench.launch_plan(world, {}, world, "gloo") == ("spawn", world)
    out = tmp_path / "chk.json"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    rc = bench.spawn_ranks(world, [str(out), "40", str(H), "3", "5"], script=REPO / "tests" / "dist_rank.py", env=env)
    assert rc == 0
    import json
    d = json.loads(out.read_text())
    assert d["world_size"] == world
    assert d["gather_bit_exact"] is True, d
    assert d["whole_frame_equal"] is True
    ranks = d["checked_rows"].split("ranks ")[1].rstrip(")")
    assert ranks == str(list(range(world))), d   # the checked rows cover every rank's shard


def test_weak_scaled_resolution():
    from cuda_raytracing_amd.multi_gpu import weak_scaled_resolution
    assert weak_scaled_resolution(1920, 1080, 1) == (1920, 1080)
    assert weak_scaled_resolution(1920, 1080, 4) == (3840, 2160)
    W, H = weak_scaled_resolution(1920, 1080, 8)
    assert abs(W * H / (1920 * 1080) - 8) < 0.01


# ---- one process, N devices through the C-ABI (rt_multi_render / rt_render_devices, rt_multi.cpp) ----
# The device code is exercised by tests/test_gpu_parity.py (N = 1 on the GPU box); here the row deal and the
# gather + un-permute are checked on the CPU: the shards the library's row map assigns, rendered by the oracle,
# padded to the longest shard and concatenated in device order (ncclGather's layout on the root), then put back
# in frame order through the same map, must give the single-process frame bit for bit.
@pytest.mark.parametrize("H,n", [(17, 1), (17, 2), (17, 3), (18, 8), (5, 8), (1, 4), (30, 7)])
def test_multi_row_map_gather_unpermute(H, n):
    import cuda_raytracing_amd as rt
    W = 20
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, W, H)
    rc, full, _ = oracle_render(w.scene(), cam, rt.make_params(s, W, H, spp=2, bounces=5))
    assert rc == 0
    maps = [rt.multi_row_map(H, n, k) for k in range(H)]
    max_rows = maps[0][3]
    assert max_rows == len(range(0, H, n))
    # the deal is a bijection onto (device, local row) with every shard's rows contiguous from 0
    assert sorted((d, l) for d, l, _, _ in maps) == sorted((d, l) for d in range(n) for l in range(len(range(d, H, n))))
    for d, l, rows_d, m in maps:
        assert rows_d == len(range(d, H, n)) and m == max_rows and l < rows_d
    gathered = np.zeros((n * max_rows, W, 3), np.float32)
    for d in range(n):
        off, stride, cnt = rt.shard_rows(H, d, n)
        assert cnt == len([1 for dd, _, _, _ in maps if dd == d])
        if cnt:
            rc, shard, _ = oracle_render(w.scene(), cam, rt.make_params(s, W, H, spp=2, bounces=5, row_offset=off,
                                                                         row_stride=stride, row_count=cnt))
            gathered[d * max_rows:d * max_rows + cnt] = shard
    frame = np.stack([gathered[d * max_rows + l] for d, l, _, _ in maps])
    assert np.array_equal(bits(frame), bits(full))


def test_multi_row_map_rejects_bad_geometry():
    import cuda_raytracing_amd as rt
    for args in ((5, 0, 0), (5, 2, 5), (5, 2, -1), (-1, 2, 0)):
        with pytest.raises(rt.RenderError):
            rt.multi_row_map(*args)
