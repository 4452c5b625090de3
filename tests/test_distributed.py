"""Multi-process (gloo, world size 2) tests of the sharded path.

The bench shards one global batch of independent trajectories across ranks
(contiguous seed ranges, no data-path collective) and takes the max of the
ranks' elapsed times.  Here both ranks run on CPU: each generates its shard with
the product's host generator and solves it with the product's host solver
(mtg_host_solve_linear_batch, the same block-Thomas algorithm as the kernels); the
union of the shards' problems and solutions must equal the global batch generated
and solved in one piece, bit for bit; the timing reduce must return the slowest rank."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, out_dir):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import mav_trajectory_generation_cmake_amd as mtg
    vals, mask, times = mtg.random_vertices_path_batch(10, 3, 10, B, seed0=bench.shard_seed0(rank, B))
    sol = mtg.host_solve_linear_batch(10, 4, vals, mask, times, free=True, cost=True, status=True, threads=2)
    el = bench.max_over_ranks(0.25 * (rank + 1), dist)
    np.savez(os.path.join(out_dir, "r%d.npz" % rank), vals=vals, mask=mask, times=times, el=el,
             coeffs=sol["coeffs"], free=sol["free"], cost=sol["cost"], status=sol["status"])
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_cover_global_batch(tmp_path):
    world, B = 2, 37
    mp.spawn(_worker, args=(world, _free_port(), B, str(tmp_path)), nprocs=world, join=True)
    import mav_trajectory_generation_cmake_amd as mtg
    gv, gm, gt = mtg.random_vertices_path_batch(10, 3, 10, world * B, seed0=0)
    gs = mtg.host_solve_linear_batch(10, 4, gv, gm, gt, free=True, cost=True, status=True)
    for r in range(world):
        d = np.load(tmp_path / ("r%d.npz" % r))
        np.testing.assert_array_equal(d["vals"], gv[r * B:(r + 1) * B])
        np.testing.assert_array_equal(d["mask"], gm[r * B:(r + 1) * B])
        np.testing.assert_array_equal(d["times"], gt[r * B:(r + 1) * B])
        for k in ("coeffs", "free", "cost", "status"):
            np.testing.assert_array_equal(d[k], gs[k][r * B:(r + 1) * B])
        assert float(d["el"]) == 0.5  # max over ranks of (0.25, 0.5)
