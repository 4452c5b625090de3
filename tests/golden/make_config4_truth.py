#!/usr/bin/env python3
"""Fixture config4_truth_sample.npz: 60-digit truth (make_golden.truth_solve, the reference algorithm
of polynomial_optimization_linear_impl.h:329-369 evaluated in mpmath) for a random sample of 256
trajectories of the full-size config-4 batch (1e4 x N = 12, K = 20, JERK; the bench's generator,
createRandomVertices(SNAP, 20, [-10,-20,-10], [10,20,10]) + estimateSegmentTimes(3, 5), seed0 = 0).

The GPU test regenerates the whole batch, solves all 1e4 on the default path and compares the sampled
trajectories with this truth; the SHA-256 of the sampled inputs is stored so a generator change cannot
pass silently.  About 7.6 s per trajectory: run here with 8 processes (~4 min)."""
import hashlib
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

N, K, r, B, S = 12, 20, 3, 10000, 256


def batch():
    from mav_trajectory_generation_cmake_amd import random_vertices_batch
    return random_vertices_batch(N, 3, K, B, [-10.0, -20.0, -10.0], [10.0, 20.0, 10.0], seed0=0,
                                 max_derivative=4, v_max=3.0, a_max=5.0)


def sample_index():
    return np.sort(np.random.default_rng(20).choice(B, S, replace=False))


def inputs_digest(vals, mask, times, idx):
    h = hashlib.sha256()
    for a in (vals[idx], mask[idx], times[idx]):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def _one(args):
    from make_golden import truth_solve
    return truth_solve(N, r, *args)[0]


def main():
    vals, mask, times = batch()
    idx = sample_index()
    with Pool(int(os.environ.get("JOBS", "8"))) as p:
        tr = p.map(_one, [(vals[b], mask[b], times[b]) for b in idx], chunksize=1)
    np.savez_compressed(os.path.join(HERE, "config4_truth_sample.npz"), index=idx,
                        coeffs=np.stack(tr).astype(np.float64),
                        inputs_sha256=np.array(inputs_digest(vals, mask, times, idx)))


if __name__ == "__main__":
    main()
