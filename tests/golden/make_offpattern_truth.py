#!/usr/bin/env python3
"""Fixture offpattern_truth_n12.npz: 60-digit truth (make_golden.truth_solve, the reference algorithm
of polynomial_optimization_linear_impl.h:329-369 in mpmath) for the first S = 64 trajectories of each
N = 12 / K = 20 off-pattern batch of test_gpu_parity.test_dl_off_pattern_masks_vs_general_kernel
(tests/_util.off_pattern_batch, B = 437, seed 900 + N + D).  At N = 12 the FP64 reference algorithm is
itself ~1e-5 from truth, so these trajectories are gated against truth at 1e-9, not
against the oracle.  Keys: "<kind>_d<D>_coeffs" [S][K][D][N] and "<kind>_d<D>_sha256" (the inputs).
About 7.6 s per trajectory: ~4 min with 8 processes.

  python tests/golden/make_offpattern_truth.py"""
import hashlib
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

N, K, r, B, S = 12, 20, 3, 437, 64
CASES = [(3, "random"), (3, "accel"), (3, "ends"), (4, "mixed")]
FILE = os.path.join(HERE, "offpattern_truth_n12.npz")


def batch(D, kind):
    from _util import off_pattern_batch
    return off_pattern_batch(N, D, K, B, 900 + N + D, kind)


def digest(vals, mask, times):
    h = hashlib.sha256()
    for a in (vals[:S], mask[:S], times[:S]):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def _one(args):
    from make_golden import truth_solve
    return truth_solve(N, r, *args)[0]


def main():
    out = {}
    jobs = []
    for D, kind in CASES:
        vals, mask, times = batch(D, kind)
        out["%s_d%d_sha256" % (kind, D)] = np.array(digest(vals, mask, times))
        jobs += [(vals[b], mask[b], times[b]) for b in range(S)]
    with Pool(int(os.environ.get("JOBS", "8"))) as p:
        tr = p.map(_one, jobs, chunksize=1)
    for i, (D, kind) in enumerate(CASES):
        out["%s_d%d_coeffs" % (kind, D)] = np.stack(tr[i * S:(i + 1) * S]).astype(np.float64)
    np.savez_compressed(FILE, **out)


if __name__ == "__main__":
    main()
