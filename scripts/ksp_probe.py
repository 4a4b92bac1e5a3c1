#!/usr/bin/env python3
"""KSP2 cost by source type on the fabric (tuning aid): one source of each tier x all
destinations per call, wall time per call and path statistics."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401

    from openr_amd import topology as T
    from openr_amd.engine import SpfEngine, decode_paths

    g = T.fabric(5000)
    V = g.num_nodes
    eng = SpfEngine([0])
    eng.set_graph(g)
    deg = np.diff(g.row_ptr)
    picks = {f"id{v}": v for v in [0, 150, 287, 288, 292, 300, 340, 1000, 2500, 4991]}
    for key, s in picks.items():
        dst = np.arange(V, dtype=np.uint32)
        src = np.full(V, s, dtype=np.uint32)
        eng.ksp2_tokens(src[:8], dst[:8], 1024, allow_overflow=True)
        t0 = time.perf_counter()
        t1, t2 = eng.ksp2_tokens(src, dst, 1024, allow_overflow=True)
        dt = time.perf_counter() - t0
        n1 = np.array([r[0] for r in t1]); n2 = np.array([r[0] for r in t2])
        print(f"{key:>8} src={s} deg={deg[s]} ms={dt*1e3:.1f} k1_paths_mean={n1[n1 < 2**31].mean():.2f} "
              f"k2_paths_mean={n2[n2 < 2**31].mean():.2f} overflow={int((n1 >= 2**31).sum() + (n2 >= 2**31).sum())}",
              flush=True)


if __name__ == "__main__":
    main()
