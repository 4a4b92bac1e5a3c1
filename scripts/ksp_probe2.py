#!/usr/bin/env python3
"""KSP2 cost by destination tier for one RSW and one FSW source (tuning aid)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401

    from openr_amd import topology as T
    from openr_amd.engine import SpfEngine

    g = T.fabric(5000)
    eng = SpfEngine([0])
    eng.set_graph(g)
    groups = {"ssw": range(0, 288), "fsw_own": range(288, 296), "fsw_other": range(296, 960),
              "rsw_own": range(960, 1008), "rsw_other": range(1008, 4992)}
    for src in (960, 300, 5):
        for name, rg in groups.items():
            dst = np.array(list(rg), dtype=np.uint32)
            dst = dst[dst != src]
            srcs = np.full(len(dst), src, dtype=np.uint32)
            eng.ksp2_tokens(srcs[:4], dst[:4], 1024, allow_overflow=True)
            t0 = time.perf_counter()
            t1, t2 = eng.ksp2_tokens(srcs, dst, 1024, allow_overflow=True)
            dt = (time.perf_counter() - t0) * 1e3
            print(f"src={src} {name:10s} n={len(dst):5d} ms={dt:7.1f} us/pair={dt * 1e3 / len(dst):7.1f} "
                  f"k1={np.mean(t1[:, 0]):.2f} k2={np.mean(t2[:, 0]):.2f}", flush=True)


if __name__ == "__main__":
    main()
