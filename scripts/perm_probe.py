#!/usr/bin/env python3
"""All-sources kernel time of G100 under node renumberings (tuning aid: ELL-row locality).

  python scripts/perm_probe.py [--reps 10]

Each variant relabels the nodes (new id = p[old]) and keeps every row's edge order, so
the solves are the same up to relabelling; only the memory locality of the frontier's
ELL rows changes. Orders: row-major (the generator's), random, Morton (Z-order of the
grid coordinates), anti-diagonal (r + c major: reverse Cuthill-McKee from a corner).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def relabel(g, p):
    from openr_amd.topology import CsrGraph

    V = g.num_nodes
    inv = np.empty(V, dtype=np.int64)
    inv[p] = np.arange(V)
    rows = [g.col[g.row_ptr[o]:g.row_ptr[o + 1]] for o in inv]
    row_ptr = np.zeros(V + 1, dtype=np.uint32)
    row_ptr[1:] = np.cumsum([len(r) for r in rows])
    col = np.concatenate([p[r] for r in rows]).astype(np.uint32)
    pick = np.concatenate([np.arange(g.row_ptr[o], g.row_ptr[o + 1]) for o in inv])
    names = [g.names[o] for o in inv]
    return CsrGraph(names, row_ptr, col, g.metric[pick], g.link_id[pick], g.edge_up[pick],
                    g.node_overloaded[inv], g.name_rank[inv], g.num_links, g.link_ends,
                    {n: i for i, n in enumerate(names)})


def morton(n):
    def spread(x):
        x = x.astype(np.uint64)
        out = np.zeros_like(x)
        for b in range(8):
            out |= ((x >> b) & 1) << (2 * b)
        return out
    r, c = np.divmod(np.arange(n * n), n)
    key = spread(r) | (spread(c) << 1)
    order = np.argsort(key, kind="stable")
    p = np.empty(n * n, dtype=np.int64)
    p[order] = np.arange(n * n)
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch

    from openr_amd import topology as T
    from openr_amd.engine import SpfEngine

    n = 100
    g0 = T.grid_fast(n)
    V = g0.num_nodes
    r, c = np.divmod(np.arange(V), n)
    rng = np.random.default_rng(7)
    antidiag = np.empty(V, dtype=np.int64)
    antidiag[np.lexsort((c, r + c))] = np.arange(V)
    variants = {"row-major": np.arange(V), "random": rng.permutation(V), "morton": morton(n),
                "anti-diagonal": antidiag}
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    eng = SpfEngine([0])
    for name, p in variants.items():
        g = relabel(g0, np.asarray(p, dtype=np.int64))
        eng.set_graph(g)
        nb = eng.nh_bytes
        src = torch.arange(0, V, dtype=torch.int32, device=dev)
        d_dist = torch.empty((V, V), dtype=torch.int64, device=dev)
        d_nh = torch.empty((V, V, nb), dtype=torch.uint8, device=dev)
        ts = []
        for i in range(args.reps + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            eng.solve_device(src.data_ptr(), V, d_dist.data_ptr(), d_nh.data_ptr(), nb, True,
                             stream=stream.cuda_stream)
            b.record(stream)
            torch.cuda.synchronize(dev)
            if i:
                ts.append(a.elapsed_time(b))
        # a relabelling permutes rows and columns of the distance matrix: its sum is invariant
        print(json.dumps({"order": name, "median_ms": float(np.median(ts)), "min_ms": float(np.min(ts)),
                          "dist_sum": int(d_dist.sum().item())}), flush=True)
        del d_dist, d_nh


if __name__ == "__main__":
    main()
