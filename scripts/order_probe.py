#!/usr/bin/env python3
"""Does the order of sources in an all-sources launch matter? (tuning probe)

Times one all-sources launch with the sources in id order and in descending
eccentricity order (longest-processing-time first: the dynamically scheduled
workgroups finish together instead of ending on a tail of deep solves). Rows are
permuted back and checked equal.

  python scripts/order_probe.py --topology grid100 --rounds 7
"""
import argparse
import json
import os
import sys
from collections import deque

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def eccentricity(g):
    """Exact hop eccentricity per node (host BFS from every node; probe only)."""
    V = g.num_nodes
    rp, col = g.row_ptr, g.col
    ecc = np.zeros(V, np.int32)
    for s in range(V):
        lv = np.full(V, -1, np.int32)
        lv[s] = 0
        q = deque([s])
        m = 0
        while q:
            u = q.popleft()
            for e in range(rp[u], rp[u + 1]):
                v = int(col[e])
                if lv[v] < 0:
                    lv[v] = lv[u] + 1
                    m = lv[v]
                    q.append(v)
        ecc[s] = m
    return ecc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--topology", default="grid100")
    ap.add_argument("--rounds", type=int, default=7)
    args = ap.parse_args()
    import torch

    from bench import build_topology
    from openr_amd.engine import SpfEngine

    g, _ = build_topology(args.topology)
    V = g.num_nodes
    if args.topology == "grid100":
        n = 100
        ecc = np.array([max(r, n - 1 - r) + max(c, n - 1 - c) for r in range(n) for c in range(n)])
    else:
        ecc = eccentricity(g)
    eng = SpfEngine([0])
    eng.set_graph(g)
    nb = eng.nh_bytes
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    orders = {"id": np.arange(V), "lpt": np.argsort(-ecc, kind="stable"), "spt": np.argsort(ecc, kind="stable"),
              "rev": np.arange(V)[::-1].copy()}
    srcs = {k: torch.tensor(v.astype(np.int32), device=dev) for k, v in orders.items()}
    d_dist = torch.empty((V, V), dtype=torch.int64, device=dev)
    d_nh = torch.empty((V, V, nb), dtype=torch.uint8, device=dev)
    times = {k: [] for k in orders}
    rows = {}
    for r in range(args.rounds):
        for k in orders:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(stream)
            eng.solve_device(srcs[k].data_ptr(), V, d_dist.data_ptr(), d_nh.data_ptr(), nb, True,
                             stream=stream.cuda_stream)
            ev1.record(stream)
            torch.cuda.synchronize(dev)
            if r:
                times[k].append(ev0.elapsed_time(ev1))
            if r == 0:
                inv = np.empty(V, np.int64)
                inv[orders[k]] = np.arange(V)
                rows[k] = d_dist[torch.tensor(inv, device=dev)][:, :64].cpu().numpy()
    for k in orders:
        assert np.array_equal(rows[k], rows["id"]), k
    print(json.dumps({k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v))} for k, v in times.items()}))
    eng.close()


if __name__ == "__main__":
    main()
