#!/usr/bin/env python3
"""A/B kernel variants in ONE process on the same device buffers (tuning aid).

  python scripts/sweep.py --topology grid100 --variants "FAM=lvl;FAM=code;WAVE=1"

Each variant is a ';'-separated list of env overrides read by the engine at
launch (OPENR_SPF_GROUP_LANES, OPENR_SPF_BFS_FULL). Rounds are interleaved
(variant A, B, C, A, B, C, ...) and the per-variant median/min kernel time is
reported; results of every variant are checked equal to the first one's.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KEYS = {"FULL": "OPENR_SPF_BFS_FULL", "FAM": "OPENR_SPF_BFS_FAMILY", "GEN": "OPENR_SPF_GENERAL",
        "RING": "OPENR_SPF_RING_CAP", "WAVE": "OPENR_SPF_BFS_WAVE", "PROF": "OPENR_SPF_PROF"}


def parse(v):
    env = {}
    for kv in filter(None, v.split(",")):
        k, val = kv.split("=")
        env[KEYS[k]] = val
    return env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--topology", default="grid100")
    ap.add_argument("--variants", default="FAM=lvl;FAM=code")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--no-metric", action="store_true")
    args = ap.parse_args()
    import torch

    from bench import algorithmic_bytes, build_topology
    from openr_amd.engine import SpfEngine

    g, cfg = build_topology(args.topology)
    V = g.num_nodes
    eng = SpfEngine([0])
    eng.set_graph(g)
    nb = eng.nh_bytes
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    src = torch.arange(0, V, dtype=torch.int32, device=dev)
    d_dist = torch.empty((V, V), dtype=torch.int64, device=dev)
    d_nh = torch.empty((V, V, nb), dtype=torch.uint8, device=dev)
    variants = args.variants.split(";")
    times = {v: [] for v in variants}
    ref = None
    base_env = {k: os.environ.get(k) for k in KEYS.values()}
    for r in range(args.rounds + 1):
        for v in variants:
            for k, val in base_env.items():
                if val is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = val
            os.environ.update(parse(v))
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            eng.solve_device(src.data_ptr(), V, d_dist.data_ptr(), d_nh.data_ptr(), nb, not args.no_metric,
                             stream=stream.cuda_stream)
            b.record(stream)
            torch.cuda.synchronize(dev)
            if r == 0:  # warmup round doubles as the cross-variant equality check
                h = (int(d_dist.sum().item()), int(d_nh.to(torch.int64).sum().item()))
                if ref is None:
                    ref = h
                assert h == ref, f"variant {v} differs: {h} vs {ref}"
                continue
            times[v].append(a.elapsed_time(b))
    B = algorithmic_bytes(g, np.arange(V))
    for v in variants:
        t = np.array(times[v])
        print(json.dumps({"topology": args.topology, "variant": v, "median_ms": float(np.median(t)),
                          "min_ms": float(t.min()), "solves_per_s": V / (np.median(t) / 1e3),
                          "roofline_frac": B / (np.median(t) / 1e3) / 8e12}), flush=True)


if __name__ == "__main__":
    main()
