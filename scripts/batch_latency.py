#!/usr/bin/env python3
"""Kernel time of one all-sources launch vs batch size (strong-scaling shard sizes).

  python scripts/batch_latency.py --topology grid100 --sizes 1250,2500,5000,10000

Each size is the source count one rank of an N-GPU strong-scaling run gets (V / N); the
kernel time at V / N is the per-GPU step time of that run. Tuning aid (no oracle).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--topology", default="grid100")
    ap.add_argument("--sizes", default="1250,2500,5000,10000")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="",
                    help="';'-separated env settings (K=V,K2=V2 with full OPENR_* names) timed interleaved per size")
    args = ap.parse_args()
    import torch

    from bench import build_topology
    from openr_amd.engine import SpfEngine

    g, _ = build_topology(args.topology)
    V = g.num_nodes
    eng = SpfEngine([0])
    eng.set_graph(g)
    nb = eng.nh_bytes
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    d_dist = torch.empty((V, V), dtype=torch.int64, device=dev)
    d_nh = torch.empty((V, V, nb), dtype=torch.uint8, device=dev)
    variants = [v for v in args.variants.split(";")] if args.variants else [""]
    keys = {kv.split("=")[0] for v in variants for kv in v.split(",") if kv}
    for n in [int(x) for x in args.sizes.split(",")]:
        src = torch.arange(0, n, dtype=torch.int32, device=dev)
        ts = {v: [] for v in variants}
        ref = None
        for r in range(args.reps + 2):
            for v in variants:
                for k in keys:
                    os.environ.pop(k, None)
                os.environ.update(dict(kv.split("=") for kv in v.split(",") if kv))
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                eng.solve_device(src.data_ptr(), n, d_dist.data_ptr(), d_nh.data_ptr(), nb, True,
                                 stream=stream.cuda_stream)
                b.record(stream)
                b.synchronize()
                if r == 0 and len(variants) > 1:  # cross-variant equality of the rows
                    h = (int(d_dist[:n].sum().item()), int(d_nh[:n].to(torch.int64).sum().item()))
                    ref = ref or h
                    assert h == ref, f"variant {v} differs"
                if r >= 2:
                    ts[v].append(a.elapsed_time(b))
        for v in variants:
            t = sorted(ts[v])
            print(json.dumps({"topology": args.topology, "variant": v, "sources": n, "ideal_gpus": V / n,
                              "median_ms": t[len(t) // 2], "min_ms": t[0],
                              "solves_per_s": n / (t[len(t) // 2] / 1e3)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
