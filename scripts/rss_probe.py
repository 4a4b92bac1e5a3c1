#!/usr/bin/env python3
"""Resident set of the routes workload by stage (tuning aid): interpreter + numpy, the
topology, the AdjDbBatch / RouteBuilder (engine context), an 8-node build, the all-node
build."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rss_mb():
    with open("/proc/self/status") as f:
        for l in f:
            if l.startswith("VmRSS:"):
                return int(l.split()[1]) / 1024.0
    return -1.0


def top_maps(tag, k=12):
    """The largest mappings by resident size (/proc/self/smaps)."""
    maps, cur = [], None
    with open("/proc/self/smaps") as f:
        for l in f:
            parts = l.split()
            if "-" in parts[0] and len(parts) >= 5 and ":" in parts[3]:
                cur = [parts[5] if len(parts) > 5 else "[anon]", 0]
                maps.append(cur)
            elif parts[0] == "Rss:" and cur is not None:
                cur[1] = int(parts[1])
    by = {}
    for name, kb in maps:
        by[name] = by.get(name, 0) + kb
    top = sorted(by.items(), key=lambda x: -x[1])[:k]
    print(f"{tag}: " + ", ".join(f"{n.split('/')[-1]} {kb / 1024:.0f} MB" for n, kb in top), flush=True)


def main():
    import resource

    import numpy as np

    print(f"start {rss_mb():.0f} MB", flush=True)
    from bench import build_topology
    from openr_amd import adjdb

    g, _ = build_topology("grid100")
    print(f"topology {rss_mb():.0f} MB", flush=True)
    if os.environ.get("RSS_ENGINE", "1") == "1":  # the engine alone, in this process
        from openr_amd.engine import SpfEngine

        eng = SpfEngine([0])
        print(f"engine created {rss_mb():.0f} MB", flush=True)
        eng.set_graph(g)
        print(f"graph set {rss_mb():.0f} MB", flush=True)
        eng.solve(list(range(8)), True)
        print(f"8 solves {rss_mb():.0f} MB", flush=True)
        top_maps("engine only")
        eng.close()
        print(f"engine closed {rss_mb():.0f} MB", flush=True)
    batch = adjdb.AdjDbBatch.from_columns(adjdb.columns_for_graph(g))
    print(f"adjdb batch {rss_mb():.0f} MB", flush=True)
    rb = adjdb.RouteBuilder(batch, "0")
    print(f"route builder {rss_mb():.0f} MB", flush=True)
    ids = np.arange(rb.num_nodes)
    rb.build(ids[:8], 0)
    print(f"8-node build {rss_mb():.0f} MB (peak {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024:.0f})",
          flush=True)
    top_maps("after 8-node build")
    rb.build(ids, 0)
    print(f"all-node build {rss_mb():.0f} MB (peak {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024:.0f})",
          flush=True)
    top_maps("after all-node build")
    rb.close()
    batch.close()


if __name__ == "__main__":
    main()
