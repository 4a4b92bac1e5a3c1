#!/usr/bin/env python3
"""Benchmark: all-sources SPF on the 100x100 grid (BASELINE.json metric).

A "step" = one all-sources pass per rank: every node of the topology is a
source, one engine launch through the C-ABI (openr_spf_solve_device) on
device-resident buffers. Inputs (CSR replica, source list) are resident in HBM
before the timed region; outputs (u64 distances + next-hop bitsets) are written
to HBM.

Scaling (one process per GPU, --gpus N under torch.distributed.run):
  weak (default)  per-GPU work is fixed: each rank runs the all-sources SPF of its
                  own LinkState replica (one OpenR area per GPU: Decision keeps one
                  LinkState per area, Decision.cpp areaLinkStates_). N x V solves per
                  step, no collective on the data path.
  strong          the V sources of ONE topology are split in contiguous blocks over
                  the ranks (shard.py); the RCCL all-gather of the result shards is
                  measured after the timed region and reported as "gather".

Timed region: barrier + synchronize, K steps, barrier + synchronize; the max
over ranks is reported.

roofline.achieved = algorithmic bytes per launch / mean kernel duration, with
B(src) = 4(V+1) + 8E + V(8 + ceil(deg(src)/8))  (SURVEY.md §8d).
cpu_baseline = the CPU oracle (C restatement of LinkState::runSpf) on a bounded
sample of the same sources, rank 0 at N=1 only.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "all-sources SPF solves/sec + edge relax/s (% HBM roofline), 10k-node grid, 1-8 GPU"
# The faithful-cost CPU model (oracle/spf_faithful.cpp) against the reference's own runSpf
# (BASELINE.md "Calibration ratio"): SURVEY.md section 6 times the shim-compiled reference at
# 15.3 ms per G100 solve (1 core, the survey container); the faithful model took 14.5 / 21.7 /
# 31.5 ms per G100 solve in the build container across sessions (host load), 0.085 vs ~0.1 ms
# on G10: its figures stand for the reference within a factor of about 2 either way.
CPU_CALIBRATION = {"reference_ms_per_g100_solve": 15.3, "faithful_ms_per_g100_solve": [14.5, 21.7, 31.5],
                   "faithful_over_reference_range": [0.95, 2.1],
                   "reference_ms_per_g10_solve": 0.1, "faithful_ms_per_g10_solve": 0.085,
                   "source": "SURVEY.md section 6 (reference, shim-compiled) vs oracle/spf_faithful.cpp, 1 core; "
                             "BASELINE.md Calibration ratio"}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md


def build_topology(name: str):
    from openr_amd import topology as T

    if name == "grid100":
        return T.grid_fast(100), {"workload": "grid100-all-sources", "nodes": 10000, "links": 19800}
    if name == "grid10":  # BASELINE config 1 (DecisionBenchmark 10x10 grid)
        return T.grid_fast(10), {"workload": "grid10-all-sources", "nodes": 100, "links": 180}
    if name == "fabric":
        g = T.fabric(5000)
        return g, {"workload": "fabric5000-all-sources", "nodes": g.num_nodes, "links": g.num_links}
    if name == "wan":
        g = T.wan(1000, 3000, 64, seed=1)
        return g, {"workload": "wan1k-all-sources", "nodes": g.num_nodes, "links": g.num_links}
    raise SystemExit(f"unknown --topology {name}")


def algorithmic_bytes(g, sources: np.ndarray) -> int:
    """Σ B(src), B = 4(V+1) + 8E + V(8 + ceil(deg(src)/8))."""
    V, E = g.num_nodes, g.num_dir_edges
    deg = np.array([len(set(g.col[g.row_ptr[u]:g.row_ptr[u + 1]].tolist())) for u in range(V)], dtype=np.int64)
    per = 4 * (V + 1) + 8 * E + V * (8 + (deg[sources] + 7) // 8)
    return int(per.sum())


def hash_rows(a) -> str:
    """64-bit digest (blake2b) of an array's bytes: the per-rank result checksum."""
    import hashlib

    return hashlib.blake2b(np.ascontiguousarray(a).view(np.uint8).tobytes(), digest_size=8).hexdigest()


def gather_hashes(h: str, world: int, dev) -> list:
    """all_gather of every rank's 64-bit digest (outside the timed region)."""
    if world == 1:
        return [h]
    import torch
    import torch.distributed as dist

    t = torch.tensor([int(h, 16) - (1 << 63)], dtype=torch.int64, device=dev)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [format(int(x.item()) + (1 << 63), "016x") for x in out]


def token_prefix(row: np.ndarray) -> np.ndarray:
    """The used prefix of a KSP2 token row ([n_paths, len, e.., len, e.., ...])."""
    n, k = int(row[0]), 1
    if n == 0xFFFFFFFF:
        return row[:1]
    for _ in range(n):
        k += 1 + int(row[k])
    return row[:k]


def rows_check(g, d_dist, d_nh, lo: int, n_local: int, use_metric: bool, nrows: int = 8):
    """The post-run check of the all-sources line: `nrows` evenly spaced rows of the rank's
    result (u64 distances and every next-hop byte) compared with oracle runSpf rows
    (oracle/spf_oracle.c, the tests' checker) outside the timed region. Raises on a
    mismatch."""
    from oracle.oracle import Oracle

    o = Oracle(g)
    idx = np.unique(np.linspace(0, n_local - 1, min(nrows, n_local)).astype(np.int64))
    srcs = (idx + lo).astype(np.uint32)
    want_d, want_nh = o.all_sources(srcs, use_metric, nthreads=1)
    got_d = d_dist[idx.tolist()].cpu().numpy().view(np.uint64)
    got_nh = d_nh[idx.tolist()].cpu().numpy()
    if got_nh.shape[-1] != want_nh.shape[-1]:
        raise AssertionError(f"next-hop width {got_nh.shape[-1]} != oracle {want_nh.shape[-1]}")
    for i, s in enumerate(srcs.tolist()):
        if not np.array_equal(got_d[i], want_d[i]):
            raise AssertionError(f"bench result check failed: dist row of source {s}")
        if not np.array_equal(got_nh[i], want_nh[i]):
            raise AssertionError(f"bench result check failed: next-hop row of source {s}")
    return {"rows": len(srcs), "sources": srcs.tolist(), "compared": "u64 dist + next-hop bytes vs oracle runSpf",
            "result": "ok"}


def cpu_baseline(g, seconds: float, use_metric: bool):
    """CPU baselines on the host cores of this box, same all-sources workload, evenly spaced
    source samples sized to ~`seconds` of wall time in all:

      faithful  oracle/spf_faithful.cpp: LinkState::runSpf restated with the reference's own
                data structures (std::string-keyed maps, shared_ptr DijkstraQ heap,
                unordered_set<string> next hops) — the reference's cost model. `value`.
      dense     oracle/spf_oracle.c: the same semantics on dense integer ids (the parity
                checker; an optimised CPU port, far cheaper than the reference).

    Each at 1 thread and at every thread of this process's CPU share (one LinkState
    replica per thread, sources strided)."""
    from oracle.oracle import Oracle, default_threads

    o = Oracle(g)
    V = g.num_nodes
    nthreads = default_threads()
    rng_all = np.arange(V, dtype=np.uint32)

    def sample(n):
        n = int(max(1, min(V, n)))
        return np.linspace(0, V - 1, n).astype(np.uint32)

    def dense(nt, budget):
        probe = sample(16)
        t0 = time.perf_counter()
        o.all_sources(probe, use_metric, nthreads=1, want_dist=True, want_nh=False)
        per = (time.perf_counter() - t0) / len(probe)
        want = max(nt, int(budget * nt / max(per, 1e-9)))
        srcs = sample(want)
        passes = max(1, want // len(srcs))
        t0 = time.perf_counter()
        for _ in range(passes):
            o.all_sources(srcs, use_metric, nthreads=nt, want_dist=True, want_nh=True)
        dt = time.perf_counter() - t0
        return {"solves_per_s": len(srcs) * passes / dt, "threads": nt, "solves": len(srcs) * passes,
                "seconds": dt}

    def faithful(nt, budget):
        _, _, sec = o.faithful_all_sources(sample(2), use_metric, nthreads=1)
        per = sec / 2
        srcs = sample(max(nt, int(budget * nt / max(per, 1e-9))))
        _, _, dt = o.faithful_all_sources(srcs, use_metric, nthreads=nt)
        return {"solves_per_s": len(srcs) / dt, "threads": nt, "solves": len(srcs), "seconds": dt}

    variants = {
        "faithful_1thread": faithful(1, 0.25 * seconds),
        f"faithful_{nthreads}threads": faithful(nthreads, 0.35 * seconds),
        "dense_1thread": dense(1, 0.15 * seconds),
        f"dense_{nthreads}threads": dense(nthreads, 0.25 * seconds),
    }
    del rng_all
    try:
        cpu_model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        cpu_model = "unknown"
    main = variants[f"faithful_{nthreads}threads"]
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        affinity = os.cpu_count() or 1
    return {
        "value": main["solves_per_s"],
        "unit": "solves/s",
        "cores": nthreads,
        "kind": "port",
        "cost_model": "faithful: reference data structures (oracle/spf_faithful.cpp)",
        "sample": f"{main['solves']} evenly spaced sources of {V}, runSpf with std::string-keyed LinkState "
                  f"replicas, {nthreads} threads, {main['seconds']:.1f}s; {cpu_model}",
        "cores_cap": 16,
        "affinity_cpus": affinity,
        "threads_note": f"cores = {nthreads} = min(affinity {affinity}, 16), a CAP: the GPU box grants one GPU's job a "
                        f"16-CPU share (its rules size worker pools to 16) although affinity lists {affinity} CPUs; "
                        f"the faithful value stands for the reference within ~2x (calibration)",
        "calibration": CPU_CALIBRATION,
        "variants": variants,
    }


def whatif_cpu_baseline(g, seconds: float, use_metric: bool):
    """The oracle on a bounded sample of what-if units: runSpf(src, {link}) per unit,
    no skipping of unaffected units (the reference has no what-if path to skip with)."""
    from oracle import Oracle

    o = Oracle(g)
    rng = np.random.default_rng(0)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(64):
            o.run_spf(int(rng.integers(g.num_nodes)), use_metric, [int(rng.integers(g.num_links))])
        n += 64
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "units/s", "cores": 1, "kind": "port",
            "sample": f"{n} random (link, source) units, one oracle runSpf with a 1-link ignore set each, "
                      f"dist+next-hops+pathLinks, 1 thread, {dt:.1f}s"}


def whatif_main(args):
    """BASELINE config 4: per-link-failure what-if sweep on the 1k-node WAN topology
    (heterogeneous metrics U[1,64]); a step = every (failed link, source) unit, one
    openr_spf_whatif_device call (base SPF, affected-unit filter, incremental repairs,
    row comparison). Strong scaling: rank r takes the contiguous block
    shard_range(L, r, N) of the links (shard.py), no collective on the data path."""
    import torch
    import torch.distributed as dist

    from openr_amd.engine import SpfEngine
    from openr_amd.shard import max_over_ranks

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    g, cfg = build_topology("wan")
    V, L = g.num_nodes, g.num_links
    eng = SpfEngine([local_rank])
    eng.set_graph(g)
    use_metric = not args.no_metric
    from openr_amd.shard import shard_range

    llo, lhi = shard_range(L, rank, world)  # strong: the ranks split ONE WAN's links
    n_links = lhi - llo
    links = torch.arange(llo, lhi, dtype=torch.int32, device=dev)
    srcs = torch.arange(0, V, dtype=torch.int32, device=dev)
    changed = torch.empty((max(n_links, 1), V), dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    solved = [0]

    kernel_ms = []

    def step():
        solved[0] = eng.whatif_device(links.data_ptr(), n_links, srcs.data_ptr(), V, changed.data_ptr(), use_metric,
                                      stream=stream.cuda_stream)
        kernel_ms.append(eng.stats().last_kernel_ms)  # the repair kernel (HIP events in the engine)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        step()
    barrier()
    kernel_ms.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    units = L * V
    value = units * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    # self-check outside the timed region: every rank's changed rows as a 64-bit digest,
    # all-gathered; rank 0 re-solves a sampled shard (the last rank's links) on its own
    # engine and compares digests, and at N = 1 checks 8 sources x its links against the
    # oracle re-solves runSpf(src, true, {link})
    mine = hash_rows(changed[:n_links].cpu().numpy().view(np.uint32))
    hashes = gather_hashes(mine, world, dev)
    check = None
    if rank == 0:
        r = world - 1
        rlo, rhi = shard_range(L, r, world)
        c_r, _ = eng.whatif(np.arange(rlo, rhi), np.arange(V), use_metric)
        check = {"rank_digests": hashes, "recomputed_rank": r, "recomputed_digest": hash_rows(c_r),
                 "recomputed_match": hash_rows(c_r) == hashes[r]}
        if world == 1:
            from oracle import Oracle

            samp = np.linspace(0, V - 1, 8).astype(np.uint32)
            want = Oracle(g).whatif(np.arange(llo, lhi, dtype=np.uint32), samp, use_metric)
            got = changed[:n_links].cpu().numpy().view(np.uint32)[:, samp]
            check.update(oracle_sample_units=int(want.size), oracle_sample_match=bool(np.array_equal(got, want)))
        check["ok"] = bool(check["recomputed_match"] and check.get("oracle_sample_match", True))
    # the delta leg (openr_spf_whatif_delta_device): the same sweep also writing each unit's
    # changed nodes with their new distance and next-hop bytes into a device pool; its own
    # clock, after the counts-only timed region
    delta = None
    if not args.no_delta:
        nbh = eng.nh_bytes
        cap = int(changed[:n_links].sum().item()) if n_links else 0
        d_ptr = torch.empty(n_links * V + 1, dtype=torch.int64, device=dev)
        d_node = torch.empty(max(cap, 1), dtype=torch.int32, device=dev)
        d_dist = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        d_nh = torch.empty((max(cap, 1), nbh), dtype=torch.uint8, device=dev)

        def dstep():
            return eng.whatif_delta_device(links.data_ptr(), n_links, srcs.data_ptr(), V, changed.data_ptr(),
                                           d_ptr.data_ptr(), d_node.data_ptr(), d_dist.data_ptr(), d_nh.data_ptr(),
                                           cap, nbh, use_metric, stream=stream.cuda_stream)[0]

        for _ in range(max(1, args.warmup)):
            dstep()
        barrier()
        td = time.perf_counter()
        for _ in range(args.steps):
            used = dstep()
        barrier()
        dt = max_over_ranks(time.perf_counter() - td, dev)
        delta = {"ms_per_step": dt / args.steps * 1e3, "units_per_s": units * args.steps / dt,
                 "entries_per_step": int(used), "pool_bytes": int(used) * (4 + 8 + nbh),
                 "note": "openr_spf_whatif_delta_device: counts + a CSR of every unit's changed nodes with their "
                         "new u64 distance and next-hop bytes, from the repair overlays (no second solve)"}
    srcs_np = np.arange(V)
    per_src = algorithmic_bytes(g, srcs_np) / V  # mean B(src)
    bytes_step = per_src * units
    bytes_solved = per_src * solved[0]
    kern_s = float(np.mean(kernel_ms)) / 1e3 if kernel_ms else elapsed / args.steps
    pmc = load_pmc("whatif")
    traffic = pmc.get("hbm_bytes_per_launch") if (pmc and "whatif_group" in pmc.get("kernel", "")
                                                  and world == 1) else None
    ucmp = None
    if rank == 0 and not args.no_ucmp:
        # config 4's "+ UCMP": the WAN's UCMP-weighted route DBs (RibPolicy
        # set_weight, default 1, neighbour wan{i} 1 + i % 4 for i % 3 == 0) for every node, through
        # the route-build C-ABI (openr_routes.h): one all-sources SPF batch on the GPU engine, then
        # SpfSolver + RibPolicy on the host. Outside the sweep's timed region; its own clock.
        from openr_amd import adjdb

        batch = adjdb.AdjDbBatch.from_columns(adjdb.columns_for_graph(g))
        rb = adjdb.RouteBuilder(batch, "0")
        wts = adjdb.wan_ucmp_weights(rb.names())
        ids = np.arange(rb.num_nodes)
        rb.build(ids[:16], adjdb.ROUTES_UCMP, 1, wts)  # warm-up (engine context, prefixes)
        tu = time.perf_counter()
        st = rb.build(ids, adjdb.ROUTES_UCMP, 1, wts)
        du = time.perf_counter() - tu
        ucmp = {"nodes": int(rb.num_nodes), "unicast_routes": int(st.unicast_routes), "nexthops": int(st.nexthops),
                "ucmp_weighted_nexthops": int(st.weighted_nexthops), "ms": du * 1e3,
                "routes_per_s": st.unicast_routes / du, "ms_spf_and_route_build": st.ms_build,
                "ms_rib_policy": st.ms_policy, "checksum": f"{st.checksum:016x}",
                "note": "SpfSolver::buildRouteDbs (GPU all-sources SPF prefetch + host route build) + "
                        "RibPolicy::applyPolicy, every node of the WAN"}
        rb.close()
        batch.close()
    if rank == 0:
        out = {
            "metric": "per-link-failure what-if SPF units/sec (link x source), 1k-node WAN, U[1,64] metrics",
            "value": value, "unit": "units/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "u64", "data": "synthetic (seeded WAN generator, SURVEY.md Appendix B)",
            "config": dict(cfg, workload="wan1k-whatif-all-links-x-all-sources", units_per_step=units,
                           spf_solved_per_step=solved[0], use_link_metric=use_metric,
                           parallelism=f"link-sharded x{world}"),
            "solved_per_s": solved[0] * world * args.steps / elapsed,
            "roofline": dict(roofline_with_physical(
                bytes_step, kern_s, traffic,
                "dominant kernel whatif_group_kernel (grouped repair), HIP events around its launch; SURVEY.md 8d: "
                "B(src) credited per what-if unit (link x source), units resolved by its fused tight-edge filter "
                f"included (affected units only: {bytes_solved / kern_s / 1e9:.1f} GB/s credited). The repair reads "
                "base rows staged once per (source, link chunk) in LDS instead of solving, so credited frac > 1; "
                "its bound is LDS latency, not HBM (DESIGN.md 5.3)", pmc=pmc,
                scope="one launch of whatif_group_kernel"), kernel_ms_mean=kern_s * 1e3),
        }
        if ucmp is not None:
            out["ucmp_routes"] = ucmp
        out["check"] = check
        if delta is not None:
            out["delta"] = delta
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = whatif_cpu_baseline(g, min(args.cpu_seconds, 10.0), use_metric)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()


PMC_ROUNDS = ("r06", "r05", "r04", "r03", "r02")  # newest first: the PMC summaries bench lines carry


def pmc_path(name):
    """profiles/<round>/pmc_traffic_<name>.json of the newest round that has one (written by
    scripts/pmc_traffic.sh), or None."""
    for rnd in PMC_ROUNDS:
        path = os.path.join(ROOT, "profiles", rnd, f"pmc_traffic_{name}.json")
        if os.path.exists(path):
            return path
    return None


def load_pmc(name):
    path = pmc_path(name)
    try:
        return dict(json.load(open(path)), _path=os.path.relpath(path, ROOT)) if path else None
    except (OSError, ValueError):
        return None


def roofline_with_physical(credited_bytes, seconds, traffic, note, pmc=None, scope=None):
    """HBM roofline of a launch / step: `credited_bytes` are SURVEY.md 8d's algorithmic bytes,
    `traffic` the PMC-measured HBM bytes of the same launch (or None), taken from the tracked
    summary `pmc` (load_pmc: its path goes into traffic_label.source). Where the credited
    fraction exceeds 1 (the kernel does not move the bytes the formula credits), the
    reported achieved / frac are the physical ones, the credited ones kept."""
    credited = credited_bytes / seconds / 1e9 if seconds > 0 else 0.0
    phys = traffic / seconds / 1e9 if (traffic and seconds > 0) else None
    r = {"bound": "hbm", "achieved": credited, "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": credited / HBM_PEAK_GBS, "traffic": traffic, "credited_bytes": credited_bytes,
         "credited_gbs": credited, "credited_frac": credited / HBM_PEAK_GBS,
         "physical_gbs": phys, "physical_frac": phys / HBM_PEAK_GBS if phys is not None else None,
         "seconds_per_launch": seconds, "note": note}
    if traffic is not None and pmc:
        r["traffic_label"] = {"source": pmc.get("_path"), "scope": scope, "correction": pmc.get("correction")}
    if credited / HBM_PEAK_GBS > 1.0 and phys is not None:
        r["achieved"], r["frac"] = phys, phys / HBM_PEAK_GBS
        r["note"] = note + "; credited frac > 1, so achieved / frac are the PMC-measured (physical) bytes"
    return r


def ksp2_cpu_baseline(g, seconds: float):
    """The oracle's getKthPaths(s, d, 2) (k = 1 SPF + trace, second SPF + trace) on random
    pairs, 1 thread, for about `seconds`."""
    from oracle import Oracle

    o = Oracle(g)
    rng = np.random.default_rng(0)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(8):
            o.kth_paths(int(rng.integers(g.num_nodes)), int(rng.integers(g.num_nodes)), 2)
        n += 8
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"{n} random (src, dst) pairs, oracle getKthPaths(k=2) each (2 SPFs + traces), 1 thread, "
                      f"{dt:.1f}s"}


def ksp2_main(args):
    """BASELINE config 5: KSP2 edge-disjoint second paths (getKthPaths k=1 and k=2) for
    all (src, dst) pairs of the fabric topology. A step = every pair of this rank's
    contiguous block of sources (shard.py; strong scaling: the ranks split ONE
    fabric's all-pairs job, no collective on the data path), one
    openr_spf_ksp2_device call: base SPF per source, device traces, one second SPF per
    pair with its k=1 links ignored."""
    import torch
    import torch.distributed as dist

    from openr_amd.engine import SpfEngine, SpfError
    from openr_amd.shard import max_over_ranks, shard_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    g, cfg = build_topology("fabric")
    V = g.num_nodes
    eng = SpfEngine([local_rank])
    eng.set_graph(g)
    n_src_total = args.ksp_sources or V
    lo, hi = shard_range(n_src_total, rank, world)
    nsrc = hi - lo
    tok_cap = 1024  # FSW -> FSW k=2: 48 edge-disjoint 6-hop paths = 337 tokens
    srcs = (torch.arange(lo, hi, dtype=torch.int64, device=dev) * V // n_src_total).to(torch.int32)  # spread
    blk = max(1, min(args.ksp_block, nsrc))
    prow = torch.arange(blk, dtype=torch.int32, device=dev).repeat_interleave(V)
    pdst = torch.arange(V, dtype=torch.int32, device=dev).repeat(blk)
    n_pairs = nsrc * V
    tok1 = torch.empty((blk * V, tok_cap), dtype=torch.int32, device=dev)
    tok2 = torch.empty((blk * V, tok_cap), dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)

    def step():
        for b in range(0, nsrc, blk):  # a block of sources x all destinations per call
            m = min(blk, nsrc - b)
            eng.ksp2_device(srcs[b:].data_ptr(), m, prow.data_ptr(), pdst.data_ptr(), m * V, tok_cap,
                            tok1.data_ptr(), tok2.data_ptr(), stream=stream.cuda_stream)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    pairs_total = n_src_total * V * args.steps
    value = pairs_total / elapsed
    s_np = srcs.cpu().numpy()
    if world == 1 and not args.no_cpu_baseline:
        # with the CPU leg only: spot check a few pairs against the oracle (outside the
        # timed region; the oracle is the checker, never the measured path)
        from openr_amd.engine import decode_paths
        from oracle import Oracle

        o = Oracle(g)
        last_b = ((nsrc - 1) // blk) * blk  # the token rows hold the last block's pairs
        m_last = nsrc - last_b
        idx = list(range(0, m_last * V, max(1, m_last * V // 7)))
        t1 = tok1[idx].cpu().numpy().view(np.uint32)
        t2 = tok2[idx].cpu().numpy().view(np.uint32)
        d_np, p_np = pdst.cpu().numpy(), prow.cpu().numpy()
        for r, i in enumerate(idx):
            s, d = int(s_np[last_b + p_np[i]]), int(d_np[i])
            assert decode_paths(t1[r]) == o.kth_paths(s, d, 1) and decode_paths(t2[r]) == o.kth_paths(s, d, 2), \
                "ksp2 bench result check failed"
    # self-check outside the timed region: 64 pairs of each rank's last block (what the
    # token buffers hold after the loop), their token prefixes as a 64-bit digest per rank,
    # all-gathered; rank 0 traces every rank's sample again with its own engine and
    # compares digests
    def sample_of(r):
        rlo, rhi = shard_range(n_src_total, r, world)
        rs = (np.arange(rlo, rhi, dtype=np.int64) * V // n_src_total).astype(np.uint32)
        rn = rhi - rlo
        lb = ((rn - 1) // blk) * blk
        m_l = rn - lb
        rows = np.linspace(0, m_l * V - 1, 64).astype(np.int64)
        return rows, rs[lb + rows // V], (rows % V).astype(np.uint32)

    rows, _, _ = sample_of(rank)
    ridx = torch.from_numpy(rows).to(dev)
    t1s = tok1.index_select(0, ridx).cpu().numpy().view(np.uint32)
    t2s = tok2.index_select(0, ridx).cpu().numpy().view(np.uint32)
    mine = hash_rows(np.concatenate([np.concatenate([token_prefix(a), token_prefix(b)]) for a, b in zip(t1s, t2s)]))
    hashes = gather_hashes(mine, world, dev)
    check = None
    if rank == 0:
        check = {"rank_digests": hashes, "pairs_per_rank": int(len(rows)), "recomputed_match": []}
        for r in range(world):
            _, ss, dd = sample_of(r)
            a1, a2 = eng.ksp2_tokens(ss, dd, tok_cap)
            d = hash_rows(np.concatenate([np.concatenate([token_prefix(a), token_prefix(b)]) for a, b in zip(a1, a2)]))
            check["recomputed_match"].append(d == hashes[r])
        check["ok"] = all(check["recomputed_match"])
    srcs_np = np.asarray(s_np, dtype=np.int64)
    per_pair = algorithmic_bytes(g, srcs_np) / max(nsrc, 1)  # B(src) per second SPF
    step_s = elapsed / args.steps
    pmc = load_pmc("ksp2")  # PMC_AGG summary: every engine kernel of a step, per pair
    traffic = None
    if pmc and pmc.get("hbm_bytes_per_step") and pmc.get("ksp_sources") and world == 1:
        traffic = pmc["hbm_bytes_per_step"] / (pmc["ksp_sources"] * V) * n_pairs
    if rank == 0:
        out = {
            "metric": "KSP2 (getKthPaths k=1,2) all-pairs throughput, pairs/sec, fabric ~5k nodes",
            "value": value, "unit": "pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u64", "data": "synthetic (fabric generator, unit metrics)",
            "config": dict(cfg, workload="fabric5000-ksp2-all-pairs" if not args.ksp_sources else
                           f"fabric5000-ksp2-{n_src_total}-sources-x-all-dests", pairs_per_step=n_src_total * V,
                           tok_cap=tok_cap, sources_per_call=blk, parallelism=f"source-sharded x{world}"),
            "roofline": roofline_with_physical(
                per_pair * n_pairs, step_s, traffic,
                "per GPU, whole step (base SPFs, k=1 / k=2 traces, second SPFs): SURVEY.md 8d B(src) per second "
                "SPF (one per pair), k=1 base SPFs and traces not credited; traffic = PMC HBM bytes of every engine "
                "kernel per pair (" + (pmc or {}).get("_path", "no PMC summary") + ") x this step's pairs",
                pmc=pmc, scope="every engine kernel of a KSP2 step on the summary's sources, per pair, x this "
                              "step's pairs"),
        }
        out["check"] = check
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = ksp2_cpu_baseline(g, min(args.cpu_seconds, 10.0))
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()


def update_main(args):
    """Convergence after an attribute change: the BM_DecisionGrid /
    BM_DecisionFabric update loop of the reference benchmark (RoutingBenchmarkUtils.cpp:
    407-479) toggles the overload bit of a random node (grid: any node; fabric: an RSW),
    then reverts it on the next update. A step = one such update applied to the resident
    mirror (openr_spf_patch_graph) + every source's dist / next-hop row brought up to date
    (openr_spf_refresh_device: affected-row filter, re-solve of the affected rows in
    place). The reference clears its memo and re-runs Dijkstra per source instead
    (LinkState.cpp:714-717), so cpu_baseline = the oracle's all-sources pass / V, i.e.
    full re-solves per second divided by the sources one update invalidates."""
    import torch
    import torch.distributed as dist

    from openr_amd.engine import SpfEngine
    from openr_amd.shard import max_over_ranks

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    g, cfg = build_topology(args.topology)
    V = g.num_nodes
    eng = SpfEngine([local_rank])
    eng.set_graph(g)
    nb = eng.nh_bytes
    use_metric = not args.no_metric
    src = torch.arange(0, V, dtype=torch.int32, device=dev)
    d_dist = torch.empty((V, V), dtype=torch.int64, device=dev)
    d_nh = torch.empty((V, V, nb), dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    # candidates: the reference's toggled node kinds (fabric: RSWs, marker 3)
    cand = [i for i, nm in enumerate(g.names) if nm.startswith("3-")] if args.topology == "fabric" else list(range(V))
    rng = np.random.default_rng(1 + rank)
    sel = [None]
    resolved = []

    def step():
        if sel[0] is None:
            sel[0] = int(cand[int(rng.integers(len(cand)))])
            flag = 1
        else:
            flag = 0
        eng.patch(nodes=[sel[0]], node_overloaded=[flag], track=False)
        if flag == 0:
            sel[0] = None
        resolved.append(eng.refresh_device(src.data_ptr(), V, d_dist.data_ptr(), d_nh.data_ptr(), nb, use_metric,
                                           stream=stream.cuda_stream))

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    # resident rows of the unpatched graph, and the full re-solve time for comparison
    eng.solve_device(src.data_ptr(), V, d_dist.data_ptr(), d_nh.data_ptr(), nb, use_metric, stream=stream.cuda_stream)
    barrier()
    tf = time.perf_counter()
    for _ in range(3):
        eng.solve_device(src.data_ptr(), V, d_dist.data_ptr(), d_nh.data_ptr(), nb, use_metric,
                         stream=stream.cuda_stream)
    barrier()
    full_ms = (time.perf_counter() - tf) / 3 * 1e3
    steps = args.steps + (args.steps % 2)  # whole set/revert pairs
    for _ in range(args.warmup + (args.warmup % 2)):
        step()
    barrier()
    resolved.clear()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    # the rows must equal a fresh solve of the final (reverted) graph
    chk = torch.empty((2, V), dtype=torch.int64, device=dev)
    eng.solve_device(src.data_ptr(), 2, chk.data_ptr(), 0, nb, use_metric, stream=stream.cuda_stream)
    barrier()
    assert torch.equal(chk, d_dist[:2]), "refreshed rows differ from a fresh solve"
    value = steps * world / elapsed
    per_src = algorithmic_bytes(g, np.arange(V)) / V
    mean_resolved = float(np.mean(resolved)) if resolved else 0.0
    achieved = per_src * mean_resolved / (elapsed / steps) / 1e9
    if rank == 0:
        out = {
            "metric": "node-overload updates/sec with all-sources SPF rows kept current (BM_Decision update loop)",
            "value": value, "unit": "updates/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
            "ms_per_step": elapsed / steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u64", "data": "synthetic (reference benchmark generators, unit metrics)",
            "config": dict(cfg, workload=cfg["workload"].replace("all-sources", "overload-toggle-refresh"),
                           rows=V, mean_rows_resolved=mean_resolved, full_resolve_ms=full_ms,
                           use_link_metric=use_metric, parallelism=f"area-per-GPU x{world}"),
            "speedup_vs_full_resolve": full_ms / (elapsed / steps * 1e3),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "note": "SURVEY.md 8d B(src) per re-solved row / step time (host patch, filter and the "
                                 "count read-back included)"},
        }
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(g, args.cpu_seconds, use_metric)
            cb = dict(cb, value=cb["value"] / V, unit="updates/s",
                      sample=cb["sample"] + f"; updates/s = solves/s / {V} (the reference re-solves every source)")
            out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()


def adjdb_main(args):
    """Bulk AdjacencyDatabase input path: a KvStore full sync of
    every node's "adj:" value. A step = native compact-protocol decode of all V values
    on host threads (Decision.cpp:1755-1757 readThriftObjStr per key in the reference)
    -> LinkState::updateAdjacencyDatabase for each (host mirror, :1773-1777) -> CSR
    mirror -> openr_spf_set_graph (H2D) -> all-sources SPF on the device. Values are
    originated once, untimed, by the native writer (LinkMonitor.cpp:620 form).
    value = decoded values/s of the decode phase; ms_per_step = the whole cold start.
    cpu_baseline = the pure-Python oracle decoder (oracle/thrift_compact.py) on a
    sample of the same values: a restatement, not fbthrift (absent here)."""
    import torch

    from openr_amd import adjdb
    from openr_amd.engine import SpfEngine

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    g, cfg = build_topology(args.topology)
    V = g.num_nodes
    data, offsets = adjdb.AdjDbBatch.from_columns(adjdb.columns_for_graph(g)).encode_all()
    threads = min(16, os.cpu_count() or 1)
    eng = SpfEngine([0])
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    src = torch.arange(0, V, dtype=torch.int32, device=dev)
    d_dist = torch.empty((V, V), dtype=torch.int64, device=dev)
    phases = {"decode": [], "linkstate_csr": [], "set_graph": [], "solve": []}
    holder = {}

    def step(record):
        t0 = time.perf_counter()
        batch = adjdb.AdjDbBatch(data, offsets, n_threads=threads)
        t1 = time.perf_counter()
        g2 = batch.to_csr("0")
        t2 = time.perf_counter()
        eng.set_graph(g2)
        t3 = time.perf_counter()
        nb = eng.nh_bytes
        if holder.get("nb") != nb:
            holder["nh"] = torch.empty((V, V, nb), dtype=torch.uint8, device=dev)
            holder["nb"] = nb
        eng.solve_device(src.data_ptr(), V, d_dist.data_ptr(), holder["nh"].data_ptr(), nb, True,
                         stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        t4 = time.perf_counter()
        batch.close()
        if record:
            for k, dt in zip(phases, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
                phases[k].append(dt * 1e3)
        holder["g2"] = g2

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    # the graph built from the bytes has the topology's links
    g2 = holder["g2"]
    assert g2.num_nodes == V and g2.num_dir_edges == g.num_dir_edges and g2.num_links == g.num_links
    ph = {k: float(np.mean(v)) for k, v in phases.items()}
    dec_s = ph["decode"] / 1e3
    mb = float(data.size) / 1e6
    out = {
        "metric": "AdjacencyDatabase decode (KvStore adj: values/s) + cold start to all-sources SPF",
        "value": V / dec_s, "unit": "values/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic (benchmark generators, values from the native writer)",
        "config": dict(cfg, workload=cfg["workload"].replace("all-sources", "adjdb-coldstart"), values=V,
                       value_bytes=int(data.size), adjacencies=g.num_dir_edges, decode_threads=threads),
        "phases_ms": ph, "decode_mb_per_s": mb / dec_s,
        "roofline": None,
        "note": "host-side byte parsing (decode) and host mirror build; the device solve is the config-2/3 kernel",
    }
    if not args.no_cpu_baseline:
        from oracle import thrift_compact as tc

        vals = [data[int(offsets[i]):int(offsets[i + 1])].tobytes() for i in range(V)]
        n, t = 0, time.perf_counter()
        while time.perf_counter() - t < min(args.cpu_seconds, 10.0):
            tc.read_adjacency_database(vals[n % V])
            n += 1
        dt = time.perf_counter() - t
        out["cpu_baseline"] = {"value": n / dt, "unit": "values/s", "cores": 1, "kind": "port",
                               "sample": f"{n} values decoded by the pure-Python oracle decoder in {dt:.1f}s"}
    print(json.dumps(out), flush=True)
    eng.close()


def routes_main(args):
    """SURVEY.md §8f rank 1 / VERDICT r2 f1: SpfSolver::buildRouteDbs for EVERY node of the
    topology (G100: the getRouteMap-scale grid workload of DecisionTest.cpp:4289-4355 at
    n = 100), through the route-build C-ABI (include/openr_routes.h): one all-sources SPF
    batch on the GPU engine, its rows kept dense in the LinkState memo, then the per-node
    route builds on host worker threads reading them through LinkState::SpfView (no
    SpfResult map materialised). Each node's DB is tallied and freed as it is built
    (streaming form), so host memory stays at the dense rows. value = unicast routes/s;
    peak_rss_mb = this process's peak resident set (getrusage)."""
    import resource

    from openr_amd import adjdb

    # no torch here: the route build drives the engine through its C-ABI on device 0, and
    # the framework's own resident set is what peak_rss_mb reports
    g, cfg = build_topology(args.topology)
    batch = adjdb.AdjDbBatch.from_columns(adjdb.columns_for_graph(g))
    rb = adjdb.RouteBuilder(batch, "0")
    ids = np.arange(rb.num_nodes)
    flags = adjdb.ROUTES_LFA if args.lfa else 0
    rb.build(ids[:8], flags)  # warm-up (engine context, prefixes)
    rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0
    times, st = [], None
    for _ in range(max(1, args.steps)):
        t0 = time.perf_counter()
        st = rb.build(ids, flags)
        times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0
    out = {
        "metric": "route DBs of every node (SpfSolver::buildRouteDbs, GPU SPF + host route build), unicast routes/s",
        "value": st.unicast_routes / dt, "unit": "routes/s", "n_gpus": 1, "steps": len(times), "warmup": 1,
        "ms_per_step": dt * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u64", "data": "synthetic (benchmark generators, one prefix per node)",
        "config": dict(cfg, workload=cfg["workload"].replace("all-sources", "route-dbs-all-nodes"), lfa=bool(args.lfa),
                       # HostParallel.h: OPENR_HOST_THREADS, else min(hardware threads, 16)
                       host_threads=int(os.environ.get("OPENR_HOST_THREADS", "0")) or min(16, os.cpu_count() or 1)),
        "unicast_routes": int(st.unicast_routes), "mpls_routes": int(st.mpls_routes), "nexthops": int(st.nexthops),
        "checksum": f"{st.checksum:016x}", "ms_spf_and_route_build": st.ms_build,
        "peak_rss_mb": rss, "rss_before_build_mb": rss0,
        "roofline": None,
        "note": "host route build over dense SPF rows (LinkState::SpfView); the device solve is the config-2/3 kernel",
    }
    print(json.dumps(out), flush=True)
    rb.close()
    batch.close()


def relaunch_distributed(n: int) -> int:
    """`bench.py --gpus N` started without torch.distributed.run: launch N ranks (one
    process per GPU) under torch.distributed.run as a CHILD process and return its exit
    code. This process never touches the GPU (no HIP call before or after), so no exec
    of an initialised process happens (the box forbids it)."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--topology", default="grid100", choices=["grid100", "grid10", "fabric", "wan"])
    ap.add_argument("--no-metric", action="store_true", help="hop-count SPF (useLinkMetric=false)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--gather", default="compact", choices=["compact", "full"],
                    help="strong scaling exchange: compact = u8/u16 level rows + next hops (uniform-cost graphs), "
                         "full = u64 dist + next hops")
    ap.add_argument("--no-ucmp", action="store_true", help="whatif: skip the UCMP route-build leg")
    ap.add_argument("--no-delta", action="store_true", help="whatif: skip the delta-output leg")
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="strong (default, BASELINE config 3): the V sources of ONE topology are split over the "
                         "ranks and the result shards all-gathered over RCCL; weak: every rank solves its own "
                         "full all-sources replica (one OpenR area per GPU)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary (scripts/pmc_traffic.sh); default profiles/<newest round>/pmc_traffic_<topology>.json")
    ap.add_argument("--ksp-sources", type=int, default=0,
                    help="ksp2: sources per step (0 = all; each source pairs with every node)")
    ap.add_argument("--ksp-block", type=int, default=1024,
                    help="ksp2: sources per device call within a step (token rows are reused; 1 024 x all "
                         "destinations x 2 x 4 KB = 42 GB of token rows: fewer, longer launches, "
                         "1.696 vs 1.711 s per step at 256, r06)")
    ap.add_argument("--lfa", action="store_true", help="routes: SpfSolver computeLfaPaths")
    ap.add_argument("--decision-cases",
                    default="grid:10:sp,grid:100:sp,grid:1000:sp,grid:10000:sp,grid:10:ksp2,grid:100:ksp2,grid:1000:ksp2,"
                            "grid:10000:ksp2,fabric:344:sp,fabric:1000:sp,fabric:5000:sp,fabricp:5000:sp",
                    help="decision: topology:size:algo list. The reference registers BM_DecisionGrid {10, 100, 1000, "
                         "10000} x SP_ECMP and {10, 100, 1000} x KSP2_ED_ECMP and BM_DecisionFabric {344, 1000, 5000} "
                         "(DecisionBenchmark.cpp:12-29; a grid of N is (int)sqrt(N) squared, "
                         "RoutingBenchmarkUtils.cpp:527); grid:10000:ksp2 is added, and fabricp = the fabric with "
                         "one prefix per node (the reference's createFabric advertises none)")
    ap.add_argument("--workload", default="all-sources",
                    choices=["all-sources", "whatif", "ksp2", "update", "adjdb", "routes", "decision"],
                    help="whatif: per-link-failure sweep, every (link, source) unit of the WAN topology "
                         "(BASELINE config 4)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return relaunch_distributed(args.gpus)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world_env}")
    if args.workload == "whatif":
        return whatif_main(args)
    if args.workload == "ksp2":
        return ksp2_main(args)
    if args.workload == "update":
        return update_main(args)
    if args.workload == "adjdb":
        return adjdb_main(args)
    if args.workload == "routes":
        return routes_main(args)
    if args.workload == "decision":
        return decision_main(args)
    return all_sources_main(args)


def decision_main(args):
    """DecisionBenchmark through the drop-in (DecisionBenchmark.cpp:12-29,
    RoutingBenchmarkUtils.cpp:406-479, 517-630): per step, one node's adjacency database is
    re-advertised with its overload bit toggled and Decision (LFA on) rebuilds its own
    route DB: LinkState::updateAdjacencyDatabase + SpfSolver::buildRouteDb on the GPU
    engine. The harness is tests/cpp/decision_bench.cpp (C++, as the reference's
    benchmark is); it checks the last route DB against oracle SPF rebuilds and prices the
    reference's cost of the same step on the faithful CPU restatement. One JSON line per
    (topology, algorithm)."""
    binary = os.path.join(ROOT, "tests", "cpp", "build", "decision_bench")
    if not os.path.exists(binary):
        raise SystemExit("build first: make (tests/cpp/build/decision_bench)")
    for case in args.decision_cases.split(","):
        topo, size, algo = case.split(":")
        fabric_prefixes = topo == "fabricp"
        topo = "fabric" if fabric_prefixes else topo
        steps = args.steps
        cmd = [binary, "--topology", topo, "--size", size, "--algo", algo, "--iters", str(steps),
               "--warmup", str(max(1, args.warmup)), "--check"] + (["--fabric-prefixes"] if fabric_prefixes else [])
        if not args.no_cpu_baseline:
            cmd += ["--cpu-iters", "1", "--cpu-threads", "16"]
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=1200)
        if p.returncode != 0:
            sys.stderr.write(p.stdout + p.stderr)
            raise SystemExit(f"decision_bench failed for {case} (rc {p.returncode})")
        line = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
        cpu = line.get("cpu_baseline")
        out = {
            "metric": "DecisionBenchmark: adjacency update (overload toggle) + buildRouteDb(my node), LFA on",
            "value": 1e3 / line["ms_per_update"],
            "unit": "updates/s",
            "n_gpus": 1,
            "steps": steps,
            "warmup": max(1, args.warmup),
            "ms_per_step": line["ms_per_update"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (reference benchmark generators: createGrid / createFabric)",
            "config": {"workload": f"BM_Decision{'Grid' if topo == 'grid' else 'Fabric'}({size}, "
                                   f"{line['algo']})" + (", one prefix per node" if fabric_prefixes else ""),
                       "topology": topo, "size": int(size), "nodes": line["nodes"],
                       "my_node": line["my_node"], "lfa": True, "fabric_prefixes": fabric_prefixes},
            "decision": line,
        }
        if cpu:
            out["cpu_baseline"] = {"value": 1e3 / cpu["ms_per_update"], "unit": "updates/s", "cores": 1,
                                   "kind": "port", "sample": cpu["sample"], "ms_per_update": cpu["ms_per_update"],
                                   "spf_runs_per_update": cpu["spf_runs_per_update"], "ms_per_spf": cpu["ms_per_spf"],
                                   "ms_route_construction": cpu["ms_route_construction"],
                                   "ms_update_adjdb": cpu.get("ms_update_adjdb")}
        print(json.dumps(out), flush=True)


def all_sources_main(args):
    """BASELINE config 3 (default; config 2 with --topology fabric): all-sources SPF.

    strong: rank r solves the contiguous source block shard_range(V, r, N) of the one
    topology (no collective on the data path); `value` = V solves per step / the slowest
    rank's step time. The RCCL all-gather of the dist / next-hop shards (the exchange
    step of config 3) is timed in a second loop of K (solve + all-gather) steps and
    reported as gather.gather_inclusive_value / ms_per_step."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from openr_amd.engine import SpfEngine
    from openr_amd.shard import max_over_ranks, shard_range

    g, cfg = build_topology(args.topology)
    V = g.num_nodes
    eng = SpfEngine([local_rank])
    eng.set_graph(g)
    nb = eng.nh_bytes
    use_metric = not args.no_metric
    strong = args.scaling == "strong"

    lo, hi = shard_range(V, rank, world) if strong else (0, V)
    n_local = hi - lo
    src = torch.arange(lo, hi, dtype=torch.int32, device=dev)
    d_dist = torch.empty((max(n_local, 1), V), dtype=torch.int64, device=dev)
    d_nh = torch.empty((max(n_local, 1), V, nb), dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)  # a real (non-null) stream shared by launches and events
    torch.cuda.set_stream(stream)

    def step():
        eng.solve_device(src.data_ptr(), n_local, d_dist.data_ptr(), d_nh.data_ptr(), nb, use_metric,
                         stream=stream.cuda_stream)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        step()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    barrier()
    t0 = time.perf_counter()
    for a, b in evs:
        a.record(stream)
        step()
        b.record(stream)
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = [a.elapsed_time(b) for a, b in evs]
    elapsed = max_over_ranks(elapsed, dev)  # the slowest rank's clock

    # correctness check outside the timed region: a handful of full rows of the last step,
    # distances AND next-hop bytes, against the CPU oracle (tests' checker) on the same graph
    grid_n = {"grid100": 100, "grid10": 10}.get(args.topology)
    check = None
    if n_local:
        check = rows_check(g, d_dist, d_nh, lo, n_local, use_metric)

    gather = None
    if world > 1 and strong and not args.no_gather:
        from openr_amd.shard import CompactGather, GatherBuffers

        # compact form (default) on uniform-cost graphs: u8/u16 level rows + next-hop rows
        # (dist = level x cost on the receiver); the full u64 form otherwise / --gather full
        mets = np.unique(np.asarray(g.metric)[np.asarray(g.edge_up) != 0]) if use_metric else np.array([1])
        cost = int(mets[0]) if mets.size == 1 else (1 if mets.size == 0 else 0)
        form = "full"
        native = False
        gstep = step
        if args.gather == "compact" and cost > 0:
            fin = d_dist[:n_local][d_dist[:n_local] != -1]
            mx = torch.tensor([float(fin.max().item()) if fin.numel() else 0.0], dtype=torch.float64, device=dev)
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            max_level = int(mx.item()) // cost
            if max_level <= 65534:
                form = "levels-u8" if max_level <= 254 else "levels-u16"
                # fused: the solve writes the level rows itself (OPENR_SPF_EMIT_LEVELS8/16);
                # the device-side encode of u64 rows only where the engine cannot
                gb = CompactGather.native(d_nh[:n_local], V, world, cost, max_level, V, dev)

                def gstep():
                    eng.solve_device(src.data_ptr(), n_local, gb.level_send.data_ptr(), d_nh.data_ptr(), nb, use_metric,
                                     stream=stream.cuda_stream, level_bytes=gb.level_bytes)
                try:
                    gstep()
                    torch.cuda.synchronize(dev)
                    native = eng.take_status() == 0
                except SpfError:
                    native = False
                if not native:
                    gb = CompactGather(d_dist[:n_local], d_nh[:n_local], V, world, cost, max_level)
                    gstep = step
        if form == "full":
            gb = GatherBuffers(d_dist[:n_local], d_nh[:n_local], V, world)
        for _ in range(max(1, args.warmup)):
            gstep()
            gb.allgather()
        barrier()
        tg = time.perf_counter()
        for _ in range(args.steps):
            gstep()
            gb.allgather()
        barrier()
        gel = max_over_ranks(time.perf_counter() - tg, dev)
        # the gathered rows are the full all-sources result on every rank
        if grid_n:
            full = gb.full_dist()
            r_chk = [0, V // 2, V - 1]
            host = full[r_chk].cpu().numpy().view(np.uint64)
            a = np.arange(V)
            for i, s in enumerate(r_chk):
                exp = np.abs(s % grid_n - a % grid_n) + np.abs(s // grid_n - a // grid_n)
                assert np.array_equal(host[i].astype(np.int64), exp), "gathered result check failed"
        m_rows = max(shard_range(V, r, world)[1] - shard_range(V, r, world)[0] for r in range(world))
        full_bytes = int(m_rows * V * (8 + nb))
        gather = {"form": form, "fused_level_rows": native, "ms_per_step": gel / args.steps * 1e3,
                  "bytes_per_rank": int(gb.bytes_per_rank) if form != "full" else full_bytes,
                  "bytes_per_rank_full_form": full_bytes,
                  "compute_only_value": None,  # filled below (= value)
                  "gather_inclusive_value": V * args.steps / gel,
                  "collective": ("all_gather_into_tensor (RCCL) of " +
                                 (("u8/u16 level rows written by the solve itself (OPENR_SPF_EMIT_LEVELS8/16; "
                                   "dist = level x cost on receipt)" if native else
                                   "u8/u16 level rows (dist = level x cost on receipt, encoded on the device after "
                                   "each solve)") + " + next-hop rows" if form != "full" else "dist u64 + next-hop rows") +
                                 ", solve included")}

    solves_total = (V if strong else V * world) * args.steps
    value = solves_total / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    sources_local = np.arange(lo, hi)
    bytes_launch = algorithmic_bytes(g, sources_local) if n_local else 0
    mean_kernel_s = float(np.mean(kernel_ms)) / 1e3
    achieved = bytes_launch / mean_kernel_s / 1e9 if mean_kernel_s > 0 else 0.0
    traffic = None
    traffic_label = None
    if args.traffic_json is None:
        args.traffic_json = pmc_path(args.topology) or ""
    if args.traffic_json and not os.path.relpath(os.path.abspath(args.traffic_json), ROOT).startswith("profiles" + os.sep):
        # a bench line cites only tracked evidence: copy the summary into profiles/ first
        sys.stderr.write(f"bench: ignoring --traffic-json {args.traffic_json} (not under profiles/)\n")
        args.traffic_json = ""
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("topology") == args.topology and tj.get("n_sources") in (None, n_local):
                # a whole step's engine kernels (PMC_AGG) or the dominant kernel's launch
                traffic = tj.get("hbm_bytes_per_step", tj.get("hbm_bytes_per_launch"))
                traffic_label = {
                    "source": os.path.relpath(args.traffic_json, ROOT),
                    "scope": ("every engine kernel of one all-sources call (the timed step)"
                              if "hbm_bytes_per_step" in tj else f"one launch of {tj.get('kernel', '?')[:80]}"),
                    "correction": tj.get("correction"),
                }
        except Exception:
            traffic = None

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (reference benchmark grid generator, unit metrics)"
                    if grid_n else "synthetic (benchmark generators)",
            "config": dict(cfg, **{"sources_per_step": solves_total // args.steps, "sources_per_rank": n_local,
                                   "use_link_metric": use_metric,
                                   "parallelism": (f"source-sharded x{world}" if strong else f"area-per-GPU x{world}")}),
            "edge_relax_per_s": value * g.num_dir_edges,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_label": traffic_label,
                "kernel_ms_mean": mean_kernel_s * 1e3,
                "bytes_per_launch": bytes_launch,
                "note": "per GPU (rank 0): SURVEY.md 8d B(src) summed over the rank's sources / mean launch "
                        "duration (HIP events on the launch stream)",
            },
        }
        if gather is not None:
            gather["compute_only_value"] = value
            out["gather"] = gather
        if check is not None:
            out["check"] = check
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(g, args.cpu_seconds, use_metric)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    sys.exit(main() or 0)
