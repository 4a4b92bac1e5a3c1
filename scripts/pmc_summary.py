#!/usr/bin/env python3
"""Per-launch HBM bytes of the bench's dominant kernel from rocprofv3 --pmc CSVs.

usage: pmc_summary.py <pmc_out_dir> [bench args...]

FETCH_SIZE / WRITE_SIZE are KiB per dispatch (counter_defs.yaml). Per
/opt/skills/guides/MI355X_MICROARCH.md (HBM section), gfx950 FETCH_SIZE counts
128-B requests as 64 B, i.e. reports half of a wide coalesced read: the corrected
figure doubles it. Writes of this kernel are 8-B-per-lane coalesced u64 rows
(uncalibrated width per the guide): reported as counted.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(out_dir, counter):
    rows = []
    for path in glob.glob(os.path.join(out_dir, counter, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") == counter:
                    rows.append((r["Kernel_Name"], int(r.get("Grid_Size", 0) or 0), float(r["Counter_Value"])))
    return rows


def main():
    out_dir = sys.argv[1]
    bench_args = sys.argv[2:]
    topo = "grid100"
    if "--topology" in bench_args:
        topo = bench_args[bench_args.index("--topology") + 1]
    res = {"topology": topo, "bench_args": " ".join(bench_args)}
    if "--workload" in bench_args:
        res["workload"] = bench_args[bench_args.index("--workload") + 1]
        # workloads with a fixed topology (bench.py: whatif = WAN, ksp2 = fabric)
        res["topology"] = {"whatif": "wan", "ksp2": "fabric"}.get(res["workload"], topo)
    want = os.environ.get("PMC_KERNEL", "")  # pick this kernel instead of the dominant one
    kinds = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        for name, grid, v in per_dispatch(out_dir, ctr):
            if "openr_spf" not in name or want not in name:
                continue
            k = kinds.setdefault(name, {"grid": grid, "FETCH_SIZE": [], "WRITE_SIZE": []})
            k[ctr].append(v)
    if not kinds:
        raise SystemExit("no openr_spf dispatches found")
    # PMC_AGG=1: every engine kernel of a step (multi-kernel pipelines such as KSP2), per step
    if os.environ.get("PMC_AGG") == "1":
        steps = int(bench_args[bench_args.index("--steps") + 1]) + int(bench_args[bench_args.index("--warmup") + 1])
        tot = 0.0
        per = {}
        for n, k in kinds.items():
            b = 2.0 * sum(k["FETCH_SIZE"]) * 1024.0 + sum(k["WRITE_SIZE"]) * 1024.0
            per[n] = b / steps
            tot += b
        res.update({"kernels": per, "steps_profiled": steps, "hbm_bytes_per_step": tot / steps,
                    "correction": "FETCH_SIZE x2 (gfx950 counts 128-B requests at 64 B); WRITE_SIZE as counted"})
        if "--ksp-sources" in bench_args:
            res["ksp_sources"] = int(bench_args[bench_args.index("--ksp-sources") + 1])
        print(json.dumps(res, indent=1))
        return
    # dominant kernel = largest total fetch+write
    name = max(kinds, key=lambda n: sum(kinds[n]["FETCH_SIZE"]) + sum(kinds[n]["WRITE_SIZE"]))
    k = kinds[name]
    f = sum(k["FETCH_SIZE"]) / max(len(k["FETCH_SIZE"]), 1) * 1024.0
    w = sum(k["WRITE_SIZE"]) / max(len(k["WRITE_SIZE"]), 1) * 1024.0
    res.update({
        "kernel": name,
        "dispatches": len(k["FETCH_SIZE"]),
        "fetch_bytes_counted": f,
        "write_bytes_counted": w,
        "hbm_bytes_per_launch": 2.0 * f + w,
        "correction": "FETCH_SIZE x2 (gfx950 counts 128-B requests at 64 B); WRITE_SIZE as counted",
    })
    # n_sources of the launch: all V of the topology (bench default weak scaling, 1 rank)
    if "workload" not in res:
        res["n_sources"] = {"grid100": 10000, "fabric": 4992, "wan": 1000}.get(topo)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
