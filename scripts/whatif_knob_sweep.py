"""Interleaved A/B of a what-if tuning knob on the config-4 WAN (tuning aid).

  python scripts/whatif_knob_sweep.py OPENR_SPF_WHATIF_CAP 96,128,160,192 [rounds] [steps]
  python scripts/whatif_knob_sweep.py - "A=1+B=2,A=4+B=0" ...   (several variables per value)

Every round runs each value once, `steps` timed steps each. For each value the script prints
the median step time and the median repair-kernel time. The `changed` rows of every value
must equal those of the first value; the script exits non-zero when they do not."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import topology as T  # noqa: E402
from openr_amd.engine import SpfEngine  # noqa: E402

knob, values = sys.argv[1], sys.argv[2].split(",")
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
g = T.wan(1000, 3000, 64, seed=1)
eng = SpfEngine([0])
eng.set_graph(g)
V, L = g.num_nodes, g.num_links
links = torch.arange(L, dtype=torch.int32, device=dev)
srcs = torch.arange(V, dtype=torch.int32, device=dev)
changed = torch.empty((L, V), dtype=torch.int32, device=dev)
s = torch.cuda.Stream(device=dev)
torch.cuda.set_stream(s)


def run():
    eng.whatif_device(links.data_ptr(), L, srcs.data_ptr(), V, changed.data_ptr(), True, stream=s.cuda_stream)


ref = None
step_ms = {v: [] for v in values}
kern_ms = {v: [] for v in values}
for r in range(rounds):
    for v in values:
        if knob == "-":
            for kv in v.split("+"):
                name, val = kv.split("=", 1)
                os.environ[name] = val
        else:
            os.environ[knob] = v
        run()
        torch.cuda.synchronize()
        if ref is None:
            ref = changed.clone()
        elif r == 0 and not torch.equal(ref, changed):
            print(f"MISMATCH: {knob}={v} changes the results", flush=True)
            sys.exit(1)
        t0 = time.perf_counter()
        ks = []
        for _ in range(steps):
            run()
            ks.append(eng.stats().last_kernel_ms)
        torch.cuda.synchronize()
        step_ms[v].append((time.perf_counter() - t0) / steps * 1e3)
        kern_ms[v].append(statistics.median(ks))
    print(f"round {r} done", flush=True)
for v in values:
    print(f"{knob}={v}: step median {statistics.median(step_ms[v]):.3f} ms (min {min(step_ms[v]):.3f}), "
          f"repair kernel median {statistics.median(kern_ms[v]):.3f} ms", flush=True)
eng.close()
