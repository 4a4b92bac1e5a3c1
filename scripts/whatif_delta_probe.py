"""What-if sweep with and without the delta output (tuning aid): per-step wall time of
openr_spf_whatif_device vs openr_spf_whatif_delta_device on the config-4 WAN. Under
`rocprofv3 --kernel-trace` the two phases' kernels come in time order, count-only first."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openr_amd import topology as T  # noqa: E402
from openr_amd.engine import SpfEngine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
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
eng.whatif_device(links.data_ptr(), L, srcs.data_ptr(), V, changed.data_ptr(), True, stream=s.cuda_stream)
cap = int(changed.sum().item())
nb = eng.nh_bytes
ptr = torch.empty(L * V + 1, dtype=torch.int64, device=dev)
node = torch.empty(cap, dtype=torch.int32, device=dev)
dist = torch.empty(cap, dtype=torch.int64, device=dev)
nh = torch.empty((cap, nb), dtype=torch.uint8, device=dev)
for name, f in (("count", lambda: eng.whatif_device(links.data_ptr(), L, srcs.data_ptr(), V, changed.data_ptr(), True,
                                                    stream=s.cuda_stream)),
                ("delta", lambda: eng.whatif_delta_device(links.data_ptr(), L, srcs.data_ptr(), V, changed.data_ptr(),
                                                          ptr.data_ptr(), node.data_ptr(), dist.data_ptr(),
                                                          nh.data_ptr(), cap, nb, True, stream=s.cuda_stream))):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"{name}: {dt * 1e3:.3f} ms per step, repair kernel {eng.stats().last_kernel_ms:.3f} ms", flush=True)
eng.close()
