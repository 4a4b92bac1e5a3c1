"""The what-if repair kernel's loop nest has only wave-uniform exits (CPU: compiles only).

Round 5 shipped `whatif_group_kernel` with a live profiling register that kept it from
hanging. The cause ("The hang"): LLVM's uniformity analysis saw the bucket
loop's exits as divergent. The wave index was `threadIdx.x >> 6`, so every per-wave LDS
pointer and every load through one was divergent. The lanes' entry loads also joined at
the loop's latch. The loop was therefore compiled with per-lane exit masks, and the
observed failure was lane 0 being dropped at the latch.

This test compiles the kernel for gfx950 and checks the fix holds. Only leaf loops with a
per-lane trip count (a lane per edge of a row) may have a divergent exit. The item, unit
and bucket loops and the dirty-node loops around process() may not. Before the fix the
bucket-loop nest showed up as cycles of 156, 72 and 66 basic blocks with divergent exits;
the leaf loops are at most 9.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import uniformity_check as uc  # noqa: E402

pytestmark = pytest.mark.skipif(not (os.path.exists(uc.HIPCC) and os.path.exists(uc.OPT)),
                                reason="needs hipcc and the ROCm LLVM opt")

MAX_LEAF_BLOCKS = 12


def test_whatif_repair_loops_have_uniform_exits():
    res = uc.divergent_exit_cycles(os.path.join(ROOT, "openr_amd", "csrc", "spf_sweep.hip"), "whatif_group_kernel",
                                   [os.path.join(ROOT, "include")])
    assert len(res) == 24, sorted(res)  # {u16, u32, u64 distances} x {global, LDS graph} x {1, 8 words} x {delta}
    for name, cycles in res.items():
        big = [c for c in cycles if c[1] > MAX_LEAF_BLOCKS]
        assert not big, f"{name}: loops with divergent exits {big}"
