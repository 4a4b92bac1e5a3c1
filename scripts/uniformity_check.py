#!/usr/bin/env python3
"""Report the loops of a HIP kernel whose exits LLVM's uniformity analysis calls divergent.

A loop with a divergent exit is compiled with per-lane exit masks: lanes leave one by one
and the loop keeps running with the rest. For a loop whose exits are all wave-uniform in
fact (ballots, readfirstlane'd counters), that machinery is pure overhead, and in the
what-if repair kernel it was where the round-5 hang lived ("The hang").

    python3 scripts/uniformity_check.py openr_amd/csrc/spf_sweep.hip whatif_group_kernel

prints, per matching kernel, every cycle with a divergent exit and its size in basic
blocks. tests/test_uniformity.py asserts that no large loop nest of the repair kernel has
one. Needs hipcc and the ROCm LLVM `opt`; compiles for gfx950 at -O3, as the Makefile does.
"""
import os
import re
import subprocess
import sys
import tempfile

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
OPT = os.path.join(ROCM, "lib", "llvm", "bin", "opt")


def divergent_exit_cycles(src, kernel_pattern, include_dirs=()):
    """{kernel mangled name: [(depth, n_blocks), ...]} for the kernels matching the pattern."""
    with tempfile.TemporaryDirectory() as td:
        ll = os.path.join(td, "k.ll")
        cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-emit-llvm",
               "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "-o", ll, src]
        for d in include_dirs:
            cmd += ["-I", d]
        subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        r = subprocess.run([OPT, "-mtriple=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-passes=print<uniformity>",
                            "-disable-output", ll], check=True, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                           text=True)
    out = {}
    parts = re.split(r"^UniformityInfo for function '([^']+)':$", r.stderr, flags=re.M)
    for name, body in zip(parts[1::2], parts[2::2]):
        if not re.search(kernel_pattern, name):
            continue
        head = body.split("TEMPORAL DIVERGENCE LIST:")[0].split("\nBLOCK ")[0]
        cycles = []
        if "CYCLES WITH DIVERGENT EXIT:" in head:
            for m in re.finditer(r"depth=(\d+): entries\(([^)]*)\)([^\n]*)", head):
                cycles.append((int(m.group(1)), 1 + len(m.group(3).split())))
        out[name] = sorted(cycles, key=lambda c: -c[1])
    return out


def main():
    if len(sys.argv) < 3:
        print(__doc__)
        return 2
    src, pat = sys.argv[1], sys.argv[2]
    inc = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "include")]
    for name, cycles in divergent_exit_cycles(src, pat, inc).items():
        print(name)
        for depth, n in cycles:
            print(f"  depth {depth}: {n} blocks")
    return 0


if __name__ == "__main__":
    sys.exit(main())
