import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine through the C-ABI)")
    # torch ships its own HIP runtime (libamdhip64.so) next to the engine's
    # (/opt/rocm/lib/libamdhip64.so.7): the two coexist in one process only when torch
    # initialises the device first, so GPU runs bring torch up before any engine.
    if "not gpu" not in (config.getoption("-m") or ""):
        try:
            import torch

            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:  # pragma: no cover - CPU-only hosts
            pass
