import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built HIP library")


def pytest_sessionstart(session):
    # torch's HIP runtime must initialise before the engine library's in a process that uses both (bench.py and the
    # device-buffer tests do): once libsentinel_gpu.so has created a context, torch reports no HIP GPU.  On a machine
    # without a GPU this is a no-op.
    try:
        import torch
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda")
    except Exception:
        pass
