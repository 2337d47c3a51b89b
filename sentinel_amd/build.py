"""In-tree build of the product libraries (hipcc for gfx950; g++ for the trace generator)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")


def build(jobs: int = 4) -> None:
    subprocess.run(["make", "-C", CSRC, "-j%d" % jobs, "-s"], check=True)


def build_trace() -> None:
    subprocess.run(["make", "-C", CSRC, "-s", os.path.join("..", "libsentinel_trace.so")], check=True)
