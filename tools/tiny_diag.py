"""Diagnostics: test_gpu_tiny's contexts / args trace in batches of 1 ... 256 events under the environment given,
first mismatch and its batch (one line).  Usage: python tools/tiny_diag.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import test_gpu_context_args as CA  # noqa: E402
import test_gpu_tiny as TT  # noqa: E402


def main():
    n_res = 36
    eng, orc, io, ic, _ = CA._pair(n_res, True)
    ev, ext, table = CA._trace(7, n_res, 4_000, io, ic)
    cuts = TT._cuts(len(ev))
    first = None
    nbad = 0
    for bi, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        g, o = CA._replay(eng, orc, ev[a:b], ext[a:b], table, 1)
        bad = np.nonzero(g != o)[0]
        if len(bad) and first is None:
            i = a + int(bad[0])
            first = (bi, a, b, i, ev[i], hex(int(g[bad[0]])), hex(int(o[bad[0]])))
        nbad += len(bad)
    print({k: os.environ.get(k) for k in ("SG_LIB_PATH", "SG_TINY", "SG_DEBUG_FLAGS")}, "mismatches", nbad, "first",
          first, flush=True)


if __name__ == "__main__":
    main()
