"""Token-server A/B on one box: bench.token_line under each SG_TOK_* setting given as an argument
(e.g. "SG_TOK_WIDE=512" "SG_TOK_WIDE=1024" "SG_TOK_LIGHT=0,SG_TOK_WIDE=1024"); one JSON line each."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    import torch
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    for k, var in enumerate(sys.argv[1:] or [""]):
        env = dict(kv.split("=") for kv in var.split(",") if kv)
        for kk in ("SG_TOK_WIDE", "SG_TOK_LIGHT"):
            os.environ.pop(kk, None)
        os.environ.update(env)
        r = bench.token_line(dev, cpu_requests=2_000_000 if k == 0 else 0)
        print(json.dumps({"variant": var, **r}), flush=True)


if __name__ == "__main__":
    main()
