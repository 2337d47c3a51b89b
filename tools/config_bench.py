"""Throughput of the engine on the SURVEY.md §8(d) configs besides the headline C4 (bench.py): C2 (10k
resources, QPS DefaultController), C3 (100k resources: QPS / thread-grade / WarmUp / RateLimiter /
WarmUpRateLimiter), C5 (10k resources, hot-parameter rules over 10M Zipf values plus uniform churn, hot
items, thread-grade param rules).  Same method as bench.py: the trace is generated on the host, copied
into HBM, cut into global batches; the first batch is submitted untimed, the rest back to back through the
two-stage pipeline and timed (inputs resident in HBM).  Parity of these shapes against the oracle is
tests/test_gpu_parity.py's; this only measures.

usage: python tools/config_bench.py [OUT.json] [configs, default 2,3,5]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

# config -> (entries, events per batch, engine kwargs, tracegen variant, description)
CONFIGS = {
    2: (50_000_000, 1 << 25, {}, 0, "C2: 10k resources, QPS DefaultController flow rules, Zipf(1.1), 100M events"),
    3: (24_000_000, 1 << 24, {}, "warm_rl",
        "C3: 100k resources, 40% QPS / 20% thread / 20% WarmUp / 10% WarmUpRateLimiter / 10% RateLimiter"),
    5: (16_000_000, 1 << 23, {"param_table_log2": 28, "status_ring_log2": 27}, "c5",
        "C5: 10k resources, ParamFlow QPS (20% throttle) + thread-grade rules, hot items, 10M Zipf values + 50% uniform"),
    # bench.py's C5 sub-line: QPS-grade param rules only, Zipf values
    50: (12_000_000, 1 << 23, {"param_table_log2": 28, "status_ring_log2": 26}, 0,
         "C5 (bench.py sub-line): 10k resources, ParamFlow QPS rules (20% throttle) over 10M Zipf values"),
}


def run(cfg: int):
    import torch
    from sentinel_amd import engine as E
    from sentinel_amd import tracegen as T
    n_entries, gb, kw, var, desc = CONFIGS[cfg]
    variant = {0: 0, "warm_rl": T.V_WARM_RL, "c5": T.V_UNIFORM | T.V_HOT | T.V_THREAD}[var]
    t = time.time()
    c = 5 if cfg == 50 else cfg
    w = T.Workload(c, seed=T.SEED_BASE + c, n_entries=n_entries, variant=variant)
    ev = w.events
    gen_s = time.time() - t
    nb = (len(ev) + gb - 1) // gb
    cuts = [min(len(ev), b * gb) for b in range(nb + 1)]
    eng = E.Engine(max_resources=max(w.n_res, 1 << 10), max_slot_chain_size=0, max_batch_events=gb, **kw)
    w.install(eng)
    dev = torch.device("cuda", 0)
    buf = torch.from_numpy(np.ascontiguousarray(ev).view(np.uint8)).to(dev)
    out = torch.empty(gb, dtype=torch.int32, device=dev)
    p0 = buf.data_ptr()
    eng.submit_ptr(p0, cuts[1], out.data_ptr(), sync=True)  # warmup: the first batch
    eng.timing_log()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(1, nb):
        eng.submit_ptr(p0 + cuts[b] * 24, cuts[b + 1] - cuts[b], out.data_ptr(), sync=False)
    eng.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = np.array(eng.timing_log())
    timed = ev[cuts[1]:]
    entries = int((timed["kind"] == 0).sum())
    res = {"config": desc, "value": entries / dt, "unit": "entries/s", "events_timed": len(timed),
           "entries_timed": entries, "batches_timed": nb - 1, "batch_events": gb, "seconds": dt,
           "ms_per_batch": dt / (nb - 1) * 1e3,
           "stage_ms_mean": {"group": float(st[:, 0].mean()), "decide": float(st[:, 1].mean()),
                             "post": float(st[:, 2].mean())},
           "resources": w.n_res, "gen_s": gen_s}
    eng.close()
    w.close()
    del buf, out
    torch.cuda.empty_cache()
    return res


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    cfgs = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [2, 3, 5]
    import bench
    rows = []
    for c in cfgs:
        r = run(c)
        print(json.dumps(r), flush=True)
        rows.append(r)
    if out:
        with open(out, "w") as f:
            json.dump({"src_sha": bench.src_sha(), "configs": rows}, f, indent=1)


if __name__ == "__main__":
    main()
