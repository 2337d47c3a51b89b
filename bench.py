#!/usr/bin/env python3
"""Bench: decided entries/sec (whole node) at 1M resources; % of HBM roofline.

Workload = SURVEY.md §8(d) config C4 (the metric's "1M resources" config): 1M
resources, each with a QPS DefaultController flow rule and one DegradeRule
(1/3 RT 50 ms, 1/3 exception ratio 0.2, 1/3 exception count 20; timeWindow 10 s),
Zipf(1.1) popularity, 10^6 entries per trace-second, every entry followed by an
EXIT at t+RT (RT ~ Exp(20 ms), clipped at 4900) and a TRACE with p = 0.05, chain
cap lifted (max_slot_chain_size = 0).  A "step" is one sg_submit of one batch of
--batch-events events already resident in HBM.  Synthetic data (no network).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
resources are hash-sharded -- each rank owns an independent 1M-resource shard
with its own seeded trace, decides with no data-path collective, and the step
time is the max over ranks (weak scaling).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Algorithmic bytes: every event record is read once (24 B), every
# decision word written once (4 B), and every resource touched by a batch reads its
# state once (S_r = 352 B) and writes it once (S_w = 256 B).
EVENT_B, DECISION_B, STATE_RW_B = 24, 4, 352 + 256


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch-events", type=int, default=1 << 25)
    p.add_argument("--resources", type=int, default=1_000_000)
    p.add_argument("--cpu-sample-events", type=int, default=4_000_000)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--profile-out", default="")
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from sentinel_amd import engine as E
    from sentinel_amd import tracegen as T

    steps, warmup = args.steps, args.warmup
    nb = steps + warmup
    # ---- synthetic trace: enough entries for warmup + timed batches
    per_entry_events = 2.05
    n_entries = int(args.batch_events * nb / per_entry_events) + 1
    t0 = time.time()
    w = T.Workload(4, seed=T.SEED_BASE + 4 + 1000 * rank, n_res=args.resources, n_entries=n_entries)
    gen_s = time.time() - t0
    ev = w.events
    n_batches = min(nb, len(ev) // args.batch_events)
    if n_batches < nb:
        steps = max(1, n_batches - warmup)
    eng = E.Engine(device=local if world > 1 else 0, max_resources=1 << 20, max_slot_chain_size=0,
                   param_table_log2=16, status_ring_log2=28, max_batch_events=args.batch_events)
    w.install(eng)

    # ---- events resident in HBM before the timed region
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    dptr = C.c_void_p()
    total = n_batches * args.batch_events
    assert hip.hipSetDevice(local if world > 1 else 0) == 0
    assert hip.hipMalloc(C.byref(dptr), C.c_size_t(total * 24)) == 0
    assert hip.hipMemcpy(dptr, C.c_void_p(ev.ctypes.data), C.c_size_t(total * 24), 1) == 0
    optr = C.c_void_p()
    assert hip.hipMalloc(C.byref(optr), C.c_size_t(args.batch_events * 4)) == 0
    kinds = ev["kind"][:total].reshape(n_batches, args.batch_events)
    entries_per_batch = (kinds == 0).sum(axis=1)
    res_per_batch = [len(np.unique(ev["res_id"][i * args.batch_events:(i + 1) * args.batch_events]))
                     for i in range(n_batches)]

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    # Batches go through the engine's two-stage pipeline (sg_submit_async): the group stage of batch
    # k+1 runs while batch k is being decided; sg_sync at the end of the timed region waits for the
    # last decision.  Per-batch stage times come from HIP events on the engine's streams.
    for i in range(warmup):
        eng.submit_ptr(dptr.value + i * args.batch_events * 24, args.batch_events, optr.value, sync=False)
    eng.sync()
    eng.timing_log()
    barrier()
    t_start = time.perf_counter()
    for i in range(warmup, warmup + steps):
        eng.submit_ptr(dptr.value + i * args.batch_events * 24, args.batch_events, optr.value, sync=False)
    eng.sync()
    barrier()
    elapsed = time.perf_counter() - t_start
    stage_ms = eng.timing_log()  # per timed step: [group, decide, post, total] device ms
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        e = torch.tensor([float(sum(entries_per_batch[warmup:warmup + steps]))], device="cuda", dtype=torch.float64)
        dist.all_reduce(e)
        entries_total = float(e.item())
    else:
        entries_total = float(sum(entries_per_batch[warmup:warmup + steps]))

    # Roofline of the dominant stage: the decide kernels (k_jac<16>/<4>/<1> and k_lane, forked over
    # four streams and joined; HIP events bracket the fork and the join on the engine stream).
    # Algorithmic bytes per launch: every event record read once (24 B), every
    # decision word written once (4 B), every resource touched by the batch reads (352 B) and writes
    # (256 B) its state once.  Sorting/grouping/re-reads are implementation cost, not counted.
    sel = range(warmup, warmup + steps)
    alg_bytes = np.mean([args.batch_events * (EVENT_B + DECISION_B) + res_per_batch[i] * STATE_RW_B for i in sel])
    sm = np.array(stage_ms)
    decide_ms = float(sm[:, 1].mean())
    achieved = alg_bytes / (decide_ms / 1e3) / 1e9
    pipe_ms = elapsed / steps * 1e3
    pipe_achieved = alg_bytes / (pipe_ms / 1e3) / 1e9
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if os.path.exists(pmc):  # rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this same command (tools/profile.sh)
        with open(pmc) as f:
            pj = json.load(f)
        traffic, traffic_src = pj.get("decide_stage_traffic_bytes"), "profiles/pmc_latest.json"
    cpu = None
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(w, args.cpu_sample_events)

    if rank == 0:
        line = {
            "metric": "decided entries/sec (whole node) at 1M resources; % of HBM roofline",
            "value": entries_total / elapsed,
            "unit": "entries/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": elapsed / steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64/f64",
            "data": "synthetic (seeded C4 trace: Zipf(1.1), RT~Exp(20ms), 5% traces)",
            "config": {"workload": "C4: 1M resources, QPS DefaultController + DegradeRule (RT/ratio/count)",
                       "resources_per_gpu": args.resources, "batch_events": args.batch_events,
                       "entries_per_step": float(np.mean(entries_per_batch[warmup:warmup + steps])),
                       "resources_touched_per_step": float(np.mean([res_per_batch[i] for i in sel])),
                       "parallelism": "resource-sharded x%d" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "decide stage: k_jac<16,..> | k_jac<4,..> then k_jac<1,..> | k_lite + k_lane (concurrent streams), then k_fill",
                         "kernel_ms": decide_ms, "alg_bytes_per_launch": float(alg_bytes)},
            "pipeline": {"achieved_GBs": pipe_achieved, "frac": pipe_achieved / HBM_PEAK_GBS,
                         "group_ms": float(sm[:, 0].mean()), "decide_ms": decide_ms, "post_ms": float(sm[:, 2].mean()),
                         "device_ms": float(sm[:, 3].mean()), "wall_ms": pipe_ms},
            "cpu_baseline": cpu,
            "gen_s": gen_s,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(w, n_events):
    """The oracle (C restatement of the Java path, 1 thread) on a bounded prefix of the same trace."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    o = O.Oracle(max_slot_chain_size=0)
    w.install(o)
    ev = w.events[:n_events]
    t = time.perf_counter()
    d = o.submit(ev)
    dt = time.perf_counter() - t
    n_ent = int((ev["kind"] == 0).sum())
    return {"value": n_ent / dt, "unit": "entries/s", "cores": 1, "kind": "port",
            "sample": "first %d events (%d entries) of the C4 trace, oracle/liboracle.so single thread" % (len(ev), n_ent)}


if __name__ == "__main__":
    main()
