#!/usr/bin/env python3
"""Bench: decided entries/sec (whole node) at 1M resources; % of HBM roofline.

Workload = SURVEY.md §8(d) config C4 (the metric's "1M resources" config): 1M resources, each with
a QPS DefaultController flow rule and one DegradeRule (1/3 RT 50 ms, 1/3 exception ratio 0.2, 1/3
exception count 20; timeWindow 10 s), Zipf(1.1) popularity, 10^6 entries per trace-second, every
entry followed by an EXIT at t+RT (RT ~ Exp(20 ms), clipped at 4900) and a TRACE with p = 0.05,
chain cap lifted (max_slot_chain_size = 0).  Synthetic data (no network).

Batches: the trace is cut into global batches of --batch-events events (2^25).  --base-batches of
them are generated on the host; later batches are time-shifted copies built on the device before
each timed chunk (timestamps + k x the trace span, EXIT/TRACE references + k x the events of the
trace), so every batch is fresh to the engine -- time only moves forward, windows roll, breakers
trip and reset -- and nothing is replayed.  A step is --sub-batches global batches submitted back to
back through the engine's two-stage pipeline (sg_submit_async: the group stage of batch k+1 overlaps
the decide stage of batch k).  The K timed steps run in chunks whose inputs fit in HBM: before each
chunk its fresh batches are built (untimed), the chunk is bracketed by barrier + synchronize and
timed, and the step time is the chunks' total over K.  Inputs are resident in HBM whenever a timed
chunk starts.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N, or bench.py --gpus N
alone, which starts the N rank processes itself): ONE C4 trace,
resources partitioned over the ranks (strong scaling).  Every rank generates the same trace and
keeps its shard (EXIT/TRACE references rewritten to its own numbering).  The partition is a resource ->
rank table balanced by the event counts of a history window, the first global batch
(sentinel_amd/dist.py balanced_table; --sharding
hash: splitmix64(res_id) % N), and each rank submits its shard either as one batch per global batch (~--batch-events
/ N events, S a step: --rank-batches global, the default) or in rank-local batches of ~--batch-events
events (S / N a step: --rank-batches local), so the ranks advance independently: the decision path has
no collective, and only the per-second MetricNode all-gather (RCCL) inside the timed chunks and the
chunk barriers synchronise them.  The step time is the max over ranks and value = every rank's
entries / that time.

After the C4 line's measurement (N = 1), the same pipeline measures the other SURVEY.md §8(d) configs
C2, C3, C5 and C6 (bounded traces, inputs in HBM) and reports them under "configs" (--no-configs: skip).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Algorithmic bytes: every event record is read once (24 B), every ENTRY's decision
# word written once (4 B), and every resource touched by a batch reads its state once (S_r = 352 B)
# and writes it once (S_w = 256 B).
EVENT_B, DECISION_B, STATE_RW_B = 24, 4, 352 + 256
REF_MASK = 0xFFFFFFFFFFFF
EPE = 2.05  # C4 events per entry (entry + exit + 5 % traces)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # defaults: ~4 s of timed GPU work (20 steps x 48 global batches) so an outside utilisation sampler sees it
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch-events", type=int, default=1 << 25, help="events per global batch")
    p.add_argument("--base-batches", type=int, default=8, help="global batches generated on the host")
    p.add_argument("--sub-batches", type=int, default=48, help="global batches per step (a multiple of N)")
    p.add_argument("--max-sub-batches", type=int, default=0, help="(kept for old scripts; unused)")
    p.add_argument("--hbm-budget", type=float, default=0.8,
                   help="fraction of free HBM for one timed chunk's inputs")
    p.add_argument("--sharding", choices=("balanced", "hash"), default="balanced",
                   help="resource -> GPU partition: balanced by event counts, or splitmix64(res_id) %% N")
    p.add_argument("--no-configs", action="store_true", help="skip the C2 / C3 / C5 / C6 sub-lines")
    p.add_argument("--only-config", default="", metavar="C2|C3|C5|C5-ext|C6",
                   help="measure only that config sub-line (no headline; tools/pmc_configs.py profiles it)")
    p.add_argument("--resources", type=int, default=1_000_000)
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="partitioned oracle threads (0: this job's CPU share -- cgroup cpu.max, else min(16, cores))")
    p.add_argument("--cpu-sample-events", type=int, default=24_000_000)
    p.add_argument("--cpu-single-events", type=int, default=6_000_000)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--balance-alpha", type=float, default=0.9,
                   help="--sharding balanced: a resource's load = its history-window events ** alpha")
    p.add_argument("--rank-batches", default="auto",
                   help="N > 1: global batches per rank batch -- an integer k (a rank's batch = its shard of k consecutive "
                        "global batches, ~k * batch-events / N events), 'local' (k = N: batches of ~--batch-events), "
                        "'global' (k = 1) or 'auto' (tools/shard_rehearsal.sh, DESIGN.md §7)")
    p.add_argument("--shard", default="", metavar="R/N",
                   help="rehearsal: run rank R's shard of an N-GPU run alone on this GPU (no collectives; "
                        "the per-rank step time of the N-GPU run, NOT a measurement of it)")
    return p.parse_args()


def src_sha() -> str:
    """Content hash of the product sources (the GPU box has no .git): profiles/ files carry it, and
    bench.py only reports PMC traffic measured on these exact sources."""
    h = hashlib.sha256()
    for d, exts in (("sentinel_amd/csrc", (".hip", ".cpp", ".h")), ("include", (".h",))):
        for f in sorted(os.listdir(os.path.join(ROOT, d))):
            if f.endswith(exts):
                h.update(f.encode())
                with open(os.path.join(ROOT, d, f), "rb") as fh:
                    h.update(fh.read())
    return h.hexdigest()[:16]


# global batches per rank batch by N (bench --rank-batches auto): one at every N measured (tools/shard_rehearsal.sh,
# N = 2 / 4 / 8 slowest rank 2.30 / 1.83 / 1.46 ms per global batch, against 2.45 / 2.16 / 1.90 with two)
AUTO_RANK_BATCHES = {}


def rank_batch_k(spec: str, nparts: int) -> int:
    """--rank-batches: global batches per rank batch (local = N, global = 1, auto by N, or an integer)."""
    if spec == "local":
        return nparts
    if spec == "global":
        return 1
    if spec == "auto":
        return AUTO_RANK_BATCHES.get(nparts, 1)
    return int(spec)


def rank_batch_cuts(pos, n_base: int, gb: int, B: int, S: int, nparts: int, kb: int):
    """A rank's batches of its shard of the B base batches: (batches LB, batches a step, event cuts [LB + 1]).

    k = N (or one GPU): B / N batches of ~gb events cut evenly (each spans N global batches' time, S / N a step);
    otherwise the shard of kb consecutive global batches each (pos: the shard's global event positions), S / kb a step.
    """
    if nparts <= 1 or kb == nparts:
        LB = max(1, B // nparts)
        return LB, max(1, S // nparts), np.linspace(0, n_base, LB + 1).astype(np.int64)
    assert kb >= 1 and B % kb == 0 and S % kb == 0, "--rank-batches k must divide --base-batches and --sub-batches"
    cuts = np.searchsorted(pos, np.arange(0, B + 1, kb, dtype=np.int64) * gb).astype(np.int64)
    cuts[-1] = n_base
    return B // kb, S // kb, cuts


def make_trace(n_res: int, batch_events: int, base_batches: int, seed: int):
    """The C4 trace, cut to base_batches whole global batches (the Workload owns the memory)."""
    from sentinel_amd import tracegen as T
    need = batch_events * base_batches
    n_entries = int(need / EPE * 1.01) + 1000
    while True:
        w = T.Workload(4, seed=seed, n_res=n_res, n_entries=n_entries)
        if len(w.events) >= need:
            return w, w.events[:need]
        n_entries = int(n_entries * 1.05)
        w.close()


def shifted_batch(base64, a: int, e: int, copy: int, tspan: int, n_base: int, out64):
    """Global-batch copy `copy` of base rows [a, e) into out64 (torch int64 [n, 3] views of sg_event
    records: ts | res_id,count,kind,flags | aux): ts + copy*tspan, references + copy*n_base."""
    import torch
    src = base64[a:e]
    out64.copy_(src)
    if copy:
        out64[:, 0] += copy * tspan
        kind = (src[:, 1] >> 48) & 0xFF
        isref = (kind != 0) & ((src[:, 2] & REF_MASK) != REF_MASK)
        out64[:, 2] += torch.where(isref, copy * n_base, 0)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.shard:
        # `bench.py --gpus N` alone: start the N ranks here (sentinel_amd/launch.py), before anything imports
        # torch -- this parent never touches a GPU; rank 0 prints the JSON line
        from sentinel_amd.launch import launch_ranks
        sys.exit(launch_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    if args.only_config:
        import torch
        dev = torch.device("cuda", 0)
        rows = config_lines(dev, None, 0, only=[args.only_config])
        print(json.dumps({"only_config": args.only_config, "configs": rows, "src_sha": src_sha()}), flush=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not args.shard and world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d: launch one process per GPU (torchrun "
                 "--nproc-per-node %d, or bench.py --gpus %d alone)" % (args.gpus, world, args.gpus, args.gpus))
    import torch
    # SG_BENCH_GLOO=1 rehearses the multi-rank path on a one-GPU box: gloo instead of RCCL, every rank on
    # device local % device_count (never used for a reported number)
    rehearse = os.environ.get("SG_BENCH_GLOO") == "1"
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local % ndev if rehearse else local)
    dev = torch.device("cuda", local % ndev if rehearse else local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    cdev = torch.device("cpu") if rehearse else dev  # where collective tensors live

    from sentinel_amd import dist as D
    from sentinel_amd import engine as E
    from sentinel_amd import tracegen as T

    steps, warmup, gb, B = args.steps, args.warmup, args.batch_events, args.base_batches
    S = max(1, args.sub_batches)
    # ---- one trace for the whole node; this rank's shard of it
    t_gen = time.time()
    w, ev = make_trace(args.resources, gb, B, T.SEED_BASE + 4)
    gen_s = time.time() - t_gen
    tspan = int(ev["ts"][-1] - ev["ts"][0]) + 1000  # copy k starts a second after copy k-1 ends
    shard = tuple(int(x) for x in args.shard.split("/")) if args.shard else None  # (R, N)
    if shard:
        assert world == 1 and 0 <= shard[0] < shard[1], "--shard R/N: one process, 0 <= R < N"
    nparts = shard[1] if shard else world
    me = shard[0] if shard else rank
    table = None
    if nparts > 1:
        # every rank computes the same table from the same history window: the event counts of the first
        # global batch only (a router knows past load, not the future), so 7/8 of the timed events are
        # batches the partition never saw (not the timed trace)
        if args.sharding == "balanced":
            table = D.balanced_table(np.bincount(ev["res_id"][:gb], minlength=args.resources), nparts,
                                     args.balance_alpha)
        mine, pos = D.shard_stream(ev, nparts, me, table)
    else:
        mine = ev
    n_base = len(mine)
    kb = rank_batch_k(args.rank_batches, nparts)
    rank_batches = kb
    LB, per_step, cuts = rank_batch_cuts(pos if nparts > 1 else None, n_base, gb, B, S, nparts, kb)
    sizes = np.diff(cuts)
    ent_b = np.array([int((mine["kind"][cuts[b]:cuts[b + 1]] == 0).sum()) for b in range(LB)])
    res_b = np.array([len(np.unique(mine["res_id"][cuts[b]:cuts[b + 1]])) for b in range(LB)])
    end_b = np.array([int(mine["ts"][max(cuts[b], cuts[b + 1] - 1)]) for b in range(LB)])

    eng = E.Engine(device=dev.index, max_resources=1 << 20, max_slot_chain_size=0, param_table_log2=16,
                   status_ring_log2=28, max_batch_events=int(sizes.max()))
    w.install(eng)

    # ---- the shard's base batches into HBM (pinned host -> device; the PCIe rate is reported, never value)
    host = torch.from_numpy(np.ascontiguousarray(mine).view(np.uint8)).pin_memory()
    base = torch.empty(host.numel(), dtype=torch.uint8, device=dev)
    h0, h1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    h0.record()
    base.copy_(host, non_blocking=True)
    h1.record()
    torch.cuda.synchronize()
    h2d_ms = h0.elapsed_time(h1)
    del host
    base64 = base.view(torch.int64).view(-1, 3)

    # ---- one timed chunk's inputs in HBM at once, after the engine's two batch slots (~120 B per event each)
    free = torch.cuda.mem_get_info(dev)[0]
    mean_b = float(sizes.mean()) * 24
    snap_cap = min(60 * args.resources // max(1, world) + 4096, 1 << 26)
    reserve = 2 * 120 * int(sizes.max()) + snap_cap * 64
    chunk_steps = int(max(1, min(steps, args.hbm_budget * (free - reserve) // (per_step * mean_b * 1.15))))
    if dist is not None:
        t = torch.tensor([chunk_steps], device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        chunk_steps = int(t.item())
    gidx = lambda i: (i % LB, i // LB)  # rank-local batch i -> (base batch, copy)
    max_ev = max(int(sum(sizes[gidx(i)[0]] for i in range(g0, g0 + chunk_steps * per_step)))
                 for g0 in range(0, (warmup + steps) * per_step, chunk_steps * per_step))
    buf = torch.empty((max_ev, 3), dtype=torch.int64, device=dev)
    out = torch.empty(int(sizes.max()), dtype=torch.int32, device=dev)
    snap = torch.empty(snap_cap * 64, dtype=torch.uint8, device=dev) if dist is not None else None

    def build(g0, n):
        """Rank-local batches g0..g0+n-1 into buf: [(row offset, rows, entries, touched, end ts)]."""
        plan, off = [], 0
        for g in range(g0, g0 + n):
            b, k = gidx(g)
            m = int(sizes[b])
            shifted_batch(base64, int(cuts[b]), int(cuts[b + 1]), k, tspan, n_base, buf[off:off + m])
            plan.append((off, m, int(ent_b[b]), int(res_b[b]), int(end_b[b]) + k * tspan))
            off += m
        torch.cuda.synchronize()
        return plan

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    def gather_metrics(now):
        """MetricTimerListener across the node: every rank's MetricNode rows, device to device."""
        n = eng.snapshot_to(now, snap.data_ptr(), snap_cap)
        n = min(n, snap_cap)
        cnt = torch.tensor([n], device=cdev)
        cnts = [torch.zeros_like(cnt) for _ in range(world)]
        dist.all_gather(cnts, cnt)
        width = int(max(c.item() for c in cnts)) * 64
        if width:
            outs = [torch.empty(width, dtype=torch.uint8, device=cdev) for _ in range(world)]
            dist.all_gather(outs, snap[:width].to(cdev))
        return sum(int(c.item()) for c in cnts)

    base_ptr = buf.data_ptr()
    # ---- warmup (untimed): the first W steps of the stream
    g = 0
    for c0 in range(0, warmup, chunk_steps):
        n = min(chunk_steps, warmup - c0) * per_step
        for off, m, _, _, _ in build(g, n):
            eng.submit_ptr(base_ptr + off * 24, m, out.data_ptr(), sync=False)
        eng.sync()
        g += n
    eng.timing_log()
    if dist is not None:  # the first fetch (lastFetchTime = -1) outside the timed region
        gather_metrics(int(end_b[(g - 1) % LB]) + ((g - 1) // LB) * tspan)
    # ---- timed: the next K steps (fresh, time-shifted batches), chunk by chunk
    n_gather, rows_gathered = 0, 0
    elapsed, entries, touched, events, stage_rows = 0.0, 0.0, 0.0, 0.0, []
    chunks = 0
    for c0 in range(0, steps, chunk_steps):
        ns = min(chunk_steps, steps - c0)
        plan = build(g, ns * per_step)
        g += ns * per_step
        barrier()
        t_start = time.perf_counter()
        t_last = t_start
        for s in range(ns):
            for off, m, _, _, _ in plan[s * per_step:(s + 1) * per_step]:
                eng.submit_ptr(base_ptr + off * 24, m, out.data_ptr(), sync=False)
            if dist is not None and time.perf_counter() - t_last >= 1.0:
                rows_gathered += gather_metrics(plan[(s + 1) * per_step - 1][4])  # drains this rank's pipeline
                n_gather += 1
                t_last = time.perf_counter()
        eng.sync()
        barrier()
        elapsed += time.perf_counter() - t_start
        chunks += 1
        stage_rows.extend(eng.timing_log().tolist())  # per timed batch: [group, decide, post, total] device ms
        entries += float(sum(p[2] for p in plan))
        touched += float(sum(p[3] for p in plan))
        events += float(sum(p[1] for p in plan))
    n_untimed = 0
    if dist is not None and n_gather == 0:  # at least one all-gather per run, untimed
        rows_gathered += gather_metrics(plan[-1][4])
        n_untimed = 1
    stage_ms = np.array(stage_rows)
    if dist is not None:
        t = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        t = torch.tensor([entries, touched, events], device=cdev, dtype=torch.float64)
        dist.all_reduce(t)
        entries, touched, events = (float(x) for x in t.tolist())
        lb = torch.tensor([float(n_base)], device=cdev, dtype=torch.float64)
        lbs = [torch.zeros_like(lb) for _ in range(world)]
        dist.all_gather(lbs, lb)
        shares = [float(x.item()) for x in lbs]
    else:
        shares = [float(n_base)]

    nb = steps * S  # global-batch equivalents timed (all ranks)
    batch_ms = elapsed / nb * 1e3
    # algorithmic bytes per global batch (all ranks), SURVEY.md §8(d)
    alg = (events * EVENT_B + entries * DECISION_B + touched * STATE_RW_B) / nb
    achieved = alg / (batch_ms / 1e3) / 1e9
    decide_ms = float(stage_ms[:, 1].mean())
    dec_alg = alg * nb / (steps * per_step) / world  # one rank-local batch's share, over its decide-stage time
    traffic, tnote, traffic_rw = None, None, None
    pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
    sha = src_sha()
    if os.path.exists(pmc):  # rocprofv3 FETCH_SIZE/WRITE_SIZE passes (tools/profile.sh) on these sources
        with open(pmc) as f:
            pj = json.load(f)
        if pj.get("src_sha") == sha and pj.get("batch_events") == gb and world == 1 and not shard:
            traffic = pj.get("traffic_bytes_per_batch")
            traffic_rw = {"read": pj.get("read_bytes_per_batch"), "write": pj.get("write_bytes_per_batch"),
                          "all_fetches_doubled": pj.get("traffic_upper_bytes_per_batch")}
            tnote = ("profiles/pmc_latest.json (src_sha %s, git %s): FETCH_SIZE doubled for the streaming kernels, "
                     "as counted for the random-access ones" % (sha, pj.get("git_head")))
        else:
            why = ("src_sha %s != %s" % (pj.get("src_sha"), sha) if pj.get("src_sha") != sha else
                   "batch_events %s != %s" % (pj.get("batch_events"), gb) if pj.get("batch_events") != gb else
                   "measured on one GPU, this run has %d ranks" % world if world > 1 else
                   "measured on the whole trace, this run is one shard")
            tnote = "profiles/pmc_latest.json is for other sources/config (%s): not used" % why
    stream = stream_copy_gbps(dev) if rank == 0 else None
    cpu = None
    if rank == 0 and world == 1 and not shard and not args.no_cpu_baseline:
        cpu = cpu_baseline(w, ev, args)
    configs = None
    if rank == 0 and world == 1 and not shard and not args.no_configs:
        del buf, base, base64, out
        eng.close()
        torch.cuda.empty_cache()
        configs = config_lines(dev, (w, ev), 0 if args.no_cpu_baseline else 4_000_000)

    if rank == 0:
        line = {
            "metric": "decided entries/sec (whole node) at 1M resources; % of HBM roofline",
            "value": entries / elapsed,
            "unit": "entries/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": elapsed / steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",   # one trace partitioned over the ranks: total work is fixed as N grows
            "vs_baseline": None,
            "dtype": "int64/f64",
            "data": "synthetic (seeded C4 trace: Zipf(1.1), RT~Exp(20ms), 5% traces; time-shifted fresh batches)",
            "config": {"workload": "C4: 1M resources, QPS DefaultController + DegradeRule (RT/ratio/count)",
                       "resources": args.resources, "batch_events": gb, "sub_batches_per_step": S,
                       "events_per_step": events / steps, "entries_per_step": entries / steps,
                       "resources_touched_per_batch": touched / nb, "base_batches": B,
                       "timed_chunks": chunks, "rank_local_batches_per_step": per_step,
                       "rank_batches": rank_batches if nparts > 1 else None,
                       "parallelism": ("resource-sharded x%d (%s)" % (world, "balanced by the event counts of a "
                                                                      "history window: base batch 0 of %d" % B
                                                                      if args.sharding == "balanced" else
                                                                      "splitmix64(res_id) %% %d" % world))
                                      if world > 1 else "one GPU",
                       "rank_event_shares": [x / sum(shares) for x in shares]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tnote,
                         "traffic_split": traffic_rw,
                         "traffic_GBps": traffic / (batch_ms / 1e3) / 1e9 if traffic else None,
                         "stream_copy_GBps": stream,
                         "frac_of_stream_copy": achieved / stream if stream else None,
                         "kernel": "one global batch through the whole pipeline (sort/group, decide, post)",
                         "batch_ms": batch_ms, "alg_bytes_per_batch": alg,
                         "decide_stage": {"ms": decide_ms, "achieved": dec_alg / (decide_ms / 1e3) / 1e9,
                                          "frac": dec_alg / (decide_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                                          "kernels": "k_jac<8> (or k_jac<16>) | k_jac<4>, k_pq | k_lite, k_lane, k_jac<1> (streams), k_fill"}},
            "pipeline": {"group_ms": float(stage_ms[:, 0].mean()), "decide_ms": decide_ms,
                         "post_ms": float(stage_ms[:, 2].mean()), "device_ms": float(stage_ms[:, 3].mean()),
                         "wall_ms_per_batch": batch_ms},
            "h2d": {"GBps": n_base * 24 / (h2d_ms / 1e3) / 1e9, "pcie_inclusive_entries_per_s":
                    entries / (elapsed + h2d_ms / 1e3 * events / max(1, n_base) / world),
                    "note": "pinned host -> HBM copy of the events, measured on the base trace; not in value"},
            "metric_gathers": {"count": n_gather + n_untimed, "timed": n_gather, "rows": rows_gathered}
                              if world > 1 else None,
            "rehearsal": ("gloo, all ranks on one GPU: NOT a measurement" if rehearse else
                          "rank %d of %d alone on one GPU (per-rank step of an N-GPU run): NOT a measurement" % shard
                          if shard else None),
            "cpu_baseline": cpu,
            "configs": configs,
            "src_sha": sha,
            "gen_s": gen_s,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def stream_copy_gbps(dev) -> float:
    """Device-to-device copy bandwidth (read + write bytes / time) of a 4 GiB buffer: the attainable
    HBM rate, the second roofline denominator."""
    import torch
    n = 1 << 31
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    b = torch.empty(n, dtype=torch.uint8, device=dev)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbps = 2.0 * n * 10 / (e0.elapsed_time(e1) / 1e3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return gbps


# SURVEY.md §8(d) configs besides C4, measured as bench.py measures C4 (first batch untimed, the rest back to back
# through the pipeline, inputs in HBM): (config, entries, events per batch, engine kwargs, tracegen variant, name)
CONFIGS = [
    (2, 50_000_000, 1 << 25, {}, 0, "C2: 10k resources, QPS DefaultController flow rules, Zipf(1.1)"),
    (3, 24_000_000, 1 << 24, {}, 1, "C3: 100k resources, QPS / thread / WarmUp / RateLimiter / WarmUpRateLimiter"),
    (5, 12_000_000, 1 << 23, {"param_table_log2": 28, "status_ring_log2": 26}, 0,
     "C5: 10k resources, ParamFlow QPS rules (20 % throttle) over 10M Zipf values"),
    (6, 49_500_000, 1 << 25, {"param_table_log2": 29, "status_ring_log2": 28, "max_rules": 1 << 22}, 0,
     "C6 (north_star's mixed rules): 1M resources, each a QPS flow rule + a DegradeRule + a QPS ParamFlowRule on "
     "args[0] (values Zipf(1.1) over 10M), Zipf(1.1) traffic"),
]
EXT_NOTE = ("sg_submit_ex, the Java drop-in's call: every event in one of 4 named contexts (ContextUtil.enter) from "
            "one of 16 origins, uniformly (an EXIT carries its ENTRY's); origin StatisticNodes and context "
            "DefaultNodes kept on the device")


def alg_bytes(ev, args_keyed: bool) -> float:
    """SURVEY.md §8(d) algorithmic bytes of one batch: 24 B per event record, 4 B per ENTRY decision, 608 B of state
    (S_r + S_w) per touched resource, and for hot-parameter rules 2 x 16 B per distinct (resource, args[0]) pair of
    the batch's ENTRYs (the param term 2 * 16 * U_b; one param rule per resource in C5 / C6)."""
    from sentinel_amd import _abi as A
    ent = ev["kind"] == A.EV_ENTRY
    b = len(ev) * EVENT_B + int(ent.sum()) * DECISION_B + len(np.unique(ev["res_id"])) * STATE_RW_B
    if args_keyed:
        has = ent & ((ev["flags"] & A.F_HAS_ARG) != 0)
        pairs = np.empty(int(has.sum()), dtype=[("r", np.uint32), ("k", np.uint64)])
        pairs["r"], pairs["k"] = ev["res_id"][has], ev["aux"][has]
        b += 2 * 16 * len(np.unique(pairs))
    return float(b)


def config_roofline(cfg_key: str, ms_per_batch: float, alg: float, gb: int) -> dict:
    """roofline of a config sub-line: its algorithmic bytes per batch over the wall time per batch; traffic = the
    rocprofv3 FETCH / WRITE passes of that config (profiles/pmc_configs.json, tools/pmc_configs.py) when they were
    measured on these sources."""
    traffic, src = None, None
    pj = os.path.join(ROOT, "profiles", "pmc_configs.json")
    if os.path.exists(pj):
        with open(pj) as f:
            rec = json.load(f).get(cfg_key)
        if rec and rec.get("src_sha") == src_sha() and rec.get("batch_events") == gb:
            traffic = rec["traffic_bytes_per_batch"]
            src = "profiles/pmc_configs.json[%s] (src_sha %s)" % (cfg_key, rec["src_sha"])
        elif rec:
            src = "profiles/pmc_configs.json[%s] is for other sources (src_sha %s): not used" % (cfg_key, rec.get("src_sha"))
    ach = alg / (ms_per_batch / 1e3) / 1e9
    return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "alg_bytes_per_batch": alg, "traffic": traffic, "traffic_source": src,
            "kernel": "one batch through the whole pipeline (group, decide, post)"}


def run_batches(eng, ev, gb, dev, ext=None, args=None, cfg_key=None, args_keyed=False):
    """Batch 0 untimed, the rest back to back through the pipeline; inputs (events, ext, args) in HBM."""
    import torch
    nb = (len(ev) + gb - 1) // gb
    cuts = [min(len(ev), b * gb) for b in range(nb + 1)]
    buf = torch.from_numpy(np.ascontiguousarray(ev).view(np.uint8)).to(dev)
    xb = torch.from_numpy(np.ascontiguousarray(ext).view(np.uint8)).to(dev) if ext is not None else None
    ab = torch.from_numpy(np.ascontiguousarray(args).view(np.uint8)).to(dev) if args is not None else None
    out = torch.empty(gb, dtype=torch.int32, device=dev)
    p0 = buf.data_ptr()

    def sub(b, sync):
        if xb is None:
            eng.submit_ptr(p0 + cuts[b] * 24, cuts[b + 1] - cuts[b], out.data_ptr(), sync=sync)
        else:
            eng.submit_ex_ptr(p0 + cuts[b] * 24, xb.data_ptr() + cuts[b] * 16, cuts[b + 1] - cuts[b], out.data_ptr(),
                              sync=sync, args_ptr=ab.data_ptr() if ab is not None else 0,
                              n_args=len(args) if args is not None else 0)
    sub(0, True)
    eng.timing_log()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(1, nb):
        sub(b, False)
    eng.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = np.array(eng.timing_log())
    ent = int((ev[cuts[1]:]["kind"] == 0).sum())
    del buf, xb, ab, out
    torch.cuda.empty_cache()
    r = {"value": ent / dt, "unit": "entries/s", "batches_timed": nb - 1, "batch_events": gb, "entries_timed": ent,
         "ms_per_batch": dt / (nb - 1) * 1e3, "stage_ms_mean": {"group": float(st[:, 0].mean()),
                                                                "decide": float(st[:, 1].mean()),
                                                                "post": float(st[:, 2].mean())}}
    if cfg_key:
        alg = float(np.mean([alg_bytes(ev[cuts[b]:cuts[b + 1]], args_keyed) for b in range(1, nb)]))
        r["roofline"] = config_roofline(cfg_key, r["ms_per_batch"], alg, gb)
    return r


def param_args(ev):
    """C5's argument through the sg_submit_ex table: args = {args[0]} for every ENTRY (its interned key)."""
    from sentinel_amd import _abi as A
    ent = ev["kind"] == A.EV_ENTRY
    ext = np.zeros(len(ev), dtype=A.EXT_DTYPE)
    ext["arg_off"] = np.arange(len(ev), dtype=np.uint32)
    ext["n_args"] = ent.astype(np.uint32)
    table = np.zeros(len(ev), dtype=A.ARG_DTYPE)
    table["key"] = ev["aux"]
    table["kind"] = np.where(ent, A.ARG_SCALAR, A.ARG_NULL)
    return ext, table


def config_cpu_baseline(w, ev, n_events):
    """The oracle on the config's first n_events events (rounded down to whole EXIT references: a prefix of the
    trace is self-contained), this job's CPU share partitioned by resource, as the C4 line's cpu_baseline."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    T = cpu_share()
    sample = ev[:min(len(ev), n_events)]
    po = O.PartitionedOracle(w, T, max_slot_chain_size=0)
    spent = []
    po.submit(sample, timed=spent)
    po.close()
    n_ent = int((sample["kind"] == 0).sum())
    return {"value": n_ent / spent[0], "unit": "entries/s", "cores": T, "kind": "port",
            "sample": "first %d events (%d entries) of the config's trace, oracle/liboracle.so, %d threads partitioned "
                      "by splitmix64(res_id) %% %d (routing excluded)" % (len(sample), n_ent, T, T)}


def ext_cpu_baseline(w, ev, ext, n_events):
    """config_cpu_baseline through or_submit_ex: the same contexts / origins on every event (the oracle keeps each
    entry's origin StatisticNode and context DefaultNode, as the device does)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    T = cpu_share()
    sample = ev[:min(len(ev), n_events)]
    po = O.PartitionedOracle(w, T, max_slot_chain_size=0)
    for o in po.orcs:
        w.intern_names(o)
    spent = []
    po.submit_ex(sample, ext[:len(sample)], timed=spent)
    po.close()
    n_ent = int((sample["kind"] == 0).sum())
    return {"value": n_ent / spent[0], "unit": "entries/s", "cores": T, "kind": "port",
            "sample": "first %d events (%d entries) of the line's trace with its contexts / origins, "
                      "oracle/liboracle.so or_submit_ex, %d threads partitioned by splitmix64(res_id) %% %d "
                      "(routing excluded)" % (len(sample), n_ent, T, T)}


def _oracle_for(w, ev, eng_names=True):
    """One oracle (one thread: a lone caller's view) holding the resources ev touches, names interned as the
    engine's (w.intern_names)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(orc, np.unique(ev["res_id"]))
    if eng_names:
        w.intern_names(orc)
    return orc


def config_lines(dev, c4=None, cpu_events=4_000_000, only=None):
    """The SURVEY.md configs besides the headline: C2, C3, C5, C6 (mixed rules); with c4 = (workload, events) of the headline trace,
    C4 and C4-ext on its first 3 global batches (the same events through sg_submit and sg_submit_ex), C5-ext, and
    the drop-in's operating point (dropin_line)."""
    import torch
    from sentinel_amd import engine as E
    from sentinel_amd import tracegen as T
    rows = []
    if c4 is not None:
        w, ev = c4
        gb = 1 << 25
        sub = ev[:3 * gb]
        for ext_on in (False, True):
            eng = E.Engine(device=dev.index, max_resources=1 << 20, max_slot_chain_size=0, param_table_log2=16,
                           status_ring_log2=28, max_batch_events=gb, aux_node_capacity=(1 << 24) if ext_on else 1 << 16)
            w.install(eng)
            ext = None
            if ext_on:
                io, ic = w.intern_names(eng)
                ext = T.ext_for(sub, io, ic, seed=T.SEED_BASE + 44)
            r = run_batches(eng, sub, gb, dev, ext=ext, cfg_key="C4-ext" if ext_on else "C4")
            r.update({"config": "C4%s: 1M resources, QPS DefaultController + DegradeRule, first 3 batches of the "
                                "headline trace" % ("-ext" if ext_on else ""), "resources": w.n_res})
            if ext_on:
                r["note"] = EXT_NOTE
                if cpu_events:
                    r["cpu_baseline"] = ext_cpu_baseline(w, sub, ext, cpu_events)
            rows.append(r)
            eng.close()
            torch.cuda.empty_cache()
    for cfg, n_entries, gb, kw, var, name in CONFIGS:
        if only and not any(o.split("-")[0] == "C%d" % cfg for o in only):
            continue
        w = T.Workload(cfg, seed=T.SEED_BASE + cfg, n_entries=n_entries, variant=var)
        ev = w.events
        ext_ons = (False, True) if cfg == 5 else (False,)
        if only:
            ext_ons = tuple(e for e in ext_ons if ("C%d%s" % (cfg, "-ext" if e else "")) in only)
        for ext_on in ext_ons:
            eng = E.Engine(device=dev.index, max_resources=max(w.n_res, 1 << 10), max_slot_chain_size=0,
                           max_batch_events=gb, aux_node_capacity=1 << 20, **kw)
            w.install(eng)
            ext = args = None
            if ext_on:
                io, ic = w.intern_names(eng)
                ext, args = param_args(ev)
                oc = T.ext_for(ev, io, ic, seed=T.SEED_BASE + 45)
                ext["origin_id"], ext["context_id"] = oc["origin_id"], oc["context_id"]
            r = run_batches(eng, ev, gb, dev, ext=ext, args=args, cfg_key="C%d%s" % (cfg, "-ext" if ext_on else ""),
                            args_keyed=cfg in (5, 6))
            r.update({"config": name if not ext_on else name.replace("C5:", "C5-ext:") + "; args[0] from the table",
                      "resources": w.n_res})
            if ext_on:
                r["note"] = EXT_NOTE
            eng.close()
            torch.cuda.empty_cache()
            if not ext_on and cpu_events:
                r["cpu_baseline"] = config_cpu_baseline(w, ev, cpu_events)
            rows.append(r)
        w.close()
    if only:  # (tools/pmc_configs.py: one config's batches under rocprofv3)
        return rows
    if c4 is not None:
        rows.append(dropin_line(dev, *c4, cpu=bool(cpu_events)))
        rows.append(latency_line(dev, *c4, cpu=bool(cpu_events)))
    rows.append(token_line(dev))
    return rows


def latency_line(dev, w, ev, sizes=(1, 64, 256, 1024), calls=2000, warm=200, cpu=False):
    """The drop-in under light load: every SphU.entry is synchronous (core/CtSph.java:117-168), so a
    lightly loaded service pays one engine call per few events.  Synchronous sg_submit_ex of 1, 64, 256 and 1,024 events
    of the C4 trace from pageable host memory (contexts and origins on every event, as the Java batcher sends them):
    p50 / p99 / mean host wall time per call.  Up to 256 events a call is one k_tiny launch (engine.cpp tiny_impl)."""
    import torch
    from sentinel_amd import engine as E
    from sentinel_amd import tracegen as T
    eng = E.Engine(device=dev.index, max_resources=1 << 20, max_slot_chain_size=0, param_table_log2=16,
                   status_ring_log2=28, max_batch_events=max(sizes), aux_node_capacity=1 << 22)
    w.install(eng)
    io, ic = w.intern_names(eng)
    out = {}
    off = 0
    total = sum(n * (calls + warm) for n in sizes)  # one prefix of the trace, in order (the engine's event indices)
    prefix = np.ascontiguousarray(ev[:total])
    ext_all = T.ext_for(prefix, io, ic, seed=T.SEED_BASE + 47)
    got = np.zeros(total, np.uint32)
    for n in sizes:
        need = n * (calls + warm)
        sub = prefix[off:off + need]
        ext = ext_all[off:off + need]
        lat = []
        for b in range(calls + warm):
            e, x = sub[b * n:(b + 1) * n], ext[b * n:(b + 1) * n]
            t = time.perf_counter()
            d = eng.submit_ex(e, x)
            dt = time.perf_counter() - t
            got[off + b * n:off + (b + 1) * n] = d
            if b >= warm:
                lat.append(dt)
        lat = np.array(lat) * 1e3
        out[str(n)] = {"p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99)),
                       "mean_ms": float(lat.mean()), "calls": calls}
        off += need
    eng.close()
    torch.cuda.empty_cache()
    r = {"config": "drop-in latency floor: synchronous sg_submit_ex of %s C4 events from pageable host memory, "
                   "contexts + origins" % " / ".join(str(n) for n in sizes), "unit": "ms per call", "latency": out,
         "note": "<= 256 events: the events in, one k_tiny launch (every stage in one workgroup), the decisions back; "
                 "larger: the group stage, one host round trip for the bins, the decide stage, the decisions back"}
    if cpu:  # the same calls through the oracle, one thread (ctypes call overhead included)
        orc = _oracle_for(w, prefix)
        cl, off, want = {}, 0, np.zeros(total, np.uint32)
        for n in sizes:
            lat = []
            for b in range(calls + warm):
                a = off + b * n
                t = time.perf_counter()
                want[a:a + n] = orc.submit_ex(prefix[a:a + n], ext_all[a:a + n])
                dt = time.perf_counter() - t
                if b >= warm:
                    lat.append(dt)
            lat = np.array(lat) * 1e3
            cl[str(n)] = {"p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99))}
            off += n * (calls + warm)
        orc.close()
        r["cpu_baseline"] = {"latency": cl, "unit": "ms per call", "cores": 1, "kind": "port",
                             "sample": "the same %d calls, oracle/liboracle.so or_submit_ex, one thread" % (
                                 len(sizes) * (calls + warm)),
                             "gpu_results_equal": bool(np.array_equal(got, want))}
    return r


def token_line(dev, n_flows=10_000, n_req=16_000_000, batch=1 << 21, seconds=60, cpu_requests=2_000_000):
    """C5's cluster half: the token server over 10k GLOBAL flowIds (thresholds 10^3..10^5 per
    window, 1-10 samples of 0.5-2 s), Zipf(1.1) requests in time order, requests and results in HBM
    (sg_cluster_request_tokens with device buffers, as dist.request_tokens_tensor calls it); first batch untimed.
    cpu_baseline: the oracle (ClusterFlowChecker restated in C, one thread: the token server is one sequential
    state machine per namespace) on the first cpu_requests requests, which the GPU result is checked against."""
    import torch
    from sentinel_amd import _abi as A
    from sentinel_amd import engine as E
    rng = np.random.default_rng(20240601 + 15)
    fids = np.arange(1_000_001, 1_000_001 + n_flows)
    eng = E.Engine(device=dev.index, max_resources=max(1 << 14, n_flows + 16), cluster_max_allowed_qps=10 ** 9)
    eng.register_many(["r%d" % f for f in fids])
    rules = [A.flow_rule("r%d" % f, float(int(np.exp(rng.uniform(np.log(1e3), np.log(1e5))))), cluster_mode=True,
                         cluster_flow_id=int(f), cluster_threshold_type=A.CLUSTER_THRESHOLD_GLOBAL,
                         cluster_sample_count=int(rng.choice([1, 2, 5, 10])),
                         cluster_window_interval_ms=int(rng.choice([500, 1000, 2000]))) for f in fids]
    eng.load_flow_rules(rules)
    orc = None
    if cpu_requests:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as O
        orc = O.Oracle(cluster_max_allowed_qps=10 ** 9)
        for f in fids:
            orc.register("r%d" % f)
        orc.load_flow_rules(rules)
    p = 1.0 / np.arange(1, n_flows + 1) ** 1.1
    p /= p.sum()
    reqs = np.zeros(n_req, dtype=A.TOKEN_REQ_DTYPE)
    reqs["ts"] = 1_700_000_000_000 + np.sort(rng.integers(0, seconds * 1000, n_req))
    reqs["flow_id"] = fids[rng.choice(n_flows, n_req, p=p)]
    reqs["acquire_count"] = rng.integers(1, 4, n_req)
    reqs["prioritized"] = rng.random(n_req) < 0.2
    rq, rs = A.TOKEN_REQ_DTYPE.itemsize, A.TOKEN_RES_DTYPE.itemsize
    dq = torch.from_numpy(reqs.view(np.uint8)).to(dev)
    dr = torch.empty(n_req * rs, dtype=torch.uint8, device=dev)
    cuts = list(range(0, n_req, batch)) + [n_req]
    eng.cluster_request_ptr(dq.data_ptr(), cuts[1], dr.data_ptr())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, b in zip(cuts[1:-1], cuts[2:]):
        eng.cluster_request_ptr(dq.data_ptr() + a * rq, b - a, dr.data_ptr() + a * rs)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = dr.view(torch.int32).view(-1, 4).cpu().numpy()
    st = res[:, 0]
    n_t = n_req - cuts[1]
    eng.close()
    del dq, dr
    torch.cuda.empty_cache()
    cpu = None
    if orc is not None:
        m = min(cpu_requests, n_req)
        t1 = time.perf_counter()
        want = orc.cluster_request_array(reqs[:m])
        dt1 = time.perf_counter() - t1
        got = res[:m].copy().view(A.TOKEN_RES_DTYPE).reshape(-1)
        same = bool(np.array_equal(np.asarray(want).view(np.uint8), got.view(np.uint8)))
        cpu = {"value": m / dt1, "unit": "token requests/s", "cores": 1, "kind": "port",
               "sample": "first %d requests of the same stream, oracle/liboracle.so (ClusterFlowChecker / "
                         "GlobalRequestLimiter restated), one thread" % m, "gpu_results_equal": same}
        orc.close()
    return {"config": "C5 cluster half: token server, %d GLOBAL flowIds (counts 1e3-1e5), Zipf(1.1) requests over %d s, "
                      "buffers in HBM, %d-request calls" % (n_flows, seconds, batch),
            "value": n_t / dt, "unit": "token requests/s", "requests_timed": n_t, "ms_per_call": dt / (len(cuts) - 2) * 1e3,
            "status_counts": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
            "cpu_baseline": cpu}


def dropin_line(dev, w, ev, batch=1 << 16, n_batches=400, cpu=False, cpu_batches=20):
    """The Java batcher's operating point (java/.../GpuEngine.java): batches of <= 65,536 events
    from pageable host memory, sg_submit_ex synchronous (one batch decided and back before the next), contexts and
    origins on every event.  Entries/s and the per-batch latency distribution (host wall clock around each call)."""
    import torch
    from sentinel_amd import engine as E
    from sentinel_amd import tracegen as T
    eng = E.Engine(device=dev.index, max_resources=1 << 20, max_slot_chain_size=0, param_table_log2=16,
                   status_ring_log2=28, max_batch_events=batch, aux_node_capacity=1 << 22)
    w.install(eng)
    io, ic = w.intern_names(eng)
    sub = np.ascontiguousarray(ev[:batch * (n_batches + 20)])
    ext = T.ext_for(sub, io, ic, seed=T.SEED_BASE + 46)
    lat = []
    ent = 0
    nc = 20 + cpu_batches
    got = []
    for b in range(n_batches + 20):
        e = sub[b * batch:(b + 1) * batch]
        t = time.perf_counter()
        d = eng.submit_ex(e, ext[b * batch:(b + 1) * batch])
        dt = time.perf_counter() - t
        if b < nc:
            got.append(d)
        if b >= 20:  # warm-up batches untimed
            lat.append(dt)
            ent += int((e["kind"] == 0).sum())
    lat = np.array(lat)
    eng.close()
    torch.cuda.empty_cache()
    r = {"config": "drop-in operating point: C4 trace, %d-event batches from pageable host memory, sg_submit_ex "
                   "synchronous" % batch, "value": ent / lat.sum(), "unit": "entries/s", "batches_timed": n_batches,
         "batch_events": batch, "latency_ms": {"p50": float(np.percentile(lat, 50) * 1e3),
                                               "p99": float(np.percentile(lat, 99) * 1e3),
                                               "mean": float(lat.mean() * 1e3)},
         "note": EXT_NOTE + "; PCIe copies of events, ext and decisions inside every call"}
    if cpu:  # the oracle, one thread, on the same first batches (the last cpu_batches of them timed)
        orc = _oracle_for(w, sub[:nc * batch])
        spent, cent, want = 0.0, 0, []
        for b in range(nc):
            e = sub[b * batch:(b + 1) * batch]
            t = time.perf_counter()
            want.append(orc.submit_ex(e, ext[b * batch:(b + 1) * batch]))
            if b >= 20:
                spent += time.perf_counter() - t
                cent += int((e["kind"] == 0).sum())
        orc.close()
        r["cpu_baseline"] = {"value": cent / spent, "unit": "entries/s", "cores": 1, "kind": "port",
                             "sample": "batches 20-%d of the same calls, oracle/liboracle.so or_submit_ex, one thread"
                                       % (nc - 1),
                             "gpu_results_equal": bool(np.array_equal(np.concatenate(got), np.concatenate(want)))}
    return r


def cpu_share() -> int:
    """This job's CPUs: the cgroup v2 cpu.max quota (the GPU box gives a one-GPU job 16 of its host's
    cores), else min(16, the affinity set)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            return max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return min(16, len(os.sched_getaffinity(0)))


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(w, ev, args):
    """The oracle (C restatement of the Java path) on bounded prefixes of the same trace: T threads
    partitioned by resource (SURVEY.md §8(d) CPU fallback), plus one thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    avail = len(os.sched_getaffinity(0))
    T = args.cpu_threads or cpu_share()
    sample = ev[:args.cpu_sample_events]
    po = O.PartitionedOracle(w, T, max_slot_chain_size=0)
    spent = []
    po.submit(sample, timed=spent)
    po.close()
    n_ent = int((sample["kind"] == 0).sum())
    one = O.Oracle(max_slot_chain_size=0)
    w.install(one)
    s1 = ev[:args.cpu_single_events]
    t = time.perf_counter()
    one.submit(s1)
    dt1 = time.perf_counter() - t
    n1 = int((s1["kind"] == 0).sum())
    return {"value": n_ent / spent[0], "unit": "entries/s", "cores": T, "kind": "port",
            "sample": "first %d events (%d entries) of the C4 trace, oracle/liboracle.so, %d threads partitioned "
                      "by splitmix64(res_id) %% %d (routing excluded)" % (len(sample), n_ent, T, T),
            "single_thread": {"value": n1 / dt1, "cores": 1, "sample": "first %d events (%d entries)" % (len(s1), n1)},
            "full_width": {"value": n_ent / spent[0] * (os.cpu_count() or T) / T, "cores": os.cpu_count(),
                           "note": "the measured %d-thread rate scaled linearly to nproc: this job may use %d of "
                                   "the host's %d CPUs (the box's CPU share), so nproc threads are not run" %
                                   (T, T, os.cpu_count() or T)},
            "cpu_model": cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": avail}


if __name__ == "__main__":
    main()
