"""Multi-GPU plumbing around the decision path.

One process and one engine per GPU (torch.distributed: "nccl" is RCCL over xGMI here, "gloo" on
CPU).  Every decision reads and writes only its own resource's state, so resources shard by
``splitmix64(res_id) % world`` and the decision path has no collective at all.  Two exchanges
remain, and they live here:

* ``gather_metrics``: once per second every rank's ``sg_snapshot_metrics`` output is all-gathered
  (the MetricTimerListener role, core/node/metric/MetricTimerListener.java:39-56, over the whole
  node).  Resource ids are local to a rank's engine, so each row carries its rank in ``reserved``.
* ``request_tokens``: token requests go to the token-server rank.  The namespace's
  GlobalRequestLimiter (csrv/flow/statistic/limit/GlobalRequestLimiter.java:46-54) is shared by all
  flowIds of the namespace, so the exact server is one engine: every rank's requests are gathered
  there, decided in one merged time order (ts, rank, local order), and the results broadcast back.
  The server's request rate is bounded by that same limiter, so one GPU is plenty.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import _abi as A

def splitmix64(x) -> np.ndarray:
    """splitmix64 finaliser of x (uint64 arithmetic, wrapping)."""
    z = np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def shard_of(res_ids, world: int) -> np.ndarray:
    """Owning rank of each resource: splitmix64(res_id) % world."""
    return (splitmix64(res_ids) % np.uint64(world)).astype(np.int64)


def route_events(events: np.ndarray, world: int):
    """Split a time-ordered sg_event batch into the per-rank batches (stable: each rank's events
    keep their order, so each shard sees a time-ordered batch).  Returns (batches, positions) where
    positions[r] are the indices of rank r's events in the input (to put decisions back)."""
    owner = shard_of(events["res_id"], world)
    order = np.argsort(owner, kind="stable")
    cuts = np.searchsorted(owner[order], np.arange(world + 1))
    pos = [order[cuts[r]:cuts[r + 1]] for r in range(world)]
    return [events[p] for p in pos], pos


def _device(group=None):
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")


def _all_gather_rows(rows: np.ndarray, group=None):
    """All-gather a 1-D structured array of any length per rank; returns the list of per-rank arrays."""
    world = dist.get_world_size(group)
    dev = _device(group)
    dt = rows.dtype
    n = torch.tensor([len(rows)], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    width = max(ns) * dt.itemsize
    if width == 0:
        return [np.zeros(0, dtype=dt) for _ in range(world)]
    buf = np.zeros(width, dtype=np.uint8)
    raw = np.ascontiguousarray(rows).view(np.uint8)
    buf[: len(raw)] = raw
    mine = torch.from_numpy(buf).to(dev)
    outs = [torch.empty(width, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(outs, mine, group=group)
    return [outs[r].cpu().numpy()[: ns[r] * dt.itemsize].view(dt).copy() for r in range(world)]


def gather_metrics(snapshot: np.ndarray, group=None) -> np.ndarray:
    """All-gather of this second's MetricNode rows of every rank (A.METRIC_NODE_DTYPE; ``reserved``
    is overwritten with the source rank).  Rows are ordered by (timestamp, rank, res_id)."""
    rows = np.ascontiguousarray(snapshot, dtype=A.METRIC_NODE_DTYPE).copy()
    rows["reserved"] = dist.get_rank(group)
    allr = np.concatenate(_all_gather_rows(rows, group))
    return allr[np.lexsort((allr["res_id"], allr["reserved"], allr["timestamp"]))]


def request_tokens(reqs: np.ndarray, decide=None, server: int = 0, group=None) -> np.ndarray:
    """Token requests of this rank (A.TOKEN_REQ_DTYPE, time-ordered) -> results (A.TOKEN_RES_DTYPE).

    ``decide`` is the server rank's batched TokenService (``Engine.cluster_request_array``); other
    ranks pass None.  Collective: every rank must call it, with its own (possibly empty) batch."""
    rank = dist.get_rank(group)
    reqs = np.ascontiguousarray(reqs, dtype=A.TOKEN_REQ_DTYPE)
    parts = _all_gather_rows(reqs, group)
    sizes = [len(p) for p in parts]
    total = sum(sizes)
    res = np.zeros(total, dtype=A.TOKEN_RES_DTYPE)
    if rank == server and total:
        if decide is None:
            raise ValueError("the token-server rank needs a decide function")
        allq = np.concatenate(parts)
        src = np.concatenate([np.full(s, r, dtype=np.int64) for r, s in enumerate(sizes)])
        loc = np.concatenate([np.arange(s, dtype=np.int64) for s in sizes])
        order = np.lexsort((loc, src, allq["ts"]))  # one time order for the whole namespace
        out = decide(allq[order])
        res[order] = out
    if total == 0:
        return res
    dev = _device(group)
    t = torch.from_numpy(res.view(np.uint8).copy()).to(dev)
    dist.broadcast(t, src=server, group=group)
    res = t.cpu().numpy().view(A.TOKEN_RES_DTYPE)
    off = sum(sizes[:rank])
    return res[off: off + sizes[rank]].copy()
