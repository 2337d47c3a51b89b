"""Multi-GPU plumbing around the decision path.

One process and one engine per GPU (torch.distributed: "nccl" is RCCL over xGMI here, "gloo" on
CPU).  Every decision reads and writes only its own resource's state, so resources shard by
``splitmix64(res_id) % world`` and the decision path has no collective at all.  Under Zipf popularity a
hash leaves the hottest resource's GPU with its share plus 1/world of the rest (C4 at 8 GPUs: 23 % of the
events on one GPU, a 4.3x ceiling), so a ``ShardMap`` may instead place resources by their observed event
counts (largest first onto the least loaded GPU; unseen resources by the hash): still a fixed partition of
resources, still no data-path traffic.  Two exchanges remain, and they live here:

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


def shard_of(res_ids, world: int, table=None) -> np.ndarray:
    """Owning rank of each resource: table[res_id] where a ShardMap table gives one (>= 0), else
    splitmix64(res_id) % world."""
    h = (splitmix64(res_ids) % np.uint64(world)).astype(np.int64)
    if table is None or len(table) == 0:  # an empty table places nothing: every resource by the hash
        return h
    r = np.asarray(res_ids, dtype=np.int64)
    t = np.where(r < len(table), table[np.minimum(r, len(table) - 1)], -1)
    return np.where(t >= 0, t, h)


def balanced_table(counts, world: int, alpha: float = 1.0) -> np.ndarray:
    """A resource -> rank table from per-resource event counts: largest first onto the least loaded rank
    (longest-processing-time greedy) with a resource's load counts**alpha (alpha < 1: a long segment costs less per
    event -- its owner skips the frozen rest of each round); resources with no events stay on their hash rank (-1)."""
    counts = np.asarray(counts, dtype=np.int64)
    table = np.full(len(counts), -1, dtype=np.int64)
    load = np.zeros(world, dtype=np.float64)
    seen = np.nonzero(counts)[0]
    cost = counts.astype(np.float64) ** alpha
    for r in seen[np.argsort(-counts[seen], kind="stable")]:
        k = int(np.argmin(load))
        table[r] = k
        load[k] += cost[r]
    return table


_REF = np.uint64(A.REF_NONE)


class EventRouter:
    """Routes one submitting stream of sg_event batches to ``world`` engines, batch by batch.

    Each rank's batch keeps the input order (a time-ordered stream stays time-ordered per shard).
    An EXIT/TRACE names its ENTRY by the ENTRY's global index in the stream the engine receives
    (include/sentinel_gpu.h, low 48 bits of ``aux``), so every reference is rewritten from the
    submitting stream's numbering to the ENTRY's index in its rank's stream.  An ENTRY and its
    EXIT/TRACE share the resource, hence the rank.  The index map is a ring of 2^ring_log2 events:
    a reference older than that (or to a later event) cannot be mapped and is rewritten to point at
    the referencing event itself, which the engine rejects as a bad reference (SG_EINVAL).
    """

    def __init__(self, world: int, ring_log2: int = 24, table=None):
        self.world = world
        self.table = table
        self.mask = (1 << ring_log2) - 1
        self.local = np.zeros(1 << ring_log2, dtype=np.int64)  # submitting index -> rank-local index
        self.owner = np.zeros(1 << ring_log2, dtype=np.int64)  # submitting index -> its rank
        self.gin = 0                                  # submitting index of the next input event
        self.gout = np.zeros(world, dtype=np.int64)   # rank-local index of each rank's next event

    def _grow(self):
        old, size = self.local, self.mask + 1
        idx = np.arange(max(0, self.gin - size), self.gin, dtype=np.int64)  # the history the ring holds
        self.mask = 2 * size - 1
        self.local = np.zeros(2 * size, dtype=np.int64)
        self.local[idx & self.mask] = old[idx & (size - 1)]
        oown = self.owner
        self.owner = np.zeros(2 * size, dtype=np.int64)
        self.owner[idx & self.mask] = oown[idx & (size - 1)]

    def route(self, events: np.ndarray):
        """Returns (batches, positions): positions[r] are the indices of rank r's events in the
        input batch (to put decisions back in submission order)."""
        n = len(events)
        while n > (self.mask + 1) // 2:  # keep room for the batch plus as much history again
            self._grow()
        owner = shard_of(events["res_id"], self.world, self.table)
        order = np.argsort(owner, kind="stable")
        cuts = np.searchsorted(owner[order], np.arange(self.world + 1))
        pos = [order[cuts[r]:cuts[r + 1]] for r in range(self.world)]
        gidx = self.gin + np.arange(n, dtype=np.int64)
        loc = np.empty(n, dtype=np.int64)
        for r, p in enumerate(pos):
            loc[p] = self.gout[r] + np.arange(len(p), dtype=np.int64)
            self.gout[r] += len(p)
        self.local[gidx & self.mask] = loc
        self.owner[gidx & self.mask] = owner
        aux = events["aux"].astype(np.uint64)
        isref = (events["kind"] != A.EV_ENTRY) & ((aux & _REF) != _REF)
        ref = (aux & _REF).astype(np.int64)
        ok = isref & (ref < gidx) & (ref >= self.gin + n - 1 - self.mask)  # ring slot not reused yet
        # a reference to an event another rank holds (another resource's ENTRY) cannot be mapped: it would alias
        # an unrelated event of this rank's numbering, so it becomes a self-reference the engine rejects
        ok &= self.owner[ref & self.mask] == owner
        bad = isref & ~ok
        new = np.where(ok, self.local[ref & self.mask], loc)
        aux2 = np.where(isref, (aux & ~_REF) | (new.astype(np.uint64) & _REF), aux)
        if bad.any():  # self-reference: rejected by the engine (an EXIT/TRACE must follow its ENTRY)
            aux2 = np.where(bad, (aux & ~_REF) | (loc.astype(np.uint64) & _REF), aux2)
        self.gin += n
        out = []
        for p in pos:
            b = events[p].copy()
            b["aux"] = aux2[p]
            out.append(b)
        return out, pos


def shard_stream(events: np.ndarray, world: int, rank: int, table=None):
    """Rank ``rank``'s share of a whole sg_event stream that starts at global index 0 (what one
    process of a multi-GPU run keeps of a trace every rank generates alike): its events in order,
    with EXIT/TRACE references rewritten to the rank's numbering, and their positions in the
    input.  O(n + m log m) for m events of the rank, no sort of the whole stream."""
    pos = np.nonzero(shard_of(events["res_id"], world, table) == rank)[0]
    mine = events[pos].copy()
    aux = mine["aux"].astype(np.uint64)
    isref = (mine["kind"] != A.EV_ENTRY) & ((aux & _REF) != _REF)
    ref = (aux & _REF).astype(np.int64)
    k = np.searchsorted(pos, ref)
    kk = np.minimum(k, len(pos) - 1) if len(pos) else k
    ok = isref & (k < len(pos)) & (pos[kk] == ref) & (ref < pos) if len(pos) else isref
    own = np.arange(len(pos), dtype=np.int64)
    new = np.where(ok, k, own)  # an unmappable reference names the event itself: rejected as bad
    mine["aux"] = np.where(isref, (aux & ~_REF) | (new.astype(np.uint64) & _REF), aux)
    return mine, pos


def route_events(events: np.ndarray, world: int, table=None):
    """Split a time-ordered sg_event stream that starts at global index 0 into the per-rank
    streams, with EXIT/TRACE references rewritten to each rank's numbering (see EventRouter).
    Returns (batches, positions)."""
    ring = 1
    while ring < max(2, len(events)):
        ring <<= 1
    return EventRouter(world, ring_log2=ring.bit_length() - 1, table=table).route(events)


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


def request_tokens_tensor(reqs: "torch.Tensor", decide_ptr=None, server: int = 0, group=None) -> "torch.Tensor":
    """Device-resident token requests: ``reqs`` = this rank's A.TOKEN_REQ_DTYPE rows (time-ordered) as a uint8
    tensor on the group's device (HBM under RCCL), returns its A.TOKEN_RES_DTYPE rows as a uint8 tensor there.
    Nothing goes through host memory: the rows are all-gathered, the server rank orders the whole namespace by time
    (a stable sort on ts of the rank-ordered concatenation = (ts, rank, index) order), decides them in one call of
    ``decide_ptr(req_ptr, n, out_ptr)`` (``Engine.cluster_request_ptr``: sg_cluster_request_tokens takes device
    buffers) and broadcasts the results.  Collective, like request_tokens."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    rq, rs = A.TOKEN_REQ_DTYPE.itemsize, A.TOKEN_RES_DTYPE.itemsize
    dev = reqs.device
    n = reqs.numel() // rq
    cnt = torch.tensor([n], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    ns = [int(c.item()) for c in cnts]
    total = sum(ns)
    if total == 0:
        return torch.zeros(0, dtype=torch.uint8, device=dev)
    width = max(ns) * rq
    mine = torch.zeros(width, dtype=torch.uint8, device=dev)
    mine[: n * rq] = reqs.reshape(-1)
    outs = [torch.empty(width, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(outs, mine, group=group)
    res = torch.zeros(total * rs, dtype=torch.uint8, device=dev)
    if rank == server:
        if decide_ptr is None:
            raise ValueError("the token-server rank needs a decide function")
        allq = torch.cat([outs[r][: ns[r] * rq] for r in range(world)]).view(total, rq)
        ts = allq[:, :8].contiguous().view(torch.int64).view(-1)
        order = torch.sort(ts, stable=True).indices
        q = allq.index_select(0, order).contiguous()
        out = torch.empty((total, rs), dtype=torch.uint8, device=dev)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)  # (the engine's own stream reads q)
        decide_ptr(q.data_ptr(), total, out.data_ptr())
        res.view(total, rs).index_copy_(0, order, out)
    dist.broadcast(res, src=server, group=group)
    off = sum(ns[:rank])
    return res[off * rs: (off + n) * rs]


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
