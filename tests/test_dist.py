"""Multi-process paths of sentinel_amd.dist on gloo, world size 2.

CPU: resource sharding, the MetricNode all-gather and token routing to the server rank, with the
oracle deciding at the server.  GPU (-m gpu): the same routing with the HIP token server on cuda:0
behind rank 0 (rank 1 stays on the CPU), so the device path is what the ranks exchange with.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T0 = 1_700_000_000_000


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    for p in (ROOT, os.path.join(ROOT, "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    return dist


def _cluster_rules(A, fids):
    return [A.flow_rule("r%d" % f, float(5 + (f * 37) % 30), cluster_mode=True, cluster_flow_id=f,
                        cluster_threshold_type=A.CLUSTER_THRESHOLD_GLOBAL, cluster_sample_count=5)
            for f in fids]


PLAN = [[300, 250], [0, 120]]  # PLAN[round][rank]: batch sizes (an empty batch on rank 0 in round 1)


def _batch(A, rank, rnd):
    n = PLAN[rnd][rank]
    rng = np.random.default_rng(1000 * rnd + 7 + rank)
    out = np.zeros(n, dtype=A.TOKEN_REQ_DTYPE)
    out["ts"] = T0 + 10_000 * rnd + np.cumsum(rng.integers(0, 12, n))  # > 1 s: the window head fills
    out["flow_id"] = rng.integers(11, 19, n)
    out["acquire_count"] = 1  # PASS tokens == PASS_REQUEST: the occupy path (SHOULD_WAIT) is reachable
    out["prioritized"] = rng.random(n) < 0.25
    return out


def _oracle_decider(O, A, fids, **cfg):
    o = O.Oracle(**cfg)
    o.load_flow_rules(_cluster_rules(A, fids))

    def decide(q):
        r = o.cluster_request([tuple(int(v) for v in x) for x in q])
        out = np.zeros(len(q), dtype=A.TOKEN_RES_DTYPE)
        for i, (s, rem, w) in enumerate(r):
            out[i] = (s, rem, w, 0)
        return out
    return decide


def _w_tokens(rank, world, port, use_gpu):
    dist = _init(rank, world, port)
    import pyoracle as O
    from sentinel_amd import _abi as A
    from sentinel_amd import dist as D
    fids = list(range(11, 19))
    decide = None
    if rank == 0:
        if use_gpu:
            from sentinel_amd import engine as E
            eng = E.Engine(max_resources=64, cluster_max_allowed_qps=250)
            eng.load_flow_rules(_cluster_rules(A, fids))
            decide = eng.cluster_request_array
        else:
            decide = _oracle_decider(O, A, fids, cluster_max_allowed_qps=250)
    ref = _oracle_decider(O, A, fids, cluster_max_allowed_qps=250)  # one server on the merged stream
    seen = {s: 0 for s in (A.TOKEN_OK, A.TOKEN_BLOCKED, A.TOKEN_SHOULD_WAIT, A.TOKEN_TOO_MANY_REQUEST)}
    for rnd in range(len(PLAN)):
        got = D.request_tokens(_batch(A, rank, rnd), decide)
        allq = [_batch(A, r, rnd) for r in range(world)]
        cat = np.concatenate(allq)
        src = np.concatenate([np.full(len(q), r) for r, q in enumerate(allq)])
        loc = np.concatenate([np.arange(len(q)) for q in allq])
        order = np.lexsort((loc, src, cat["ts"]))
        res = np.zeros(len(cat), dtype=A.TOKEN_RES_DTYPE)
        res[order] = ref(cat[order])
        off = sum(len(q) for q in allq[:rank])
        assert np.array_equal(got, res[off: off + len(got)]), (rank, rnd)
        for s in res["status"]:
            seen[int(s)] = seen.get(int(s), 0) + 1
    assert all(v > 0 for v in seen.values()), seen  # every outcome is exercised by the merged stream
    dist.barrier()
    dist.destroy_process_group()


def _w_tokens_tensor(rank, world, port, backend):
    # request_tokens_tensor: the requests and results stay tensors on the group's device (HBM under RCCL), the
    # server decides through a pointer call (the engine's device buffers, or the oracle's host ones under gloo)
    import torch
    import torch.distributed as dist
    for p in (ROOT, os.path.join(ROOT, "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend, init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    import pyoracle as O
    from sentinel_amd import _abi as A
    from sentinel_amd import dist as D
    fids = list(range(11, 19))
    dev = torch.device("cuda", 0) if backend == "nccl" else torch.device("cpu")
    decide = None
    if rank == 0:
        if backend == "nccl":
            from sentinel_amd import engine as E
            eng = E.Engine(max_resources=64, cluster_max_allowed_qps=250)
            eng.load_flow_rules(_cluster_rules(A, fids))
            decide = eng.cluster_request_ptr
        else:
            o = O.Oracle(cluster_max_allowed_qps=250)
            o.load_flow_rules(_cluster_rules(A, fids))
            decide = o.cluster_request_ptr
    ref = _oracle_decider(O, A, fids, cluster_max_allowed_qps=250)
    for rnd in range(len(PLAN)):
        mine = _batch(A, rank, rnd)
        t = torch.from_numpy(mine.view(np.uint8).copy()).to(dev)
        got = D.request_tokens_tensor(t, decide)
        assert got.device.type == dev.type
        got = got.cpu().numpy().view(A.TOKEN_RES_DTYPE)
        allq = [_batch(A, r, rnd) for r in range(world)]
        cat = np.concatenate(allq)
        src = np.concatenate([np.full(len(q), r) for r, q in enumerate(allq)])
        loc = np.concatenate([np.arange(len(q)) for q in allq])
        order = np.lexsort((loc, src, cat["ts"]))
        res = np.zeros(len(cat), dtype=A.TOKEN_RES_DTYPE)
        res[order] = ref(cat[order])
        off = sum(len(q) for q in allq[:rank])
        assert np.array_equal(got, res[off: off + len(mine)]), (rank, rnd)
    dist.barrier()
    dist.destroy_process_group()


def _w_metrics(rank, world, port):
    dist = _init(rank, world, port)
    from sentinel_amd import _abi as A
    from sentinel_amd import dist as D
    n = [3, 0][rank]
    rows = np.zeros(n, dtype=A.METRIC_NODE_DTYPE)
    rows["timestamp"] = T0 + 1000 * np.arange(n)
    rows["res_id"] = 10 + np.arange(n)
    rows["pass_qps"] = 100 + rank
    g = D.gather_metrics(rows)
    assert len(g) == 3 and (g["reserved"] == 0).all()
    rows2 = np.zeros(2 + rank, dtype=A.METRIC_NODE_DTYPE)
    rows2["timestamp"] = T0
    rows2["res_id"] = np.arange(2 + rank)[::-1]
    rows2["pass_qps"] = rank
    g = D.gather_metrics(rows2)
    assert len(g) == 5
    assert list(g["reserved"]) == [0, 0, 1, 1, 1] and list(g["res_id"]) == [0, 1, 0, 1, 2]
    assert list(g["pass_qps"]) == [0, 0, 1, 1, 1]
    dist.barrier()
    dist.destroy_process_group()


def _w_routed_decisions(rank, world, port, balanced=False):
    """Each rank decides its splitmix64 shard of one C4 stream (ENTRY/EXIT/TRACE, three batches) with its
    own engine; the merged decisions and the owned resources' node states equal one engine's run over the
    whole stream.  The oracle is the engine here (CPU), so this checks the routing: shards, order and the
    rewriting of EXIT/TRACE references to each rank's numbering."""
    dist = _init(rank, world, port)
    import pyoracle as O
    from sentinel_amd import _abi as A
    from sentinel_amd import dist as D
    from sentinel_amd import tracegen as T
    w = T.Workload(4, n_entries=40_000, n_res=300)
    ev = w.events
    mine = O.Oracle(max_slot_chain_size=0)
    w.install(mine)
    table = D.balanced_table(np.bincount(ev["res_id"], minlength=w.n_res), world) if balanced else None
    router = D.EventRouter(world, ring_log2=18, table=table)
    cuts = np.linspace(0, len(ev), 4).astype(np.int64)
    dec = np.zeros(len(ev), dtype=np.uint32)
    for a, b in zip(cuts[:-1], cuts[1:]):
        parts, pos = router.route(np.ascontiguousarray(ev[a:b]))
        rows = np.zeros(len(pos[rank]), dtype=[("i", "<i8"), ("d", "<u4"), ("pad", "<u4")])
        rows["i"] = a + pos[rank]
        rows["d"] = mine.submit(parts[rank])
        for got in D._all_gather_rows(rows):
            dec[got["i"]] = got["d"]
    whole = O.Oracle(max_slot_chain_size=0)
    w.install(whole)
    ref = whole.submit(ev)
    assert np.array_equal(dec, ref), (rank, int(np.nonzero(dec != ref)[0][0]))
    owned = np.nonzero(D.shard_of(np.arange(w.n_res), world, table) == rank)[0]
    for r in owned[:60]:
        g, o = mine.read_node(int(r)), whole.read_node(int(r))
        assert g["thread"] == o["thread"] and np.array_equal(g["minute"], o["minute"]), r
    st = ref[ev["kind"] == A.EV_ENTRY] & 0xFF
    assert (st == A.BLOCK_FLOW).sum() > 0 and (st == A.BLOCK_DEGRADE).sum() > 0
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("balanced", [False, True])
def test_routed_decisions_equal_single_engine_gloo(balanced):
    mp.spawn(_w_routed_decisions, args=(2, _port(), balanced), nprocs=2, join=True)


def test_balanced_table_and_cross_rank_references():
    from sentinel_amd import _abi as A
    from sentinel_amd import dist as D
    from sentinel_amd import tracegen as T
    # C4 popularity: the hottest resource holds ~12 % of the events; by hash its GPU also gets 1/8 of the rest
    w = T.Workload(4, n_entries=300_000, n_res=100_000)
    cnt = np.bincount(w.events["res_id"], minlength=w.n_res)
    table = D.balanced_table(cnt, 8)
    share = lambda own: np.bincount(own, weights=cnt, minlength=8) / cnt.sum()
    hashed = share(D.shard_of(np.arange(w.n_res), 8))
    bal = share(D.shard_of(np.arange(w.n_res), 8, table))
    assert bal.max() < hashed.max() and bal.max() <= max(cnt.max() / cnt.sum(), 1 / 8) * 1.02, (bal, hashed)
    assert (table[cnt == 0] == -1).all()  # unseen resources keep their hash rank
    # an EXIT naming another resource's ENTRY held by another rank becomes a self-reference (rejected)
    ev = np.zeros(3, dtype=A.EVENT_DTYPE)
    ev["ts"] = T0 + np.arange(3)
    tab = np.array([0, 1], dtype=np.int64)  # resource 0 on rank 0, resource 1 on rank 1
    ev["res_id"] = [0, 1, 1]
    ev["kind"] = [A.EV_ENTRY, A.EV_ENTRY, A.EV_EXIT]
    ev["aux"] = [0, 0, A.aux_exit(0, 5)]  # rank 1's EXIT names rank 0's ENTRY
    parts, pos = D.EventRouter(2, ring_log2=4, table=tab).route(ev)
    assert list(pos[1]) == [1, 2] and int(parts[1]["aux"][1]) & A.REF_NONE == 1  # its own local index


def test_router_rewrites_references():
    from sentinel_amd import _abi as A
    from sentinel_amd import dist as D
    ev = np.zeros(6, dtype=A.EVENT_DTYPE)
    ev["ts"] = T0 + np.arange(6)
    ev["res_id"] = [1, 2, 1, 2, 1, 1]
    ev["kind"] = [A.EV_ENTRY, A.EV_ENTRY, A.EV_EXIT, A.EV_EXIT, A.EV_TRACE, A.EV_EXIT]
    ev["aux"] = [0, 0, A.aux_exit(0, 7), A.aux_exit(1, 3), 0, A.aux_exit(A.REF_NONE, 2)]
    router = D.EventRouter(2, ring_log2=4)
    parts, pos = router.route(ev)
    o1, o2 = int(D.shard_of(1, 2)), int(D.shard_of(2, 2))
    REF = np.uint64(A.REF_NONE)
    if o1 != o2:
        p1 = parts[o1]
        assert list(p1["aux"] & REF) == [0, 0, 0, A.REF_NONE]  # the EXIT and TRACE name local index 0
        assert int(p1["aux"][1]) >> 48 == 7 and int(p1["aux"][3]) >> 48 == 2  # RT bits kept
        assert list(parts[o2]["aux"] & REF) == [0, 0]
    # next batch: a reference into the previous batch maps through the ring; a future reference is rejected
    ev2 = np.zeros(2, dtype=A.EVENT_DTYPE)
    ev2["ts"] = T0 + 10
    ev2["res_id"] = [2, 2]
    ev2["kind"] = [A.EV_EXIT, A.EV_EXIT]
    ev2["aux"] = [A.aux_exit(1, 1), A.aux_exit(9, 1)]
    parts2, _ = router.route(ev2)
    got = parts2[o2]["aux"] & REF
    n2_before = 2 if o1 != o2 else 6
    assert int(got[0]) == (0 if o1 != o2 else 1) and int(got[1]) == n2_before + 1


def test_shard_and_route_events():
    from sentinel_amd import _abi as A
    from sentinel_amd import dist as D
    rng = np.random.default_rng(3)
    ev = np.zeros(5000, dtype=A.EVENT_DTYPE)
    ev["ts"] = T0 + np.sort(rng.integers(0, 10_000, len(ev)))
    ev["res_id"] = rng.integers(0, 1000, len(ev))
    parts, pos = D.route_events(ev, 4)
    assert sorted(np.concatenate(pos).tolist()) == list(range(len(ev)))
    for r, (p, q) in enumerate(zip(parts, pos)):
        assert (D.shard_of(p["res_id"], 4) == r).all()
        assert (np.diff(q) > 0).all() and (np.diff(p["ts"]) >= 0).all()
    # splitmix64 known values (Vigna's reference generator, state 0 -> first output)
    assert int(D.splitmix64(0)) == 0xE220A8397B1DCDAF


def test_gather_metrics_gloo():
    mp.spawn(_w_metrics, args=(2, _port()), nprocs=2, join=True)


def test_request_tokens_gloo():
    mp.spawn(_w_tokens, args=(2, _port(), False), nprocs=2, join=True)


@pytest.mark.gpu
def test_request_tokens_gpu_server():
    mp.spawn(_w_tokens, args=(2, _port(), True), nprocs=2, join=True)


def test_request_tokens_tensor_gloo():
    mp.spawn(_w_tokens_tensor, args=(2, _port(), "gloo"), nprocs=2, join=True)


@pytest.mark.gpu
def test_request_tokens_tensor_rccl():
    # one GPU on the box: a one-rank RCCL group, every buffer in HBM (the ordering, the pointer call into the
    # engine and the broadcast on device tensors)
    mp.spawn(_w_tokens_tensor, args=(1, _port(), "nccl"), nprocs=1, join=True)


def test_partitioned_oracle_equals_one_oracle():
    # bench.py's multi-core CPU baseline (and the large-trace parity replays): 4 resource-partitioned oracles
    # in threads, rules installed per shard, decisions and node states equal one oracle's over 3 batches
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as O
    from sentinel_amd import tracegen as T
    w = T.Workload(4, n_entries=60_000, n_res=2_000)
    po = O.PartitionedOracle(w, 4, max_slot_chain_size=0)
    one = O.Oracle(max_slot_chain_size=0)
    w.install(one)
    ev = w.events
    cuts = np.linspace(0, len(ev), 4).astype(np.int64)
    for a, b in zip(cuts[:-1], cuts[1:]):
        assert np.array_equal(po.submit(ev[a:b]), one.submit(ev[a:b]))
    for r in np.argsort(-np.bincount(ev["res_id"], minlength=w.n_res))[:30]:
        g, o = po.read_node(int(r)), one.read_node(int(r))
        assert np.array_equal(g["minute"], o["minute"]) and g["thread"] == o["thread"]
    po.close()
