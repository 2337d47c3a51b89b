"""Wire-compatible token server front-end (sentinel_amd/token_server.py).

CPU tests: byte layouts of the reference's Netty codecs (NettyTransportServer framing,
DefaultRequestEntityDecoder, FlowRequestDataDecoder, PingRequestDataDecoder,
DefaultResponseEntityWriter, FlowResponseDataWriter), and the asyncio server with a recording
stub service (batching, ping/connected counts, BAD for types without a processor, oversize frames).
GPU test: real clients against the server on the device engine; every response equals the
oracle's TokenService answer for the same requests at the same times.
"""
import asyncio
import struct

import numpy as np
import pytest

from sentinel_amd import _abi as A
from sentinel_amd import token_server as S


def test_flow_request_bytes():
    b = S.encode_flow_request(7, 0x0102030405060708, 3, True)
    # u16 length 18 | int xid | byte type 1 | long flowId | int count | bool priority
    assert b == bytes.fromhex("0012" "00000007" "01" "0102030405060708" "00000003" "01")
    req = S.decode_request(b[2:])
    assert (req.xid, req.type, req.data) == (7, S.MSG_TYPE_FLOW, S.FlowRequest(0x0102030405060708, 3, True))
    # priority byte absent -> false (FlowRequestDataDecoder.java:36-40); short body -> null data
    assert S.decode_request(b[2:-1]).data == S.FlowRequest(0x0102030405060708, 3, False)
    assert S.decode_request(b[2:12]).data is None
    assert S.decode_request(b[2:6]) is None  # < 5 bytes
    assert S.decode_request(struct.pack(">ib", 1, 9)) is None  # unknown type


def test_ping_and_response_bytes():
    b = S.encode_ping_request(-2, "app-ns")
    req = S.decode_request(b[2:])
    assert (req.xid, req.type, req.data) == (-2, S.MSG_TYPE_PING, "app-ns")
    assert S.decode_request(struct.pack(">ibi", 1, 0, 0)).data is None
    assert S.encode_flow_response(5, A.TOKEN_SHOULD_WAIT, 0, 200) == bytes.fromhex("000e" "00000005" "01" "02" "00000000" "000000c8")
    assert S.encode_ping_response(5, 3) == bytes.fromhex("0007" "00000005" "00" "00" "03")
    assert S.encode_bad_response(5, 2) == bytes.fromhex("0006" "00000005" "02" "ff")
    assert S.decode_response(S.encode_flow_response(9, A.TOKEN_BLOCKED, -1, 0)[2:]) == (9, 1, A.TOKEN_BLOCKED, (-1, 0))


def test_frame_decoder_split_and_oversize():
    d = S.FrameDecoder()
    stream = S.encode_flow_request(1, 10, 1, False) + S.encode_ping_request(2, "ns")
    got = []
    for i in range(len(stream)):
        got += d.feed(stream[i:i + 1])
    assert [S.decode_request(g).xid for g in got] == [1, 2]
    with pytest.raises(ValueError):
        S.FrameDecoder().feed(struct.pack(">H", 1023))


class _Stub:
    """Records what reaches the device boundary; answers OK with remaining = flowId + count."""

    def __init__(self):
        self.connected = {}

    def cluster_set_connected(self, fid, n):
        self.connected[fid] = n

    def cluster_request_array(self, reqs):
        out = np.zeros(len(reqs), dtype=A.TOKEN_RES_DTYPE)
        out["status"] = A.TOKEN_OK
        out["remaining"] = reqs["flow_id"] + reqs["acquire_count"]
        out["wait_in_ms"] = reqs["prioritized"]
        return out


async def _client(port, frames, n_resp):
    r, w = await asyncio.open_connection("127.0.0.1", port)
    w.write(b"".join(frames))
    await w.drain()
    dec, out = S.FrameDecoder(), []
    while len(out) < n_resp:
        data = await asyncio.wait_for(r.read(65536), 10)
        assert data
        out += [S.decode_response(b) for b in dec.feed(data)]
    return r, w, out


def test_server_batches_and_pings():
    async def run():
        stub = _Stub()
        srv = S.TokenServer(stub, flow_namespaces={11: "ns-a", 12: "ns-b"}, clock=lambda: 1000)
        port = await srv.start(port=0)
        r1, w1, a = await _client(port, [S.encode_ping_request(1, "ns-a")] +
                                  [S.encode_flow_request(10 + i, 11, i + 1, i % 2 == 1) for i in range(50)], 51)
        assert a[0] == (1, S.MSG_TYPE_PING, S.RESPONSE_STATUS_OK, 1)
        assert sorted(a[1:]) == [(10 + i, 1, A.TOKEN_OK, (12 + i, i % 2)) for i in range(50)]
        assert stub.connected == {11: 1}
        r2, w2, b = await _client(port, [S.encode_ping_request(3, "ns-a"), S.encode_ping_request(4, " "),
                                         S.frame(struct.pack(">ib", 5, S.MSG_TYPE_PARAM_FLOW))], 3)
        assert b == [(3, 0, 0, 2), (4, 0, S.RESPONSE_STATUS_BAD, None), (5, S.MSG_TYPE_PARAM_FLOW, S.RESPONSE_STATUS_BAD, None)]
        assert stub.connected == {11: 2}
        w2.close()
        await asyncio.sleep(0.05)
        assert stub.connected == {11: 1}
        # far fewer device calls than requests: frames that arrive together are decided together
        assert sum(srv.batches) == 50 and len(srv.batches) < 50
        w1.close()
        await srv.stop()

    asyncio.run(run())


@pytest.mark.gpu
def test_server_on_device_matches_oracle():
    import pyoracle as O
    from sentinel_amd import engine as E

    T0 = 1_700_000_000_000
    rules = [A.flow_rule("abc", c, cluster_mode=True, cluster_flow_id=fid,
                         cluster_threshold_type=A.CLUSTER_THRESHOLD_GLOBAL)
             for fid, c in ((101, 20), (102, 5), (103, 50))]
    eng = E.Engine(max_resources=64)
    eng.register("abc")
    eng.load_flow_rules(rules)
    tick = [T0]

    def clock():
        tick[0] += 37
        return tick[0]

    async def run():
        srv = S.TokenServer(eng, clock=clock, record=True)
        port = await srv.start(port=0)
        rng = np.random.default_rng(3)
        clients = []
        for c in range(4):
            frames = [S.encode_flow_request(c * 1000 + i, int(rng.choice([101, 102, 103, 999])),
                                            int(rng.integers(1, 4)), bool(rng.random() < 0.2)) for i in range(300)]
            clients.append(_client(port, frames, 300))
        res = await asyncio.gather(*clients)
        for _, w, _ in res:
            w.close()
        await srv.stop()
        return srv, [x for _, _, out in res for x in out]

    srv, got = asyncio.run(run())
    orc = O.Oracle()
    orc.register("abc")
    orc.load_flow_rules(rules)
    by_xid = {}
    for xids, reqs, res in srv.submitted:
        want = orc.cluster_request([(int(r["ts"]), int(r["flow_id"]), int(r["acquire_count"]),
                                     bool(r["prioritized"])) for r in reqs])
        dev = [(int(o["status"]), int(o["remaining"]), int(o["wait_in_ms"])) for o in res]
        assert dev == want
        by_xid.update(zip(xids, dev))
    assert len(got) == 1200 and len(by_xid) == 1200 and len(srv.batches) < 1200
    for xid, typ, st, data in got:
        assert (st,) + tuple(data) == by_xid[xid]
    assert {s for s, _, _ in by_xid.values()} >= {A.TOKEN_OK, A.TOKEN_NO_RULE_EXISTS}


def test_param_flow_request_bytes():
    b = S.encode_param_flow_request(9, 77, 2, [(S.PARAM_TYPE_INTEGER, -3), (S.PARAM_TYPE_STRING, "ab"),
                                               (S.PARAM_TYPE_BOOLEAN, True), (S.PARAM_TYPE_DOUBLE, 0.1)])
    # int xid | byte 2 | long flowId | int count | int amount | (byte type, value)*
    assert b[2:] == bytes.fromhex("00000009" "02" "000000000000004d" "00000002" "00000004"
                                  "00" "fffffffd" "07" "00000002" "6162" "06" "01" "03" "3fb999999999999a")
    req = S.decode_request(b[2:])
    assert req.data == S.ParamFlowRequest(77, 2, [("java.lang.Integer", -3), ("java.lang.String", "ab"),
                                                  ("java.lang.Boolean", True), ("java.lang.Double", 0.1)])
    # fewer than 16 bytes or amount <= 0 -> null data (ParamFlowRequestDataDecoder.java:33-50)
    assert S.decode_request(struct.pack(">ibqii", 1, 2, 77, 1, 0)).data is None
    assert S.decode_request(struct.pack(">ibqi", 1, 2, 77, 1)).data is None
    assert S.decode_response(S.encode_param_flow_response(9, A.TOKEN_OK, 4)[2:]) == (9, 2, A.TOKEN_OK, (4, 0))
    assert [S.param_value_text(c, v) for c, v in req.data.params] == ["-3", "ab", "true", "0.1"]


@pytest.mark.gpu
def test_server_param_flow_on_device_matches_oracle():
    import pyoracle as O
    from sentinel_amd import engine as E

    T0 = 1_700_000_000_000
    rules = [A.param_rule("abc", 0, c, cluster_mode=True, cluster_flow_id=fid,
                          cluster_threshold_type=A.CLUSTER_THRESHOLD_GLOBAL,
                          items=[("7", "java.lang.Integer", 9)])
             for fid, c in ((201, 4), (202, 2))]
    eng = E.Engine(max_resources=64)
    eng.register("abc")
    eng.load_param_rules(rules)
    tick = [T0]

    def clock():
        tick[0] += 53
        return tick[0]

    async def run():
        srv = S.TokenServer(eng, clock=clock, record=True, param_key=E.param_key)
        port = await srv.start(port=0)
        rng = np.random.default_rng(5)
        clients = []
        for c in range(3):
            frames = []
            for i in range(200):
                ps = [(S.PARAM_TYPE_INTEGER, int(rng.integers(0, 10))) if rng.random() < 0.5 else
                      (S.PARAM_TYPE_STRING, "u%d" % int(rng.integers(0, 5))) for _ in range(int(rng.integers(1, 3)))]
                frames.append(S.encode_param_flow_request(c * 1000 + i, int(rng.choice([201, 202, 203])), 1, ps))
            clients.append(_client(port, frames, 200))
        res = await asyncio.gather(*clients)
        for _, w, _ in res:
            w.close()
        await srv.stop()
        return srv, [x for _, _, out in res for x in out]

    srv, got = asyncio.run(run())
    orc = O.Oracle()
    orc.register("abc")
    orc.load_param_rules(rules)
    by_xid = {}
    for xids, (reqs, vals), res in srv.submitted:
        q = [(int(r["ts"]), int(r["flow_id"]), int(r["acquire_count"]),
              vals[int(r["value_off"]):int(r["value_off"]) + int(r["n_values"])]) for r in reqs]
        want = orc.cluster_request_param(q)
        dev = [(int(o["status"]), int(o["remaining"]), int(o["wait_in_ms"])) for o in res]
        assert dev == want
        by_xid.update(zip(xids, dev))
    assert len(got) == 600 and len(by_xid) == 600
    for xid, typ, st, data in got:
        assert typ == S.MSG_TYPE_PARAM_FLOW and (st,) + tuple(data) == by_xid[xid]
    assert {s for s, _, _ in by_xid.values()} >= {A.TOKEN_OK, A.TOKEN_BLOCKED, A.TOKEN_NO_RULE_EXISTS}


def test_param_flow_decoder_unknown_type_and_truncation():
    # ParamFlowRequestDataDecoder.java:34-94: the loop runs `amount` times and ignores decodeParam's false
    # return, so an unknown type byte is consumed and the next byte is read as the next type.
    head = struct.pack(">ibqii", 3, 2, 77, 1, 3)
    body = head + bytes([0x7F]) + struct.pack(">bi", S.PARAM_TYPE_INTEGER, 5) + struct.pack(">bq", S.PARAM_TYPE_LONG, 6)
    assert S.decode_request(body).data == S.ParamFlowRequest(77, 1, [("java.lang.Integer", 5), ("java.lang.Long", 6)])
    # a read past the end throws out of the decoder: the request is dropped (no partial param list)
    assert S.decode_request(head + struct.pack(">bi", S.PARAM_TYPE_INTEGER, 5)).data is None
    short_str = struct.pack(">ibqii", 3, 2, 77, 1, 1) + struct.pack(">bi", S.PARAM_TYPE_STRING, 10) + b"abc"
    assert S.decode_request(short_str).data is None
    neg_str = struct.pack(">ibqii", 3, 2, 77, 1, 1) + struct.pack(">bi", S.PARAM_TYPE_STRING, -1)
    assert S.decode_request(neg_str).data is None
    assert S.decode_request(struct.pack(">ibqii", 3, 2, 77, 1, 2) + struct.pack(">bh", S.PARAM_TYPE_SHORT, 1)).data is None


class _MixedStub(_Stub):
    """Records the order and clock of every device call; the first FLOW call raises."""

    def __init__(self):
        super().__init__()
        self.calls = []

    def cluster_request_array(self, reqs):
        self.calls.append(("flow", int(reqs["ts"][0]), len(reqs)))
        if len(self.calls) == 1:
            raise RuntimeError("device error")
        return super().cluster_request_array(reqs)

    def cluster_request_param_array(self, reqs, vals):
        self.calls.append(("param", int(reqs["ts"][0]), len(reqs)))
        out = np.zeros(len(reqs), dtype=A.TOKEN_RES_DTYPE)
        out["status"] = A.TOKEN_OK
        return out


def test_server_tick_order_clock_and_error_recovery():
    # One tick: FLOW x2, PARAM x1, FLOW x1 in arrival order -> three device calls in that order, one clock
    # reading for the whole tick.  The first call raises: its requests get FAIL, the loop keeps serving.
    stub = _MixedStub()
    ticks = []

    def clock():
        ticks.append(1)
        return 1_700_000_000_000 + len(ticks)

    async def run():
        srv = S.TokenServer(stub, clock=clock, param_key=lambda text, cls: 5)
        port = await srv.start(port=0)
        frames = [S.encode_flow_request(1, 10, 1, False), S.encode_flow_request(2, 10, 1, False),
                  S.encode_param_flow_request(3, 11, 1, [(S.PARAM_TYPE_INTEGER, 1)]),
                  S.encode_flow_request(4, 10, 1, False)]
        _, w, out = await _client(port, frames, 4)
        _, w2, out2 = await _client(port, [S.encode_flow_request(5, 10, 2, False)], 1)
        w.close()
        w2.close()
        await srv.stop()
        return srv, out, out2

    srv, out, out2 = asyncio.run(run())
    by = {x: st for x, _, st, _ in out}
    assert by == {1: A.TOKEN_FAIL, 2: A.TOKEN_FAIL, 3: A.TOKEN_OK, 4: A.TOKEN_OK}
    assert [c[0] for c in stub.calls[:3]] == ["flow", "param", "flow"] and [c[2] for c in stub.calls[:3]] == [2, 1, 1]
    assert len({c[1] for c in stub.calls[:3]}) == 1  # one clock reading per tick
    assert out2[0][2] == A.TOKEN_OK and len(srv.errors) == 1
