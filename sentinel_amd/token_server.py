"""Wire-compatible cluster token server front-end over the device token service
(SURVEY.md §8(f) rank 2).

Real `DefaultClusterTokenClient`s connect unchanged: the framing and entity layouts are those of
the reference's Netty server, and every FLOW request of a tick is decided in ONE
`sg_cluster_request_tokens` call (the device GlobalRequestLimiter + ClusterFlowChecker), instead of
one `TokenService.requestToken` per request on a Netty worker thread.

Reference (csrv/ = sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster/):
  csrv/server/NettyTransportServer.java:80-87      LengthFieldBasedFrameDecoder(1024, 0, 2, 0, 2) +
                                                   LengthFieldPrepender(2): u16 big-endian frame length
  csrv/server/codec/DefaultRequestEntityDecoder.java:36-55   int xid, byte type, then the body
  csrv/server/codec/data/FlowRequestDataDecoder.java:32-44   long flowId, int count [, bool priority]
  csrv/server/codec/data/PingRequestDataDecoder.java:30-41   int length, namespace bytes
  csrv/server/codec/DefaultResponseEntityWriter.java:33-51   int xid, byte type, byte status, then the body
  csrv/server/codec/data/FlowResponseDataWriter.java:29-33   int remaining, int waitInMs
  csrv/server/codec/data/PingResponseDataWriter.java:29-35   byte connectedCount
  csrv/server/handler/TokenServerHandler.java:58-110         ping -> ConnectionManager; no processor -> BAD
  csrv/processor/FlowRequestProcessor.java:33-52             TokenResult -> (status, remaining, wait)
  cluster/ClusterConstants.java:24-40 (sentinel-cluster-common-default)  message types, status codes

  csrv/server/codec/data/ParamFlowRequestDataDecoder.java:33-90  long flowId, int count, int amount,
                                                   typed params (ClusterConstants.PARAM_TYPE_*)
  csrv/processor/ParamFlowRequestProcessor.java:33-52        requestParamToken -> (status, remaining, 0)

PARAM_FLOW requests of a tick are decided in one `sg_cluster_request_param_tokens` call; their
typed values are interned with the same 64-bit keys as the rules' hot items (`sg_param_key`).
"""
from __future__ import annotations

import asyncio
import struct
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

from . import _abi as A

MSG_TYPE_PING = 0
MSG_TYPE_FLOW = 1
MSG_TYPE_PARAM_FLOW = 2
RESPONSE_STATUS_BAD = -1
RESPONSE_STATUS_OK = 0
DEFAULT_CLUSTER_SERVER_PORT = 18730
MAX_FRAME_LENGTH = 1024          # LengthFieldBasedFrameDecoder maxFrameLength (includes the 2-byte field)
DEFAULT_NAMESPACE = "default"   # ServerConstants.DEFAULT_NAMESPACE


@dataclass
class ClusterRequest:
    xid: int
    type: int
    data: object  # FlowRequest, str (ping namespace) or None


PARAM_TYPE_INTEGER, PARAM_TYPE_LONG, PARAM_TYPE_BYTE, PARAM_TYPE_DOUBLE = 0, 1, 2, 3
PARAM_TYPE_FLOAT, PARAM_TYPE_SHORT, PARAM_TYPE_BOOLEAN, PARAM_TYPE_STRING = 4, 5, 6, 7
# wire type -> (struct format, Java class of the decoded object, as sg_param_key names it)
_PARAM_WIRE = {PARAM_TYPE_INTEGER: (">i", "java.lang.Integer"), PARAM_TYPE_LONG: (">q", "java.lang.Long"),
               PARAM_TYPE_BYTE: (">b", "java.lang.Byte"), PARAM_TYPE_DOUBLE: (">d", "java.lang.Double"),
               PARAM_TYPE_FLOAT: (">f", "java.lang.Float"), PARAM_TYPE_SHORT: (">h", "java.lang.Short"),
               PARAM_TYPE_BOOLEAN: (">?", "java.lang.Boolean")}


@dataclass
class ParamFlowRequest:
    flow_id: int
    count: int
    params: list  # [(java class, value)]


@dataclass
class FlowRequest:
    flow_id: int
    count: int
    priority: bool = False


# ---------------------------------------------------------------- codec
def decode_request(body: bytes) -> Optional[ClusterRequest]:
    """DefaultRequestEntityDecoder.decode: None when fewer than 5 bytes or the type has no decoder."""
    if len(body) < 5:
        return None
    xid, typ = struct.unpack_from(">ib", body, 0)
    rest = body[5:]
    if typ == MSG_TYPE_FLOW:
        data = None
        if rest:
            if len(rest) >= 12:  # FlowRequestDataDecoder
                fid, cnt = struct.unpack_from(">qi", rest, 0)
                data = FlowRequest(fid, cnt, len(rest) >= 13 and rest[12] != 0)
        return ClusterRequest(xid, typ, data)
    if typ == MSG_TYPE_PING:
        data = None
        if len(rest) >= 4:  # PingRequestDataDecoder
            n = struct.unpack_from(">i", rest, 0)[0]
            if n > 0 and len(rest) > 4:
                data = rest[4:4 + n].decode("utf-8", "replace")
        return ClusterRequest(xid, typ, data)
    if typ == MSG_TYPE_PARAM_FLOW:
        return ClusterRequest(xid, typ, decode_param_flow(rest) if rest else None)
    return None  # "Unknown type of request data decoder": dropped


def decode_param_flow(b: bytes) -> Optional[ParamFlowRequest]:
    """ParamFlowRequestDataDecoder.decode (sentinel-cluster-server-default .../codec/data/
    ParamFlowRequestDataDecoder.java:34-94): None unless >= 16 bytes and amount > 0.  The loop runs
    `amount` times; decodeParam's false return for an unknown type byte is ignored, so the next byte is
    read as the next value's type.  A read past the end of the body (ByteBuf IndexOutOfBoundsException,
    including a string whose declared length exceeds the remaining bytes or is negative) throws out of
    the decoder, so the request is dropped: None."""
    if len(b) < 16:
        return None
    fid, cnt, amount = struct.unpack_from(">qii", b, 0)
    if amount <= 0:
        return None
    off, params = 16, []
    try:
        for _ in range(amount):
            t = struct.unpack_from(">b", b, off)[0]
            off += 1
            if t == PARAM_TYPE_STRING:
                n = struct.unpack_from(">i", b, off)[0]
                if n < 0 or off + 4 + n > len(b):
                    return None
                params.append(("java.lang.String", b[off + 4:off + 4 + n].decode("utf-8", "replace")))
                off += 4 + n
            elif t in _PARAM_WIRE:
                fmt, cls = _PARAM_WIRE[t]
                v = struct.unpack_from(fmt, b, off)[0]
                params.append((cls, v))
                off += struct.calcsize(fmt)
            # else: unknown type, decodeParam returns false and the loop goes on
    except struct.error:
        return None
    return ParamFlowRequest(fid, cnt, params)


def encode_param_flow_request(xid: int, flow_id: int, count: int, params) -> bytes:
    """Client side (ParamFlowRequestDataWriter): params = [(PARAM_TYPE_*, value)]."""
    body = struct.pack(">ibqii", xid, MSG_TYPE_PARAM_FLOW, flow_id, count, len(params))
    for t, v in params:
        if t == PARAM_TYPE_STRING:
            raw = v.encode("utf-8")
            body += struct.pack(">bi", t, len(raw)) + raw
        else:
            body += struct.pack(">b", t) + struct.pack(_PARAM_WIRE[t][0], v)
    return frame(body)


def param_value_text(cls: str, v) -> str:
    """Text of a decoded value as sg_param_key parses it (Java's toString for the boxed types)."""
    if cls == "java.lang.Boolean":
        return "true" if v else "false"
    if cls in ("java.lang.Double", "java.lang.Float"):
        return repr(float(v))
    return str(v)


def encode_flow_request(xid: int, flow_id: int, count: int, priority: bool) -> bytes:
    """Client side (FlowRequestDataWriter + DefaultRequestEntityWriter), framed."""
    return frame(struct.pack(">ibqi?", xid, MSG_TYPE_FLOW, flow_id, count, priority))


def encode_ping_request(xid: int, namespace: str) -> bytes:
    ns = namespace.encode("utf-8")
    return frame(struct.pack(">ibi", xid, MSG_TYPE_PING, len(ns)) + ns)


def encode_flow_response(xid: int, status: int, remaining: int, wait_ms: int) -> bytes:
    return frame(struct.pack(">ibbii", xid, MSG_TYPE_FLOW, status, remaining, wait_ms))


def encode_ping_response(xid: int, connected: int) -> bytes:
    # ByteBuf.writeByte keeps the low 8 bits of the connected count
    return frame(struct.pack(">ibbB", xid, MSG_TYPE_PING, RESPONSE_STATUS_OK, connected & 0xFF))


def encode_param_flow_response(xid: int, status: int, remaining: int) -> bytes:
    """ParamFlowRequestProcessor.toResponse + FlowResponseDataWriter (waitInMs is always 0)."""
    return frame(struct.pack(">ibbii", xid, MSG_TYPE_PARAM_FLOW, status, remaining, 0))


def encode_bad_response(xid: int, typ: int) -> bytes:
    return frame(struct.pack(">ibb", xid, typ, RESPONSE_STATUS_BAD))


def decode_response(body: bytes) -> Tuple[int, int, int, object]:
    """Client side (DefaultResponseEntityDecoder): (xid, type, status, data)."""
    xid, typ, st = struct.unpack_from(">ibb", body, 0)
    rest = body[6:]
    if typ in (MSG_TYPE_FLOW, MSG_TYPE_PARAM_FLOW) and len(rest) >= 8:
        return xid, typ, st, struct.unpack_from(">ii", rest, 0)
    if typ == MSG_TYPE_PING and len(rest) >= 1:
        return xid, typ, st, struct.unpack_from(">b", rest, 0)[0]
    return xid, typ, st, None


def frame(body: bytes) -> bytes:
    """LengthFieldPrepender(2)."""
    return struct.pack(">H", len(body)) + body


class FrameDecoder:
    """LengthFieldBasedFrameDecoder(1024, 0, 2, 0, 2): u16 length, field stripped.  A frame whose
    length field + 2 exceeds 1024 is a TooLongFrameException: the connection is closed."""

    def __init__(self):
        self.buf = bytearray()

    def feed(self, data: bytes) -> List[bytes]:
        self.buf += data
        out = []
        while len(self.buf) >= 2:
            n = (self.buf[0] << 8) | self.buf[1]
            if n + 2 > MAX_FRAME_LENGTH:
                raise ValueError("frame length %d exceeds %d" % (n + 2, MAX_FRAME_LENGTH))
            if len(self.buf) < n + 2:
                break
            out.append(bytes(self.buf[2:2 + n]))
            del self.buf[:2 + n]
        return out


# ---------------------------------------------------------------- server
class ConnectionManager:
    """ConnectionManager (csrv/connection/ConnectionManager.java): namespace -> client addresses."""

    def __init__(self):
        self.groups: Dict[str, set] = {}

    def add(self, namespace: str, addr: str) -> int:
        self.groups.setdefault(namespace, set()).add(addr)
        return len(self.groups[namespace])

    def remove(self, addr: str) -> List[str]:
        hit = [ns for ns, s in self.groups.items() if addr in s]
        for ns in hit:
            self.groups[ns].discard(addr)
        return hit

    def count(self, namespace: str) -> int:
        return len(self.groups.get(namespace, ()))


class TokenServer:
    """asyncio transport server.  `service` is the device engine (`sentinel_amd.engine.Engine`):
    `cluster_request_array(A.TOKEN_REQ_DTYPE array)` and `cluster_set_connected(flow_id, n)`.
    `flow_namespaces` maps flowId -> namespace (ClusterFlowRuleManager's namespace of a rule) so a
    ping updates the AVG_LOCAL connected count of every flow of its namespace.  `clock` returns ms
    (TimeUtil.currentTimeMillis); tests inject a replay clock.  `max_batch` bounds one device call."""

    def __init__(self, service, flow_namespaces: Optional[Dict[int, str]] = None,
                 clock: Optional[Callable[[], int]] = None, max_batch: int = 65536, record: bool = False,
                 param_key: Optional[Callable[[str, str], int]] = None):
        self.service = service
        self.flow_ns = dict(flow_namespaces or {})
        self.clock = clock or (lambda: int(time.time() * 1000))
        self.max_batch = max_batch
        self.record = record
        self.conns = ConnectionManager()
        # FLOW and PARAM_FLOW requests in arrival order: (writer, xid, type, request)
        self._pending: List[Tuple[asyncio.StreamWriter, int, int, object]] = []
        self.param_key = param_key  # (text, java class) -> interned 64-bit key
        self._wake = asyncio.Event()
        self._server = None
        self._batcher = None
        self.batches: List[int] = []      # sizes of the device calls (observability)
        self.submitted: List[tuple] = []  # (xids, requests, results) of every device call, in order
        self.errors: List[str] = []       # device-call failures answered with FAIL (observability)

    async def start(self, host: str = "127.0.0.1", port: int = DEFAULT_CLUSTER_SERVER_PORT):
        self._server = await asyncio.start_server(self._serve, host, port)
        self._batcher = asyncio.ensure_future(self._batch_loop())
        return self._server.sockets[0].getsockname()[1]

    async def stop(self):
        if self._server is not None:
            self._server.close()
            await self._server.wait_closed()
        if self._batcher is not None:
            self._batcher.cancel()
            try:
                await self._batcher
            except asyncio.CancelledError:
                pass

    def _update_connected(self, namespace: str):
        n = self.conns.count(namespace)
        for fid, ns in self.flow_ns.items():
            if ns == namespace:
                self.service.cluster_set_connected(fid, n)

    async def _serve(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        peer = writer.get_extra_info("peername")
        addr = "%s:%s" % (peer[0], peer[1]) if peer else "?"
        dec = FrameDecoder()
        try:
            while True:
                data = await reader.read(65536)
                if not data:
                    break
                for body in dec.feed(data):
                    req = decode_request(body)
                    if req is None:
                        continue
                    if req.type == MSG_TYPE_PING:
                        if not req.data or not req.data.strip():
                            writer.write(encode_bad_response(req.xid, req.type))
                        else:
                            n = self.conns.add(req.data, addr)
                            self._update_connected(req.data)
                            writer.write(encode_ping_response(req.xid, n))
                    elif req.type == MSG_TYPE_FLOW:
                        if req.data is not None:  # the reference's processor NPEs on a null body
                            self._pending.append((writer, req.xid, MSG_TYPE_FLOW, req.data))
                            self._wake.set()
                    elif req.type == MSG_TYPE_PARAM_FLOW and self.param_key is not None:
                        if req.data is not None:  # the reference's processor NPEs on a null body
                            self._pending.append((writer, req.xid, MSG_TYPE_PARAM_FLOW, req.data))
                            self._wake.set()
                    else:
                        writer.write(encode_bad_response(req.xid, req.type))
        except (ValueError, ConnectionError):
            pass
        finally:
            for ns in self.conns.remove(addr):
                self._update_connected(ns)
            writer.close()

    async def _batch_loop(self):
        """One tick = every request queued since the last one, decided with ONE clock reading, in arrival
        order: consecutive requests of one type form one device call (FLOW and PARAM_FLOW share the
        namespace's GlobalRequestLimiter, so the order of the calls is the order of arrival).  A device
        error fails the requests of that call (TokenResultStatus.FAIL) and the loop keeps serving."""
        while True:
            await self._wake.wait()
            self._wake.clear()
            await asyncio.sleep(0)  # let every readable connection queue its frames first
            if not self._pending:
                continue
            now = self.clock()
            queue, self._pending = self._pending, []
            i = 0
            while i < len(queue):
                typ, j = queue[i][2], i
                while j < len(queue) and queue[j][2] == typ and j - i < self.max_batch:
                    j += 1
                run = [(w, x, r) for w, x, _, r in queue[i:j]]
                try:
                    (self._decide if typ == MSG_TYPE_FLOW else self._decide_param)(run, now)
                except Exception as exc:  # e.g. SentinelError from the device call
                    self.errors.append(repr(exc))
                    for w, xid, _ in run:
                        if not w.is_closing():
                            w.write(encode_flow_response(xid, A.TOKEN_FAIL, 0, 0) if typ == MSG_TYPE_FLOW
                                    else encode_param_flow_response(xid, A.TOKEN_FAIL, 0))
                i = j

    def _decide(self, batch, now: int):
        reqs = np.zeros(len(batch), dtype=A.TOKEN_REQ_DTYPE)
        reqs["ts"] = now
        reqs["flow_id"] = [r.flow_id for _, _, r in batch]
        reqs["acquire_count"] = [r.count for _, _, r in batch]
        reqs["prioritized"] = [int(r.priority) for _, _, r in batch]
        res = self.service.cluster_request_array(reqs)
        self.batches.append(len(batch))
        if self.record:
            self.submitted.append(([x for _, x, _ in batch], reqs, res))
        for (w, xid, _), o in zip(batch, res):
            if not w.is_closing():
                w.write(encode_flow_response(xid, int(o["status"]), int(o["remaining"]), int(o["wait_in_ms"])))

    def _decide_param(self, batch, now: int):
        reqs = np.zeros(len(batch), dtype=A.PARAM_TOKEN_REQ_DTYPE)
        vals: List[int] = []
        for j, (_, _, r) in enumerate(batch):
            reqs[j] = (now, r.flow_id, r.count, len(r.params), len(vals))
            vals += [self.param_key(param_value_text(c, v), c) for c, v in r.params]
        res = self.service.cluster_request_param_array(reqs, np.array(vals, dtype=np.uint64))
        self.batches.append(len(batch))
        if self.record:
            self.submitted.append(([x for _, x, _ in batch], (reqs, vals), res))
        for (w, xid, _), o in zip(batch, res):
            if not w.is_closing():
                w.write(encode_param_flow_response(xid, int(o["status"]), int(o["remaining"])))
