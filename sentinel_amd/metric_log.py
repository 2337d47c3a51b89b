"""Metric log writer and searcher fed by the device snapshot.

Keeps the dashboard's `metric` command and every consumer of `{app}-metrics.log` working when
node statistics live on the GPU: `MetricTimerListener.run` takes `sg_snapshot_metrics` (the
per-second `StatisticNode.metrics()` of every ClusterNode, computed on the device) instead of
walking Java ClusterNodes, and writes the same files the reference writes.

Reference (paths under sentinel-core/src/main/java/com/alibaba/csp/sentinel/):
  node/metric/MetricNode.java:116-209     thin/fat line formats
  node/metric/MetricWriter.java:121-409   file naming, rolling, .idx (second, offset) pairs
  node/metric/MetricTimerListener.java:39-71  TreeMap aggregation by timestamp
  node/metric/MetricSearcher.java:84-222  index-driven search (cached last position)
  node/metric/MetricsReader.java:33-141   line reading across rolled files

Differences, each deliberate:
  * the writer's clock is injectable (`now_ms`), because replay runs on event time; the
    reference seeds `lastSecond` from System.currentTimeMillis() (MetricWriter.java:104-105);
  * within one timestamp, nodes follow resource-id order (the reference iterates a HashMap of
    ClusterNodes, MetricTimerListener.java:42 -- an order no caller relies on);
  * the `__total_inbound_traffic__` row (Constants.ENTRY_NODE) is not produced: the global
    ENTRY_NODE belongs to SystemSlot, which is out of scope.
"""
from __future__ import annotations

import os
import re
import struct
import time as _time
from dataclasses import dataclass
from functools import cmp_to_key
from typing import Dict, Iterable, List, Optional

import numpy as np

METRIC_FILE = "metrics.log"
METRIC_FILE_INDEX_SUFFIX = ".idx"
MAX_LINES_RETURN = 100000  # MetricsReader.java:33
CHARSET = "utf-8"


def _fmt_local(ts_ms: int) -> str:
    """SimpleDateFormat("yyyy-MM-dd HH:mm:ss") in the JVM default zone = the process zone."""
    return _time.strftime("%Y-%m-%d %H:%M:%S", _time.localtime(ts_ms // 1000))


def _fmt_day(ts_ms: int) -> str:
    return _time.strftime("%Y-%m-%d", _time.localtime(ts_ms // 1000))


@dataclass
class MetricNode:
    """MetricNode.java:30-42."""
    timestamp: int = 0
    resource: str = ""
    pass_qps: int = 0
    block_qps: int = 0
    success_qps: int = 0
    exception_qps: int = 0
    rt: int = 0
    occupied_pass_qps: int = 0

    def to_thin_string(self) -> str:  # MetricNode.java:125-137
        name = self.resource.replace("|", "_")
        return "%d|%s|%d|%d|%d|%d|%d|%d" % (self.timestamp, name, self.pass_qps, self.block_qps,
                                             self.success_qps, self.exception_qps, self.rt,
                                             self.occupied_pass_qps)

    @staticmethod
    def from_thin_string(line: str) -> "MetricNode":  # MetricNode.java:145-159
        s = line.split("|")
        n = MetricNode(int(s[0]), s[1], int(s[2]), int(s[3]), int(s[4]), int(s[5]), int(s[6]))
        if len(s) == 8:
            n.occupied_pass_qps = int(s[7])
        return n

    def to_fat_string(self) -> str:  # MetricNode.java:170-186
        name = self.resource.replace("|", "_")
        return "%d|%s|%s|%d|%d|%d|%d|%d|%d\n" % (self.timestamp, _fmt_local(self.timestamp), name,
                                                  self.pass_qps, self.block_qps, self.success_qps,
                                                  self.exception_qps, self.rt, self.occupied_pass_qps)

    @staticmethod
    def from_fat_string(line: str) -> "MetricNode":  # MetricNode.java:194-209
        s = line.rstrip("\n").split("|")
        n = MetricNode(int(s[0]), s[2], int(s[3]), int(s[4]), int(s[5]), int(s[6]), int(s[7]))
        if len(s) == 9:
            n.occupied_pass_qps = int(s[8])
        return n


def form_metric_file_name(app_name: Optional[str], pid: int, use_pid: bool = True) -> str:
    """MetricWriter.formMetricFileName (MetricWriter.java:377-392); LogBase.isLogNameUsePid."""
    app = (app_name or "").replace(".", "-")
    name = app + "-" + METRIC_FILE
    if use_pid:
        name += ".pid%d" % pid
    return name


def form_index_file_name(metric_file_name: str) -> str:
    return metric_file_name + METRIC_FILE_INDEX_SUFFIX


_NAME_TAIL = re.compile(r"\.[0-9]{4}-[0-9]{2}-[0-9]{2}(\.[0-9]*)?")


def file_name_matches(file_name: str, base_file_name: str) -> bool:
    """MetricWriter.fileNameMatches (MetricWriter.java:312-320): whole-tail match."""
    if not file_name.startswith(base_file_name):
        return False
    return _NAME_TAIL.fullmatch(file_name[len(base_file_name):]) is not None


def _name_cmp(o1: str, o2: str) -> int:
    """MetricFileNameComparator (MetricWriter.java:240-268): date, then name length, then name."""
    n1, n2 = os.path.basename(o1), os.path.basename(o2)
    d1, d2 = n1.split(".")[2], n2.split(".")[2]
    if d1.startswith("pid"):
        d1, d2 = n1.split(".")[3], n2.split(".")[3]
    if d1 != d2:
        return -1 if d1 < d2 else 1
    if len(n1) != len(n2):
        return len(n1) - len(n2)
    return (n1 > n2) - (n1 < n2)


METRIC_FILE_NAME_KEY = cmp_to_key(_name_cmp)


def list_metric_files(base_dir: str, base_file_name: str) -> List[str]:
    """MetricWriter.listMetricFiles (MetricWriter.java:282-300)."""
    if not os.path.isdir(base_dir):
        return []
    out = []
    for f in os.listdir(base_dir):
        p = os.path.abspath(os.path.join(base_dir, f))
        if (os.path.isfile(p) and file_name_matches(f, base_file_name)
                and not f.endswith(METRIC_FILE_INDEX_SUFFIX) and not f.endswith(".lck")):
            out.append(p)
    out.sort(key=METRIC_FILE_NAME_KEY)
    return out


class MetricWriter:
    """MetricWriter.java:47-409.  `write(time, nodes)` appends fat lines and, on each new second,
    an (second, byte offset) pair of big-endian int64s to the `.idx` file (DataOutputStream)."""

    def __init__(self, single_file_size: int, total_file_count: int = 6, *, base_dir: str,
                 app_name: str = "", pid: Optional[int] = None, use_pid: bool = True,
                 now_ms: Optional[int] = None):
        if single_file_size <= 0 or total_file_count <= 0:
            raise ValueError("singleFileSize and totalFileCount must be positive")
        self.base_dir = base_dir if base_dir.endswith(os.sep) else base_dir + os.sep
        os.makedirs(self.base_dir, exist_ok=True)
        self.single_file_size = single_file_size
        self.total_file_count = total_file_count
        self.app_name = app_name
        self.pid = os.getpid() if pid is None else pid
        self.use_pid = use_pid
        now = int(_time.time() * 1000) if now_ms is None else int(now_ms)
        self.last_second = now // 1000
        # df.parse("1970-01-01 00:00:00") in the local zone (MetricWriter.java:109)
        self.time_second_base = int(_time.mktime(_time.strptime("1970-01-02 00:00:00", "%Y-%m-%d %H:%M:%S"))) - 86400
        self.base_file_name: Optional[str] = None
        self.cur_metric_file: Optional[str] = None
        self.cur_index_file: Optional[str] = None
        self._out = None
        self._idx = None

    # -- MetricWriter.java:121-175
    def write(self, time_ms: int, nodes: Optional[Iterable[MetricNode]]):
        if nodes is None:
            return
        nodes = list(nodes)
        for n in nodes:
            n.timestamp = time_ms
        if self.cur_metric_file is None:
            self.base_file_name = form_metric_file_name(self.app_name, self.pid, self.use_pid)
            self._close_and_new_file(self._next_file_name_of_day(time_ms))
        if not (os.path.exists(self.cur_metric_file) and os.path.exists(self.cur_index_file)):
            self._close_and_new_file(self._next_file_name_of_day(time_ms))
        second = time_ms // 1000
        if second < self.last_second:
            return  # earlier seconds are ignored (MetricWriter.java:143-144)
        if second > self.last_second:
            self._write_index(second, self._out.tell())
            if self._is_new_day(self.last_second, second):
                self._close_and_new_file(self._next_file_name_of_day(time_ms))
        self._write_lines(nodes, time_ms)
        if second > self.last_second:
            self.last_second = second

    def _write_lines(self, nodes, time_ms):
        self._out.write("".join(n.to_fat_string() for n in nodes).encode(CHARSET))
        self._out.flush()
        if self._out.tell() >= self.single_file_size:  # validSize (MetricWriter.java:355-358)
            self._close_and_new_file(self._next_file_name_of_day(time_ms))

    def close(self):
        for f in (self._out, self._idx):
            if f is not None:
                f.close()
        self._out = self._idx = None

    def _write_index(self, second: int, offset: int):
        self._idx.write(struct.pack(">qq", second, offset))
        self._idx.flush()

    def _next_file_name_of_day(self, time_ms: int) -> str:  # MetricWriter.java:192-217
        model = "%s.%s" % (self.base_file_name, _fmt_day(time_ms))
        names = [os.path.abspath(os.path.join(self.base_dir, f)) for f in os.listdir(self.base_dir)
                 if model in f and not f.endswith(METRIC_FILE_INDEX_SUFFIX) and not f.endswith(".lck")]
        names.sort(key=METRIC_FILE_NAME_KEY)
        if not names:
            return self.base_dir + model
        tail = names[-1].split(".")[-1]
        n = int(tail) if re.fullmatch(r"[0-9]{1,10}", tail) else 0
        return "%s%s.%d" % (self.base_dir, model, n + 1)

    def _remove_more_files(self):  # MetricWriter.java:322-335
        files = list_metric_files(self.base_dir, self.base_file_name)
        for f in files[: max(0, len(files) - self.total_file_count + 1)]:
            for p in (f, form_index_file_name(f)):
                if os.path.exists(p):
                    os.remove(p)

    def _close_and_new_file(self, name: str):  # MetricWriter.java:337-353 (append=false)
        self._remove_more_files()
        self.close()
        self._out = open(name, "wb")
        self.cur_metric_file = name
        self.cur_index_file = form_index_file_name(name)
        self._idx = open(self.cur_index_file, "wb")

    def _is_new_day(self, last_second: int, second: int) -> bool:  # MetricWriter.java:360-364
        return (second - self.time_second_base) // 86400 > (last_second - self.time_second_base) // 86400


class MetricTimerListener:
    """MetricTimerListener.java:34-71: one run per second; `engine.snapshot(now)` replaces the walk
    over ClusterBuilderSlot.getClusterNodeMap() and ClusterNode.metrics()."""

    def __init__(self, engine, writer: MetricWriter, names: Dict[int, str]):
        self.engine, self.writer, self.names = engine, writer, names

    def run(self, now_ms: int) -> int:
        snap = self.engine.snapshot(now_ms)
        snap = snap[np.lexsort((snap["res_id"], snap["timestamp"]))]
        maps: Dict[int, List[MetricNode]] = {}
        for r in snap:
            node = MetricNode(int(r["timestamp"]), self.names.get(int(r["res_id"]), str(int(r["res_id"]))),
                              int(r["pass_qps"]), int(r["block_qps"]), int(r["success_qps"]),
                              int(r["exception_qps"]), int(r["rt"]), int(r["occupied_pass_qps"]))
            maps.setdefault(node.timestamp, []).append(node)
        for ts in sorted(maps):  # TreeMap order
            self.writer.write(ts, maps[ts])
        return len(snap)


class MetricsReader:
    """MetricsReader.java:28-141."""

    @staticmethod
    def _lines(file_name: str, offset: int):
        with open(file_name, "rb") as f:
            f.seek(offset)
            for raw in f:
                line = raw.decode(CHARSET).rstrip("\n")
                if line:
                    yield line

    def read_in_one_file_by_end_time(self, out, file_name, offset, begin_ms, end_ms, identity) -> bool:
        begin_s, end_s = begin_ms // 1000, end_ms // 1000
        for line in self._lines(file_name, offset):
            node = MetricNode.from_fat_string(line)
            cur = node.timestamp // 1000
            if cur < begin_s or cur > end_s:
                return False
            if identity is None or node.resource == identity:
                out.append(node)
            if len(out) >= MAX_LINES_RETURN:
                return False
        return True

    def read_in_one_file(self, out, file_name, offset, recommend_lines):
        last = out[-1].timestamp // 1000 if out else -1
        for line in self._lines(file_name, offset):
            node = MetricNode.from_fat_string(line)
            cur = node.timestamp // 1000
            if len(out) < recommend_lines or cur == last:
                out.append(node)
            else:
                break
            last = cur

    def read_metrics_by_end_time(self, names, pos, offset, begin_ms, end_ms, identity):
        out: List[MetricNode] = []
        if self.read_in_one_file_by_end_time(out, names[pos], offset, begin_ms, end_ms, identity):
            pos += 1
            while pos < len(names) and self.read_in_one_file_by_end_time(out, names[pos], 0, begin_ms,
                                                                            end_ms, identity):
                pos += 1
        return out

    def read_metrics(self, names, pos, offset, recommend_lines):
        out: List[MetricNode] = []
        self.read_in_one_file(out, names[pos], offset, recommend_lines)
        pos += 1
        while len(out) < recommend_lines and pos < len(names):
            self.read_in_one_file(out, names[pos], 0, recommend_lines)
            pos += 1
        return out


class MetricSearcher:
    """MetricSearcher.java:34-222, including its cached index position."""

    def __init__(self, base_dir: str, base_file_name: str):
        if base_dir is None or base_file_name is None:
            raise ValueError("baseDir and baseFileName can't be null")
        self.base_dir = base_dir if base_dir.endswith(os.sep) else base_dir + os.sep
        self.base_file_name = base_file_name
        self.reader = MetricsReader()
        self._pos_file = self._pos_idx = None
        self._pos_off = 0
        self._pos_second = 0

    def _start(self, begin_ms, names):
        if self._valid_position(begin_ms) and self._pos_file in names:
            return names.index(self._pos_file), self._pos_off
        return 0, 0

    def find(self, begin_ms: int, recommend_lines: int):
        names = list_metric_files(self.base_dir, self.base_file_name)
        i, off_in_idx = self._start(begin_ms, names)
        for j in range(i, len(names)):
            off = self._find_offset(begin_ms, names[j], form_index_file_name(names[j]), off_in_idx)
            off_in_idx = 0
            if off != -1:
                return self.reader.read_metrics(names, j, off, recommend_lines)
        return None

    def find_by_time_and_resource(self, begin_ms: int, end_ms: int, identity: Optional[str]):
        names = list_metric_files(self.base_dir, self.base_file_name)
        i, off_in_idx = self._start(begin_ms, names)
        for j in range(i, len(names)):
            off = self._find_offset(begin_ms, names[j], form_index_file_name(names[j]), off_in_idx)
            off_in_idx = 0
            if off != -1:
                return self.reader.read_metrics_by_end_time(names, j, off, begin_ms, end_ms, identity)
        return None

    def _valid_position(self, begin_ms: int) -> bool:  # MetricSearcher.java:163-191
        if begin_ms // 1000 < self._pos_second or self._pos_idx is None:
            return False
        try:
            with open(self._pos_idx, "rb") as f:
                f.seek(self._pos_off)
                b = f.read(8)
                return len(b) == 8 and struct.unpack(">q", b)[0] == self._pos_second
        except OSError:
            return False

    def _find_offset(self, begin_ms, metric_file, idx_file, off_in_idx) -> int:  # :193-222
        self._pos_file = self._pos_idx = None
        if not os.path.exists(idx_file):
            return -1
        begin_s = begin_ms // 1000
        with open(idx_file, "rb") as f:
            f.seek(off_in_idx)
            self._pos_off = f.tell()
            while True:
                b = f.read(16)
                if len(b) < 8:
                    return -1  # EOFException
                second = struct.unpack(">q", b[:8])[0]
                if second >= begin_s:
                    if len(b) < 16:
                        return -1
                    self._pos_file, self._pos_idx, self._pos_second = metric_file, idx_file, second
                    return struct.unpack(">q", b[8:])[0]
                if len(b) < 16:
                    return -1
                self._pos_off = f.tell()
