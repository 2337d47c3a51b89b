"""Metric log writer / searcher (sentinel_amd/metric_log.py) against the reference's MetricWriter
contract (sentinel-core/.../node/metric/MetricWriter.java, MetricSearcher.java, MetricsReader.java).

CPU tests: the reference's own MetricWriterTest cases (file-name order and matching), line
formats, the .idx layout and searcher behaviour over rolled files.  GPU test: the device
snapshot written through MetricTimerListener gives the same files as the oracle's snapshot.
"""
import os
import struct

import numpy as np
import pytest

from sentinel_amd import _abi as A
from sentinel_amd import metric_log as M

T0 = 1_700_000_000_000


# ---- MetricWriterTest.java:17-80 (transcribed)
def test_file_name_cmp():
    arr = ["metrics.log.2018-03-06", "metrics.log.2018-03-07", "metrics.log.2018-03-07.51",
           "metrics.log.2018-03-07.10", "metrics.log.2018-03-06.100"]
    key = ["metrics.log.2018-03-06", "metrics.log.2018-03-06.100", "metrics.log.2018-03-07",
           "metrics.log.2018-03-07.10", "metrics.log.2018-03-07.51"]
    assert sorted(arr, key=M.METRIC_FILE_NAME_KEY) == key


def test_file_name_pid_cmp():
    arr = ["metrics.log.pid1234.2018-03-06", "metrics.log.pid1234.2018-03-07",
           "metrics.log.pid1234.2018-03-07.51", "metrics.log.pid1234.2018-03-07.10",
           "metrics.log.pid1234.2018-03-06.100"]
    key = ["metrics.log.pid1234.2018-03-06", "metrics.log.pid1234.2018-03-06.100",
           "metrics.log.pid1234.2018-03-07", "metrics.log.pid1234.2018-03-07.10",
           "metrics.log.pid1234.2018-03-07.51"]
    assert sorted(arr, key=M.METRIC_FILE_NAME_KEY) == key


def test_file_name_matches():
    assert M.file_name_matches("Sentinel-SDK-Demo-metrics.log.2018-03-06", "Sentinel-SDK-Demo-metrics.log")
    assert M.file_name_matches("Sentinel-Admin-metrics.log.pid22568.2018-12-24", "Sentinel-Admin-metrics.log.pid22568")
    assert M.file_name_matches("Sentinel-SDK-Demo-metrics.log.2018-03-06.11", "Sentinel-SDK-Demo-metrics.log")
    assert not M.file_name_matches("Sentinel-SDK-Demo-metrics.log.XXX.2018-03-06.11", "Sentinel-SDK-Demo-metrics.log")
    assert not M.file_name_matches("Sentinel-SDK-Demo-metrics.log.2018-03-06.11XXX", "Sentinel-SDK-Demo-metrics.log")


def test_form_metric_file_name():
    assert M.form_metric_file_name("com.foo.app", 42) == "com-foo-app-metrics.log.pid42"
    assert M.form_metric_file_name(None, 7, use_pid=False) == "-metrics.log"


def test_line_formats_round_trip():
    n = M.MetricNode(T0, "a|b", 3, 1, 2, 0, 17, 5)
    assert n.to_thin_string() == "%d|a_b|3|1|2|0|17|5" % T0
    back = M.MetricNode.from_thin_string(n.to_thin_string())
    assert back == M.MetricNode(T0, "a_b", 3, 1, 2, 0, 17, 5)
    fat = n.to_fat_string()
    assert fat.endswith("\n") and fat.count("|") == 8 and fat.split("|")[1] == M._fmt_local(T0)
    assert M.MetricNode.from_fat_string(fat) == back
    # a thin line without occupiedPassQps (MetricNode.java:155-157)
    assert M.MetricNode.from_thin_string("1|r|1|2|3|4|5").occupied_pass_qps == 0


def _nodes(sec, k):
    return [M.MetricNode(0, "res%d" % i, sec + i, i, sec, 0, 10 + i, 0) for i in range(k)]


def test_writer_index_and_search(tmp_path):
    w = M.MetricWriter(1 << 20, 6, base_dir=str(tmp_path), app_name="app", pid=1, now_ms=T0 - 5000)
    for s in range(10):
        w.write(T0 + 1000 * s, _nodes(s, 3))
    w.close()
    files = M.list_metric_files(str(tmp_path), "app-metrics.log.pid1")
    assert len(files) == 1
    idx = open(M.form_index_file_name(files[0]), "rb").read()
    pairs = [struct.unpack(">qq", idx[i:i + 16]) for i in range(0, len(idx), 16)]
    lines = open(files[0], "rb").read().split(b"\n")[:-1]
    assert len(lines) == 30 and [p[0] for p in pairs] == [T0 // 1000 + s for s in range(10)]
    # each index offset points at the first line of its second
    data = open(files[0], "rb").read()
    for sec, off in pairs:
        assert int(data[off:].split(b"|", 1)[0]) // 1000 == sec
    srch = M.MetricSearcher(str(tmp_path), "app-metrics.log.pid1")
    got = srch.find(T0 + 4000, 4)
    # a second is never split: 4 lines requested -> seconds 4 and 5 complete = 6 lines
    assert [n.timestamp for n in got] == [T0 + 4000] * 3 + [T0 + 5000] * 3
    got = srch.find_by_time_and_resource(T0 + 2000, T0 + 3999, "res1")
    assert [(n.timestamp, n.pass_qps) for n in got] == [(T0 + 2000, 3), (T0 + 3000, 4)]
    assert srch.find(T0 + 60_000, 4) is None


def test_same_second_writes_no_index_and_earlier_seconds_ignored(tmp_path):
    w = M.MetricWriter(1 << 20, base_dir=str(tmp_path), app_name="x", pid=2, now_ms=T0)
    w.write(T0 + 10, _nodes(0, 2))      # second == lastSecond: lines, no index (MetricWriter.java:145-152)
    w.write(T0 - 2000, _nodes(9, 2))    # earlier second: ignored
    w.write(T0 + 1000, _nodes(1, 1))
    w.close()
    f = M.list_metric_files(str(tmp_path), "x-metrics.log.pid2")[0]
    assert len(open(f, "rb").read().split(b"\n")) - 1 == 3
    assert len(open(M.form_index_file_name(f), "rb").read()) == 16


def test_rolling_by_size_and_file_count(tmp_path):
    w = M.MetricWriter(200, 3, base_dir=str(tmp_path), app_name="r", pid=3, now_ms=T0 - 1000)
    for s in range(12):
        w.write(T0 + 1000 * s, _nodes(s, 2))
    w.close()
    files = M.list_metric_files(str(tmp_path), "r-metrics.log.pid3")
    # removeMoreFiles keeps totalFileCount - 1 old files before opening a new one
    assert len(files) == 3
    assert all(os.path.exists(M.form_index_file_name(f)) for f in files)
    suffixes = [f.rsplit(".", 1)[1] for f in files]
    assert suffixes == sorted(suffixes, key=int)


class _FakeEngine:
    def __init__(self, rows):
        self.rows = rows

    def snapshot(self, now):
        a = np.zeros(len(self.rows), dtype=A.METRIC_NODE_DTYPE)
        for i, r in enumerate(self.rows):
            a[i]["timestamp"], a[i]["res_id"], a[i]["pass_qps"], a[i]["rt"] = r
        return a


def test_timer_listener_groups_by_timestamp(tmp_path):
    eng = _FakeEngine([(T0 + 2000, 1, 5, 7), (T0 + 1000, 0, 3, 4), (T0 + 1000, 1, 2, 9), (T0 + 2000, 0, 1, 1)])
    w = M.MetricWriter(1 << 20, base_dir=str(tmp_path), app_name="t", pid=4, now_ms=T0)
    M.MetricTimerListener(eng, w, {0: "a", 1: "b"}).run(T0 + 3000)
    w.close()
    f = M.list_metric_files(str(tmp_path), "t-metrics.log.pid4")[0]
    got = [M.MetricNode.from_fat_string(l) for l in open(f).read().splitlines()]
    assert [(n.timestamp, n.resource, n.pass_qps, n.rt) for n in got] == [
        (T0 + 1000, "a", 3, 4), (T0 + 1000, "b", 2, 9), (T0 + 2000, "a", 1, 1), (T0 + 2000, "b", 5, 7)]


@pytest.mark.gpu
def test_device_snapshot_log_matches_oracle(tmp_path):
    import pyoracle as O
    from sentinel_amd import engine as E
    from sentinel_amd import tracegen as T

    w = T.Workload(2, n_entries=60_000, n_res=300)
    eng = E.Engine(max_resources=w.n_res, max_slot_chain_size=0, param_table_log2=16, status_ring_log2=22)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    names = {i: "res-%d" % i for i in range(w.n_res)}
    out = {}
    for tag, src in (("gpu", eng), ("cpu", orc)):
        d = tmp_path / tag
        wr = M.MetricWriter(1 << 16, 100, base_dir=str(d), app_name="c2", pid=9, now_ms=int(w.events["ts"][0]) - 1000)
        lis = M.MetricTimerListener(src, wr, names)
        ev = w.events
        cuts = np.linspace(0, len(ev), 6).astype(np.int64)
        for a, b in zip(cuts[:-1], cuts[1:]):
            src.submit(ev[a:b])
            lis.run(int(ev["ts"][b - 1]))
        lis.run(w.t_end + 2000)
        wr.close()
        files = M.list_metric_files(str(d), "c2-metrics.log.pid9")
        out[tag] = [(os.path.basename(f), open(f, "rb").read(), open(M.form_index_file_name(f), "rb").read())
                    for f in files]
    assert out["gpu"] and out["gpu"] == out["cpu"]
