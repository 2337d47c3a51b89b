"""The drop-in boundary: the C-ABI library loads, exports every entry point of
include/sentinel_gpu.h, and its structs have the layout the bindings assume.
CPU-only (no compute call needs a GPU); engine creation must fail loudly here."""
import ctypes as C
import os
import re
import subprocess

import pytest

from sentinel_amd import _abi as A
from sentinel_amd import build, engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(engine.LIB_PATH):
        build.build()


def test_header_declares_exactly_the_exported_api():
    hdr = open(os.path.join(ROOT, "include", "sentinel_gpu.h")).read()
    declared = set(re.findall(r"\b(sg_[a-z_]+)\s*\(", hdr)) - {"sg_engine"}
    assert declared == set(engine.EXPORTS)


def test_library_exports_every_symbol():
    L = C.CDLL(engine.LIB_PATH)
    for name in engine.EXPORTS:
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", engine.LIB_PATH], capture_output=True, text=True).stdout
    for name in engine.EXPORTS:
        assert re.search(r"\bT %s$" % name, out, re.M), name


def test_struct_layouts_match_header(tmp_path):
    exe = tmp_path / "abi_sizes"
    subprocess.run(["gcc", "-O0", "-o", str(exe), os.path.join(ROOT, "tests", "abi_sizes.c")], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                               check=True).stdout.splitlines())
    got = {k: int(v) for k, v in got.items()}
    assert got["sg_config"] == C.sizeof(A.SgConfig)
    assert got["sg_flow_rule"] == C.sizeof(A.SgFlowRule)
    assert got["sg_degrade_rule"] == C.sizeof(A.SgDegradeRule)
    assert got["sg_param_item"] == C.sizeof(A.SgParamItem)
    assert got["sg_param_rule"] == C.sizeof(A.SgParamRule)
    assert got["sg_event"] == 24 == A.EVENT_DTYPE.itemsize
    assert got["sg_metric_node"] == C.sizeof(A.SgMetricNode) == A.METRIC_NODE_DTYPE.itemsize
    assert got["sg_bucket"] == C.sizeof(A.SgBucket) == 64
    assert got["sg_node_state"] == C.sizeof(A.SgNodeState)
    assert got["sg_token_req"] == C.sizeof(A.SgTokenReq)
    assert got["sg_token_result"] == C.sizeof(A.SgTokenResult)
    assert got["sg_param_token_req"] == A.PARAM_TOKEN_REQ_DTYPE.itemsize
    assert got["ev.aux"] == A.EVENT_DTYPE.fields["aux"][1]
    assert got["cfg.cluster_exceed_count"] == A.SgConfig.cluster_exceed_count.offset
    assert got["param.items"] == A.SgParamRule.items.offset
    assert got["cfg.aux_node_capacity"] == A.SgConfig.aux_node_capacity.offset
    assert got["sg_event_ext"] == A.EXT_DTYPE.itemsize and got["sg_arg"] == A.ARG_DTYPE.itemsize


def test_config_defaults_are_the_reference_defaults():
    cfg = engine.default_config()
    assert (cfg.sample_count, cfg.interval_ms, cfg.statistic_max_rt, cfg.cold_factor, cfg.occupy_timeout_ms,
            cfg.max_slot_chain_size, cfg.switch_on) == (2, 1000, 4900, 3, 500, 6000, 1)
    assert (cfg.cluster_sample_count, cfg.cluster_interval_ms, cfg.cluster_max_allowed_qps) == (10, 1000, 30000)


def test_param_key_matches_oracle():
    import pyoracle as O
    for v, t in [("a", None), ("a", "java.lang.String"), ("1", "int"), ("1", "java.lang.Integer"),
                 ("1", "java.lang.Long"), ("1.5", "java.lang.Double"), ("1.5", "float"), ("c", "char"),
                 ("TRUE", "boolean"), ("7", "short"), ("-3", "byte"), ("123456789012345678901", "long")]:
        assert engine.param_key(v, t) == O.param_key(v, t)
    assert engine.param_key("1", "int") != engine.param_key("1", "java.lang.Long") != engine.param_key("1", None)


def test_engine_create_fails_loudly_without_gfx950():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible: covered by the gpu tests")
    with pytest.raises(engine.SentinelError) as ei:
        engine.Engine(max_resources=64)
    assert ei.value.code == A.SG_EDEVICE
