"""The device hot-parameter map code on the CPU (no GPU needed): tests/pmap_host.cpp compiles
sentinel_amd/csrc/pmap.h (its operations are __host__ __device__) and checks, against a reference LRU after
every operation, (1) the sequential CacheMap operations k_lane runs -- put / get / thread-count decrement with
removal, ring compaction -- and (2) the tile residency rule k_pq decides a tile of accesses with (param.hip).
ParameterMetric's CacheMap semantics: param/slots/block/flow/param/ParameterMetric.java:37-241."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "pmap_host.cpp")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def binary(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not installed")
    out = str(tmp_path_factory.mktemp("pmap") / "pmap_host")
    subprocess.run([HIPCC, "-O2", "-std=c++17", "--offload-arch=gfx950", "-o", out, SRC], check=True,
                   capture_output=True)
    return out


# (cap, ops, key space, seed, hot keys): churn with evictions, hot keys that keep old keys alive (ring
# compactions), capacities of the thread-count map (4000) and of a 2-second rule map (8000)
CASES = [(16, 200_000, 64, 1, 0), (100, 300_000, 1000, 5, 20), (4000, 1_500_000, 100_000, 7, 50),
         (4000, 1_500_000, 3000, 17, 5), (8000, 1_000_000, 50_000, 21, 100), (50, 500_000, 200, 11, 3)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "cap%d-ks%d-hot%d" % (c[0], c[2], c[4]))
def test_lane_operations_match_reference_lru(binary, case):
    r = subprocess.run([binary] + [str(x) for x in case], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("case", CASES, ids=lambda c: "cap%d-ks%d-hot%d" % (c[0], c[2], c[4]))
def test_tile_residency_rule_matches_reference_lru(binary, case):
    r = subprocess.run([binary] + [str(x) for x in case] + ["tile"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
