"""bench.py --gpus N without torchrun (VERDICT r3 missing #4): the launcher starts N rank processes with
torchrun's environment, waits for them, and stops the others when one fails.

CPU: the launcher (sentinel_amd/launch.py) with small child programs, and bench.py's own check that the
world it runs in is the one --gpus names.  GPU (-m gpu): `bench.py --gpus 2` itself on the one-GPU box,
ranks over gloo (SG_BENCH_GLOO=1), a small C4 shape: one JSON line with n_gpus 2, two rank shares and a
metric all-gather.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from sentinel_amd import launch as L  # noqa: E402

PROBE = ("import json, os; print(json.dumps({k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', "
         "'LOCAL_WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')}), flush=True)")


def test_launch_sets_rank_environment(tmp_path):
    out = tmp_path / "env"
    code = PROBE.replace("print(", "open(%r + os.environ['RANK'], 'w').write(" % str(out)).replace(", flush=True", "")
    rc = L.launch_ranks(3, [sys.executable, "-c", code], poll_s=0.05)
    assert rc == 0
    envs = [json.loads((tmp_path / ("env%d" % r)).read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"} and {e["LOCAL_WORLD_SIZE"] for e in envs} == {"3"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_launch_failing_rank_stops_the_others():
    # rank 1 fails at once; rank 0 would sleep for a minute (a collective waiting for rank 1) and is stopped
    code = "import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(7)\ntime.sleep(60)"
    import time
    t = time.time()
    rc = L.launch_ranks(2, [sys.executable, "-c", code], poll_s=0.05)
    assert rc == 7
    assert time.time() - t < 30


def test_launch_escalates_to_sigkill():
    # a rank that ignores SIGTERM (stuck in a collective) is killed after the grace period
    code = ("import os, signal, sys, time\nif os.environ['RANK'] == '1': sys.exit(3)\n"
            "signal.signal(signal.SIGTERM, signal.SIG_IGN)\ntime.sleep(120)")
    import time
    t = time.time()
    rc = L.launch_ranks(2, [sys.executable, "-c", code], poll_s=0.05, grace_s=1.0)
    assert rc == 3
    assert time.time() - t < 30


def test_launch_parent_interrupt_stops_ranks(monkeypatch):
    # an exception in the parent (Ctrl-C) stops every rank before it propagates: no orphan keeps a GPU
    started = []
    real = L.subprocess.Popen

    def popen(*a, **k):
        p = real(*a, **k)
        started.append(p)
        return p

    def boom(_):
        raise KeyboardInterrupt

    import types
    monkeypatch.setattr(L.subprocess, "Popen", popen)
    monkeypatch.setattr(L, "time", types.SimpleNamespace(sleep=boom, monotonic=L.time.monotonic))
    with pytest.raises(KeyboardInterrupt):
        L.launch_ranks(2, [sys.executable, "-c", "import time; time.sleep(120)"], grace_s=2.0)
    assert len(started) == 2 and all(p.poll() is not None for p in started)


def test_launch_ranks_rendezvous_gloo():
    # the environment is enough for torch.distributed's env:// rendezvous (what bench.py's ranks do)
    code = ("import torch, torch.distributed as d; d.init_process_group('gloo'); t = torch.ones(1); "
            "d.all_reduce(t); assert t.item() == d.get_world_size() == 2; d.destroy_process_group()")
    assert L.launch_ranks(2, [sys.executable, "-c", code], poll_s=0.05) == 0


def test_bench_rejects_a_world_that_is_not_gpus():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "--gpus 2 but WORLD_SIZE=1" in p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("rank_batches,k", [("auto", 1), ("local", 2)])
def test_bench_gpus2_launches_two_ranks(rank_batches, k):
    # each global batch's shard as one batch (the default) and rank-local batches of ~--batch-events
    env = dict(os.environ, SG_BENCH_GLOO="1")
    for key in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(key, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--resources", "20000",
                        "--batch-events", str(1 << 20), "--base-batches", "2", "--sub-batches", "2", "--steps", "2",
                        "--warmup", "1", "--no-configs", "--no-cpu-baseline", "--rank-batches", rank_batches], env=env,
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-4000:]
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2
    assert len(j["config"]["rank_event_shares"]) == 2
    assert j["metric_gathers"]["count"] >= 1
    assert j["value"] > 0
    assert j["config"]["rank_batches"] == k and j["config"]["rank_local_batches_per_step"] == 2 // k
