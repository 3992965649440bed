"""bench.py's N-rank launcher on the CPU (gloo): `python bench.py --gpus N` without torchrun starts N child ranks
itself (env:// on 127.0.0.1, one LOCAL_RANK per GPU) before any GPU call, rank 0 prints the one line; under torchrun a
WORLD_SIZE that is not --gpus exits non-zero before anything runs"""
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _bench():
    spec = importlib.util.spec_from_file_location("bench_launch_under_test", BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    e.update(kw)
    return e


def test_child_envs_bookkeeping():
    b = _bench()
    envs = b.child_envs(4, {"KEEP": "1"}, 29511)
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4" for e in envs)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511" and e["KEEP"] == "1" for e in envs)


def test_check_world():
    b = _bench()
    assert b.check_world(2, {}) is None
    assert b.check_world(2, {"WORLD_SIZE": "2"}) is None
    assert b.check_world(8, {"WORLD_SIZE": "2"}) is not None
    assert b.check_world(1, {"WORLD_SIZE": "x"}) is not None


def test_world_size_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--workload", "launchcheck", "--backend", "gloo"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr and r.stdout == ""


def test_self_launch_two_ranks_gloo():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--workload", "launchcheck", "--backend", "gloo"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["rank_sum"] == 1 and out["launcher"] == "bench.py"


def test_self_launch_failing_rank_fails_the_run():
    # a workload that needs libspg: on a CPU-only host every rank fails (no gfx950 device), so the launcher must
    # return non-zero and print no line
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--workload", "msm", "--backend", "gloo", "--log-msm", "4",
                        "--steps", "1", "--warmup", "0", "--no-cpu-baseline"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and r.stdout.strip() == ""
