"""bench.py's own rank launcher (``python bench.py --gpus N`` without torchrun), on CPU with stub
children: the environment each rank gets, rank 0's output only, and a failing or hung rank ending
the whole job with a non-zero status (the launch the reference leaves to
``accelerate launch``, utils/common.py:58-90)."""
import io
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (numpy-only at import; no GPU)

STUB = r'''
import json, os, sys, time
mode = sys.argv[1]
r = int(os.environ["RANK"])
env = {k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
open(os.path.join(sys.argv[2], f"env{r}.json"), "w").write(json.dumps(env))
print(json.dumps({"rank": r, "line": "result"}), flush=True)
if mode == "fail" and r == 1:
    time.sleep(0.3)
    sys.exit(3)
if mode in ("fail", "hang") and r != 1 or mode == "hang":
    time.sleep(120)
'''


def _stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return p


def test_launcher_env_and_rank0_output(tmp_path):
    stub = _stub(tmp_path)
    out = io.StringIO()
    rc = bench.launch_ranks(4, [sys.executable, str(stub), "ok", str(tmp_path)], timeout=60, out=out)
    assert rc == 0
    lines = [json.loads(x) for x in out.getvalue().splitlines()]
    assert lines == [{"rank": 0, "line": "result"}]            # rank 0's stdout only
    envs = [json.load(open(tmp_path / f"env{r}.json")) for r in range(4)]
    ports = {e["MASTER_PORT"] for e in envs}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1"


def test_launcher_failing_rank_stops_the_job(tmp_path):
    stub = _stub(tmp_path)
    t = time.monotonic()
    rc = bench.launch_ranks(3, [sys.executable, str(stub), "fail", str(tmp_path)], timeout=100, out=io.StringIO())
    assert rc == 3                                    # the failing rank's status
    assert time.monotonic() - t < 60                  # the sleeping siblings were killed


def test_launcher_timeout(tmp_path):
    stub = _stub(tmp_path)
    rc = bench.launch_ranks(2, [sys.executable, str(stub), "hang", str(tmp_path)], timeout=2, out=io.StringIO())
    assert rc == 124


def test_bench_refuses_more_gpus_than_visible():
    """This container shows no GPU: ``--gpus 2`` exits non-zero with the message and prints no
    JSON line (on a one-GPU lease the same)."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode != 0
    assert p.stdout.strip() == ""
    assert "visible GPUs" in p.stderr


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--no-cpu-baseline"], capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode != 0 and p.stdout.strip() == ""
    assert "WORLD_SIZE 1" in p.stderr
