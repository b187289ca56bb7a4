"""bench.py's launch decision (`--gpus N` is authoritative) and its child-rank launcher, on the CPU.

No GPU is touched: launch_plan() is pure, run_ranks() is driven with stand-in child commands, and the
`--dry-launch` subprocess never reaches the benchmark body.
"""
import argparse
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _args(*argv):
    return bench.parse(list(argv))


def test_single_process_without_launcher():
    assert bench.launch_plan(_args("--gpus", "1"), {}, ["--gpus", "1"]) == ("run", 1)


def test_world_size_must_match_gpus():
    kind, msg = bench.launch_plan(_args("--gpus", "8"), {"WORLD_SIZE": "1"}, [])
    assert kind == "error" and "WORLD_SIZE=1" in msg and "--gpus 8" in msg
    assert bench.launch_plan(_args("--gpus", "4"), {"WORLD_SIZE": "4"}, []) == ("run", 4)


def test_self_launch_builds_one_child_per_rank():
    argv = ["--gpus", "3", "--backend", "gloo", "--steps", "7", "--dry-launch"]
    kind, ranks = bench.launch_plan(_args(*argv), {}, argv)
    assert kind == "launch" and len(ranks) == 3
    ports = {e["MASTER_PORT"] for e, _ in ranks}
    assert len(ports) == 1
    for r, (e, cmd) in enumerate(ranks):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r) and e["WORLD_SIZE"] == "3"
        assert e["MASTER_ADDR"] == "127.0.0.1"
        assert cmd[1].endswith("bench.py") and "--dry-launch" not in cmd
        assert cmd[2:] == ["--gpus", "3", "--backend", "gloo", "--steps", "7"]


def test_nccl_self_launch_needs_enough_devices():
    kind, msg = bench.launch_plan(_args("--gpus", "2"), {}, ["--gpus", "2"], device_count=lambda: 1)
    assert kind == "error" and "needs 2 GPUs" in msg and "gloo" in msg
    kind, _ = bench.launch_plan(_args("--gpus", "2"), {}, ["--gpus", "2"], device_count=lambda: 8)
    assert kind == "launch"


def test_dry_launch_cli():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--dry-launch"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["launch"] == "children" and d["world_size"] == 2
    assert [x["env"]["RANK"] for x in d["ranks"]] == ["0", "1"]
    # nccl on a host without 2 GPUs (this container has none): refused before anything starts
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-launch"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "needs 2 GPUs" in r.stderr
    # a launcher's world size that differs from --gpus
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--dry-launch"],
                       capture_output=True, text=True, timeout=120, env=dict(os.environ, WORLD_SIZE="1"))
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


def _fake_ranks(scripts):
    return [({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(len(scripts)), "MASTER_ADDR": "127.0.0.1",
              "MASTER_PORT": "1"}, [sys.executable, "-c", s]) for r, s in enumerate(scripts)]


def test_run_ranks_relays_rank0_line(capsys):
    line = json.dumps({"metric": "m", "value": 1.0, "n_gpus": 2})
    ok0 = f"import json; print('banner'); print({line!r})"
    rc = bench.run_ranks(_fake_ranks([ok0, "pass"]), sys.stdout)
    out = capsys.readouterr()
    assert rc == 0
    assert out.out.strip() == line
    assert "banner" in out.err


def test_run_ranks_worst_exit_code_and_watchdog(capsys):
    line = json.dumps({"metric": "m", "value": 1.0})
    # rank 0 prints its line and exits 3 (the c4 watchdog); rank 1 fails with 1: the worst code is 3
    rc = bench.run_ranks(_fake_ranks([f"import os,sys; print({line!r}); sys.stdout.flush(); os._exit(3)",
                                      "raise SystemExit(1)"]), sys.stdout)
    assert rc == 3
    assert capsys.readouterr().out.strip() == line


def test_run_ranks_terminates_blocked_peer(capsys):
    # rank 1 fails at once; rank 0 would block forever in a collective: terminated after the grace period
    rc = bench.run_ranks(_fake_ranks(["import time; time.sleep(600)", "raise SystemExit(4)"]), sys.stdout,
                         grace_s=1.0)
    assert rc != 0
    assert "terminating rank" in capsys.readouterr().err


def test_run_ranks_no_line_is_failure(capsys):
    rc = bench.run_ranks(_fake_ranks(["pass", "pass"]), sys.stdout)
    assert rc == 1
