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


def test_c4_scaling_keys():
    """The c4 leg's speed-up is against the same job's one-GPU c3 frame, never the group's own N = 1 figure."""
    W, H, rays = 3840, 2160, 18_956_255
    k = bench.c4_scaling_keys(8, W, H, rays, c4_ms=0.020, c3_ms_inflight=0.1265, c3_ms_serial=0.128)
    assert k["speedup_vs_c3_1gpu"] == round(0.1265 / 0.020, 3)
    assert k["efficiency"] == round(0.1265 / 0.020 / 8, 3)
    assert k["speedup_vs_c3_1gpu_serial"] == round(0.128 / 0.020, 3)
    assert k["mray_s_per_gpu"] == round(rays / 20e-6 / 1e6 / 8, 3)
    assert k["hbm_write_frac_per_gpu"] == round(W * H * 4 / 8 / 20e-6 / 8e12, 5)
    assert k["c3_1gpu_ms_per_frame"] == 0.1265
    # a leg that did not time anything carries the baseline only
    assert "speedup_vs_c3_1gpu" not in bench.c4_scaling_keys(8, W, H, rays, None, 0.1265, 0.128)
    txt = bench.c4_parallelism_text(8, dict(k, value=947.8))
    assert "8 GPUs" in txt and "efficiency" in txt and str(k["speedup_vs_c3_1gpu"]) in txt
    assert bench.c4_parallelism_text(8, {"error": "x"}) == ""


def test_cpu_baseline_labels_threads_not_cores():
    """The CPU baseline names what it ran on: OpenMP threads of the lease's share, not physical cores."""
    lab = bench.cpu_baseline_labels(16, env={"OMP_NUM_THREADS": "16"})
    assert lab["threads"] == 16 and lab["cores"] == lab["threads"]
    assert "not physical cores" in lab["threads_note"] and "OMP_NUM_THREADS=16" in lab["threads_note"]
    assert lab["nproc"] == os.cpu_count() and lab["affinity_threads"] >= 1
    assert lab["omp_num_threads_env"] == "16" and "host_cpu" in lab and lab["unit"] == "Mray/s"


def test_c4_projection_keys():
    """The one-GPU projection of the 8-rank c4 frame: the slowest of rank 0's pipeline (its bands + unpack, measured
    or, without it, summed) and the peers' band renders, or the nominal gather when longer; speed-up bound against
    the one-GPU c3 frame."""
    k = bench.c4_projection_keys(8, 0.112, [0.015, 0.0165, 0.016], 0.003, 1_044_480)
    assert k["n8_rank_render_ms_max"] == 0.0165 and k["n8_unpack_ms"] == 0.003
    assert k["n8_rank0_ms"] == 0.018 and k["n8_projected_frame_ms"] == 0.018
    assert k["n8_speedup_bound"] == round(0.112 / 0.018, 3)
    assert k["n8_limiting_stage"] == "rank 0 (bands + unpack)"
    assert abs(k["n8_gather_ms_nominal"] - 1_044_480 / 153e9 * 1e3) < 1e-5
    m = bench.c4_projection_keys(8, 0.112, [0.015, 0.0165, 0.016], 0.003, 1_044_480, root_ms=0.016)
    assert m["n8_projected_frame_ms"] == 0.0165 and m["n8_limiting_stage"] == "a peer's band render"
    assert m["n8_speedup_bound"] == round(0.112 / 0.0165, 3)
    # rank 0 only assembles: the seven renderers are all peers, rank 0 is its unpack pipeline
    a = bench.c4_projection_keys(8, 0.112, [0.016] * 6 + [0.017], 0.007, 1_200_000, root_ms=0.0075, root_renders=False)
    assert a["n8_root_renders"] is False and a["n8_projected_frame_ms"] == 0.017
    assert a["n8_limiting_stage"] == "a peer's band render" and a["n8_speedup_bound"] == round(0.112 / 0.017, 3)
    b = bench.c4_projection_keys(8, 0.112, [0.016] * 7, 0.02, 1_200_000, root_renders=False)
    assert b["n8_rank0_ms"] == 0.02 and b["n8_limiting_stage"] == "rank 0 (unpack)"
    slow = bench.c4_projection_keys(8, 0.112, [0.001], 0.0005, 10_000_000)      # gather-bound
    assert slow["n8_limiting_stage"] == "gather (nominal xGMI)"
    assert slow["n8_projected_frame_ms"] == slow["n8_gather_ms_nominal"]
