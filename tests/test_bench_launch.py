"""bench.py's multi-GPU launch contract, checked without a GPU: `--gpus N` with no WORLD_SIZE starts
N worker processes (one per GPU, torch.distributed.run on 127.0.0.1) before anything touches the
GPU; a WORLD_SIZE that differs from --gpus is refused (no line is printed for a world the flags do
not name)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=e, timeout=120)


def test_gpus_n_launches_n_workers():
    r = _run(["--gpus", "4", "--workload", "c3", "--steps", "3", "--dry-launch"])
    assert r.returncode == 0, r.stderr
    cmd = json.loads(r.stdout.strip().splitlines()[-1])["launch"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    # the workers get the same flags (so each asserts WORLD_SIZE == --gpus)
    tail = cmd[cmd.index(BENCH) + 1:]
    assert tail == ["--gpus", "4", "--workload", "c3", "--steps", "3"]
    fields = json.loads(r.stdout.strip().splitlines()[-1])["fields_at_n_gt_1"]
    assert {"roundtrip_ok", "gather", "value"} <= set(fields)


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "2"], WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr and r.stdout.strip() == ""


def test_too_few_devices_refused():
    import torch
    if torch.cuda.device_count() >= 2:  # pragma: no cover - a multi-GPU host would really launch
        return
    r = _run(["--gpus", "2"])
    assert r.returncode == 2 and "visible" in r.stderr
