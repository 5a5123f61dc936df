"""bench.py's N > 1 launch on CPU: `--gpus 2` starts two ranks itself (torch.distributed.run
child), they rendezvous over gloo, run the bucketed gradient exchange around a toy model,
time with barrier + max-over-ranks, and rank 0 prints ONE JSON line with n_gpus 2.
(--device cpu is the plumbing mode: no libmdemi, not a measurement.)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    return p


def test_bench_gpus2_launches_two_ranks_cpu():
    p = _run(["--gpus", "2", "--device", "cpu", "--steps", "3", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # only rank 0 prints
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["config"]["parallelism"] == "dp2"
    assert rec["buckets"] >= 2 and rec["launch_order"] == list(range(rec["buckets"]))
    assert rec["replicas_identical"]


def test_bench_gpus1_cpu_single_process():
    p = _run(["--gpus", "1", "--device", "cpu", "--steps", "2", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["n_gpus"] == 1


def test_bench_rejects_more_gpus_than_visible():
    # no GPU in the CPU container: asking for 2 GPU ranks must fail loudly, not time one rank
    p = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], timeout=120)
    assert p.returncode != 0
    assert "GPU(s) visible" in p.stderr
