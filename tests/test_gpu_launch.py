"""The multi-GPU launch path of bench.py, end to end, as a fresh child process.

`python bench.py --gpus 2` outside a launcher starts `torch.distributed.run` itself (one rank per GPU, as the
reference's trainer.py:237-242 spawns one process per GPU) and every rank runs the DDP + SyncBatchNorm train
step (trainer.py:143-147).  On a one-GPU box both ranks share cuda:0 and talk over gloo
(EBC_BENCH_ONE_DEVICE=1 EBC_BENCH_BACKEND=gloo): a rehearsal of the launch, rendezvous, per-rank timing and the
max-over-ranks reduction, not a scaling number.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_rank_launch():
    env = dict(os.environ, EBC_BENCH_ONE_DEVICE="1", EBC_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)                      # not under a launcher: bench.py must start one itself
    proc = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                           "--no-probe"], cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert proc.returncode == 0, proc.stdout[-2000:] + proc.stderr[-4000:]
    lines = [l for l in proc.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, proc.stdout[-2000:]              # rank 0 prints the one JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["config"]["parallelism"] == "dp2"
    assert len(out["per_rank_crops_s"]) == 2 and all(v > 0 for v in out["per_rank_crops_s"])
    assert out["config"]["global_batch"] == 64                # configs[3]: 32 crops per rank at N > 1
    # value = all ranks' crops over the max-over-ranks time
    assert out["value"] <= sum(out["per_rank_crops_s"]) * 1.0001
