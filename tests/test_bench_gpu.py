"""The multi-rank GPU path of bench.py on a one-GPU box: two ranks share GPU 0 and gloo moves
the CUDA tensors in place of RCCL.  Everything else is the code the 8-GPU driver run takes
(self-spawned ranks, flat-buffer bucketer fed by the gradient side stream, fused LAMB / SGD,
barrier + max-over-ranks timing, one JSON line), for plain data parallelism and ZeRO-1."""
import json
import math
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--model", "tiny", "--gpus", "2",
                          "--dist-backend", "gloo", "--steps", "3", "--warmup", "1", *extra],
                         capture_output=True, text=True, env=env, timeout=300, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("zero", [False, True])
def test_bench_two_ranks_share_one_gpu(zero):
    r = _run(*(["--zero"] if zero else []))
    # two ranks, ONE physical GPU: n_gpus counts devices, the world size comes from a collective
    assert r["n_gpus"] == 1 and r["world_size"] == 2 and r["backend"] == "gloo" and "note" in r
    assert r["env"]["world_size_seen_by_collective"] == 2 and r["env"]["distinct_devices"] == 1
    assert r["dtype"] == "bf16" and r["config"]["zero1"] is zero
    assert len(r["per_rank_ms_per_step"]) == 2 and len(r["resnet50_per_rank_ms_per_step"]) == 2
    assert r["value"] > 0 and r["resnet50_images_per_sec"] > 0
    assert math.isfinite(r["config"]["loss_last_step"]) and math.isfinite(r["resnet50_loss_last_step"])
