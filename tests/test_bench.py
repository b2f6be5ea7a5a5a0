"""bench.py contract: `--gpus N` without a launcher spawns N ranks itself, both halves of the
metric (BERT tokens/s + ResNet-50 images/s) land in ONE JSON line, and the world size seen
by the process group is N."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--device", "cpu", "--model", "tiny",
                          "--steps", "2", "--warmup", "1", *extra], capture_output=True, text=True, env=env,
                         timeout=600, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_spawns_two_ranks_and_reports_both_metrics():
    r = _run("--gpus", "2")
    # CPU/gloo: no GPU behind the ranks; the world size comes from a real collective
    assert r["n_gpus"] == 0 and r["world_size"] == 2 and r["backend"] == "gloo"
    assert r["env"]["world_size_seen_by_collective"] == 2 and r["world_size_seen_by_rccl"] is None
    assert r["step_ms_mean"] > 0 and r["step_ms_ci95"] >= 0 and r["value_ci95"] >= 0
    assert r["bucket_plan"]["buckets"] >= 1 and r["resnet50_bucket_plan"]["buckets"] >= 1
    assert r["metric"] == "bert_large_pretrain_tokens_per_sec" and r["value"] > 0
    assert r["resnet50_images_per_sec"] > 0
    assert len(r["per_rank_ms_per_step"]) == 2
    assert r["config"]["parallelism"] == "dp2" and r["config"]["global_batch"] == 8
    assert r["steps"] == 2 and r["warmup"] == 1


def test_bench_single_process_eager_impl():
    r = _run("--gpus", "1", "--impl", "eager")
    assert r["world_size"] == 1 and r["config"]["impl"] == "eager"
    assert r["value"] > 0 and r["resnet50_images_per_sec"] > 0


def test_bench_eight_ranks_one_node_layout():
    """The N = 8 launch of the driver's scaling run, rehearsed on gloo: 8 ranks, one JSON
    line, the max over 8 ranks, both halves through the same bucketed data-parallel path."""
    r = _run("--gpus", "8")
    assert r["world_size"] == 8 and r["env"]["world_size_seen_by_collective"] == 8
    assert len(r["per_rank_ms_per_step"]) == 8 and len(r["resnet50_per_rank_ms_per_step"]) == 8
    assert r["ms_per_step"] >= max(r["per_rank_ms_per_step"]) * 0.999
    assert r["config"]["parallelism"] == "dp8" and r["config"]["global_batch"] == 32
    assert r["value"] > 0 and r["resnet50_images_per_sec"] > 0
