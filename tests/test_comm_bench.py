"""bench/comm_bench.py: the collective sweep runs end to end over gloo with 2 ranks on the CPU
(the same code path the 8-GPU RCCL run takes), and the bus-bandwidth / bucket / crossover
arithmetic is right for the N = 8 node."""
import importlib.util
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("comm_bench", os.path.join(REPO, "bench", "comm_bench.py"))
cb = importlib.util.module_from_spec(spec)
spec.loader.exec_module(cb)


def test_bus_factor_and_recommendations_for_eight_ranks():
    assert cb.bus_factor("all_reduce", 8) == 2 * 7 / 8
    assert cb.bus_factor("reduce_scatter", 8) == 7 / 8 and cb.bus_factor("all_gather", 1) == 0.0
    rows = [{"op": "all_reduce", "bytes": b << 20, "busbw_gbs": bw}
            for b, bw in [(1, 40), (2, 90), (4, 160), (8, 250), (16, 290), (32, 300), (64, 305)]]
    assert cb.recommend_bucket(rows, 0.8) == 8 << 20          # 250 >= 0.8 * 305
    assert cb.recommend_bucket([], 0.8) is None
    small = [{"bytes": 16 << 10, "rccl_us": 30, "p2p_us": 8}, {"bytes": 256 << 10, "rccl_us": 40, "p2p_us": 25},
             {"bytes": 1 << 20, "rccl_us": 60, "p2p_us": 70}]
    assert cb.crossover(small) == 256 << 10
    assert cb.crossover([{"bytes": 1, "rccl_us": 1}]) is None
    assert cb.sizes(1 << 20, 8 << 20) == [1 << 20, 2 << 20, 4 << 20, 8 << 20]


def test_two_gloo_ranks_end_to_end(tmp_path):
    env = dict(os.environ, PYTHONPATH=REPO)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench", "comm_bench.py"), "--device", "cpu",
                        "--gpus", "2", "--min-bytes", str(1 << 16), "--max-bytes", str(1 << 18),
                        "--p2p-min-bytes", str(1 << 12), "--p2p-max-bytes", str(1 << 13), "--iters", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=240, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["world_size"] == 2 and out["backend"] == "gloo"
    ops = {(x["op"], x["dtype"]) for x in out["rows"]}
    assert ops == {(o, d) for o in ("all_reduce", "reduce_scatter", "all_gather") for d in ("bf16", "fp32")}
    assert all(x["us"] > 0 and x["busbw_gbs"] >= 0 for x in out["rows"])
    assert len(out["small"]) == 4 and out["recommended_bucket_bytes"] in {None, 1 << 16, 1 << 17, 1 << 18}
    assert "| all_reduce |" in r.stderr
