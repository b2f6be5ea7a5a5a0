"""Trial parallelism (reference Hyperopt SparkTrials): concurrent trial
processes, failure isolation, refinement toward the optimum, GPU pinning per slot."""
import os

from cloudtik_amd.runtime.ai.tune import choice, loguniform, tune, uniform


def quadratic(p):
    if p["mode"] == "bad":
        raise ValueError("bad configuration")
    return {"loss": (p["x"] - 0.3) ** 2 + (0.0 if p["mode"] == "good" else 0.5), "pid": os.getpid(),
            "gpu": os.environ.get("HIP_VISIBLE_DEVICES")}


def test_tune_runs_concurrently_isolates_failures_and_improves():
    r = tune(quadratic, {"x": uniform(-2.0, 2.0), "mode": choice(["good", "ok", "bad"]),
                         "lr": loguniform(1e-4, 1e-1)}, num_trials=24, max_concurrent=3, seed=1)
    assert len(r.trials) == 24
    assert any(t.error and "bad configuration" in t.error for t in r.trials)
    best = r.best
    assert best.params["mode"] == "good" and abs(best.params["x"] - 0.3) < 0.35
    assert len({t.result["pid"] for t in r.trials if t.result}) > 1
    assert all(1e-4 <= t.params["lr"] <= 1e-1 for t in r.trials)


def test_tune_pins_one_gpu_per_slot(monkeypatch):
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "4,5")
    r = tune(quadratic, {"x": uniform(0, 1), "mode": choice(["good"])}, num_trials=4)
    assert {t.result["gpu"] for t in r.trials} <= {"4", "5"} and {t.gpu for t in r.trials} == {4, 5}
