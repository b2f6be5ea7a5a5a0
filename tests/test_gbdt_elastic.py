"""Elastic / fault-tolerant GBDT training (modeling/gbdt/elastic.py; reference
xgboost/modeling/run.py:90-106 RayParams: num_actors, elastic_training, max_failed_actors,
max_actor_restarts, checkpoint_frequency) on CPU actors over gloo:

* an actor killed mid-run with a restart left is restarted and the job resumes from the last
  checkpoint: the model equals the uninterrupted run's (row / feature sampling is seeded by
  the global round);
* elastic: an actor killed with no restarts is dropped and training finishes on the others;
* without elastic training, or past max_failed_actors, the job fails.
Parity with xgboost_ray itself is unpinned (neither it nor xgboost is importable here)."""
import numpy as np
import pytest

from cloudtik_amd.modeling.gbdt import DMatrix
from cloudtik_amd.modeling.gbdt.elastic import ElasticParams, train_elastic

PARAMS = {"objective": "binary:logistic", "max_depth": 3, "eta": 0.3, "subsample": 0.8,
          "colsample_bytree": 0.8, "seed": 5}


def _data(n=1800, f=6, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, f)).astype(np.float32)
    logit = 2 * X[:, 0] - X[:, 1] ** 2 + X[:, 2] * X[:, 3]
    y = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(np.float32)
    return X, y


def shard(actor_id, num_actors):
    X, y = _data()
    return DMatrix(X[:1500][actor_id::num_actors], y[:1500][actor_id::num_actors])


def _run(tmp_path, name, **kw):
    ep = ElasticParams(num_actors=3, checkpoint_frequency=2, checkpoint_dir=str(tmp_path / name),
                       collective_timeout_s=60, attempt_timeout_s=240, **kw)
    return train_elastic(PARAMS, shard, 8, ep)


def test_restarted_actor_resumes_from_checkpoint_and_matches_uninterrupted(tmp_path):
    ref, rep0 = _run(tmp_path, "ref")
    assert rep0["attempts"] == [{"actors": [0, 1, 2], "failed": [], "resumed_trees": 0}]
    b, rep = _run(tmp_path, "restart", max_actor_restarts=1, fail_at={1: 4})
    a0, a1 = rep["attempts"]
    assert a0["failed"] == [1] and a1["actors"] == [0, 1, 2] and a1["failed"] == []
    assert a1["resumed_trees"] == 4       # died after round 4 (0-based): resumes from the checkpoint at 4
    assert b.num_trees == ref.num_trees == 8
    X, _ = _data()
    np.testing.assert_allclose(b.predict(X[1500:]), ref.predict(X[1500:]), rtol=1e-5, atol=1e-6)
    assert (b.trees.feat == ref.trees.feat).float().mean() > 0.95


def test_elastic_training_continues_without_the_failed_actor(tmp_path):
    b, rep = _run(tmp_path, "elastic", elastic_training=True, max_failed_actors=1, fail_at={2: 2})
    assert rep["final_actors"] == [0, 1] and rep["dropped_actors"] == [2]
    assert rep["attempts"][1] == {"actors": [0, 1], "failed": [], "resumed_trees": 2}
    assert b.num_trees == 8
    from sklearn.metrics import roc_auc_score
    X, y = _data()
    assert roc_auc_score(y[1500:], b.predict(X[1500:])) > 0.8


def test_failure_without_elasticity_or_past_the_limit_raises(tmp_path):
    with pytest.raises(RuntimeError, match="elastic_training is off"):
        _run(tmp_path, "rigid", fail_at={0: 1})
    # past the limit: one lost actor with max_failed_actors=0 (two simultaneous failures are
    # not deterministic -- the driver tears the group down at the FIRST exit it sees)
    with pytest.raises(RuntimeError, match="actors lost"):
        _run(tmp_path, "toomany", elastic_training=True, max_failed_actors=0, fail_at={2: 1})


def test_run_workflow_with_elastic_actors(tmp_path):
    """run.py --num-actors 2 drives the fault-tolerant trainer from the processed parquet."""
    import pandas as pd
    import yaml
    from cloudtik_amd.modeling.gbdt import run as gbdt_run
    X, y = _data(1200)
    df = pd.DataFrame(X, columns=[f"c{i}" for i in range(X.shape[1])])
    df["label"] = y
    df["year"] = np.where(np.arange(len(df)) < 1000, 2017, 2019)
    df.to_csv(tmp_path / "raw.csv", index=False)
    (tmp_path / "dp.yaml").write_text(yaml.safe_dump({"data_splitting": {"custom_rules": {
        "train": 'df["year"] < 2018', "test": 'df["year"] > 2018'}}}))
    (tmp_path / "tr.yaml").write_text(yaml.safe_dump({"model_spec": {
        "model_params": {"objective": "binary:logistic", "learning_rate": 0.3},
        "training_params": {"num_boost_round": 6}, "test_metric": "auc"}}))
    out = gbdt_run.main(["--raw-data-path", str(tmp_path / "raw.csv"), "--data-processing-config",
                         str(tmp_path / "dp.yaml"), "--training-config", str(tmp_path / "tr.yaml"),
                         "--target-col", "label", "--output-dir", str(tmp_path / "out"), "--device", "cpu",
                         "--num-actors", "2", "--checkpoint-frequency", "2", "--max-actor-restarts", "1"])
    assert out["num_trees"] == 6 and out["elastic"]["final_actors"] == [0, 1]
    assert out["test_metric"]["auc"] > 0.75
    assert (tmp_path / "out" / "checkpoints" / "latest").exists()
