#!/usr/bin/env python3
"""scikit-learn model selection with concurrent trials and tracked runs (reference
examples/runtime/ai/basics/scikit-learn/iris-scikit_learn-spark-hyperopt-mlflow.py, where
Hyperopt's SparkTrials farmed the trials out to Spark executors; here the AI runtime's
trial runner runs them as parallel processes on the node).

    python examples/ai/basics/iris_sklearn_tune.py --trials 12
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))


def objective(params):
    from sklearn.datasets import load_iris
    from sklearn.model_selection import cross_val_score
    from sklearn.svm import SVC
    from sklearn.ensemble import RandomForestClassifier
    from cloudtik_amd.runtime.ai.tracking import start_run
    x, y = load_iris(return_X_y=True)
    if params["model"] == "svc":
        clf = SVC(C=params["C"], gamma="scale")
    else:
        clf = RandomForestClassifier(n_estimators=int(params["n_estimators"]), max_depth=int(params["max_depth"]),
                                     random_state=0)
    acc = float(cross_val_score(clf, x, y, cv=5).mean())
    with start_run(params.get("experiment", "iris-sklearn")) as run:
        run.log_params({k: v for k, v in params.items() if k != "experiment"})
        run.log_metric("cv_accuracy", acc)
    return {"loss": -acc, "accuracy": acc}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=12)
    ap.add_argument("--concurrent", type=int, default=4)
    ap.add_argument("--experiment", default="iris-sklearn")
    a = ap.parse_args(argv)
    from cloudtik_amd.runtime.ai.tune import choice, loguniform, tune, uniform
    space = {"model": choice(["svc", "rf"]), "C": loguniform(1e-2, 1e2), "n_estimators": uniform(10, 200),
             "max_depth": uniform(2, 8), "experiment": choice([a.experiment])}
    res = tune(objective, space, num_trials=a.trials, max_concurrent=a.concurrent)
    out = {"best_params": {k: v for k, v in res.best.params.items() if k != "experiment"},
           "best_accuracy": res.best.result["accuracy"], "trials": len(res.trials)}
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()
