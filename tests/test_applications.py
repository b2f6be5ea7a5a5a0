"""Applications: disease prediction (vision + NLP ensemble) end to end on a
small synthetic patient set."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_disease_prediction_pipeline(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "applications", "disease_prediction", "train.py"),
                        "--patients", "300", "--epochs", "2", "--output-dir", str(tmp_path)],
                       capture_output=True, text=True, timeout=600, env=dict(os.environ, CUDA_VISIBLE_DEVICES=""))
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert 0.0 <= res["ensemble_f1"] <= 1.0 and len(res["text_weights"]) == 3
    assert res["vision_f1"] > 0.4                      # learnable signal
    assert (tmp_path / "consult-model.csv").read_text().startswith("class,text_weight")
    pred = json.loads((tmp_path / "predictions.json").read_text())
    assert len(pred["predicted"]) == res["test_patients"]
