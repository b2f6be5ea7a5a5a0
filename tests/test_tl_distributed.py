"""Transfer-learning distributed launch from the model API (modeling/transfer_learning/
distributed.py; reference image_classification_model.py:250, common/pytorch/model.py:217-237):
``train(..., distributed=True, nproc_per_node=2)`` launches 2 gloo ranks through cloudtik-run,
trains data-parallel, and loads the trained weights + history back into the calling model."""
import os

import torch

from cloudtik_amd.modeling.transfer_learning import synthetic_image_dataset
from cloudtik_amd.modeling.transfer_learning.image_classification import ImageClassificationModel


def test_image_model_trains_distributed_with_two_gloo_ranks(tmp_path, monkeypatch):
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    monkeypatch.setenv("PYTHONPATH", repo + os.pathsep + os.environ.get("PYTHONPATH", ""))
    torch.manual_seed(0)
    m = ImageClassificationModel("resnet_tiny", num_classes=2, device="cpu", freeze_backbone=True)
    before_fc = m.model.fc.weight.detach().clone()
    before_conv = m.model.conv1.weight.detach().clone()
    ds = synthetic_image_dataset(32, 2, image_size=32, seed=1)
    hist = m.train(ds, epochs=2, batch_size=4, lr=0.05, distributed=True, nproc_per_node=2,
                   shared_dir=str(tmp_path), launcher="local")
    assert len(hist) == 2 and all("loss" in h for h in hist)
    assert not torch.equal(m.model.fc.weight, before_fc)            # trained weights came back
    assert torch.equal(m.model.conv1.weight, before_conv)           # the frozen backbone stayed frozen
    (job,) = [d for d in os.listdir(tmp_path) if d.startswith("tl_job_")]
    assert {"model", "trained", "history.json", "job.json", "datasets.pkl"} <= set(os.listdir(tmp_path / job))


def test_run_command_api_launches_every_rank(tmp_path, monkeypatch):
    from cloudtik_amd.runner import run_command
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    monkeypatch.setenv("PYTHONPATH", repo)
    script = tmp_path / "w.py"
    script.write_text("import os\nopen(os.path.join(%r, 'r' + os.environ['RANK']), 'w').write(os.environ['WORLD_SIZE'])\n"
                      % str(tmp_path))
    assert run_command(["python", str(script)], nproc_per_node=3, launcher="local", no_python=True) == 0
    assert sorted(p.name for p in tmp_path.iterdir() if p.name.startswith("r")) == ["r0", "r1", "r2"]
    assert (tmp_path / "r2").read_text() == "3"


def test_multi_host_job_without_shared_dir_is_refused_up_front():
    """A job whose ranks land on other hosts cannot read a local temp dir: refused before
    anything is exported or launched (advisor r4)."""
    import pytest
    from cloudtik_amd.modeling.transfer_learning.distributed import fit_distributed, spans_hosts
    assert not spans_hosts(1, None, None) and not spans_hosts(1, "localhost:2", None)
    assert spans_hosts(2, None, None) and spans_hosts(1, "10.0.0.1:4,10.0.0.2:4", None)
    with pytest.raises(ValueError, match="shared_dir"):
        fit_distributed(object(), [], {}, nnodes=2, nproc_per_node=1)
