"""Readiness protocol of the data-parallel bucketer on the real BERT blocks (GPU kernels,
weight-gradient side stream on).  A bucket is all-reduced the moment its last parameter
reports ready, so a bucket launched before every member's gradient has landed would reduce a
partial gradient on every rank.  The check runs at world size 1 with the bucketer's own hooks
installed and its launch replaced by a recorder: every bucket must launch exactly once during
backward, and the bucket's gradient slice at launch time (ordered after both streams) must
equal the slice after backward.

The fused paths accumulate straight into the flat buffer and report through
``_ct_grad_ready``; autograd then still runs the parameter's post-accumulate hook, so every such
parameter reports twice (the first probe of this test) -- the bucketer counts one report per
parameter per backward."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bert(bucket_mb):
    from cloudtik_amd import ops
    from cloudtik_amd.models.bert import BertConfig, BertForPreTraining, synthetic_pretraining_batch
    from cloudtik_amd.parallel import GradBucketer
    from cloudtik_amd.train.optim import FlatParamSpace

    dev = torch.device("cuda", 0)
    torch.manual_seed(5)
    ops.manual_seed(5)
    cfg = BertConfig.tiny(hidden_size=256, num_attention_heads=4, intermediate_size=1024)
    model = BertForPreTraining(cfg, device=dev, dtype=torch.bfloat16)
    named = list(model.named_parameters())
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    ddp = GradBucketer(space, bucket_mb=bucket_mb)
    batch = synthetic_pretraining_batch(cfg, 8, 128, 20, device=dev, generator=torch.Generator().manual_seed(1))
    return model, named, space, ddp, batch


@pytest.mark.parametrize("bucket_mb", [0.25, 2.0, 64.0])
def test_buckets_launch_once_with_final_gradients(bucket_mb):
    model, named, space, ddp, batch = _bert(bucket_mb)
    launched = {}

    def record(b):
        torch.cuda.synchronize()                      # both streams: what the bucket holds NOW
        lo, hi, _ = ddp.buckets[b]
        launched.setdefault(b, []).append(space.grad[lo:hi].clone())

    ddp._launch = record
    ddp._register_hooks()
    try:
        for _ in range(2):                            # second step: bookkeeping reset by finish()
            launched.clear()
            model(**batch).backward()
            torch.cuda.synchronize()
            space.flush_grads()
            torch.cuda.synchronize()
            bad = []
            for b, (lo, hi, mem) in enumerate(ddp.buckets):
                got = launched.get(b, [])
                if len(got) != 1:
                    bad.append(f"bucket {b}: launched {len(got)} times")
                elif not torch.equal(got[0], space.grad[lo:hi]):
                    names = [space.names[i] for i in mem]
                    bad.append(f"bucket {b} ({names[:3]}...): launched before its gradients were final")
            assert not bad, "\n".join(bad)
            ddp.finish()
            space.zero_grad()
    finally:
        ddp.remove()


@pytest.mark.parametrize("bucket_mb", [0.25, 8.0])
def test_resnet_buckets_launch_once_with_final_gradients(bucket_mb):
    """The same on the ResNet path: conv weight gradients added into the flat buffer on the
    side stream or deferred until flush_grads(), BN affine gradients from fused kernels."""
    import torch.nn.functional as F
    from cloudtik_amd.models.resnet import resnet18_like_small
    from cloudtik_amd.parallel import GradBucketer
    from cloudtik_amd.train.optim import FlatParamSpace

    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    model = resnet18_like_small(device=dev)
    model.train()
    named = list(model.named_parameters())
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    ddp = GradBucketer(space, bucket_mb=bucket_mb)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(4, 3, 32, 32, generator=g).to(device=dev, dtype=next(model.parameters()).dtype)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (4,), generator=g).to(dev)
    launched = {}

    def record(b):
        space.flush_grads()                           # what _launch does before the collective
        torch.cuda.synchronize()
        lo, hi, _ = ddp.buckets[b]
        launched.setdefault(b, []).append(space.grad[lo:hi].clone())

    ddp._launch = record
    ddp._register_hooks()
    try:
        for _ in range(2):
            launched.clear()
            F.cross_entropy(model(x).float(), y).backward()
            space.flush_grads()
            torch.cuda.synchronize()
            bad = []
            for b, (lo, hi, mem) in enumerate(ddp.buckets):
                got = launched.get(b, [])
                if len(got) != 1:
                    bad.append(f"bucket {b}: launched {len(got)} times")
                elif not torch.equal(got[0], space.grad[lo:hi]):
                    bad.append(f"bucket {b} ({[space.names[i] for i in mem][:3]}...): launched early")
            assert not bad, "\n".join(bad)
            ddp.finish()
            space.zero_grad()
    finally:
        ddp.remove()
