"""Mask R-CNN training-step timing with / without the flat-buffer optimizer."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
from cloudtik_amd.models.detection import mask_rcnn_resnet50_fpn, synthetic_detection_batch
from cloudtik_amd.train.optim import build_optimizer
dev = torch.device("cuda")
torch.manual_seed(0)
m = mask_rcnn_resnet50_fpn(81, device=dev)
imgs, tg = synthetic_detection_batch(4, 800, 81, 8, device=dev)


def run(tag, opt=None, n=3):
    for i in range(n):
        torch.cuda.synchronize(); t = time.perf_counter()
        loss = sum(m(imgs, tg).values())
        torch.cuda.synchronize(); t1 = time.perf_counter()
        loss.backward()
        torch.cuda.synchronize(); t2 = time.perf_counter()
        if opt is not None:
            opt.step(); opt.zero_grad()
        else:
            m.zero_grad(set_to_none=True)
        torch.cuda.synchronize(); t3 = time.perf_counter()
        print(f"{tag} step {i}: fwd {(t1-t)*1e3:.1f} bwd {(t2-t1)*1e3:.1f} opt {(t3-t2)*1e3:.1f} ms", flush=True)


run("plain")
w = m.backbone.fpn.output[0].weight
print("before opt: fpn weight CL", w.is_contiguous(memory_format=torch.channels_last), flush=True)
opt = build_optimizer("sgd", m, 0.01, 1e-4, momentum=0.9)
g = w.grad if w.grad is not None else getattr(w, "_ct_flat_view", None)   # flat-buffer view
print("after opt: fpn weight CL", w.is_contiguous(memory_format=torch.channels_last),
      "grad CL", None if g is None else g.is_contiguous(memory_format=torch.channels_last), flush=True)
run("flat-opt", opt, n=8)
