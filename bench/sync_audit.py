"""List the host<->GPU synchronisation points of one training step (torch sync debug mode).

    python bench/sync_audit.py --model maskrcnn

Every sync stalls the host until the GPU queue drains, so a launch-bound step (thousands of
small kernels) loses its run-ahead at each one.  Prints one line per distinct call site.
"""
import argparse
import collections
import os
import sys
import traceback
import warnings

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="maskrcnn")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--size", type=int, default=800)
    a = ap.parse_args()
    from cloudtik_amd.models.detection import mask_rcnn_resnet50_fpn, synthetic_detection_batch
    from cloudtik_amd.train.optim import build_optimizer
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = mask_rcnn_resnet50_fpn(81, device=dev)
    imgs, tg = synthetic_detection_batch(a.batch, a.size, 81, 8, device=dev)
    opt = build_optimizer("sgd", m, 0.01, 1e-4, momentum=0.9)

    def step():
        loss = sum(m(imgs, tg).values())
        loss.backward()
        opt.step()
        opt.zero_grad()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    sites = collections.Counter()

    def hook(message, category, filename, lineno, file=None, line=None):
        stack = [f for f in traceback.extract_stack()[:-1] if "cloudtik_amd" in f.filename or "bench" in f.filename]
        where = " <- ".join(f"{os.path.relpath(f.filename)}:{f.lineno}" for f in reversed(stack[-3:]))
        sites[where] += 1

    old = warnings.showwarning
    warnings.showwarning = hook
    warnings.simplefilter("always")
    torch.cuda.set_sync_debug_mode("warn")
    step()
    torch.cuda.set_sync_debug_mode(0)
    warnings.showwarning = old
    print(f"{sum(sites.values())} synchronising calls in one step at {len(sites)} sites")
    for where, n in sites.most_common():
        print(f"{n:4d}  {where}")


if __name__ == "__main__":
    main()
