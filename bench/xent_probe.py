"""Fused MLM cross-entropy kernel on the BERT-large shape (19456 masked rows x 30720 padded
vocabulary, bf16 logits, gradient in place): time per call.

    python bench/xent_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from cloudtik_amd import ops
    C = ops.require_native()
    R, V, ld = 19456, 30522, 30720
    logits = (3 * torch.randn(R, ld, device="cuda")).bfloat16()
    labels = torch.randint(0, V, (R,), device="cuda")
    scale = torch.tensor([1.0 / R], device="cuda")
    bufs = [logits.clone() for _ in range(3)]
    for b in bufs:
        C.xent_fwd(b, b, V, labels, scale, -100, 0.0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for i in range(15):
        b = bufs[i % 3]
        C.xent_fwd(b, b, V, labels, scale, -100, 0.0)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 15 * 1e3
    gb = 2 * R * ld * 2 / 1e9
    print(json.dumps({"rows": R, "ld": ld, "us": round(us, 1), "GB_moved_once": round(gb, 2),
                      "TBs_if_read_once": round(gb / us * 1e3, 2),
                      "reg_kernel": os.environ.get("CLOUDTIK_AMD_XENT_REG", "1") != "0"}), flush=True)


if __name__ == "__main__":
    main()
