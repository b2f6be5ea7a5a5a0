"""Would the LAMB update hide behind the next step's forward?  BERT-large at the bench config:
times (HIP events) the forward alone, the fused LAMB step alone, and the two issued together on
two streams (the LAMB on a side stream, the forward on the main one), each averaged over K.

    python bench/overlap_probe.py [--steps 5]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    from cloudtik_amd.models.bert import BertConfig, BertForPreTraining, synthetic_pretraining_batch
    from cloudtik_amd.train.optim import FlatParamSpace, FusedLAMB
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = BertConfig.large()
    model = BertForPreTraining(cfg, device=dev, dtype=torch.bfloat16)
    named = list(model.named_parameters())
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    opt = FusedLAMB(space, lr=3.5e-4, weight_decay=0.01, no_decay=BertForPreTraining.no_decay)
    batch = synthetic_pretraining_batch(cfg, 256, 128, 76, device=dev)
    side = torch.cuda.Stream()

    def fwd():
        with torch.no_grad():
            model(**batch)

    def lamb():
        opt.step()

    def timeit(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(a.steps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.steps

    def both():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            lamb()
        fwd()
        torch.cuda.current_stream().wait_stream(side)

    loss = model(**batch)
    loss.backward()                       # gradients for the optimizer to chew on
    torch.cuda.synchronize()
    t_f, t_l, t_b = timeit(fwd), timeit(lamb), timeit(both)
    print(json.dumps({"forward_ms": round(t_f, 3), "lamb_ms": round(t_l, 3), "together_ms": round(t_b, 3),
                      "hidden_ms": round(t_f + t_l - t_b, 3)}), flush=True)


if __name__ == "__main__":
    main()
