"""LayerNorm forward (with / without the saved input sum) and backward (from the saved sum /
from the output y, csrc/layernorm.hip FROMY) on the BERT-large shape: 32768 x 1024 bf16, bias +
residual + dropout 0.1, dgamma / dbeta / dbias accumulated.  Median of interleaved rounds.

    python bench/ln_from_y_probe.py [--rounds 5] [--iters 20]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--p", type=float, default=0.1, help="hidden dropout probability")
    a = ap.parse_args()
    from cloudtik_amd import ops
    C = ops.require_native()
    dev = torch.device("cuda")
    M, N, p = 32768, 1024, a.p
    g = torch.Generator(device="cpu").manual_seed(0)
    mk = lambda *sh: torch.randn(*sh, generator=g).to(dev, torch.bfloat16)  # noqa: E731
    x, res, dy = mk(M, N), mk(M, N), mk(M, N)
    bias, gam, beta = mk(N) * 0.1, 1 + 0.1 * mk(N), 0.1 * mk(N)
    y, s, mean, rstd = C.layernorm_fwd(x, bias, res, gam, beta, 1e-12, False, p, 1, 0, keep_sum=True)
    dg, db, dbias = (torch.zeros(N, device=dev) for _ in range(3))
    fns = {
        "fwd_sum": lambda: C.layernorm_fwd(x, bias, res, gam, beta, 1e-12, False, p, 1, 0, keep_sum=True),
        "fwd_nosum": lambda: C.layernorm_fwd(x, bias, res, gam, beta, 1e-12, False, p, 1, 0, keep_sum=False),
        "bwd_sum": lambda: C.layernorm_bwd_into(dy, s, gam, mean, rstd, False, dg, db, dbias, True, p, 1, 0),
        "bwd_y": lambda: C.layernorm_bwd_into(dy, y, gam, mean, rstd, False, dg, db, dbias, True, p, 1, 0,
                                             beta_y=beta),
    }
    for f in fns.values():
        f()
    times = {k: [] for k in fns}
    for _ in range(a.rounds):
        for k, f in fns.items():
            times[k].append(timeit(f, a.iters))
    print(json.dumps({k: round(statistics.median(v), 1) for k, v in times.items()}), flush=True)


if __name__ == "__main__":
    main()
