"""Do the bench's library GEMMs hit the committed TunableOp table?  Times the BERT-large
decoder (MLM head) and forward projection GEMMs as bench.py issues them, with the tuned table
(private copy, tuning off -- bench.py's `--tunableop use`) and with TunableOp off, and prints
which table keys the run looked up.

    python bench/tunableop_probe.py"""
import json
import os
import shutil
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    import torch.cuda.tunable as tn
    import torch.nn.functional as F
    from bench import TUNE_FILE
    mode = sys.argv[1] if len(sys.argv) > 1 else "use"
    if mode == "use":
        fd, path = tempfile.mkstemp(suffix=".csv")
        os.close(fd)
        shutil.copyfile(TUNE_FILE, path)
        tn.enable(True)
        tn.set_filename(path)
        tn.tuning_enable(False)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    out = {"mode": mode}
    x = torch.randn(19456, 1024, device=dev, generator=g).to(bf)
    W = torch.randn(30720, 1024, device=dev, generator=g).to(bf) * 0.02
    b = torch.zeros(30720, device=dev, dtype=bf)
    out["decoder_fwd_us"] = round(timeit(lambda: F.linear(x, W, b)), 1)
    d = torch.randn(19456, 30720, device=dev, generator=g).to(bf)
    out["decoder_dgrad_us"] = round(timeit(lambda: torch.matmul(d, W)), 1)
    t = torch.randn(32768, 1024, device=dev, generator=g).to(bf)
    Wq = torch.randn(3072, 1024, device=dev, generator=g).to(bf) * 0.02
    bq = torch.zeros(3072, device=dev, dtype=bf)
    out["qkv_fwd_us"] = round(timeit(lambda: torch.addmm(bq, t, Wq.t())), 1)
    Wo = torch.randn(1024, 1024, device=dev, generator=g).to(bf) * 0.02
    out["wo_fwd_us"] = round(timeit(lambda: torch.mm(t, Wo.t())), 1)
    h = torch.randn(32768, 4096, device=dev, generator=g).to(bf)
    W2 = torch.randn(1024, 4096, device=dev, generator=g).to(bf) * 0.02
    out["ffn2_fwd_us"] = round(timeit(lambda: torch.mm(h, W2.t())), 1)
    if mode == "use":
        res = tn.get_results() or []
        out["table_hits"] = len(res)
        out["keys"] = sorted({f"{r[0]}:{r[1]}" for r in res})[:40]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
