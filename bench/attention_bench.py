"""Microbenchmark: fused MFMA attention (fwd, fwd+bwd) vs PyTorch SDPA on BERT shapes."""
import argparse, json, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloudtik_amd import ops

def timeit(fn, iters=20, warm=5):
    for _ in range(warm): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / iters * 1e3

ap = argparse.ArgumentParser(); ap.add_argument("--B", type=int, default=256); ap.add_argument("--S", type=int, default=128)
ap.add_argument("--H", type=int, default=16); a = ap.parse_args()
B, S, H, D = a.B, a.S, a.H, 64
dev = torch.device("cuda")
qkv = (torch.randn(B, S, 3 * H * D, device=dev) * 0.5).bfloat16().requires_grad_()
kb = torch.zeros(B, S, device=dev)
do = torch.randn(B, S, H * D, device=dev).bfloat16()
fl_f = 4 * B * H * S * S * D
res = {}
for p in (0.0, 0.1):
    f = lambda: ops.attention_packed(qkv, H, kb, p=p, training=True)
    res[f"ours_fwd_p{p}"] = timeit(f)
    def fb():
        o = ops.attention_packed(qkv, H, kb, p=p, training=True); o.backward(do)
    res[f"ours_fwdbwd_p{p}"] = timeit(fb)
q, k, v = [t.detach().view(B, S, H, D).transpose(1, 2).contiguous().requires_grad_() for t in qkv.view(B, S, 3, H * D).unbind(2)]
dos = do.view(B, S, H, D).transpose(1, 2).contiguous()
for p in (0.0, 0.1):
    f = lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, dropout_p=p)
    try:
        res[f"sdpa_fwd_p{p}"] = timeit(f)
        def fb():
            o = torch.nn.functional.scaled_dot_product_attention(q, k, v, dropout_p=p); o.backward(dos)
        res[f"sdpa_fwdbwd_p{p}"] = timeit(fb)
    except Exception as e:
        res[f"sdpa_p{p}"] = str(e)[:100]
out = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}
for k, v in list(out.items()):
    if isinstance(v, float):
        fl = fl_f if "fwd_" in k and "fwdbwd" not in k else 3.5 * fl_f
        out[k + "_TFLOPs"] = round(fl / (v * 1e-3) / 1e12, 1)
print(json.dumps(out))
