"""hipBLASLt fused-epilogue GEMMs vs GEMM + separate HIP elementwise kernel on the BERT-large
FFN shapes (tokens 32768, hidden 1024, ffn 4096).

    python bench/lt_epilogue_probe.py [--tokens 32768]

Prints one JSON line per case: time of the unfused pair, time of the fused call, numerics of
the fused call against an fp32 reference (erf GELU)."""
import argparse
import json
import math

import torch

GELU_AUX_BIAS, DGELU_BGRAD, DEFAULT, BIAS, BGRADB = 164, 208, 1, 4, 512


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3       # us


def gelu_ref(x):
    return 0.5 * x * (1 + torch.erf(x / math.sqrt(2)))


def gelu_grad_ref(x):
    return 0.5 * (1 + torch.erf(x / math.sqrt(2))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    a = ap.parse_args()
    from cloudtik_amd import ops
    C = ops.require_native()
    M, H, F = a.tokens, 1024, 4096
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    x2 = torch.randn(M, H, device=dev, dtype=bf, generator=g)
    W1 = (torch.randn(F, H, device=dev, generator=g) * 0.03).to(bf)
    b1 = (torch.randn(F, device=dev, generator=g) * 0.1).to(bf)
    W2 = (torch.randn(H, F, device=dev, generator=g) * 0.03).to(bf)
    df = torch.randn(M, H, device=dev, dtype=bf, generator=g)
    flops_f = 2 * M * H * F

    # ---- plain GEMM: torch (maybe TunableOp) vs lt heuristic
    zt = torch.empty(M, F, device=dev, dtype=bf)
    t_mm = timeit(lambda: torch.mm(x2, W1.t(), out=zt))
    ok = C.lt_matmul(x2, W1, zt, False, True, 1.0, 0.0, None, DEFAULT, None, None)
    t_lt = timeit(lambda: C.lt_matmul(x2, W1, zt, False, True, 1.0, 0.0, None, DEFAULT, None, None)) if ok else None
    zr = torch.mm(x2, W1.t())
    err = (zt.float() - zr.float()).abs().max().item() if ok else None
    print(json.dumps({"case": "fwd_plain", "torch_us": t_mm, "lt_us": t_lt, "lt_ok": ok, "max_abs_vs_torch": err,
                      "torch_tflops": flops_f / t_mm / 1e6}), flush=True)

    # ---- forward: z = x W1^T; h = gelu(z + b1)
    def unfused_fwd():
        z = torch.mm(x2, W1.t())
        return z, C.bias_act_fwd(z, b1, 1)
    t_u = timeit(unfused_fwd)
    h = torch.empty(M, F, device=dev, dtype=bf)
    aux = torch.empty(M, F, device=dev, dtype=bf)
    ok = C.lt_matmul(x2, W1, h, False, True, 1.0, 0.0, None, GELU_AUX_BIAS, b1, aux)
    rec = {"case": "fwd_gelu_aux_bias", "unfused_us": t_u, "lt_ok": ok}
    if ok:
        rec["fused_us"] = timeit(lambda: C.lt_matmul(x2, W1, h, False, True, 1.0, 0.0, None, GELU_AUX_BIAS, b1, aux))
        zb = x2.float() @ W1.float().t() + b1.float()
        rec["aux_max_abs"] = (aux.float() - zb).abs().max().item()
        rec["h_max_abs_vs_erf_gelu"] = (h.float() - gelu_ref(zb)).abs().max().item()
        rec["h_unfused_max_abs_vs_erf_gelu"] = (unfused_fwd()[1].float() - gelu_ref(zb)).abs().max().item()
    print(json.dumps(rec), flush=True)

    # ---- backward: dh = df W2; dz = dh * gelu'(z + b1); db1 = colsum(dz)
    z = torch.mm(x2, W1.t())
    zb_bf = (z.float() + b1.float()).to(bf)
    db = torch.zeros(F, device=dev, dtype=torch.float32)

    def unfused_bwd():
        dh = torch.mm(df, W2)
        return C.bias_act_bwd_into(dh, z, b1, 1, db, True)
    t_u = timeit(unfused_bwd)
    rec = {"case": "bwd_dgelu_bgrad", "unfused_us": t_u}
    for bdt in (torch.float32, torch.bfloat16):
        dz = torch.empty(M, F, device=dev, dtype=bf)
        dbl = torch.zeros(F, device=dev, dtype=bdt)
        key = "f32" if bdt == torch.float32 else "bf16"
        try:
            ok = C.lt_matmul(df, W2, dz, False, False, 1.0, 0.0, None, DGELU_BGRAD, dbl, zb_bf)
        except RuntimeError as e:
            ok, rec[f"err_{key}"] = False, str(e)[:200]
        rec[f"lt_ok_{key}"] = ok
        if ok:
            rec[f"fused_us_{key}"] = timeit(
                lambda: C.lt_matmul(df, W2, dz, False, False, 1.0, 0.0, None, DGELU_BGRAD, dbl, zb_bf))
            dh32 = df.float() @ W2.float()
            dz_ref = dh32 * gelu_grad_ref(zb_bf.float())
            rec[f"dz_max_abs_{key}"] = (dz.float() - dz_ref).abs().max().item()
            rec[f"dz_ref_absmax"] = dz_ref.abs().max().item()
            rec[f"db_max_rel_{key}"] = ((dbl.float() - dz_ref.sum(0)).abs().max() / dz_ref.sum(0).abs().max()).item()
    dz_u = unfused_bwd()
    dz_ref = (df.float() @ W2.float()) * gelu_grad_ref(zb_bf.float())
    rec["dz_unfused_max_abs"] = (dz_u.float() - dz_ref).abs().max().item()
    print(json.dumps(rec), flush=True)

    # ---- QKV dgrad + bias-grad: wgrad with BGRADB (dW = dqkv^T x2, db = colsum(dqkv))
    dqkv = torch.randn(M, 3 * H, device=dev, dtype=bf, generator=g)
    dW = torch.empty(3 * H, H, device=dev, dtype=bf)
    dbq = torch.zeros(3 * H, device=dev, dtype=torch.float32)
    rec = {"case": "wgrad_bgrad"}
    from cloudtik_amd.ops.linear import wgrad_accumulate
    gacc = torch.zeros(3 * H, H, device=dev, dtype=bf)

    def unfused_wg():
        C.bias_act_bwd_into(dqkv, dqkv, None, 0, dbq, False)
        wgrad_accumulate(gacc, dqkv, x2)
    rec["unfused_us"] = timeit(unfused_wg)
    for epi, name in ((BGRADB, "bgradb"), (256, "bgrada")):
        try:
            ok = C.lt_matmul(dqkv, x2, dW, True, False, 1.0, 0.0, None, epi, dbq, None)
        except RuntimeError as e:
            ok, rec[f"err_{name}"] = False, str(e)[:200]
        rec[f"ok_{name}"] = ok
        if ok:
            rec[f"fused_us_{name}"] = timeit(lambda: C.lt_matmul(dqkv, x2, dW, True, False, 1.0, 0.0, None, epi,
                                                                 dbq, None))
            ref = dqkv.float().sum(0)
            rec[f"db_max_rel_{name}"] = ((dbq - ref).abs().max() / ref.abs().max()).item()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
