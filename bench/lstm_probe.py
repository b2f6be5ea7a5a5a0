"""LSTM fwd+bwd time by dtype (bf16 -> PyTorch per-step kernels; fp16/fp32 -> MIOpen RNN)."""
import time
import torch

dev = torch.device("cuda")
B, T, I, H, L = 32, 400, 240, 1024, 2
for dt in (torch.bfloat16, torch.float16, torch.float32):
    m = torch.nn.LSTM(I, H, L, batch_first=True, device=dev, dtype=dt)
    x = torch.randn(B, T, I, device=dev, dtype=dt, requires_grad=True)
    for i in range(4):
        if i == 1:
            torch.cuda.synchronize(); t0 = time.perf_counter()
        y, _ = m(x)
        y.float().sum().backward()
    torch.cuda.synchronize()
    print(f"{dt}: {(time.perf_counter() - t0) / 3 * 1000:.1f} ms fwd+bwd", flush=True)
