// Bindings for the implicit-GEMM convolution kernels (csrc/conv.hip).  Shapes, layouts and
// alignment are validated here; the plan (row grid, taps, output addressing) comes from
// ops/conv.py.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <vector>

extern "C" {
int ct_conv_igemm(const void*, int, int, int, const void*, void*, int, int, int, int, int, int, int, int, int, int,
                  int, int, int, int, const int*, int, float*, int, hipStream_t);
int ct_conv_igemm_bn(const void*, int, int, int, const void*, void*, int, int, int, int, int, int, int, int, int, int,
                     int, int, int, int, const int*, int, int, const void*, const void*, const void*, const float*,
                     float*, long, int, hipStream_t);
int ct_conv_igemm_rows(int, int, int, int);
int ct_conv_igemm_tile_m(int);
int ct_conv_igemm_part_rows(int);
void ct_conv_stream_set_cus(int);
void ct_conv_batch_begin();
int ct_conv_batch_end(hipStream_t);
int ct_dgrad_wgather(const void*, void*, const int*, int, hipStream_t);
int ct_to_nhwc8(const void*, void*, int, int, int, int, long, long, long, long, int, hipStream_t);
int ct_bn_partials_finalize(const float*, int, int, int, int, float*, float*, hipStream_t);
int ct_conv_wgrad(const void*, const void*, int, int, int, int, int, int, int, int, int, int, const int*, float*, int,
                  int, int, hipStream_t);
int ct_conv_wgrad_cfg(int, int, int);
int ct_splitk_reduce_wide(const float*, int, long, void*, int, float*, hipStream_t);
}

// X: NHWC-dense bf16 [Nb, Hi, Wi, Ci] (any logical NCHW/NHWC view whose memory is NHWC);
// W: [Co, T*Ci] bf16 row-major; Y: bf16 memory written at the planned addresses.
// geo = {Hr, Wr, sy, sx, Ho, Wo, oys, oxs, oy0, ox0, ldy, M}; taps = {dy0, dx0, dy1, dx1, ...}.
// part (optional, fp32 [tiles, 2, Co]) receives per-tile BatchNorm (mean, M2) of Y.
bool conv_igemm(at::Tensor X, at::Tensor W, at::Tensor Y, std::vector<int64_t> geo, std::vector<int64_t> taps,
                int64_t accumulate, c10::optional<at::Tensor> part, int64_t cfg) {
  TORCH_CHECK(X.is_cuda() && W.is_cuda() && Y.is_cuda(), "conv_igemm: GPU tensors");
  TORCH_CHECK(X.scalar_type() == at::kBFloat16 && W.scalar_type() == at::kBFloat16 && Y.scalar_type() == at::kBFloat16,
              "conv_igemm: bf16 tensors");
  TORCH_CHECK(X.dim() == 4 && X.is_contiguous(at::MemoryFormat::ChannelsLast), "conv_igemm: X must be NHWC-dense");
  TORCH_CHECK(W.dim() == 2 && W.is_contiguous(), "conv_igemm: W must be [Co, T*Ci] row-major");
  TORCH_CHECK(geo.size() == 12 && taps.size() % 2 == 0, "conv_igemm: plan");
  const int Ci = (int)X.size(1), Hi = (int)X.size(2), Wi = (int)X.size(3);
  const int T = (int)taps.size() / 2, Co = (int)W.size(0);
  const int cw = (Ci == 8 || Ci == 4) ? 64 : Ci;   // stem (pixel-chunk) modes: 64 weight columns per tap
  TORCH_CHECK(W.size(1) == (int64_t)T * cw, "conv_igemm: W columns != taps * Ci");
  const long M = geo[11];
  // every output address the plan produces must lie inside Y (checked on the host before launch)
  const long Nb = X.size(0);
  TORCH_CHECK(M > 0 && M <= Nb * geo[0] * geo[1], "conv_igemm: rows exceed the row grid");
  const long last_y = (geo[0] - 1) * geo[6] + geo[8], last_x = (geo[1] - 1) * geo[7] + geo[9];
  TORCH_CHECK(geo[8] >= 0 && geo[9] >= 0 && last_y < geo[4] && last_x < geo[5], "conv_igemm: output grid");
  TORCH_CHECK((((Nb - 1) * geo[4] + last_y) * geo[5] + last_x) * geo[10] + Co <= Y.numel(), "conv_igemm: Y too small");
  std::vector<int> tp(taps.begin(), taps.end());
  float* pp = nullptr;
  if (part.has_value() && part->defined()) {
    const int cfg_r = ct_conv_igemm_rows((int)cfg, Co, (int)M, T * (cw / 64));
    const int pr = ct_conv_igemm_part_rows(cfg_r);     // rows per statistics partial
    TORCH_CHECK(part->scalar_type() == at::kFloat && part->is_contiguous() &&
                part->numel() >= (M + pr - 1) / pr * 2 * Co, "conv_igemm: part buffer");
    pp = part->data_ptr<float>();
  }
  const int rc = ct_conv_igemm(X.data_ptr(), Hi, Wi, Ci, W.data_ptr(), Y.data_ptr(), (int)geo[0], (int)geo[1],
                               (int)geo[2], (int)geo[3], (int)geo[4], (int)geo[5], (int)geo[6], (int)geo[7],
                               (int)geo[8], (int)geo[9], (int)geo[10], Co, (int)M, T, tp.data(), (int)accumulate, pp,
                               (int)cfg, at::hip::getCurrentHIPStream().stream());
  return rc == 0;
}

// Data gradient feeding a BatchNorm + ReLU backward (ReLU mask read from its output bny, or
// recomputed from its input bnx): Y = the masked gradient (after the accumulate), per-tile sums
// of dy' and dy' * xhat into part rows [tile0, tile0 + tiles) and [rows + tile0, ...) (rows =
// the buffer's tile capacity).
// Returns false (nothing launched) on an unsupported configuration.
bool conv_igemm_bn(at::Tensor X, at::Tensor W, at::Tensor Y, std::vector<int64_t> geo, std::vector<int64_t> taps,
                   bool accumulate, int64_t cfg, at::Tensor bnx, c10::optional<at::Tensor> bny, at::Tensor stat,
                   at::Tensor part, int64_t tile0, int64_t rows) {
  TORCH_CHECK(X.is_cuda() && W.is_cuda() && Y.is_cuda() && bnx.is_cuda(), "conv_igemm_bn: GPU tensors");
  TORCH_CHECK(X.scalar_type() == at::kBFloat16 && W.scalar_type() == at::kBFloat16 &&
              Y.scalar_type() == at::kBFloat16 && bnx.scalar_type() == at::kBFloat16, "conv_igemm_bn: bf16 tensors");
  TORCH_CHECK(X.dim() == 4 && X.is_contiguous(at::MemoryFormat::ChannelsLast), "conv_igemm_bn: X must be NHWC-dense");
  TORCH_CHECK(W.dim() == 2 && W.is_contiguous(), "conv_igemm_bn: W must be [Co, T*Ci] row-major");
  TORCH_CHECK(geo.size() == 12 && taps.size() % 2 == 0, "conv_igemm_bn: plan");
  // the BatchNorm input must share Y's memory layout exactly (same shape, both NHWC-dense)
  TORCH_CHECK(Y.dim() == 4 && Y.is_contiguous(at::MemoryFormat::ChannelsLast) && bnx.sizes() == Y.sizes() &&
              bnx.is_contiguous(at::MemoryFormat::ChannelsLast), "conv_igemm_bn: bnx / Y layout");
  // bny: the BatchNorm output (bf16, Y's layout) or its ReLU bitmask (uint8, one byte per 8
  // channels of every pixel: Y.numel() / 8 bytes)
  const bool has_y = bny.has_value() && bny->defined();
  const bool is_mask = has_y && bny->scalar_type() == at::kByte;
  if (is_mask) {
    TORCH_CHECK(bny->is_cuda() && bny->is_contiguous() && bny->numel() * 8 == Y.numel(), "conv_igemm_bn: bny mask");
  } else if (has_y) {
    TORCH_CHECK(bny->is_cuda() && bny->scalar_type() == at::kBFloat16 && bny->sizes() == Y.sizes() &&
                bny->is_contiguous(at::MemoryFormat::ChannelsLast), "conv_igemm_bn: bny / Y layout");
  }
  const int Ci = (int)X.size(1), Hi = (int)X.size(2), Wi = (int)X.size(3);
  const int T = (int)taps.size() / 2, Co = (int)W.size(0);
  TORCH_CHECK(Ci % 64 == 0 && W.size(1) == (int64_t)T * Ci, "conv_igemm_bn: W columns != taps * Ci");
  TORCH_CHECK(Y.size(1) == Co && geo[10] == Co, "conv_igemm_bn: Y channels");
  TORCH_CHECK(stat.is_cuda() && stat.scalar_type() == at::kFloat && stat.is_contiguous() && stat.numel() == 4L * Co,
              "conv_igemm_bn: stat must be float[4 Co]");
  const long M = geo[11];
  const long Nb = X.size(0);
  TORCH_CHECK(M > 0 && M <= Nb * geo[0] * geo[1], "conv_igemm_bn: rows exceed the row grid");
  const long last_y = (geo[0] - 1) * geo[6] + geo[8], last_x = (geo[1] - 1) * geo[7] + geo[9];
  TORCH_CHECK(geo[8] >= 0 && geo[9] >= 0 && last_y < geo[4] && last_x < geo[5], "conv_igemm_bn: output grid");
  TORCH_CHECK((((Nb - 1) * geo[4] + last_y) * geo[5] + last_x) * geo[10] + Co <= Y.numel(), "conv_igemm_bn: Y too small");
  const int bm = ct_conv_igemm_tile_m(ct_conv_igemm_rows((int)cfg, Co, (int)M, T * (Ci / 64)));
  const long tiles = (M + bm - 1) / bm;
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && tile0 >= 0 &&
              tile0 + tiles <= rows && part.numel() >= 2 * rows * Co, "conv_igemm_bn: part buffer");
  std::vector<int> tp(taps.begin(), taps.end());
  const int rc = ct_conv_igemm_bn(X.data_ptr(), Hi, Wi, Ci, W.data_ptr(), Y.data_ptr(), (int)geo[0], (int)geo[1],
                                  (int)geo[2], (int)geo[3], (int)geo[4], (int)geo[5], (int)geo[6], (int)geo[7],
                                  (int)geo[8], (int)geo[9], (int)geo[10], Co, (int)M, T, tp.data(), accumulate ? 1 : 0,
                                  (int)cfg, bnx.data_ptr(), (has_y && !is_mask) ? bny->data_ptr() : nullptr,
                                  is_mask ? bny->data_ptr() : nullptr, stat.data_ptr<float>(), part.data_ptr<float>(), rows * Co,
                                  (int)tile0, at::hip::getCurrentHIPStream().stream());
  return rc == 0;
}

int64_t conv_igemm_tile_m(int64_t cfg, int64_t Co, int64_t M, int64_t KT) {
  return ct_conv_igemm_tile_m(ct_conv_igemm_rows((int)cfg, (int)Co, (int)M, (int)KT));
}

int64_t conv_igemm_part_rows(int64_t cfg, int64_t Co, int64_t M, int64_t KT) {
  return ct_conv_igemm_part_rows(ct_conv_igemm_rows((int)cfg, (int)Co, (int)M, (int)KT));
}

void bn_partials_finalize(at::Tensor part, int64_t rows_per_tile, int64_t M, at::Tensor mean, at::Tensor var) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous(), "bn_partials_finalize");
  const int C = (int)mean.numel();
  const int tiles = (int)((M + rows_per_tile - 1) / rows_per_tile);
  TORCH_CHECK(part.numel() >= (long)tiles * 2 * C && var.numel() == C && mean.scalar_type() == at::kFloat &&
              var.scalar_type() == at::kFloat && mean.is_contiguous() && var.is_contiguous(), "bn_partials_finalize");
  TORCH_CHECK(ct_bn_partials_finalize(part.data_ptr<float>(), tiles, (int)rows_per_tile, (int)M, C,
                                      mean.data_ptr<float>(), var.data_ptr<float>(),
                                      at::hip::getCurrentHIPStream().stream()) == 0, "bn_partials_finalize launch");
}

// fp32 partials P[splits, Co, T*Ci] of the weight gradient; DY: NHWC-dense [Nb, Co, Hr, Wr]
// (the conv output grid), X: NHWC-dense input.  geo = {sy, sx, rows_per_split}.
bool conv_wgrad(at::Tensor DY, at::Tensor X, at::Tensor P, std::vector<int64_t> taps, std::vector<int64_t> geo,
                int64_t splits, int64_t cfg) {
  TORCH_CHECK(DY.is_cuda() && X.is_cuda() && P.is_cuda(), "conv_wgrad: GPU tensors");
  TORCH_CHECK(DY.scalar_type() == at::kBFloat16 && X.scalar_type() == at::kBFloat16 && P.scalar_type() == at::kFloat,
              "conv_wgrad: dtypes");
  TORCH_CHECK(DY.dim() == 4 && X.dim() == 4 && DY.is_contiguous(at::MemoryFormat::ChannelsLast) &&
              X.is_contiguous(at::MemoryFormat::ChannelsLast) && P.is_contiguous(), "conv_wgrad: layouts");
  TORCH_CHECK(geo.size() == 3 && taps.size() % 2 == 0 && DY.size(0) == X.size(0), "conv_wgrad: plan");
  const int T = (int)taps.size() / 2, Ci = (int)X.size(1), Co = (int)DY.size(1);
  const long M = DY.size(0) * DY.size(2) * DY.size(3);
  TORCH_CHECK(P.numel() >= splits * (long)Co * T * ((Ci == 8 || Ci == 4) ? 64 : Ci), "conv_wgrad: partial buffer");
  std::vector<int> tp(taps.begin(), taps.end());
  const int rc = ct_conv_wgrad(DY.data_ptr(), X.data_ptr(), (int)X.size(2), (int)X.size(3), Ci, (int)DY.size(2),
                               (int)DY.size(3), (int)geo[0], (int)geo[1], Co, (int)M, T, tp.data(),
                               P.data_ptr<float>(), (int)splits, (int)geo[2], (int)cfg,
                               at::hip::getCurrentHIPStream().stream());
  return rc == 0;
}

int64_t conv_wgrad_cfg(int64_t cfg, int64_t Co, int64_t NN) { return ct_conv_wgrad_cfg((int)cfg, (int)Co, (int)NN); }

// out (bf16, n elements, contiguous) (+)= sum of the S fp32 slabs of P [S * n]
void splitk_reduce_wide(at::Tensor P, int64_t S, at::Tensor out, bool accumulate) {
  TORCH_CHECK(P.is_cuda() && P.scalar_type() == at::kFloat && P.is_contiguous(), "splitk_reduce_wide: P");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kBFloat16 && out.is_contiguous(), "splitk_reduce_wide: out");
  const long n = out.numel();
  TORCH_CHECK(P.numel() >= S * n, "splitk_reduce_wide: P too small");
  auto ws = at::empty({n + (n + 1023) / 1024 + 4}, P.options());
  TORCH_CHECK(ct_splitk_reduce_wide(P.data_ptr<float>(), (int)S, n, out.data_ptr(), accumulate ? 1 : 0,
                                    ws.data_ptr<float>(), at::hip::getCurrentHIPStream().stream()) == 0,
              "splitk_reduce_wide launch");
}

void register_conv(pybind11::module& m) {
  m.def("splitk_reduce_wide", &splitk_reduce_wide, "sum of many fp32 split-K slabs into bf16 (+=)");
  m.def("conv_wgrad", &conv_wgrad, "implicit-GEMM conv weight gradient: fp32 split-K partials");
  m.def("conv_wgrad_cfg", &conv_wgrad_cfg, "wgrad tile configuration for (Co, T*Ci)");
  m.def("conv_igemm", &conv_igemm, "implicit-GEMM NHWC convolution (MFMA), optional BatchNorm tile statistics");
  m.def("conv_igemm_bn", &conv_igemm_bn, "conv data gradient + the BatchNorm+ReLU backward reduction in its epilogue");
  m.def("to_nhwc8", [](at::Tensor x, int64_t cp) {
          TORCH_CHECK(cp == 8 || cp == 4, "to_nhwc8: 8 or 4 output channels");
          TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.size(1) <= cp,
                      "to_nhwc8: [N, C <= cp, H, W] bf16 CUDA tensor");
          const long N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
          auto y = at::empty({N, cp, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
          TORCH_CHECK(ct_to_nhwc8(x.data_ptr(), y.data_ptr(), (int)N, (int)C, (int)H, (int)W, x.stride(0), x.stride(1),
                                  x.stride(2), x.stride(3), (int)cp, at::hip::getCurrentHIPStream().stream()) == 0,
                      "to_nhwc8 launch");
          return y;
        },
        pybind11::arg("x"), pybind11::arg("cp") = 8,
        "[N, C<=cp, H, W] bf16 -> channels_last [N, cp, H, W] zero-padded (cp = 8 or 4), one pass");
  m.def("dgrad_wgather", [](at::Tensor src, at::Tensor dst, at::Tensor desc) {
          TORCH_CHECK(src.is_cuda() && dst.is_cuda() && desc.is_cuda(), "dgrad_wgather: CUDA tensors");
          TORCH_CHECK(src.scalar_type() == at::kBFloat16 && dst.scalar_type() == at::kBFloat16, "dgrad_wgather: bf16");
          TORCH_CHECK(desc.scalar_type() == at::kInt && desc.is_contiguous() && desc.dim() == 2 && desc.size(1) == 10,
                      "dgrad_wgather: desc int32 [tiles, 10]");
          TORCH_CHECK(ct_dgrad_wgather(src.data_ptr(), dst.data_ptr(), desc.data_ptr<int>(), (int)desc.size(0),
                                       at::hip::getCurrentHIPStream().stream()) == 0, "dgrad_wgather launch");
        },
        "data-gradient weight matrices of many convs by 64x64 tiled transposes (desc: 10 ints per tile)");
  m.def("conv_batch_begin", []() { ct_conv_batch_begin(); },
        "queue the following one-tile conv launches (same configuration, <= 4) for one grid");
  m.def("conv_batch_end", []() {
          const int rc = ct_conv_batch_end(at::hip::getCurrentHIPStream().stream());
          TORCH_CHECK(rc == 0, "conv_batch_end: launch failed (", rc, ")");
        },
        "launch the queued conv launches as one grid");
  m.def("conv_stream_set_cus", [](int64_t cus) { ct_conv_stream_set_cus((int)cus); },
        "streamed conv kernels: persistent workgroups = cus x per-CU count (0: the device's CUs)");
  m.def("conv_igemm_part_rows", &conv_igemm_part_rows, "rows per BatchNorm-statistics partial (EPI 1)");
  m.def("conv_igemm_tile_m", &conv_igemm_tile_m, "rows per tile of the chosen conv configuration");
  m.def("bn_partials_finalize", &bn_partials_finalize, "Chan merge of per-tile (mean, M2) -> mean, var");
}
