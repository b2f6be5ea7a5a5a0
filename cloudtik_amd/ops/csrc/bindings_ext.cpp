// Bindings for RoPE, EmbeddingBag / interaction, detection ops and multi-tensor copy.
// Host-side shape / dtype / alignment validation happens here, before any launch.
#include <torch/extension.h>
#include <cstring>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

extern "C" {
int ct_rope(const void*, void*, long, long, int, const void*, void*, long, long, int, const float*, const float*,
            const int64_t*, int, long, int, int, int, hipStream_t);
int ct_embbag_fwd(const float*, const int64_t*, const int64_t*, const int64_t*, const float*, void*, int, int, int,
                  int, int, hipStream_t);
int ct_embbag_bwd(const void*, int, float*, float*, const int64_t*, const int64_t*, const int64_t*, const float*,
                  float*, int, int, int, int, float, hipStream_t);
int ct_interact_fwd(const void*, const void*, void*, int, int, int, int, hipStream_t);
int ct_interact_bwd(const void*, const void*, const void*, void*, void*, int, int, int, int, hipStream_t);
int ct_nms(const float*, int, float, float, uint64_t*, int64_t*, int64_t*, hipStream_t);
int ct_nms_segmented(const float*, const int64_t*, const int64_t*, int, int, float, float, uint64_t*, uint8_t*,
                     hipStream_t);
int ct_roi_align_fwd(const void*, const float*, void*, int, int, int, int, int, int, int, float, int, int, hipStream_t);
int ct_roi_align_bwd(const void*, const float*, float*, int, int, int, int, int, int, int, float, int, int, hipStream_t);
int ct_roi_align_nhwc_fwd(const void* const*, const int*, const float*, int, const int*, const float*, void*, int, int,
                          int, int, int, int, int, hipStream_t);
int ct_roi_align_nhwc_bwd(const void*, float* const*, const int*, const float*, int, const int*, const float*, int, int,
                          int, int, int, int, int, hipStream_t);
int ct_roi_pool_fwd(const void*, const float*, void*, int*, int, int, int, int, int, int, int, float, hipStream_t);
int ct_roi_pool_bwd(const void*, const float*, const int*, float*, int, int, int, int, int, int, int, hipStream_t);
int ct_focal_fwd(const void*, const int64_t*, float*, int, long, int, float, float, hipStream_t);
int ct_focal_bwd(const void*, const int64_t*, const float*, void*, int, long, int, float, float, hipStream_t);
int ct_rnnt_fwd(const void*, int, const int*, const int*, const int*, float*, float*, float*, float*, float*, int, int,
                int, int, int, hipStream_t);
int ct_rnnt_bwd(const void*, int, const int*, const int*, const int*, const float*, const float*, const float*,
                const float*, const float*, const float*, void*, int, int, int, int, int, hipStream_t);
int ct_mt_copy(const uint64_t*, const int64_t*, const int64_t*, int, long, void*, int, int, float, int, hipStream_t);
int ct_mt_add(const int64_t*, int, int, hipStream_t);
void* ct_loader_create(int, const void* const*, const long*, long, int, int, uint64_t, int, int, int, int, int, int);
long ct_loader_num_batches(void*);
void ct_loader_set_epoch(void*, long);
long ct_loader_next_device(void*, void* const*, hipStream_t, hipStream_t);
long ct_loader_next_host(void*, void* const*);
void ct_loader_destroy(void*);
int ct_image_u8_to_bf16(const uint8_t*, void*, const uint8_t*, int, int, int, const float*, const float*, hipStream_t);
}

namespace {

#define XCHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define XCHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define XCHECK_IN(x) do { XCHECK_CUDA(x); XCHECK_CONTIG(x); } while (0)
#define XCHECK_DT(x, d) TORCH_CHECK((x).scalar_type() == (d), #x " has the wrong dtype")

hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

int fb(const at::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, "expected fp32 or bf16");
  return t.scalar_type() == at::kFloat ? 0 : 1;
}

// ---------------------------------------------------------------- RoPE
// q: [T, Hq, D] view (token/head strides arbitrary, unit stride in D); k likewise (optional)
void rope(at::Tensor q, c10::optional<at::Tensor> k, at::Tensor cos, at::Tensor sin,
          c10::optional<at::Tensor> positions, int64_t seq_len, bool neox, bool backward) {
  XCHECK_CUDA(q);
  XCHECK_DT(q, at::kBFloat16);
  TORCH_CHECK(q.dim() == 3 && q.stride(2) == 1, "rope: q must be [T, H, D] with unit stride in D");
  const long T = q.size(0);
  const int D = (int)q.size(2);
  TORCH_CHECK(D % 8 == 0, "rope: head dim must be a multiple of 8");
  XCHECK_IN(cos); XCHECK_IN(sin); XCHECK_DT(cos, at::kFloat); XCHECK_DT(sin, at::kFloat);
  TORCH_CHECK(cos.dim() == 2 && cos.size(1) == D / 2 && sin.sizes() == cos.sizes(), "rope: cos/sin must be [P, D/2]");
  const int align = neox ? 4 : 8;
  TORCH_CHECK(q.stride(0) % align == 0 && q.stride(1) % align == 0, "rope: q strides must keep vector alignment");
  const void* kp = nullptr;
  long kt = 0, kh = 0;
  int hk = 0;
  if (k.has_value() && k->defined()) {
    XCHECK_CUDA(*k);
    XCHECK_DT(*k, at::kBFloat16);
    TORCH_CHECK(k->dim() == 3 && k->size(0) == T && k->size(2) == D && k->stride(2) == 1, "rope: k must be [T, Hk, D]");
    TORCH_CHECK(k->stride(0) % align == 0 && k->stride(1) % align == 0, "rope: k strides must keep vector alignment");
    kp = k->data_ptr(); kt = k->stride(0); kh = k->stride(1); hk = (int)k->size(1);
  }
  const int64_t* pp = nullptr;
  if (positions.has_value() && positions->defined()) {
    XCHECK_IN(*positions);
    XCHECK_DT(*positions, at::kLong);
    TORCH_CHECK(positions->numel() == T, "rope: one position per token");
    pp = positions->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(seq_len > 0 && seq_len <= cos.size(0), "rope: seq_len must be in (0, P]");
  }
  const int rc = ct_rope(q.data_ptr(), q.data_ptr(), q.stride(0), q.stride(1), (int)q.size(1), kp, (void*)kp, kt, kh, hk,
                         cos.data_ptr<float>(), sin.data_ptr<float>(), pp, (int)seq_len, T, D, neox ? 1 : 0,
                         backward ? 1 : 0, stream());
  TORCH_CHECK(rc == 0, "rope launch failed");
}

// ---------------------------------------------------------------- EmbeddingBag
at::Tensor embbag_fwd(at::Tensor W, at::Tensor row_base, at::Tensor idx, at::Tensor offs,
                      c10::optional<at::Tensor> psw, int64_t B, bool mean, bool bf16_out) {
  XCHECK_IN(W); XCHECK_DT(W, at::kFloat); XCHECK_IN(row_base); XCHECK_IN(idx); XCHECK_IN(offs);
  XCHECK_DT(idx, at::kLong); XCHECK_DT(offs, at::kLong); XCHECK_DT(row_base, at::kLong);
  const int T = (int)row_base.numel(), E = (int)W.size(1);
  TORCH_CHECK(offs.numel() == (long)T * B + 1, "embbag: offsets must have T*B+1 entries");
  const float* pw = nullptr;
  if (psw.has_value() && psw->defined()) {
    XCHECK_IN(*psw); XCHECK_DT(*psw, at::kFloat);
    TORCH_CHECK(psw->numel() == idx.numel());
    pw = psw->data_ptr<float>();
  }
  auto out = at::empty({B, T, E}, W.options().dtype(bf16_out ? at::kBFloat16 : at::kFloat));
  ct_embbag_fwd(W.data_ptr<float>(), row_base.data_ptr<int64_t>(), idx.data_ptr<int64_t>(), offs.data_ptr<int64_t>(),
                pw, out.data_ptr(), bf16_out ? 1 : 0, T, (int)B, E, mean ? 1 : 0, stream());
  return out;
}

// lr != 0: SGD-update W in place (sparse rows);  otherwise accumulate into dW
void embbag_bwd(at::Tensor gout, at::Tensor W, c10::optional<at::Tensor> dW, at::Tensor row_base, at::Tensor idx,
                at::Tensor offs, c10::optional<at::Tensor> psw, c10::optional<at::Tensor> dpsw, bool mean, double lr) {
  XCHECK_IN(gout); XCHECK_IN(W); XCHECK_DT(W, at::kFloat);
  const int T = (int)row_base.numel(), E = (int)W.size(1);
  TORCH_CHECK(gout.dim() == 3 && gout.size(1) == T && gout.size(2) == E, "embbag_bwd: gout must be [B, T, E]");
  const int B = (int)gout.size(0);
  TORCH_CHECK(offs.numel() == (long)T * B + 1);
  float* dwp = nullptr;
  if (dW.has_value() && dW->defined()) {
    XCHECK_IN(*dW); XCHECK_DT(*dW, at::kFloat);
    TORCH_CHECK(dW->sizes() == W.sizes());
    dwp = dW->data_ptr<float>();
  } else {
    TORCH_CHECK(lr != 0.0, "embbag_bwd: need dW or a learning rate");
  }
  const float* pw = (psw.has_value() && psw->defined()) ? psw->data_ptr<float>() : nullptr;
  float* dpw = (dpsw.has_value() && dpsw->defined()) ? dpsw->data_ptr<float>() : nullptr;
  ct_embbag_bwd(gout.data_ptr(), fb(gout), W.data_ptr<float>(), dwp, row_base.data_ptr<int64_t>(),
                idx.data_ptr<int64_t>(), offs.data_ptr<int64_t>(), pw, dpw, T, B, E, mean ? 1 : 0, (float)lr, stream());
}

at::Tensor interact_fwd(at::Tensor x, at::Tensor emb) {
  XCHECK_IN(x); XCHECK_IN(emb);
  TORCH_CHECK(x.dim() == 2 && emb.dim() == 3 && emb.size(0) == x.size(0) && emb.size(2) == x.size(1),
              "interact: x [B, E], emb [B, T, E]");
  TORCH_CHECK(x.scalar_type() == emb.scalar_type());
  const int B = (int)x.size(0), E = (int)x.size(1), T = (int)emb.size(1), F = T + 1;
  auto out = at::empty({B, E + F * (F - 1) / 2}, x.options());
  const int rc = ct_interact_fwd(x.data_ptr(), emb.data_ptr(), out.data_ptr(), fb(x), B, T, E, stream());
  TORCH_CHECK(rc == 0, "interact_fwd: too many features for LDS");
  return out;
}

std::vector<at::Tensor> interact_bwd(at::Tensor gout, at::Tensor x, at::Tensor emb) {
  XCHECK_IN(gout); XCHECK_IN(x); XCHECK_IN(emb);
  const int B = (int)x.size(0), E = (int)x.size(1), T = (int)emb.size(1), F = T + 1;
  TORCH_CHECK(gout.size(0) == B && gout.size(1) == E + F * (F - 1) / 2 && gout.scalar_type() == x.scalar_type());
  auto dx = at::empty_like(x);
  auto demb = at::empty_like(emb);
  const int rc = ct_interact_bwd(gout.data_ptr(), x.data_ptr(), emb.data_ptr(), dx.data_ptr(), demb.data_ptr(), fb(x),
                                 B, T, E, stream());
  TORCH_CHECK(rc == 0, "interact_bwd: too many features for LDS");
  return {dx, demb};
}

// ---------------------------------------------------------------- detection
// boxes must be sorted by descending score; returns kept indices (into the sorted boxes)
at::Tensor nms_sorted(at::Tensor boxes, double thr, double offset) {
  XCHECK_IN(boxes); XCHECK_DT(boxes, at::kFloat);
  TORCH_CHECK(boxes.dim() == 2 && boxes.size(1) == 4, "nms: boxes must be [N, 4]");
  const int n = (int)boxes.size(0);
  auto lo = boxes.options().dtype(at::kLong);
  if (n == 0) return at::empty({0}, lo);
  TORCH_CHECK(n <= 524288, "nms: at most 524288 boxes");
  const int cb = (n + 63) / 64;
  auto mask = at::empty({(long)n * cb}, lo);
  auto keep = at::empty({n}, lo);
  auto nkeep = at::empty({1}, lo);
  const int rc = ct_nms(boxes.data_ptr<float>(), n, (float)thr, (float)offset, (uint64_t*)mask.data_ptr<int64_t>(),
                        keep.data_ptr<int64_t>(), nkeep.data_ptr<int64_t>(), stream());
  TORCH_CHECK(rc == 0, "nms launch failed");
  return keep.narrow(0, 0, nkeep.item<int64_t>());
}

// many NMS problems in one launch: boxes sorted by (segment, score desc), segment s owning
// rows [seg_offsets[s], seg_offsets[s+1]) (host int64).  Returns uint8 keep flags per row.
at::Tensor nms_segmented(at::Tensor boxes, at::Tensor seg_offsets, double thr, double offset) {
  XCHECK_IN(boxes); XCHECK_DT(boxes, at::kFloat);
  TORCH_CHECK(boxes.dim() == 2 && boxes.size(1) == 4, "nms: boxes must be [N, 4]");
  TORCH_CHECK(!seg_offsets.is_cuda() && seg_offsets.scalar_type() == at::kLong && seg_offsets.dim() == 1 &&
                  seg_offsets.is_contiguous(), "nms_segmented: seg_offsets must be a contiguous host int64 vector");
  const long nseg = seg_offsets.numel() - 1;
  const long N = boxes.size(0);
  auto keep = at::zeros({N}, boxes.options().dtype(at::kByte));
  if (nseg <= 0 || N == 0) return keep;
  const int64_t* so = seg_offsets.data_ptr<int64_t>();
  TORCH_CHECK(so[0] == 0 && so[nseg] == N, "nms_segmented: offsets must span the boxes");
  TORCH_CHECK(nseg <= 65535, "nms_segmented: at most 65535 segments");
  auto moff = at::empty({nseg}, seg_offsets.options());
  int64_t* mo = moff.data_ptr<int64_t>();
  long total = 0, max_n = 0;
  for (long s = 0; s < nseg; ++s) {
    const long n = so[s + 1] - so[s];
    TORCH_CHECK(n >= 0, "nms_segmented: offsets must be non-decreasing");
    mo[s] = total;
    total += n * ((n + 63) / 64);
    max_n = std::max(max_n, n);
  }
  TORCH_CHECK(max_n <= 524288, "nms: at most 524288 boxes per segment");
  if (max_n == 0) return keep;
  auto seg_d = seg_offsets.to(boxes.device());
  auto moff_d = moff.to(boxes.device());
  auto mask = at::empty({std::max(total, 1L)}, boxes.options().dtype(at::kLong));
  const int rc = ct_nms_segmented(boxes.data_ptr<float>(), seg_d.data_ptr<int64_t>(), moff_d.data_ptr<int64_t>(),
                                  (int)nseg, (int)max_n, (float)thr, (float)offset,
                                  (uint64_t*)mask.data_ptr<int64_t>(), keep.data_ptr<uint8_t>(), stream());
  TORCH_CHECK(rc == 0, "nms_segmented launch failed (", rc, ")");
  return keep;
}

// ---------------------------------------------------------------- weight-gradient GEMM
// out[M, N] (+)= A[T, M]^T B[T, N] (bf16 operands, fp32 accumulation).  mode 0: out is fp32
// [splits, M, N] partials; 1: bf16 out += result; 2: bf16 out = result.  Returns false (and
// launches nothing) for shapes the kernel does not tile (M, N % 256, T % (64 * splits)).

void check_rois(const at::Tensor& feat, const at::Tensor& rois) {
  XCHECK_IN(feat); XCHECK_IN(rois); XCHECK_DT(rois, at::kFloat);
  TORCH_CHECK(feat.dim() == 4, "features must be NCHW");
  TORCH_CHECK(rois.dim() == 2 && rois.size(1) == 5, "rois must be [K, 5] (batch, x1, y1, x2, y2)");
}

at::Tensor roi_align_fwd(at::Tensor feat, at::Tensor rois, double scale, int64_t PH, int64_t PW, int64_t sr, bool aligned) {
  check_rois(feat, rois);
  const int K = (int)rois.size(0), C = (int)feat.size(1), H = (int)feat.size(2), W = (int)feat.size(3);
  auto out = at::empty({K, C, PH, PW}, feat.options());
  if (K) ct_roi_align_fwd(feat.data_ptr(), rois.data_ptr<float>(), out.data_ptr(), fb(feat), K, C, H, W, (int)PH, (int)PW,
                          (float)scale, (int)sr, aligned ? 1 : 0, stream());
  return out;
}

at::Tensor roi_align_bwd(at::Tensor gout, at::Tensor rois, std::vector<int64_t> fshape, double scale, int64_t sr, bool aligned) {
  XCHECK_IN(gout); XCHECK_IN(rois);
  TORCH_CHECK(fshape.size() == 4);
  const int K = (int)rois.size(0), C = (int)fshape[1], H = (int)fshape[2], W = (int)fshape[3];
  TORCH_CHECK(gout.dim() == 4 && gout.size(0) == K && gout.size(1) == C);
  auto g = at::zeros(fshape, gout.options().dtype(at::kFloat));
  if (K) ct_roi_align_bwd(gout.data_ptr(), rois.data_ptr<float>(), g.data_ptr<float>(), fb(gout), K, C, H, W,
                          (int)gout.size(2), (int)gout.size(3), (float)scale, (int)sr, aligned ? 1 : 0, stream());
  return gout.scalar_type() == at::kFloat ? g : g.to(gout.scalar_type());
}

// channels_last feature maps [N, C, H_l, W_l] (NHWC in memory; one per pyramid level) ->
// channels_last [K, C, PH, PW].  ``lvl`` [K] int32 picks each RoI's level (undefined when
// there is one level).  All levels in one launch.
void check_levels(const std::vector<at::Tensor>& feats, const at::Tensor& rois, const c10::optional<at::Tensor>& lvl,
                  const std::vector<double>& scales) {
  TORCH_CHECK(!feats.empty() && feats.size() <= 5 && scales.size() == feats.size(), "roi_align_nhwc: 1-5 levels");
  XCHECK_IN(rois); XCHECK_DT(rois, at::kFloat);
  TORCH_CHECK(rois.dim() == 2 && rois.size(1) == 5, "rois must be [K, 5]");
  TORCH_CHECK(feats.size() == 1 || (lvl.has_value() && lvl->defined()), "roi_align_nhwc: levels need lvl");
  if (lvl.has_value() && lvl->defined()) {
    XCHECK_IN(*lvl); XCHECK_DT(*lvl, at::kInt);
    TORCH_CHECK(lvl->numel() == rois.size(0), "roi_align_nhwc: one level per RoI");
  }
}

at::Tensor roi_align_nhwc_fwd(std::vector<at::Tensor> feats, at::Tensor rois, c10::optional<at::Tensor> lvl,
                              std::vector<double> scales, int64_t PH, int64_t PW, int64_t sr, bool aligned) {
  check_levels(feats, rois, lvl, scales);
  const auto& f0 = feats[0];
  const int K = (int)rois.size(0), C = (int)f0.size(1);
  TORCH_CHECK(C % 8 == 0, "roi_align_nhwc: channels must be a multiple of 8");
  std::vector<const void*> ptrs;
  std::vector<int> hw;
  std::vector<float> sc;
  for (size_t l = 0; l < feats.size(); ++l) {
    const auto& f = feats[l];
    TORCH_CHECK(f.is_cuda() && f.dim() == 4 && f.is_contiguous(at::MemoryFormat::ChannelsLast),
                "roi_align_nhwc: features must be channels_last");
    TORCH_CHECK(f.size(0) == f0.size(0) && f.size(1) == C && f.scalar_type() == f0.scalar_type(),
                "roi_align_nhwc: levels must share batch, channels and dtype");
    ptrs.push_back(f.data_ptr());
    hw.push_back((int)f.size(2)); hw.push_back((int)f.size(3));
    sc.push_back((float)scales[l]);
  }
  auto out = at::empty({K, C, PH, PW}, f0.options(), at::MemoryFormat::ChannelsLast);
  const int* lp = (lvl.has_value() && lvl->defined()) ? lvl->data_ptr<int>() : nullptr;
  if (K) TORCH_CHECK(ct_roi_align_nhwc_fwd(ptrs.data(), hw.data(), sc.data(), (int)feats.size(), lp,
                                           rois.data_ptr<float>(), out.data_ptr(), fb(f0), K, C, (int)PH, (int)PW,
                                           (int)sr, aligned ? 1 : 0, stream()) == 0);
  return out;
}

// shapes: 4 ints per level.  The fp32 gradients of all levels share one zeroed buffer (one
// fill, one cast); each level is returned as a channels_last view of it in gout's dtype.
std::vector<at::Tensor> roi_align_nhwc_bwd(at::Tensor gout, at::Tensor rois, c10::optional<at::Tensor> lvl,
                                           std::vector<int64_t> shapes, std::vector<double> scales, int64_t sr,
                                           bool aligned) {
  const size_t nlev = scales.size();
  TORCH_CHECK(shapes.size() == 4 * nlev && nlev >= 1 && nlev <= 5, "roi_align_nhwc_bwd: 4 dims per level");
  XCHECK_IN(rois); XCHECK_DT(rois, at::kFloat);
  TORCH_CHECK(nlev == 1 || (lvl.has_value() && lvl->defined()), "roi_align_nhwc_bwd: levels need lvl");
  gout = gout.contiguous(at::MemoryFormat::ChannelsLast);
  const int K = (int)rois.size(0), C = (int)shapes[1];
  TORCH_CHECK(gout.dim() == 4 && gout.size(0) == K && gout.size(1) == C && C % 8 == 0);
  std::vector<int64_t> offs;
  int64_t total = 0;
  for (size_t l = 0; l < nlev; ++l) {
    TORCH_CHECK(shapes[4 * l + 1] == C && shapes[4 * l] == shapes[0], "roi_align_nhwc_bwd: level shapes");
    offs.push_back(total);
    total += shapes[4 * l] * shapes[4 * l + 1] * shapes[4 * l + 2] * shapes[4 * l + 3];
  }
  auto buf = at::zeros({total}, gout.options().dtype(at::kFloat));
  std::vector<float*> ptrs;
  std::vector<int> hw;
  std::vector<float> sc;
  for (size_t l = 0; l < nlev; ++l) {
    ptrs.push_back(buf.data_ptr<float>() + offs[l]);
    hw.push_back((int)shapes[4 * l + 2]); hw.push_back((int)shapes[4 * l + 3]);
    sc.push_back((float)scales[l]);
  }
  const int* lp = (lvl.has_value() && lvl->defined()) ? lvl->data_ptr<int>() : nullptr;
  if (K) TORCH_CHECK(ct_roi_align_nhwc_bwd(gout.data_ptr(), ptrs.data(), hw.data(), sc.data(), (int)nlev, lp,
                                           rois.data_ptr<float>(), fb(gout), K, C, (int)gout.size(2),
                                           (int)gout.size(3), (int)sr, aligned ? 1 : 0, stream()) == 0);
  if (gout.scalar_type() != at::kFloat) buf = buf.to(gout.scalar_type());
  std::vector<at::Tensor> grads;
  for (size_t l = 0; l < nlev; ++l) {
    const int64_t N = shapes[4 * l], H = shapes[4 * l + 2], W = shapes[4 * l + 3];
    grads.push_back(buf.as_strided({N, C, H, W}, {H * W * C, 1, W * C, C}, offs[l]));
  }
  return grads;
}

std::vector<at::Tensor> roi_pool_fwd(at::Tensor feat, at::Tensor rois, double scale, int64_t PH, int64_t PW) {
  check_rois(feat, rois);
  const int K = (int)rois.size(0), C = (int)feat.size(1), H = (int)feat.size(2), W = (int)feat.size(3);
  auto out = at::empty({K, C, PH, PW}, feat.options());
  auto arg = at::empty({K, C, PH, PW}, feat.options().dtype(at::kInt));
  if (K) ct_roi_pool_fwd(feat.data_ptr(), rois.data_ptr<float>(), out.data_ptr(), arg.data_ptr<int>(), fb(feat), K, C, H,
                         W, (int)PH, (int)PW, (float)scale, stream());
  return {out, arg};
}

at::Tensor roi_pool_bwd(at::Tensor gout, at::Tensor rois, at::Tensor argmax, std::vector<int64_t> fshape) {
  XCHECK_IN(gout); XCHECK_IN(rois); XCHECK_IN(argmax);
  TORCH_CHECK(argmax.sizes() == gout.sizes());
  const int K = (int)rois.size(0), C = (int)fshape[1], H = (int)fshape[2], W = (int)fshape[3];
  auto g = at::zeros(fshape, gout.options().dtype(at::kFloat));
  if (K) ct_roi_pool_bwd(gout.data_ptr(), rois.data_ptr<float>(), argmax.data_ptr<int>(), g.data_ptr<float>(), fb(gout),
                         K, C, H, W, (int)gout.size(2), (int)gout.size(3), stream());
  return gout.scalar_type() == at::kFloat ? g : g.to(gout.scalar_type());
}

at::Tensor focal_fwd(at::Tensor logits, at::Tensor targets, double gamma, double alpha) {
  XCHECK_IN(logits); XCHECK_IN(targets); XCHECK_DT(targets, at::kLong);
  TORCH_CHECK(logits.dim() == 2 && targets.numel() == logits.size(0));
  auto loss = at::empty(logits.sizes(), logits.options().dtype(at::kFloat));
  ct_focal_fwd(logits.data_ptr(), targets.data_ptr<int64_t>(), loss.data_ptr<float>(), fb(logits), logits.size(0),
               (int)logits.size(1), (float)gamma, (float)alpha, stream());
  return loss;
}

at::Tensor focal_bwd(at::Tensor logits, at::Tensor targets, at::Tensor gloss, double gamma, double alpha) {
  XCHECK_IN(logits); XCHECK_IN(targets); XCHECK_IN(gloss); XCHECK_DT(gloss, at::kFloat);
  TORCH_CHECK(gloss.sizes() == logits.sizes());
  auto g = at::empty_like(logits);
  ct_focal_bwd(logits.data_ptr(), targets.data_ptr<int64_t>(), gloss.data_ptr<float>(), g.data_ptr(), fb(logits),
               logits.size(0), (int)logits.size(1), (float)gamma, (float)alpha, stream());
  return g;
}

// ---------------------------------------------------------------- RNN-T loss
// logits [B, T, U+1, V] (bf16/fp32), labels [B, U] int32, lengths int32 -> (loglik [B], state)
std::vector<at::Tensor> rnnt_fwd(at::Tensor logits, at::Tensor labels, at::Tensor tlen, at::Tensor ulen, int64_t blank) {
  XCHECK_IN(logits); XCHECK_IN(labels); XCHECK_IN(tlen); XCHECK_IN(ulen);
  XCHECK_DT(labels, at::kInt); XCHECK_DT(tlen, at::kInt); XCHECK_DT(ulen, at::kInt);
  TORCH_CHECK(logits.dim() == 4, "rnnt: logits must be [B, T, U+1, V]");
  const int B = (int)logits.size(0), Tm = (int)logits.size(1), U1 = (int)logits.size(2), V = (int)logits.size(3);
  TORCH_CHECK(labels.dim() == 2 && labels.size(0) == B && labels.size(1) == U1 - 1, "rnnt: labels must be [B, U]");
  TORCH_CHECK(tlen.numel() == B && ulen.numel() == B);
  TORCH_CHECK(blank >= 0 && blank < V, "rnnt: blank out of range");
  // lengths must fit the padded lattice (checked on the host: a bad length would index out of bounds)
  auto tl = tlen.cpu(), ul = ulen.cpu();
  for (int b = 0; b < B; ++b) {
    const int t = tl.data_ptr<int>()[b], u = ul.data_ptr<int>()[b];
    TORCH_CHECK(t >= 1 && t <= Tm && u >= 0 && u <= U1 - 1, "rnnt: length out of range for utterance ", b);
  }
  auto f = logits.options().dtype(at::kFloat);
  const long rows = (long)B * Tm * U1;
  auto lse = at::empty({rows}, f), lp = at::empty({rows, 2}, f);
  auto alpha = at::empty({B, Tm, U1}, f), beta = at::empty({B, Tm, U1}, f), loglik = at::empty({B}, f);
  const int rc = ct_rnnt_fwd(logits.data_ptr(), fb(logits), labels.data_ptr<int>(), tlen.data_ptr<int>(),
                             ulen.data_ptr<int>(), lse.data_ptr<float>(), lp.data_ptr<float>(), alpha.data_ptr<float>(),
                             beta.data_ptr<float>(), loglik.data_ptr<float>(), B, Tm, U1, V, (int)blank, stream());
  TORCH_CHECK(rc == 0, "rnnt_fwd failed (", rc, ")");
  return {loglik, lse, lp, alpha, beta};
}

at::Tensor rnnt_bwd(at::Tensor logits, at::Tensor labels, at::Tensor tlen, at::Tensor ulen, at::Tensor lse,
                    at::Tensor lp, at::Tensor alpha, at::Tensor beta, at::Tensor loglik, at::Tensor gloss,
                    int64_t blank) {
  XCHECK_IN(logits); XCHECK_IN(gloss); XCHECK_DT(gloss, at::kFloat);
  const int B = (int)logits.size(0), Tm = (int)logits.size(1), U1 = (int)logits.size(2), V = (int)logits.size(3);
  TORCH_CHECK(gloss.numel() == B);
  auto grad = at::empty_like(logits);
  const int rc = ct_rnnt_bwd(logits.data_ptr(), fb(logits), labels.data_ptr<int>(), tlen.data_ptr<int>(),
                             ulen.data_ptr<int>(), lse.data_ptr<float>(), lp.data_ptr<float>(), alpha.data_ptr<float>(),
                             beta.data_ptr<float>(), loglik.data_ptr<float>(), gloss.data_ptr<float>(), grad.data_ptr(),
                             B, Tm, U1, V, (int)blank, stream());
  TORCH_CHECK(rc == 0, "rnnt_bwd failed (", rc, ")");
  return grad;
}

// ---------------------------------------------------------------- multi-tensor copy
// pack (unpack=false): flat[offs[t]:...] = scale * tensors[t];  unpack: tensors[t] = scale * flat[...]
void mt_copy(std::vector<at::Tensor> tensors, at::Tensor flat, double scale, bool unpack) {
  XCHECK_IN(flat);
  if (tensors.empty()) return;
  const auto dt = tensors[0].scalar_type();
  std::vector<int64_t> ptrs, sizes, offs;
  long off = 0, mx = 0;
  for (auto& t : tensors) {
    XCHECK_IN(t);
    TORCH_CHECK(t.scalar_type() == dt, "mt_copy: all tensors must share a dtype");
    ptrs.push_back((int64_t)(uintptr_t)t.data_ptr());
    sizes.push_back(t.numel());
    offs.push_back(off);
    off += t.numel();
    mx = std::max<long>(mx, t.numel());
  }
  TORCH_CHECK(flat.numel() >= off, "mt_copy: flat buffer too small");
  auto meta = at::tensor(ptrs, at::kLong);
  meta = at::cat({meta, at::tensor(sizes, at::kLong), at::tensor(offs, at::kLong)}).to(flat.device(), /*non_blocking=*/true);
  const int n = (int)tensors.size();
  const int rc = ct_mt_copy((const uint64_t*)meta.data_ptr<int64_t>(), meta.data_ptr<int64_t>() + n,
                            meta.data_ptr<int64_t>() + 2 * n, n, mx, flat.data_ptr(), fb(tensors[0]), fb(flat),
                            (float)scale, unpack ? 1 : 0, stream());
  TORCH_CHECK(rc == 0, "mt_copy: too many tensors");
}

// dsts[t] += srcs[t] (same dtype, same strides, dense) for all t in one launch: chunks of
// 64K elements, table (src, dst, n) per chunk staged through pinned memory
void mt_add_(std::vector<at::Tensor> srcs, std::vector<at::Tensor> dsts) {
  TORCH_CHECK(srcs.size() == dsts.size(), "mt_add_: list lengths differ");
  if (srcs.empty()) return;
  const auto dt = srcs[0].scalar_type();
  TORCH_CHECK(dt == at::kFloat || dt == at::kBFloat16, "mt_add_: fp32 / bf16");
  constexpr long CH = 65536;
  std::vector<int64_t> tab;
  for (size_t t = 0; t < srcs.size(); ++t) {
    auto& a = srcs[t];
    auto& b = dsts[t];
    TORCH_CHECK(a.is_cuda() && b.is_cuda(), "mt_add_: GPU tensors");
    TORCH_CHECK(a.scalar_type() == dt && b.scalar_type() == dt, "mt_add_: mixed dtypes");
    bool same = a.sizes() == b.sizes();
    for (int64_t d = 0; same && d < a.dim(); ++d)
      if (a.size(d) > 1 && a.stride(d) != b.stride(d)) same = false;     // size-1 dims: any stride
    TORCH_CHECK(same && a.is_non_overlapping_and_dense() && b.is_non_overlapping_and_dense(),
                "mt_add_: src / dst layouts differ");
    TORCH_CHECK(((uintptr_t)a.data_ptr() % 16) == 0 && ((uintptr_t)b.data_ptr() % 16) == 0, "mt_add_: alignment");
    const long n = a.numel();
    const long es = a.element_size();
    for (long o = 0; o < n; o += CH) {
      tab.push_back((int64_t)((uintptr_t)a.data_ptr() + o * es));
      tab.push_back((int64_t)((uintptr_t)b.data_ptr() + o * es));
      tab.push_back(std::min(CH, n - o));
    }
  }
  auto host = at::empty({(long)tab.size()}, at::TensorOptions().dtype(at::kLong).pinned_memory(true));
  std::memcpy(host.data_ptr<int64_t>(), tab.data(), tab.size() * sizeof(int64_t));
  auto dev = host.to(srcs[0].device(), /*non_blocking=*/true);
  const int rc = ct_mt_add(dev.data_ptr<int64_t>(), (int)(tab.size() / 3), dt == at::kFloat ? 1 : 0, stream());
  TORCH_CHECK(rc == 0, "mt_add_: too many chunks");
}

// ---------------------------------------------------------------- native loader
// cols: CPU contiguous tensors whose dim 0 is the row; the Python wrapper keeps them alive
int64_t loader_create(std::vector<at::Tensor> cols, int64_t batch, bool shuffle, int64_t seed, bool drop_last,
                      int64_t workers, int64_t slots, int64_t rank, int64_t world, bool pinned) {
  TORCH_CHECK(!cols.empty(), "loader: no columns");
  const long n = cols[0].size(0);
  std::vector<const void*> ptrs;
  std::vector<long> rb;
  for (auto& c : cols) {
    TORCH_CHECK(!c.is_cuda() && c.is_contiguous(), "loader: columns must be contiguous host tensors");
    TORCH_CHECK(c.size(0) == n, "loader: all columns need the same row count");
    ptrs.push_back(c.data_ptr());
    rb.push_back((long)(c.numel() / std::max<long>(n, 1)) * (long)c.element_size());
  }
  void* h = ct_loader_create((int)cols.size(), ptrs.data(), rb.data(), n, (int)batch, shuffle, (uint64_t)seed, drop_last,
                             (int)workers, (int)slots, (int)rank, (int)world, pinned ? 1 : 0);
  TORCH_CHECK(h != nullptr, "loader: creation failed (bad arguments or pinned allocation failed)");
  return (int64_t)(uintptr_t)h;
}

int64_t loader_num_batches(int64_t h) { return ct_loader_num_batches((void*)(uintptr_t)h); }
void loader_set_epoch(int64_t h, int64_t epoch) { ct_loader_set_epoch((void*)(uintptr_t)h, epoch); }
void loader_destroy(int64_t h) { ct_loader_destroy((void*)(uintptr_t)h); }

int64_t loader_next_device(int64_t h, std::vector<at::Tensor> outs, int64_t copy_stream) {
  std::vector<void*> ptrs;
  for (auto& t : outs) { XCHECK_IN(t); ptrs.push_back(t.data_ptr()); }
  return ct_loader_next_device((void*)(uintptr_t)h, ptrs.data(), (hipStream_t)(uintptr_t)copy_stream, stream());
}

int64_t loader_next_host(int64_t h, std::vector<at::Tensor> outs) {
  std::vector<void*> ptrs;
  for (auto& t : outs) { TORCH_CHECK(!t.is_cuda() && t.is_contiguous()); ptrs.push_back(t.data_ptr()); }
  return ct_loader_next_host((void*)(uintptr_t)h, ptrs.data());
}

}  // namespace

// images: uint8 [N, H, W, 3] contiguous -> bf16 [N, 3, H, W] channels_last; flip: optional uint8 [N]
at::Tensor image_u8_to_bf16(at::Tensor images, c10::optional<at::Tensor> flip, std::vector<double> mean,
                            std::vector<double> stdv) {
  XCHECK_IN(images);
  XCHECK_DT(images, at::kByte);
  TORCH_CHECK(images.dim() == 4 && images.size(3) == 3, "image_u8_to_bf16: images must be [N, H, W, 3]");
  TORCH_CHECK(mean.size() == 3 && stdv.size() == 3, "image_u8_to_bf16: 3 means and stds");
  const int N = (int)images.size(0), H = (int)images.size(1), W = (int)images.size(2);
  TORCH_CHECK(W % 4 == 0, "image_u8_to_bf16: width must be a multiple of 4");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(images.data_ptr()) & 3) == 0, "image_u8_to_bf16: 4-byte aligned input");
  const uint8_t* fp = nullptr;
  if (flip.has_value()) {
    XCHECK_IN(*flip);
    XCHECK_DT(*flip, at::kByte);
    TORCH_CHECK(flip->numel() == N, "image_u8_to_bf16: one flip flag per image");
    fp = flip->data_ptr<uint8_t>();
  }
  auto out = at::empty({N, H, W, 3}, images.options().dtype(at::kBFloat16));
  float m[3], s[3];
  for (int i = 0; i < 3; ++i) { m[i] = (float)mean[i]; s[i] = (float)stdv[i]; }
  int rc = ct_image_u8_to_bf16(images.data_ptr<uint8_t>(), out.data_ptr(), fp, N, H, W, m, s, stream());
  TORCH_CHECK(rc == 0, "ct_image_u8_to_bf16 failed: ", rc);
  return out.permute({0, 3, 1, 2});
}

void register_ext(pybind11::module& m) {
  m.def("image_u8_to_bf16", &image_u8_to_bf16);
  m.def("loader_create", &loader_create);
  m.def("loader_num_batches", &loader_num_batches);
  m.def("loader_set_epoch", &loader_set_epoch);
  m.def("loader_destroy", &loader_destroy);
  m.def("loader_next_device", &loader_next_device, pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("loader_next_host", &loader_next_host, pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("rope", &rope);
  m.def("embbag_fwd", &embbag_fwd);
  m.def("embbag_bwd", &embbag_bwd);
  m.def("interact_fwd", &interact_fwd);
  m.def("interact_bwd", &interact_bwd);
  m.def("nms_sorted", &nms_sorted);
  m.def("nms_segmented", &nms_segmented);
  m.def("roi_align_fwd", &roi_align_fwd);
  m.def("roi_align_bwd", &roi_align_bwd);
  m.def("roi_align_nhwc_fwd", &roi_align_nhwc_fwd);
  m.def("rnnt_fwd", &rnnt_fwd);
  m.def("rnnt_bwd", &rnnt_bwd);
  m.def("roi_align_nhwc_bwd", &roi_align_nhwc_bwd);
  m.def("roi_pool_fwd", &roi_pool_fwd);
  m.def("roi_pool_bwd", &roi_pool_bwd);
  m.def("focal_fwd", &focal_fwd);
  m.def("focal_bwd", &focal_bwd);
  m.def("mt_copy", &mt_copy);
  m.def("mt_add_", &mt_add_);
}
