// Bindings for deformable convolution / deformable PS RoI pooling (deform.hip).  Every
// index the kernels dereference is validated here first (shapes, group divisibility,
// RoI batch indices, pooled channel ranges).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

extern "C" {
int ct_dcn_im2col(const void*, const float*, const float*, void*, int, const int*, hipStream_t);
int ct_dcn_col2im(const float*, const float*, const float*, float*, const int*, hipStream_t);
int ct_dcn_col2coord(const float*, const void*, const float*, const float*, float*, float*, int, const int*,
                     hipStream_t);
int ct_psroi_fwd(const float*, const float*, const float*, float*, float*, const int*, float, float, hipStream_t);
int ct_psroi_bwd(const float*, const float*, const float*, const float*, const float*, float*, float*, const int*,
                 float, float, hipStream_t);
}

namespace {

#define DCHECK(x) TORCH_CHECK((x).is_cuda() && (x).is_contiguous(), #x " must be a contiguous GPU tensor")
#define DDT(x, d) TORCH_CHECK((x).scalar_type() == (d), #x " has the wrong dtype")

hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

struct Geom {
  int v[15];
};

// input [B, C, H, W]; offset [B, dg*2*kh*kw, Ho, Wo]; mask [B, dg*kh*kw, Ho, Wo]
Geom geometry(const at::Tensor& input, const at::Tensor& offset, const c10::optional<at::Tensor>& mask,
              std::vector<int64_t> k, std::vector<int64_t> s, std::vector<int64_t> p, std::vector<int64_t> d,
              int64_t dg) {
  TORCH_CHECK(k.size() == 2 && s.size() == 2 && p.size() == 2 && d.size() == 2, "dcn: 2-D kernel/stride/pad/dil");
  TORCH_CHECK(input.dim() == 4 && offset.dim() == 4, "dcn: input and offset must be 4-D");
  const int B = input.size(0), C = input.size(1), H = input.size(2), W = input.size(3);
  const int kh = k[0], kw = k[1];
  const int Ho = (H + 2 * p[0] - (d[0] * (kh - 1) + 1)) / s[0] + 1;
  const int Wo = (W + 2 * p[1] - (d[1] * (kw - 1) + 1)) / s[1] + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "dcn: empty output");
  TORCH_CHECK(dg >= 1 && C % dg == 0, "dcn: channels must divide into deformable groups");
  TORCH_CHECK(offset.size(0) == B && offset.size(1) == dg * 2 * kh * kw && offset.size(2) == Ho && offset.size(3) == Wo,
              "dcn: offset must be [B, dg*2*kh*kw, Ho, Wo]");
  if (mask.has_value()) {
    TORCH_CHECK(mask->dim() == 4 && mask->size(0) == B && mask->size(1) == dg * kh * kw && mask->size(2) == Ho &&
                    mask->size(3) == Wo, "dcn: mask must be [B, dg*kh*kw, Ho, Wo]");
    DCHECK(*mask);
    DDT(*mask, at::kFloat);
  }
  DCHECK(input); DCHECK(offset); DDT(offset, at::kFloat);
  Geom g{{B, C, H, W, Ho, Wo, kh, kw, (int)s[0], (int)s[1], (int)p[0], (int)p[1], (int)d[0], (int)d[1], (int)dg}};
  return g;
}

int dt_of(const at::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, "dcn: fp32 or bf16 input");
  return t.scalar_type() == at::kFloat ? 0 : 1;
}

at::Tensor dcn_im2col(at::Tensor input, at::Tensor offset, c10::optional<at::Tensor> mask, std::vector<int64_t> k,
                      std::vector<int64_t> s, std::vector<int64_t> p, std::vector<int64_t> d, int64_t dg) {
  Geom g = geometry(input, offset, mask, k, s, p, d, dg);
  const int B = g.v[0], C = g.v[1], Ho = g.v[4], Wo = g.v[5], K = g.v[6] * g.v[7];
  auto col = at::empty({(long)C * K, (long)B * Ho * Wo}, input.options());
  int rc = ct_dcn_im2col(input.data_ptr(), offset.data_ptr<float>(), mask ? mask->data_ptr<float>() : nullptr,
                         col.data_ptr(), dt_of(input), g.v, stream());
  TORCH_CHECK(rc == 0, "ct_dcn_im2col failed: ", rc);
  return col;
}

at::Tensor dcn_col2im(at::Tensor gcol, at::Tensor input, at::Tensor offset, c10::optional<at::Tensor> mask,
                      std::vector<int64_t> k, std::vector<int64_t> s, std::vector<int64_t> p, std::vector<int64_t> d,
                      int64_t dg) {
  Geom g = geometry(input, offset, mask, k, s, p, d, dg);
  DCHECK(gcol); DDT(gcol, at::kFloat);
  const long K = g.v[6] * g.v[7];
  TORCH_CHECK(gcol.dim() == 2 && gcol.size(0) == g.v[1] * K && gcol.size(1) == (long)g.v[0] * g.v[4] * g.v[5],
              "dcn: grad columns shape");
  auto gim = at::zeros(input.sizes(), input.options().dtype(at::kFloat));
  int rc = ct_dcn_col2im(gcol.data_ptr<float>(), offset.data_ptr<float>(), mask ? mask->data_ptr<float>() : nullptr,
                         gim.data_ptr<float>(), g.v, stream());
  TORCH_CHECK(rc == 0, "ct_dcn_col2im failed: ", rc);
  return gim;
}

std::vector<at::Tensor> dcn_col2coord(at::Tensor gcol, at::Tensor input, at::Tensor offset,
                                      c10::optional<at::Tensor> mask, std::vector<int64_t> k, std::vector<int64_t> s,
                                      std::vector<int64_t> p, std::vector<int64_t> d, int64_t dg) {
  Geom g = geometry(input, offset, mask, k, s, p, d, dg);
  DCHECK(gcol); DDT(gcol, at::kFloat);
  const long K = g.v[6] * g.v[7];
  TORCH_CHECK(gcol.dim() == 2 && gcol.size(0) == g.v[1] * K && gcol.size(1) == (long)g.v[0] * g.v[4] * g.v[5],
              "dcn: grad columns shape");
  auto goff = at::empty(offset.sizes(), offset.options());
  at::Tensor gmask;
  if (mask) gmask = at::empty(mask->sizes(), mask->options());
  int rc = ct_dcn_col2coord(gcol.data_ptr<float>(), input.data_ptr(), offset.data_ptr<float>(),
                            mask ? mask->data_ptr<float>() : nullptr, goff.data_ptr<float>(),
                            mask ? gmask.data_ptr<float>() : nullptr, dt_of(input), g.v, stream());
  TORCH_CHECK(rc == 0, "ct_dcn_col2coord failed: ", rc);
  return {goff, mask ? gmask : at::Tensor()};
}

std::vector<int> psroi_geom(const at::Tensor& data, const at::Tensor& rois, const c10::optional<at::Tensor>& trans,
                            int64_t out_dim, int64_t group, int64_t pooled, int64_t part, int64_t spp) {
  DCHECK(data); DCHECK(rois); DDT(data, at::kFloat); DDT(rois, at::kFloat);
  TORCH_CHECK(data.dim() == 4 && rois.dim() == 2 && rois.size(1) == 5, "psroi: data [N,C,H,W], rois [K,5]");
  TORCH_CHECK(group >= 1 && pooled >= 1 && part >= 1 && spp >= 1 && out_dim >= 1, "psroi: positive sizes");
  TORCH_CHECK(data.size(1) >= out_dim * group * group, "psroi: data needs out_dim * group_size^2 channels");
  const int K = rois.size(0);
  if (K > 0) {
    auto bi = rois.select(1, 0);
    TORCH_CHECK(bi.min().item<float>() >= 0 && bi.max().item<float>() < data.size(0),
                "psroi: roi batch index out of range");
  }
  int nc = 1, no_trans = 1;
  if (trans.has_value() && trans->numel() > 0) {
    DCHECK(*trans); DDT(*trans, at::kFloat);
    TORCH_CHECK(trans->dim() == 4 && trans->size(0) == K && trans->size(1) % 2 == 0 && trans->size(2) == part &&
                    trans->size(3) == part, "psroi: trans must be [K, 2*num_classes, part, part]");
    nc = trans->size(1) / 2;
    TORCH_CHECK(nc >= 1 && out_dim % nc == 0, "psroi: output_dim must split evenly across classes");
    no_trans = 0;
  }
  return {(int)data.size(1), (int)data.size(2), (int)data.size(3), K, (int)out_dim, (int)group, (int)pooled,
          (int)part, (int)spp, nc, no_trans};
}

std::vector<at::Tensor> psroi_fwd(at::Tensor data, at::Tensor rois, c10::optional<at::Tensor> trans,
                                  double scale, int64_t out_dim, int64_t group, int64_t pooled, int64_t part,
                                  int64_t spp, double trans_std) {
  auto gi = psroi_geom(data, rois, trans, out_dim, group, pooled, part, spp);
  auto out = at::empty({rois.size(0), out_dim, pooled, pooled}, data.options());
  auto cnt = at::empty_like(out);
  const float* tp = gi[10] ? nullptr : trans->data_ptr<float>();
  int rc = ct_psroi_fwd(data.data_ptr<float>(), rois.data_ptr<float>(), tp, out.data_ptr<float>(),
                        cnt.data_ptr<float>(), gi.data(), (float)scale, (float)trans_std, stream());
  TORCH_CHECK(rc == 0, "ct_psroi_fwd failed: ", rc);
  return {out, cnt};
}

std::vector<at::Tensor> psroi_bwd(at::Tensor gout, at::Tensor data, at::Tensor rois, c10::optional<at::Tensor> trans,
                                  at::Tensor count, double scale, int64_t out_dim, int64_t group, int64_t pooled,
                                  int64_t part, int64_t spp, double trans_std) {
  auto gi = psroi_geom(data, rois, trans, out_dim, group, pooled, part, spp);
  DCHECK(gout); DCHECK(count);
  TORCH_CHECK(gout.sizes() == count.sizes() && gout.size(0) == rois.size(0) && gout.size(1) == out_dim,
              "psroi: grad shape");
  auto gdata = at::zeros_like(data);
  at::Tensor gtrans = gi[10] ? at::Tensor() : at::zeros_like(*trans);
  const float* tp = gi[10] ? nullptr : trans->data_ptr<float>();
  int rc = ct_psroi_bwd(gout.data_ptr<float>(), data.data_ptr<float>(), rois.data_ptr<float>(), tp,
                        count.data_ptr<float>(), gdata.data_ptr<float>(), gi[10] ? nullptr : gtrans.data_ptr<float>(),
                        gi.data(), (float)scale, (float)trans_std, stream());
  TORCH_CHECK(rc == 0, "ct_psroi_bwd failed: ", rc);
  return {gdata, gtrans};
}

}  // namespace

void register_deform(pybind11::module& m) {
  m.def("dcn_im2col", &dcn_im2col);
  m.def("dcn_col2im", &dcn_col2im);
  m.def("dcn_col2coord", &dcn_col2coord);
  m.def("psroi_fwd", &psroi_fwd);
  m.def("psroi_bwd", &psroi_bwd);
}
