// Deformable convolution (v1 / modulated v2) and deformable position-sensitive RoI pooling
// -- the DCN entry points of the Mask R-CNN op set (reference maskrcnn_benchmark/csrc/
// deform_conv.h:11-190, deform_pool.h:11-70; CUDA sources absent from the reference tree).
//
// Deformable convolution is split the MI355X way: the sampling work (bilinear gathers at
// learned offsets) is a memory-bound HIP kernel that writes the column matrix, and the
// FLOPs are one GEMM per group on hipBLASLt (MFMA) issued from the Python side.  Backward
// is the transposed GEMM, then two kernels: col2im scatters column gradients into the
// input (fp32 atomics, at most 4 corners per sample) and col2im_coord reduces over the
// channels of a deformable group for the offset / mask gradients (no atomics).
//
// Sampling uses the zero-padded bilinear rule: a sample at (h, w) outside (-1, H) x (-1, W)
// reads 0 and corners outside the image count as 0.
#include "common.h"

namespace ct {

template <typename T>
__device__ __forceinline__ float bilinear_zero(const T* __restrict__ im, int H, int W, float h, float w) {
  const int h0 = (int)floorf(h), w0 = (int)floorf(w);
  const int h1 = h0 + 1, w1 = w0 + 1;
  const float lh = h - h0, lw = w - w0, hh = 1.f - lh, hw = 1.f - lw;
  float v00 = 0.f, v01 = 0.f, v10 = 0.f, v11 = 0.f;
  if (h0 >= 0 && w0 >= 0) v00 = to_f<T>(im[h0 * W + w0]);
  if (h0 >= 0 && w1 <= W - 1) v01 = to_f<T>(im[h0 * W + w1]);
  if (h1 <= H - 1 && w0 >= 0) v10 = to_f<T>(im[h1 * W + w0]);
  if (h1 <= H - 1 && w1 <= W - 1) v11 = to_f<T>(im[h1 * W + w1]);
  return hh * hw * v00 + hh * lw * v01 + lh * hw * v10 + lh * lw * v11;
}

__device__ __forceinline__ bool in_range(float h, float w, int H, int W) {
  return h > -1.f && w > -1.f && h < (float)H && w < (float)W;
}

struct DcnGeom {
  int B, C, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, dh, dw, dg;
};

// columns [C * kh * kw, B * Ho * Wo]; offset [B, dg * 2 * kh * kw, Ho, Wo]; mask [B, dg * kh * kw, Ho, Wo]
template <typename T>
__global__ __launch_bounds__(256) void dcn_im2col_kernel(const T* __restrict__ im, const float* __restrict__ off,
                                                         const float* __restrict__ mask, T* __restrict__ col,
                                                         DcnGeom g) {
  const long total = (long)g.C * g.B * g.Ho * g.Wo;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int wo = idx % g.Wo;
  long t = idx / g.Wo;
  const int ho = t % g.Ho;
  t /= g.Ho;
  const int b = t % g.B;
  const int c = (int)(t / g.B);
  const int K = g.kh * g.kw;
  const int grp = c / (g.C / g.dg);
  const long HWo = (long)g.Ho * g.Wo;
  const float* op = off + ((long)b * g.dg + grp) * 2 * K * HWo + ho * g.Wo + wo;
  const float* mp = mask ? mask + ((long)b * g.dg + grp) * K * HWo + ho * g.Wo + wo : nullptr;
  const T* ip = im + ((long)b * g.C + c) * g.H * g.W;
  T* cp = col + ((long)c * K * g.B + b) * HWo + ho * g.Wo + wo;
  const int h_in = ho * g.sh - g.ph, w_in = wo * g.sw - g.pw;
  for (int i = 0; i < g.kh; ++i) {
    for (int j = 0; j < g.kw; ++j) {
      const int p = i * g.kw + j;
      const float h = h_in + i * g.dh + op[(2 * p) * HWo];
      const float w = w_in + j * g.dw + op[(2 * p + 1) * HWo];
      float v = in_range(h, w, g.H, g.W) ? bilinear_zero(ip, g.H, g.W, h, w) : 0.f;
      if (mp) v *= mp[p * HWo];
      cp[(long)p * g.B * HWo] = from_f<T>(v);
    }
  }
}

// grad_im (fp32, accumulated) from grad_col [C*K, B*Ho*Wo] (fp32)
__global__ __launch_bounds__(256) void dcn_col2im_kernel(const float* __restrict__ gcol, const float* __restrict__ off,
                                                         const float* __restrict__ mask, float* __restrict__ gim,
                                                         DcnGeom g) {
  const int K = g.kh * g.kw;
  const long HWo = (long)g.Ho * g.Wo;
  const long total = (long)g.C * K * g.B * HWo;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int wo = idx % g.Wo;
  long t = idx / g.Wo;
  const int ho = t % g.Ho;
  t /= g.Ho;
  const int b = t % g.B;
  t /= g.B;
  const int p = t % K;
  const int c = (int)(t / K);
  const int i = p / g.kw, j = p % g.kw;
  const int grp = c / (g.C / g.dg);
  const float* op = off + ((long)b * g.dg + grp) * 2 * K * HWo + ho * g.Wo + wo;
  const float h = ho * g.sh - g.ph + i * g.dh + op[(2 * p) * HWo];
  const float w = wo * g.sw - g.pw + j * g.dw + op[(2 * p + 1) * HWo];
  if (!in_range(h, w, g.H, g.W)) return;
  float gv = gcol[idx];
  if (mask) gv *= mask[((long)b * g.dg + grp) * K * HWo + p * HWo + ho * g.Wo + wo];
  if (gv == 0.f) return;
  const int h0 = (int)floorf(h), w0 = (int)floorf(w);
  const float lh = h - h0, lw = w - w0;
  float* gp = gim + ((long)b * g.C + c) * g.H * g.W;
  if (h0 >= 0 && w0 >= 0) atomicAdd(gp + h0 * g.W + w0, (1.f - lh) * (1.f - lw) * gv);
  if (h0 >= 0 && w0 + 1 <= g.W - 1) atomicAdd(gp + h0 * g.W + w0 + 1, (1.f - lh) * lw * gv);
  if (h0 + 1 <= g.H - 1 && w0 >= 0) atomicAdd(gp + (h0 + 1) * g.W + w0, lh * (1.f - lw) * gv);
  if (h0 + 1 <= g.H - 1 && w0 + 1 <= g.W - 1) atomicAdd(gp + (h0 + 1) * g.W + w0 + 1, lh * lw * gv);
}

// grad_offset [B, dg*2K, Ho, Wo] and grad_mask [B, dg*K, Ho, Wo] (written, not accumulated)
template <typename T>
__global__ __launch_bounds__(256) void dcn_col2coord_kernel(const float* __restrict__ gcol, const T* __restrict__ im,
                                                            const float* __restrict__ off,
                                                            const float* __restrict__ mask,
                                                            float* __restrict__ goff, float* __restrict__ gmask,
                                                            DcnGeom g) {
  const int K = g.kh * g.kw;
  const long HWo = (long)g.Ho * g.Wo;
  const long total = (long)g.B * g.dg * 2 * K * HWo;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int wo = idx % g.Wo;
  long t = idx / g.Wo;
  const int ho = t % g.Ho;
  t /= g.Ho;
  const int oc = t % (g.dg * 2 * K);          // offset channel
  const int b = (int)(t / (g.dg * 2 * K));
  const int grp = oc / (2 * K);
  const int p = (oc % (2 * K)) / 2;
  const int dir = oc % 2;                        // 0: h, 1: w
  const int i = p / g.kw, j = p % g.kw;
  const float* op = off + ((long)b * g.dg + grp) * 2 * K * HWo + ho * g.Wo + wo;
  const float h = ho * g.sh - g.ph + i * g.dh + op[(2 * p) * HWo];
  const float w = wo * g.sw - g.pw + j * g.dw + op[(2 * p + 1) * HWo];
  const float m = mask ? mask[((long)b * g.dg + grp) * K * HWo + p * HWo + ho * g.Wo + wo] : 1.f;
  const bool ok = in_range(h, w, g.H, g.W);
  const int h0 = (int)floorf(h), w0 = (int)floorf(w);
  const float lh = h - h0, lw = w - w0;
  const int cpg = g.C / g.dg;
  float acc = 0.f, macc = 0.f;
  for (int cc = 0; cc < cpg; ++cc) {
    const int c = grp * cpg + cc;
    const float gc = gcol[(((long)c * K + p) * g.B + b) * HWo + ho * g.Wo + wo];
    if (!ok || gc == 0.f) continue;
    const T* ip = im + ((long)b * g.C + c) * g.H * g.W;
    float v00 = 0.f, v01 = 0.f, v10 = 0.f, v11 = 0.f;
    if (h0 >= 0 && w0 >= 0) v00 = to_f<T>(ip[h0 * g.W + w0]);
    if (h0 >= 0 && w0 + 1 <= g.W - 1) v01 = to_f<T>(ip[h0 * g.W + w0 + 1]);
    if (h0 + 1 <= g.H - 1 && w0 >= 0) v10 = to_f<T>(ip[(h0 + 1) * g.W + w0]);
    if (h0 + 1 <= g.H - 1 && w0 + 1 <= g.W - 1) v11 = to_f<T>(ip[(h0 + 1) * g.W + w0 + 1]);
    const float d = dir == 0 ? (1.f - lw) * (v10 - v00) + lw * (v11 - v01)
                             : (1.f - lh) * (v01 - v00) + lh * (v11 - v10);
    acc += gc * m * d;
    if (dir == 0 && mask) {
      macc += gc * ((1.f - lh) * (1.f - lw) * v00 + (1.f - lh) * lw * v01 + lh * (1.f - lw) * v10 + lh * lw * v11);
    }
  }
  goff[idx] = acc;
  if (dir == 0 && gmask) gmask[(((long)b * g.dg + grp) * K + p) * HWo + ho * g.Wo + wo] = macc;
}

// ------------------------------------------------------------------ deformable PS RoI pooling
struct PsroiGeom {
  int C, H, W, K, out_dim, group, pooled, part, spp, num_classes, no_trans;
  float scale, trans_std;
};

__device__ __forceinline__ void psroi_bin(const float* rois, const float* trans, const PsroiGeom& g, long idx,
                                          int& n, int& b, int& ctop, int& ph, int& pw, float& wstart,
                                          float& hstart, float& sub_w, float& sub_h, float& roi_w, float& roi_h,
                                          int& part_h, int& part_w, int& cls, int& c_in) {
  pw = idx % g.pooled;
  long t = idx / g.pooled;
  ph = t % g.pooled;
  t /= g.pooled;
  ctop = t % g.out_dim;
  n = (int)(t / g.out_dim);
  const float* r = rois + n * 5;
  b = (int)r[0];
  const float x1 = roundf(r[1]) * g.scale - 0.5f, y1 = roundf(r[2]) * g.scale - 0.5f;
  const float x2 = (roundf(r[3]) + 1.f) * g.scale - 0.5f, y2 = (roundf(r[4]) + 1.f) * g.scale - 0.5f;
  roi_w = fmaxf(x2 - x1, 0.1f);
  roi_h = fmaxf(y2 - y1, 0.1f);
  const float bin_w = roi_w / g.pooled, bin_h = roi_h / g.pooled;
  sub_w = bin_w / g.spp;
  sub_h = bin_h / g.spp;
  part_h = (int)floorf((float)ph / g.pooled * g.part);
  part_w = (int)floorf((float)pw / g.pooled * g.part);
  const int per_class = g.no_trans ? g.out_dim : g.out_dim / g.num_classes;
  cls = ctop / per_class;
  float tx = 0.f, ty = 0.f;
  if (!g.no_trans) {
    tx = trans[(((long)n * g.num_classes + cls) * 2 * g.part + part_h) * g.part + part_w] * g.trans_std;
    ty = trans[((((long)n * g.num_classes + cls) * 2 + 1) * g.part + part_h) * g.part + part_w] * g.trans_std;
  }
  wstart = pw * bin_w + x1 + tx * roi_w;
  hstart = ph * bin_h + y1 + ty * roi_h;
  int gw = (int)floorf((float)pw * g.group / g.pooled), gh = (int)floorf((float)ph * g.group / g.pooled);
  gw = min(max(gw, 0), g.group - 1);
  gh = min(max(gh, 0), g.group - 1);
  c_in = (ctop * g.group + gh) * g.group + gw;
}

__device__ __forceinline__ float bilin_clamped(const float* d, int W, float x, float y) {
  const int x1 = (int)floorf(x), x2 = (int)ceilf(x), y1 = (int)floorf(y), y2 = (int)ceilf(y);
  const float dx = x - x1, dy = y - y1;
  const float v11 = d[y1 * W + x1], v12 = d[y2 * W + x1], v21 = d[y1 * W + x2], v22 = d[y2 * W + x2];
  return (1 - dx) * (1 - dy) * v11 + (1 - dx) * dy * v12 + dx * (1 - dy) * v21 + dx * dy * v22;
}

__global__ __launch_bounds__(256) void psroi_fwd_kernel(const float* __restrict__ data, const float* __restrict__ rois,
                                                        const float* __restrict__ trans, float* __restrict__ out,
                                                        float* __restrict__ count, PsroiGeom g, long total) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  int n, b, ctop, ph, pw, part_h, part_w, cls, c_in;
  float wstart, hstart, sub_w, sub_h, roi_w, roi_h;
  psroi_bin(rois, trans, g, idx, n, b, ctop, ph, pw, wstart, hstart, sub_w, sub_h, roi_w, roi_h, part_h, part_w,
            cls, c_in);
  const float* d = data + ((long)b * g.C + c_in) * g.H * g.W;
  float sum = 0.f;
  int cnt = 0;
  for (int ih = 0; ih < g.spp; ++ih) {
    for (int iw = 0; iw < g.spp; ++iw) {
      float w = wstart + iw * sub_w, h = hstart + ih * sub_h;
      if (w < -0.5f || w > g.W - 0.5f || h < -0.5f || h > g.H - 0.5f) continue;
      w = fminf(fmaxf(w, 0.f), g.W - 1.f);
      h = fminf(fmaxf(h, 0.f), g.H - 1.f);
      sum += bilin_clamped(d, g.W, w, h);
      ++cnt;
    }
  }
  out[idx] = cnt ? sum / cnt : 0.f;
  count[idx] = (float)cnt;
}

__global__ __launch_bounds__(256) void psroi_bwd_kernel(const float* __restrict__ gout, const float* __restrict__ data,
                                                        const float* __restrict__ rois, const float* __restrict__ trans,
                                                        const float* __restrict__ count, float* __restrict__ gdata,
                                                        float* __restrict__ gtrans, PsroiGeom g, long total) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const float cnt = count[idx];
  if (cnt <= 0.f) return;
  int n, b, ctop, ph, pw, part_h, part_w, cls, c_in;
  float wstart, hstart, sub_w, sub_h, roi_w, roi_h;
  psroi_bin(rois, trans, g, idx, n, b, ctop, ph, pw, wstart, hstart, sub_w, sub_h, roi_w, roi_h, part_h, part_w,
            cls, c_in);
  const float diff = gout[idx] / cnt;
  const long base = ((long)b * g.C + c_in) * g.H * g.W;
  const float* d = data + base;
  float* gd = gdata + base;
  float gx = 0.f, gy = 0.f;
  for (int ih = 0; ih < g.spp; ++ih) {
    for (int iw = 0; iw < g.spp; ++iw) {
      float w = wstart + iw * sub_w, h = hstart + ih * sub_h;
      if (w < -0.5f || w > g.W - 0.5f || h < -0.5f || h > g.H - 0.5f) continue;
      w = fminf(fmaxf(w, 0.f), g.W - 1.f);
      h = fminf(fmaxf(h, 0.f), g.H - 1.f);
      const int x0 = (int)floorf(w), x1 = (int)ceilf(w), y0 = (int)floorf(h), y1 = (int)ceilf(h);
      const float dx = w - x0, dy = h - y0;
      atomicAdd(gd + y0 * g.W + x0, (1 - dx) * (1 - dy) * diff);
      atomicAdd(gd + y1 * g.W + x0, (1 - dx) * dy * diff);
      atomicAdd(gd + y0 * g.W + x1, dx * (1 - dy) * diff);
      atomicAdd(gd + y1 * g.W + x1, dx * dy * diff);
      if (!g.no_trans) {
        const float u00 = d[y0 * g.W + x0], u01 = d[y1 * g.W + x0], u10 = d[y0 * g.W + x1], u11 = d[y1 * g.W + x1];
        gx += (dy * (u11 - u01) + (1 - dy) * (u10 - u00)) * diff;
        gy += (dx * (u11 - u10) + (1 - dx) * (u01 - u00)) * diff;
      }
    }
  }
  if (!g.no_trans) {
    const long tb = (((long)n * g.num_classes + cls) * 2 * g.part + part_h) * g.part + part_w;
    atomicAdd(gtrans + tb, gx * g.trans_std * roi_w);
    atomicAdd(gtrans + tb + (long)g.part * g.part, gy * g.trans_std * roi_h);
  }
}

}  // namespace ct

using namespace ct;

static inline unsigned blocks_for(long n) { return (unsigned)((n + 255) / 256); }

extern "C" {

int ct_dcn_im2col(const void* im, const float* off, const float* mask, void* col, int dtype, const int* geom,
                  hipStream_t st) {
  DcnGeom g{geom[0], geom[1], geom[2], geom[3], geom[4], geom[5], geom[6], geom[7], geom[8],
            geom[9], geom[10], geom[11], geom[12], geom[13], geom[14]};
  const long total = (long)g.C * g.B * g.Ho * g.Wo;
  if (total <= 0) return 0;
  if (dtype == 0)
    dcn_im2col_kernel<float><<<blocks_for(total), 256, 0, st>>>((const float*)im, off, mask, (float*)col, g);
  else
    dcn_im2col_kernel<bf16_t><<<blocks_for(total), 256, 0, st>>>((const bf16_t*)im, off, mask, (bf16_t*)col, g);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int ct_dcn_col2im(const float* gcol, const float* off, const float* mask, float* gim, const int* geom,
                  hipStream_t st) {
  DcnGeom g{geom[0], geom[1], geom[2], geom[3], geom[4], geom[5], geom[6], geom[7], geom[8],
            geom[9], geom[10], geom[11], geom[12], geom[13], geom[14]};
  const long total = (long)g.C * g.kh * g.kw * g.B * g.Ho * g.Wo;
  if (total <= 0) return 0;
  dcn_col2im_kernel<<<blocks_for(total), 256, 0, st>>>(gcol, off, mask, gim, g);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int ct_dcn_col2coord(const float* gcol, const void* im, const float* off, const float* mask, float* goff,
                     float* gmask, int dtype, const int* geom, hipStream_t st) {
  DcnGeom g{geom[0], geom[1], geom[2], geom[3], geom[4], geom[5], geom[6], geom[7], geom[8],
            geom[9], geom[10], geom[11], geom[12], geom[13], geom[14]};
  const long total = (long)g.B * g.dg * 2 * g.kh * g.kw * g.Ho * g.Wo;
  if (total <= 0) return 0;
  if (dtype == 0)
    dcn_col2coord_kernel<float><<<blocks_for(total), 256, 0, st>>>(gcol, (const float*)im, off, mask, goff, gmask, g);
  else
    dcn_col2coord_kernel<bf16_t><<<blocks_for(total), 256, 0, st>>>(gcol, (const bf16_t*)im, off, mask, goff, gmask,
                                                                     g);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// geom: C, H, W, K(rois), out_dim, group, pooled, part, spp, num_classes, no_trans
int ct_psroi_fwd(const float* data, const float* rois, const float* trans, float* out, float* count, const int* gi,
                 float scale, float trans_std, hipStream_t st) {
  PsroiGeom g{gi[0], gi[1], gi[2], gi[3], gi[4], gi[5], gi[6], gi[7], gi[8], gi[9], gi[10], scale, trans_std};
  const long total = (long)g.K * g.out_dim * g.pooled * g.pooled;
  if (total <= 0) return 0;
  psroi_fwd_kernel<<<blocks_for(total), 256, 0, st>>>(data, rois, trans, out, count, g, total);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int ct_psroi_bwd(const float* gout, const float* data, const float* rois, const float* trans, const float* count,
                 float* gdata, float* gtrans, const int* gi, float scale, float trans_std, hipStream_t st) {
  PsroiGeom g{gi[0], gi[1], gi[2], gi[3], gi[4], gi[5], gi[6], gi[7], gi[8], gi[9], gi[10], scale, trans_std};
  const long total = (long)g.K * g.out_dim * g.pooled * g.pooled;
  if (total <= 0) return 0;
  psroi_bwd_kernel<<<blocks_for(total), 256, 0, st>>>(gout, data, rois, trans, count, gdata, gtrans, g, total);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
