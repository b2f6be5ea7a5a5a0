// Multi-tensor fused optimizers over FLAT parameter buffers.
//
// The framework keeps every parameter of a model in one contiguous fp32 master buffer,
// the bf16 model weights in one contiguous bf16 buffer (the nn.Parameters are views of
// it) and the gradients in one contiguous buffer (the .grad views are also the all-reduce
// buckets, so no pack/unpack copies).  A "segment" table splits the flat space into
// <= 8K-element pieces, each tagged with its owning tensor, so ONE launch updates every
// parameter of the model.
//
//   * LAMB (reference: applications/ai/quickstart/models/language_modeling/pytorch/
//     bert_large/training/lamb.py:61-139 -- bf16 params + fp32 master copy, no bias
//     correction by default, trust ratio only for groups with weight decay, eps 1e-6;
//     IPEX `Lamb(fused=True)` at run_pretrain_mlperf.py:503):
//       stage 1: m, v update; u = m/(sqrt(v)+eps) + wd*w; per-segment partial ||w||^2, ||u||^2
//       reduce : per-tensor sums (deterministic wave reduction, no float atomics) -- these
//                [T,2] partials are what a sharded (ZeRO-1) optimizer all-reduces across ranks
//       stage 2: w -= lr * trust(tensor) * u (u recomputed: same bytes as storing it),
//                writes fp32 master + bf16 model copy.
//   * Adam / AdamW (transfer-learning Trainer default, GraphSAGE Adam): single pass.
//   * SGD + momentum / nesterov (ResNet-50 `main.py:317`, DLRM SplitSGD): single pass.
//
// Dynamic hyper-parameters (lr, grad scale, bias corrections) are read from a device array
// so a hipGraph-captured step picks up the scheduler's new values at replay.
#include "common.h"
#include <cstdlib>

namespace ct {

// dyn[0] = lr, dyn[1] = grad scale (e.g. 1/world or clip coef), dyn[2] = 1/(1-b1^t),
// dyn[3] = 1/(1-b2^t)
struct OptSegs {
  const int* seg_tensor;    // [nseg]
  const long* seg_start;    // [nseg] element offset in the flat space
  const int* seg_len;       // [nseg]
};

template <typename GT>
__device__ __forceinline__ f32x4 load4(const GT* p, long i);
template <>
__device__ __forceinline__ f32x4 load4<float>(const float* p, long i) {
  return *reinterpret_cast<const f32x4*>(p + i);
}
template <>
__device__ __forceinline__ f32x4 load4<bf16_t>(const bf16_t* p, long i) {
  const u16x4 v = *reinterpret_cast<const u16x4*>(p + i);
  return f32x4{bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3])};
}
__device__ __forceinline__ void store4(float* p, long i, f32x4 v) { *reinterpret_cast<f32x4*>(p + i) = v; }
__device__ __forceinline__ void store4(bf16_t* p, long i, f32x4 v) {
  u16x4 o = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
  *reinterpret_cast<u16x4*>(p + i) = o;
}

// 8 consecutive elements as one 16-byte (bf16) or two 16-byte (fp32) accesses
__device__ __forceinline__ void load8(const float* p, long i, float (&o)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p + i), b = *reinterpret_cast<const f32x4*>(p + i + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { o[j] = a[j]; o[4 + j] = b[j]; }
}
__device__ __forceinline__ void load8(const bf16_t* p, long i, float (&o)[8]) {
  const u16x8 v = *reinterpret_cast<const u16x8*>(p + i);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = bf2f(v[j]);
}
__device__ __forceinline__ void store8(float* p, long i, const float (&v)[8]) {
  *reinterpret_cast<f32x4*>(p + i) = f32x4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(p + i + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
__device__ __forceinline__ void store8(bf16_t* p, long i, const float (&v)[8]) {
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
  *reinterpret_cast<u16x8*>(p + i) = o;
}

// LAMB over a segment with every load of the thread's share issued before any math: U chunks
// of 8 elements per thread (a whole 8K segment in one pass at U = 4, 256 threads); segments are
// 64-element multiples, so a chunk that starts inside the segment ends inside it.  Opt-in
// (CLOUDTIK_AMD_LAMB_V8=1): in the BERT-large step stage 1 took 1.386 ms against 1.257 for the
// one-vec4-per-iteration kernel and stage 2 the same 1.13 ms (profiles/r5/steady_bert_large_head_r5a.md)
// -- the two passes are HBM-bound as they are, more bytes in flight per thread buy nothing.
constexpr int LAMB_U = 4;

template <typename GT>
__global__ __launch_bounds__(256) void lamb_stage1_v8_kernel(
    const GT* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    const float* __restrict__ w, OptSegs segs, const float* __restrict__ tensor_wd,
    const float* __restrict__ dyn, float beta1, float beta2, float eps, int bias_corr,
    float* __restrict__ seg_part) {
  __shared__ float scratch[8];
  const int s = blockIdx.x;
  const long start = segs.seg_start[s];
  const int len = segs.seg_len[s];
  const float wd = tensor_wd[segs.seg_tensor[s]];
  const float gs = dyn[1];
  const float bc1 = bias_corr ? dyn[2] : 1.f, bc2 = bias_corr ? dyn[3] : 1.f;
  float w2 = 0.f, u2 = 0.f;
  for (int i0 = threadIdx.x * 8; i0 < len; i0 += 256 * 8 * LAMB_U) {
    float gv[LAMB_U][8], mv[LAMB_U][8], vv[LAMB_U][8], wv[LAMB_U][8];
#pragma unroll
    for (int u = 0; u < LAMB_U; ++u) {
      const int i = i0 + u * 256 * 8;
      if (i < len) {
        const long k = start + i;
        load8(g, k, gv[u]);
        load8(m, k, mv[u]);
        load8(v, k, vv[u]);
        load8(w, k, wv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < LAMB_U; ++u) {
      const int i = i0 + u * 256 * 8;
      if (i < len) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gr = gv[u][j] * gs;
          mv[u][j] = beta1 * mv[u][j] + (1.f - beta1) * gr;
          vv[u][j] = beta2 * vv[u][j] + (1.f - beta2) * gr * gr;
          const float up = (mv[u][j] * bc1) / (sqrtf(vv[u][j] * bc2) + eps) + wd * wv[u][j];
          w2 += wv[u][j] * wv[u][j];
          u2 += up * up;
        }
        const long k = start + i;
        store8(m, k, mv[u]);
        store8(v, k, vv[u]);
      }
    }
  }
  w2 = block_sum(w2, scratch);
  u2 = block_sum(u2, scratch);
  if (threadIdx.x == 0) { seg_part[2 * s] = w2; seg_part[2 * s + 1] = u2; }
}

template <typename PT>
__global__ __launch_bounds__(256) void lamb_stage2_v8_kernel(
    const float* __restrict__ m, const float* __restrict__ v, float* __restrict__ w,
    PT* __restrict__ w_model, OptSegs segs, const float* __restrict__ tensor_wd,
    const float* __restrict__ tensor_part, const float* __restrict__ dyn, float eps, int bias_corr,
    int trust_all) {
  const int s = blockIdx.x;
  const long start = segs.seg_start[s];
  const int len = segs.seg_len[s];
  const int t = segs.seg_tensor[s];
  const float wd = tensor_wd[t];
  const float lr = dyn[0];
  const float bc1 = bias_corr ? dyn[2] : 1.f, bc2 = bias_corr ? dyn[3] : 1.f;
  float ratio = 1.f;
  if (wd != 0.f || trust_all) {
    const float wn = sqrtf(tensor_part[2 * t]), un = sqrtf(tensor_part[2 * t + 1]);
    ratio = (wn > 0.f && un > 0.f) ? wn / un : 1.f;
  }
  const float step = lr * ratio;
  for (int i0 = threadIdx.x * 8; i0 < len; i0 += 256 * 8 * LAMB_U) {
    float mv[LAMB_U][8], vv[LAMB_U][8], wv[LAMB_U][8];
#pragma unroll
    for (int u = 0; u < LAMB_U; ++u) {
      const int i = i0 + u * 256 * 8;
      if (i < len) {
        const long k = start + i;
        load8(m, k, mv[u]);
        load8(v, k, vv[u]);
        load8(w, k, wv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < LAMB_U; ++u) {
      const int i = i0 + u * 256 * 8;
      if (i < len) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float up = (mv[u][j] * bc1) / (sqrtf(vv[u][j] * bc2) + eps) + wd * wv[u][j];
          wv[u][j] -= step * up;
        }
        const long k = start + i;
        store8(w, k, wv[u]);
        if (w_model) store8(w_model, k, wv[u]);
      }
    }
  }
}

template <typename GT>
__global__ __launch_bounds__(256) void lamb_stage1_kernel(
    const GT* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    const float* __restrict__ w, OptSegs segs, const float* __restrict__ tensor_wd,
    const float* __restrict__ dyn, float beta1, float beta2, float eps, int bias_corr,
    float* __restrict__ seg_part) {
  __shared__ float scratch[8];
  const int s = blockIdx.x;
  const long start = segs.seg_start[s];
  const int len = segs.seg_len[s];
  const float wd = tensor_wd[segs.seg_tensor[s]];
  const float gs = dyn[1];
  const float bc1 = bias_corr ? dyn[2] : 1.f, bc2 = bias_corr ? dyn[3] : 1.f;
  float w2 = 0.f, u2 = 0.f;
  for (int i = threadIdx.x * 4; i < len; i += blockDim.x * 4) {
    const long k = start + i;
    const f32x4 gv = load4<GT>(g, k);
    f32x4 mv = load4<float>(m, k), vv = load4<float>(v, k);
    const f32x4 wv = load4<float>(w, k);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gr = gv[j] * gs;
      mv[j] = beta1 * mv[j] + (1.f - beta1) * gr;
      vv[j] = beta2 * vv[j] + (1.f - beta2) * gr * gr;
      const float u = (mv[j] * bc1) / (sqrtf(vv[j] * bc2) + eps) + wd * wv[j];
      w2 += wv[j] * wv[j];
      u2 += u * u;
    }
    store4(m, k, mv);
    store4(v, k, vv);
  }
  w2 = block_sum(w2, scratch);
  u2 = block_sum(u2, scratch);
  if (threadIdx.x == 0) { seg_part[2 * s] = w2; seg_part[2 * s + 1] = u2; }
}

// per-tensor sums of the segment partials: one wave per tensor
__global__ __launch_bounds__(256) void seg_to_tensor_kernel(const float* __restrict__ seg_part,
                                                            const int* __restrict__ tensor_first_seg,
                                                            int T, float* __restrict__ tensor_part) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T) return;
  const int a = tensor_first_seg[t], b = tensor_first_seg[t + 1];
  float w2 = 0.f, u2 = 0.f;
  for (int s = a + lane; s < b; s += 64) { w2 += seg_part[2 * s]; u2 += seg_part[2 * s + 1]; }
  w2 = wave_sum(w2);
  u2 = wave_sum(u2);
  if (lane == 0) { tensor_part[2 * t] = w2; tensor_part[2 * t + 1] = u2; }
}

template <typename PT>
__global__ __launch_bounds__(256) void lamb_stage2_kernel(
    const float* __restrict__ m, const float* __restrict__ v, float* __restrict__ w,
    PT* __restrict__ w_model, OptSegs segs, const float* __restrict__ tensor_wd,
    const float* __restrict__ tensor_part, const float* __restrict__ dyn, float eps, int bias_corr,
    int trust_all) {
  const int s = blockIdx.x;
  const long start = segs.seg_start[s];
  const int len = segs.seg_len[s];
  const int t = segs.seg_tensor[s];
  const float wd = tensor_wd[t];
  const float lr = dyn[0];
  const float bc1 = bias_corr ? dyn[2] : 1.f, bc2 = bias_corr ? dyn[3] : 1.f;
  float ratio = 1.f;
  if (wd != 0.f || trust_all) {
    const float wn = sqrtf(tensor_part[2 * t]), un = sqrtf(tensor_part[2 * t + 1]);
    ratio = (wn > 0.f && un > 0.f) ? wn / un : 1.f;
  }
  const float step = lr * ratio;
  for (int i = threadIdx.x * 4; i < len; i += blockDim.x * 4) {
    const long k = start + i;
    const f32x4 mv = load4<float>(m, k), vv = load4<float>(v, k);
    f32x4 wv = load4<float>(w, k);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float u = (mv[j] * bc1) / (sqrtf(vv[j] * bc2) + eps) + wd * wv[j];
      wv[j] -= step * u;
    }
    store4(w, k, wv);
    if (w_model) store4(w_model, k, wv);
  }
}

// Adam / AdamW.  adamw=1: decoupled decay w -= lr*wd*w; adamw=0: L2 (g += wd*w)
template <typename GT, typename PT>
__global__ __launch_bounds__(256) void adam_kernel(
    const GT* __restrict__ g, float* __restrict__ m, float* __restrict__ v, float* __restrict__ w,
    PT* __restrict__ w_model, OptSegs segs, const float* __restrict__ tensor_wd,
    const float* __restrict__ dyn, float beta1, float beta2, float eps, int adamw) {
  const int s = blockIdx.x;
  const long start = segs.seg_start[s];
  const int len = segs.seg_len[s];
  const float wd = tensor_wd[segs.seg_tensor[s]];
  const float lr = dyn[0], gs = dyn[1], bc1 = dyn[2], bc2 = dyn[3];
  for (int i = threadIdx.x * 4; i < len; i += blockDim.x * 4) {
    const long k = start + i;
    const f32x4 gv = load4<GT>(g, k);
    f32x4 mv = load4<float>(m, k), vv = load4<float>(v, k), wv = load4<float>(w, k);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gr = gv[j] * gs;
      if (!adamw) gr += wd * wv[j];
      mv[j] = beta1 * mv[j] + (1.f - beta1) * gr;
      vv[j] = beta2 * vv[j] + (1.f - beta2) * gr * gr;
      float upd = (mv[j] * bc1) / (sqrtf(vv[j] * bc2) + eps);
      if (adamw) upd += wd * wv[j];
      wv[j] -= lr * upd;
    }
    store4(m, k, mv);
    store4(v, k, vv);
    store4(w, k, wv);
    if (w_model) store4(w_model, k, wv);
  }
}

// SGD with momentum (PyTorch semantics: buf = mom*buf + (1-damp)*g; nesterov g + mom*buf)
template <typename GT, typename PT>
__global__ __launch_bounds__(256) void sgd_kernel(
    const GT* __restrict__ g, float* __restrict__ buf, float* __restrict__ w,
    PT* __restrict__ w_model, OptSegs segs, const float* __restrict__ tensor_wd,
    const float* __restrict__ dyn, float momentum, float dampening, int nesterov, int first) {
  const int s = blockIdx.x;
  const long start = segs.seg_start[s];
  const int len = segs.seg_len[s];
  const float wd = tensor_wd[segs.seg_tensor[s]];
  const float lr = dyn[0], gs = dyn[1];
  for (int i = threadIdx.x * 4; i < len; i += blockDim.x * 4) {
    const long k = start + i;
    const f32x4 gv = load4<GT>(g, k);
    f32x4 wv = load4<float>(w, k);
    f32x4 bv = f32x4{0.f, 0.f, 0.f, 0.f};
    if (momentum != 0.f) bv = load4<float>(buf, k);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gr = gv[j] * gs + wd * wv[j];
      if (momentum != 0.f) {
        bv[j] = first ? gr : momentum * bv[j] + (1.f - dampening) * gr;
        gr = nesterov ? gr + momentum * bv[j] : bv[j];
      }
      wv[j] -= lr * gr;
    }
    if (momentum != 0.f) store4(buf, k, bv);
    store4(w, k, wv);
    if (w_model) store4(w_model, k, wv);
  }
}

// sum of squares over [n] (grad-norm clipping): per-block partials, then one block adds their
// sum to *out (one atomic: up to 2048 blocks adding into one address serialise at the memory
// side, ~0.2 us each)
template <typename GT>
__global__ __launch_bounds__(256) void sumsq_kernel(const GT* __restrict__ x, long n,
                                                    float* __restrict__ part) {
  __shared__ float scratch[8];
  float acc = 0.f;
  for (long i = (blockIdx.x * (long)blockDim.x + threadIdx.x) * 4; i < n;
       i += (long)gridDim.x * blockDim.x * 4) {
    const f32x4 v = load4<GT>(x, i);
    acc += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void sumsq_finish_kernel(const float* __restrict__ part, int g,
                                                           float* __restrict__ out) {
  __shared__ float scratch[8];
  float acc = 0.f;
  for (int i = threadIdx.x; i < g; i += blockDim.x) acc += part[i];
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) atomicAdd(out, acc);     // += : callers may sum several tensors
}

// dyn[1] = base_scale * min(1, max_norm / (sqrt(sumsq)*base_scale + 1e-6))
__global__ void clip_coef_kernel(const float* __restrict__ sumsq, float* __restrict__ dyn,
                                 float base_scale, float max_norm) {
  const float norm = sqrtf(*sumsq) * base_scale;
  const float c = max_norm / (norm + 1e-6f);
  dyn[1] = base_scale * (c < 1.f ? c : 1.f);
}

}  // namespace ct

using namespace ct;

// gdt / pdt: 0 = fp32, 1 = bf16.  w_model may be null (fp32 params updated in place via w).
extern "C" int ct_lamb(const void* g, int gdt, float* m, float* v, float* w, void* w_model, int pdt,
                       const int* seg_tensor, const long* seg_start, const int* seg_len, int nseg,
                       const int* tensor_first_seg, int T, const float* tensor_wd, const float* dyn,
                       float beta1, float beta2, float eps, int bias_corr, int trust_all,
                       float* seg_part, float* tensor_part, int stage, hipStream_t stream) {
  OptSegs segs{seg_tensor, seg_start, seg_len};
  // the 8-element form needs 16-byte aligned bases (segments start at 64-element multiples)
  static const bool v8_env = [] { const char* e = getenv("CLOUDTIK_AMD_LAMB_V8"); return e && atoi(e) != 0; }();
  const bool v8 = v8_env && !(((uintptr_t)g | (uintptr_t)m | (uintptr_t)v | (uintptr_t)w | (uintptr_t)w_model) & 15);
  if (stage & 1) {
    if (v8 && gdt == 1)
      lamb_stage1_v8_kernel<bf16_t><<<nseg, 256, 0, stream>>>((const bf16_t*)g, m, v, w, segs, tensor_wd, dyn, beta1, beta2, eps, bias_corr, seg_part);
    else if (v8)
      lamb_stage1_v8_kernel<float><<<nseg, 256, 0, stream>>>((const float*)g, m, v, w, segs, tensor_wd, dyn, beta1, beta2, eps, bias_corr, seg_part);
    else if (gdt == 1)
      lamb_stage1_kernel<bf16_t><<<nseg, 256, 0, stream>>>((const bf16_t*)g, m, v, w, segs, tensor_wd, dyn, beta1, beta2, eps, bias_corr, seg_part);
    else
      lamb_stage1_kernel<float><<<nseg, 256, 0, stream>>>((const float*)g, m, v, w, segs, tensor_wd, dyn, beta1, beta2, eps, bias_corr, seg_part);
    seg_to_tensor_kernel<<<ceil_div(T, 4), 256, 0, stream>>>(seg_part, tensor_first_seg, T, tensor_part);
  }
  if (stage & 2) {
    if (v8 && pdt == 1)
      lamb_stage2_v8_kernel<bf16_t><<<nseg, 256, 0, stream>>>(m, v, w, (bf16_t*)w_model, segs, tensor_wd, tensor_part, dyn, eps, bias_corr, trust_all);
    else if (v8)
      lamb_stage2_v8_kernel<float><<<nseg, 256, 0, stream>>>(m, v, w, (float*)w_model, segs, tensor_wd, tensor_part, dyn, eps, bias_corr, trust_all);
    else if (pdt == 1)
      lamb_stage2_kernel<bf16_t><<<nseg, 256, 0, stream>>>(m, v, w, (bf16_t*)w_model, segs, tensor_wd, tensor_part, dyn, eps, bias_corr, trust_all);
    else
      lamb_stage2_kernel<float><<<nseg, 256, 0, stream>>>(m, v, w, (float*)w_model, segs, tensor_wd, tensor_part, dyn, eps, bias_corr, trust_all);
  }
  return 0;
}

extern "C" int ct_adam(const void* g, int gdt, float* m, float* v, float* w, void* w_model, int pdt,
                       const int* seg_tensor, const long* seg_start, const int* seg_len, int nseg,
                       const float* tensor_wd, const float* dyn, float beta1, float beta2,
                       float eps, int adamw, hipStream_t stream) {
  OptSegs segs{seg_tensor, seg_start, seg_len};
#define CT_ADAM(GT, PT) adam_kernel<GT, PT><<<nseg, 256, 0, stream>>>((const GT*)g, m, v, w, (PT*)w_model, segs, tensor_wd, dyn, beta1, beta2, eps, adamw)
  if (gdt == 1 && pdt == 1) CT_ADAM(bf16_t, bf16_t);
  else if (gdt == 1) CT_ADAM(bf16_t, float);
  else if (pdt == 1) CT_ADAM(float, bf16_t);
  else CT_ADAM(float, float);
#undef CT_ADAM
  return 0;
}

extern "C" int ct_sgd(const void* g, int gdt, float* buf, float* w, void* w_model, int pdt,
                      const int* seg_tensor, const long* seg_start, const int* seg_len, int nseg,
                      const float* tensor_wd, const float* dyn, float momentum, float dampening,
                      int nesterov, int first, hipStream_t stream) {
  OptSegs segs{seg_tensor, seg_start, seg_len};
#define CT_SGD(GT, PT) sgd_kernel<GT, PT><<<nseg, 256, 0, stream>>>((const GT*)g, buf, w, (PT*)w_model, segs, tensor_wd, dyn, momentum, dampening, nesterov, first)
  if (gdt == 1 && pdt == 1) CT_SGD(bf16_t, bf16_t);
  else if (gdt == 1) CT_SGD(bf16_t, float);
  else if (pdt == 1) CT_SGD(float, bf16_t);
  else CT_SGD(float, float);
#undef CT_SGD
  return 0;
}

// part: float[2048] scratch
extern "C" int ct_sumsq(const void* x, int dt, long n, float* out, float* part, hipStream_t stream) {
  long g = (n / 4 + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  if (dt == 1) sumsq_kernel<bf16_t><<<(int)g, 256, 0, stream>>>((const bf16_t*)x, n, part);
  else sumsq_kernel<float><<<(int)g, 256, 0, stream>>>((const float*)x, n, part);
  sumsq_finish_kernel<<<1, 256, 0, stream>>>(part, (int)g, out);
  return 0;
}

extern "C" int ct_clip_coef(const float* sumsq, float* dyn, float base_scale, float max_norm,
                            hipStream_t stream) {
  clip_coef_kernel<<<1, 1, 0, stream>>>(sumsq, dyn, base_scale, max_norm);
  return 0;
}
