// DLRM sparse path for gfx950: multi-table EmbeddingBag (sum / mean, per-sample weights)
// and the pairwise dot-product feature interaction, forward and backward.
//
// Reference: DLRM dlrm_s_pytorch.py:267-269 (nn.EmbeddingBag per table, mode="sum"),
// :407-418 (interact_features: bmm(T, T^T) + strictly-lower-triangle gather), IPEX
// ipex.interaction / SplitSGD (SURVEY.md §2.15 "EmbeddingBag (sum) + dot interaction").
//
// Layout (MI355X-first): all tables live in ONE [sum(V_t), E] fp32 buffer (row_base[t] is
// table t's first row), the bags of all tables form one CSR (offsets over T*B bags,
// table-major), and the forward writes straight into the [B, T, E] tensor the interaction
// consumes -- one launch for all 26 tables instead of 26 + a torch.stack.  The backward
// either scatters into a dense fp32 gradient with fp32 atomics, or applies the SGD update
// to the touched rows directly (w[row] -= lr * g; the IPEX SplitSGD/"fused backward"
// analogue), so 10^7-row tables never materialise a dense gradient.
#include "common.h"

namespace ct {

// one wave per bag; lanes stride over E
template <typename TO>
__global__ void __launch_bounds__(256) embbag_fwd_kernel(const float* __restrict__ W, const int64_t* __restrict__ row_base,
                                                          const int64_t* __restrict__ idx, const int64_t* __restrict__ offs,
                                                          const float* __restrict__ psw, TO* __restrict__ out,
                                                          int T, int B, int E, int mean) {
  const int lane = threadIdx.x & 63;
  const long nbags = (long)T * B;
  for (long bag = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6; bag < nbags;
       bag += ((long)gridDim.x * blockDim.x) >> 6) {
    const int t = (int)(bag / B), b = (int)(bag % B);
    const long s = offs[bag], e = offs[bag + 1];
    const float* Wt = W + row_base[t] * (long)E;
    TO* o = out + ((long)b * T + t) * E;
    for (int c = lane; c < E; c += 64) {
      float acc0 = 0.f, acc1 = 0.f;
      long i = s;
      for (; i + 1 < e; i += 2) {          // two rows in flight per lane
        const float w0 = psw ? psw[i] : 1.f, w1 = psw ? psw[i + 1] : 1.f;
        acc0 += w0 * Wt[idx[i] * E + c];
        acc1 += w1 * Wt[idx[i + 1] * E + c];
      }
      if (i < e) acc0 += (psw ? psw[i] : 1.f) * Wt[idx[i] * E + c];
      float acc = acc0 + acc1;
      if (mean && e > s) acc /= (float)(e - s);
      o[c] = from_f<TO>(acc);
    }
  }
}

template <typename TG>
__global__ void __launch_bounds__(256) embbag_bwd_kernel(const TG* __restrict__ gout, float* __restrict__ W,
                                                          float* __restrict__ dW, const int64_t* __restrict__ row_base,
                                                          const int64_t* __restrict__ idx, const int64_t* __restrict__ offs,
                                                          const float* __restrict__ psw, int T, int B, int E, int mean,
                                                          float neg_lr) {
  const int lane = threadIdx.x & 63;
  const long nbags = (long)T * B;
  for (long bag = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6; bag < nbags;
       bag += ((long)gridDim.x * blockDim.x) >> 6) {
    const int t = (int)(bag / B), b = (int)(bag % B);
    const long s = offs[bag], e = offs[bag + 1];
    if (e <= s) continue;
    const float scale = mean ? 1.f / (float)(e - s) : 1.f;
    const TG* g = gout + ((long)b * T + t) * E;
    const long base = row_base[t] * (long)E;
    for (int c = lane; c < E; c += 64) {
      const float gv = to_f<TG>(g[c]) * scale;
      for (long i = s; i < e; ++i) {
        const float v = gv * (psw ? psw[i] : 1.f);
        const long off = base + idx[i] * E + c;
        if (dW) atomicAdd(dW + off, v);
        else atomicAdd(W + off, neg_lr * v);
      }
    }
  }
}

// d(loss)/d(psw[i]) = <gout[bag], W[row_i]>   (per-sample-weight gradient)
template <typename TG>
__global__ void __launch_bounds__(256) embbag_psw_grad_kernel(const TG* __restrict__ gout, const float* __restrict__ W,
                                                               const int64_t* __restrict__ row_base,
                                                               const int64_t* __restrict__ idx, const int64_t* __restrict__ offs,
                                                               float* __restrict__ dpsw, int T, int B, int E, int mean) {
  const int lane = threadIdx.x & 63;
  const long nbags = (long)T * B;
  for (long bag = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6; bag < nbags;
       bag += ((long)gridDim.x * blockDim.x) >> 6) {
    const int t = (int)(bag / B), b = (int)(bag % B);
    const TG* g = gout + ((long)b * T + t) * E;
    const float* Wt = W + row_base[t] * (long)E;
    const long s = offs[bag], e = offs[bag + 1];
    const float scale = (mean && e > s) ? 1.f / (float)(e - s) : 1.f;
    for (long i = s; i < e; ++i) {
      float acc = 0.f;
      for (int c = lane; c < E; c += 64) acc += to_f<TG>(g[c]) * Wt[idx[i] * E + c];
      acc = wave_sum(acc);
      if (lane == 0) dpsw[i] = acc * scale;
    }
  }
}

// ------------------------------------------------------------------ interaction
// V = [x_b ; emb_b]  (F = T + 1 rows of E), out_b = [x_b, Z_{i,j} for i > j] row-major
// over (i, j) -- the order torch.tril_indices(F, F, -1) produces.
constexpr int kMaxF = 64;
constexpr int kIntWaves = 4;

template <typename TI>
__global__ void __launch_bounds__(256) interact_fwd_kernel(const TI* __restrict__ x, const TI* __restrict__ emb,
                                                            TI* __restrict__ out, int B, int T, int E) {
  extern __shared__ float lds[];
  const int F = T + 1, P = F * (F - 1) / 2, ld = E + 1;      // +1: rows in distinct banks
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* V = lds + w * F * ld;
  for (long b = (long)blockIdx.x * kIntWaves + w; b < B; b += (long)gridDim.x * kIntWaves) {
    const TI* xb = x + b * E;
    const TI* eb = emb + b * (long)T * E;
    TI* ob = out + b * (long)(E + P);
    for (int c = lane; c < E; c += 64) {
      const TI v = xb[c];
      V[c] = to_f<TI>(v);
      ob[c] = v;
    }
    for (int r = 0; r < T; ++r)
      for (int c = lane; c < E; c += 64) V[(r + 1) * ld + c] = to_f<TI>(eb[r * E + c]);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    for (int p = lane; p < P; p += 64) {
      // p -> (i, j), i > j, row-major:  i = floor((1 + sqrt(1 + 8p)) / 2)
      int i = (int)((1.f + sqrtf(1.f + 8.f * p)) * 0.5f);
      while (i * (i - 1) / 2 > p) --i;
      while ((i + 1) * i / 2 <= p) ++i;
      const int j = p - i * (i - 1) / 2;
      const float* vi = V + i * ld;
      const float* vj = V + j * ld;
      float acc = 0.f;
      for (int c = 0; c < E; ++c) acc += vi[c] * vj[c];
      ob[E + p] = from_f<TI>(acc);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <typename TI>
__global__ void __launch_bounds__(256) interact_bwd_kernel(const TI* __restrict__ gout, const TI* __restrict__ x,
                                                            const TI* __restrict__ emb, TI* __restrict__ dx,
                                                            TI* __restrict__ demb, int B, int T, int E) {
  extern __shared__ float lds[];
  const int F = T + 1, P = F * (F - 1) / 2, ld = E + 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* V = lds + w * (F * ld + F * F);
  float* G = V + F * ld;                                      // symmetric F x F, zero diagonal
  for (long b = (long)blockIdx.x * kIntWaves + w; b < B; b += (long)gridDim.x * kIntWaves) {
    const TI* gb = gout + b * (long)(E + P);
    for (int c = lane; c < E; c += 64) V[c] = to_f<TI>(x[b * E + c]);
    for (int r = 0; r < T; ++r)
      for (int c = lane; c < E; c += 64) V[(r + 1) * ld + c] = to_f<TI>(emb[(b * T + r) * (long)E + c]);
    for (int q = lane; q < F * F; q += 64) G[q] = 0.f;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    for (int p = lane; p < P; p += 64) {
      int i = (int)((1.f + sqrtf(1.f + 8.f * p)) * 0.5f);
      while (i * (i - 1) / 2 > p) --i;
      while ((i + 1) * i / 2 <= p) ++i;
      const int j = p - i * (i - 1) / 2;
      const float g = to_f<TI>(gb[E + p]);
      G[i * F + j] = g;
      G[j * F + i] = g;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    for (int r = 0; r < F; ++r) {
      for (int c = lane; c < E; c += 64) {
        float acc = 0.f;
        for (int j = 0; j < F; ++j) acc += G[r * F + j] * V[j * ld + c];
        if (r == 0) dx[b * E + c] = from_f<TI>(acc + to_f<TI>(gb[c]));
        else demb[(b * T + (r - 1)) * (long)E + c] = from_f<TI>(acc);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

inline int grid_waves(long waves) {
  long g = (waves * 64 + 255) / 256;
  if (g > 8192) g = 8192;
  return g < 1 ? 1 : (int)g;
}

}  // namespace ct

using namespace ct;

// dtype codes: 0 fp32, 1 bf16
extern "C" int ct_embbag_fwd(const float* W, const int64_t* row_base, const int64_t* idx, const int64_t* offs,
                             const float* psw, void* out, int out_dt, int T, int B, int E, int mean,
                             hipStream_t stream) {
  const int g = grid_waves((long)T * B);
  if (out_dt == 0) embbag_fwd_kernel<float><<<g, 256, 0, stream>>>(W, row_base, idx, offs, psw, (float*)out, T, B, E, mean);
  else embbag_fwd_kernel<bf16_t><<<g, 256, 0, stream>>>(W, row_base, idx, offs, psw, (bf16_t*)out, T, B, E, mean);
  return 0;
}

extern "C" int ct_embbag_bwd(const void* gout, int g_dt, float* W, float* dW, const int64_t* row_base,
                             const int64_t* idx, const int64_t* offs, const float* psw, float* dpsw,
                             int T, int B, int E, int mean, float lr, hipStream_t stream) {
  const int g = grid_waves((long)T * B);
  if (dpsw) {   // before the SGD update touches W
    if (g_dt == 0) embbag_psw_grad_kernel<float><<<g, 256, 0, stream>>>((const float*)gout, W, row_base, idx, offs, dpsw, T, B, E, mean);
    else embbag_psw_grad_kernel<bf16_t><<<g, 256, 0, stream>>>((const bf16_t*)gout, W, row_base, idx, offs, dpsw, T, B, E, mean);
  }
  if (g_dt == 0) embbag_bwd_kernel<float><<<g, 256, 0, stream>>>((const float*)gout, W, dW, row_base, idx, offs, psw, T, B, E, mean, -lr);
  else embbag_bwd_kernel<bf16_t><<<g, 256, 0, stream>>>((const bf16_t*)gout, W, dW, row_base, idx, offs, psw, T, B, E, mean, -lr);
  return 0;
}

extern "C" int ct_interact_fwd(const void* x, const void* emb, void* out, int dt, int B, int T, int E,
                               hipStream_t stream) {
  const int F = T + 1;
  if (F > kMaxF) return -1;
  const size_t lds = (size_t)kIntWaves * F * (E + 1) * sizeof(float);
  if (lds > 160 * 1024) return -2;
  int g = (B + kIntWaves - 1) / kIntWaves;
  if (g > 8192) g = 8192;
  if (dt == 0) interact_fwd_kernel<float><<<g, 256, lds, stream>>>((const float*)x, (const float*)emb, (float*)out, B, T, E);
  else interact_fwd_kernel<bf16_t><<<g, 256, lds, stream>>>((const bf16_t*)x, (const bf16_t*)emb, (bf16_t*)out, B, T, E);
  return 0;
}

extern "C" int ct_interact_bwd(const void* gout, const void* x, const void* emb, void* dx, void* demb, int dt,
                               int B, int T, int E, hipStream_t stream) {
  const int F = T + 1;
  if (F > kMaxF) return -1;
  const size_t lds = (size_t)kIntWaves * (F * (E + 1) + F * F) * sizeof(float);
  if (lds > 160 * 1024) return -2;
  int g = (B + kIntWaves - 1) / kIntWaves;
  if (g > 8192) g = 8192;
  if (dt == 0) interact_bwd_kernel<float><<<g, 256, lds, stream>>>((const float*)gout, (const float*)x, (const float*)emb,
                                                                   (float*)dx, (float*)demb, B, T, E);
  else interact_bwd_kernel<bf16_t><<<g, 256, lds, stream>>>((const bf16_t*)gout, (const bf16_t*)x, (const bf16_t*)emb,
                                                            (bf16_t*)dx, (bf16_t*)demb, B, T, E);
  return 0;
}
