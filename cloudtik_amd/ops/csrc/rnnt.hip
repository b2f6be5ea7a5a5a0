// RNN-Transducer loss for gfx950 (the MLPerf RNN-T workload of the reference quickstart,
// SURVEY.md §2.12 "RNN-T"; the reference relies on a third-party CUDA/C++ transducer loss).
//
// Three kernels, no host synchronisation, fp32 arithmetic on bf16 or fp32 joint logits:
//
//  1. rnnt_logprob: one wave per lattice node (b, t, u) -- a wave-wide log-sum-exp over the
//     vocabulary, then the two log-probabilities the lattice needs: blank and the next label.
//     The [B, T, U+1, V] logits are read exactly once here (and once in the gradient kernel).
//  2. rnnt_alpha_beta: one workgroup per (utterance, direction).  The forward variables
//     alpha(t, u) and backward variables beta(t, u) are swept along anti-diagonals
//     t + u = n (every node of a diagonal depends only on the previous one), lanes over u,
//     one barrier per diagonal; alpha and beta run concurrently in separate workgroups.
//  3. rnnt_grad: d loss / d logits of every node (row-wise, 8-lane groups over V):
//        g_v = softmax_v * exp(alpha + beta - logP)
//              - [v = blank] exp(alpha + lp_blank + beta(t+1, u) - logP)
//              - [v = y_u]   exp(alpha + lp_label + beta(t, u+1) - logP),
//     scaled by the incoming per-utterance loss gradient, written in the logits' dtype.
#include "common.h"

namespace ct {

constexpr float kNegInf = -INFINITY;

__device__ __forceinline__ float log_add(float a, float b) {
  if (a == kNegInf) return b;
  if (b == kNegInf) return a;
  const float m = fmaxf(a, b);
  return m + log1pf(__expf(-fabsf(a - b)));
}

// logits [B, T, U1, V]; labels [B, U1-1] (int32); lens: T_b, U_b (labels per utterance)
template <typename T>
__global__ void __launch_bounds__(256) rnnt_logprob_kernel(const T* __restrict__ logits,
                                                           const int* __restrict__ labels,
                                                           const int* __restrict__ tlen, const int* __restrict__ ulen,
                                                           float* __restrict__ lse_out, float2* __restrict__ lp,
                                                           int B, int Tm, int U1, int V, int blank) {
  const long rows = (long)B * Tm * U1;
  const int lane = threadIdx.x & 63;
  const long wave = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wave; r < rows; r += nwaves) {
    const int u = r % U1, t = (r / U1) % Tm, b = r / ((long)U1 * Tm);
    if (t >= tlen[b] || u > ulen[b]) {                // outside this utterance's lattice
      if (lane == 0) { lse_out[r] = 0.f; lp[r] = make_float2(kNegInf, kNegInf); }
      continue;
    }
    const T* x = logits + r * V;
    float m = kNegInf;
    for (int v = lane; v < V; v += 64) m = fmaxf(m, to_f<T>(x[v]));
    m = wave_max(m);
    float s = 0.f;
    for (int v = lane; v < V; v += 64) s += __expf(to_f<T>(x[v]) - m);
    s = wave_sum(s);
    if (lane == 0) {
      const float lse = m + __logf(s);
      lse_out[r] = lse;
      const float pb = to_f<T>(x[blank]) - lse;
      const float pl = u < ulen[b] ? to_f<T>(x[labels[(long)b * (U1 - 1) + u]]) - lse : kNegInf;
      lp[r] = make_float2(pb, pl);
    }
  }
}

// grid (B, 2): y = 0 -> alpha, y = 1 -> beta.  alpha / beta [B, T, U1]; loglik [B]
__global__ void __launch_bounds__(256) rnnt_alpha_beta_kernel(const float2* __restrict__ lp,
                                                              const int* __restrict__ tlen,
                                                              const int* __restrict__ ulen,
                                                              float* __restrict__ alpha, float* __restrict__ beta,
                                                              float* __restrict__ loglik, int Tm, int U1) {
  const int b = blockIdx.x;
  const int Tb = tlen[b], Ub = ulen[b];
  const long base = (long)b * Tm * U1;
  const float2* L = lp + base;
  if (blockIdx.y == 0) {
    float* A = alpha + base;
    for (int n = 0; n < Tb + Ub; ++n) {               // diagonal t + u = n
      for (int u = threadIdx.x; u <= Ub; u += blockDim.x) {
        const int t = n - u;
        if (t < 0 || t >= Tb) continue;
        float a;
        if (t == 0 && u == 0) a = 0.f;
        else {
          const float from_t = t > 0 ? A[(long)(t - 1) * U1 + u] + L[(long)(t - 1) * U1 + u].x : kNegInf;
          const float from_u = u > 0 ? A[(long)t * U1 + u - 1] + L[(long)t * U1 + u - 1].y : kNegInf;
          a = log_add(from_t, from_u);
        }
        A[(long)t * U1 + u] = a;
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) loglik[b] = A[(long)(Tb - 1) * U1 + Ub] + L[(long)(Tb - 1) * U1 + Ub].x;
  } else {
    float* Bt = beta + base;
    for (int n = Tb + Ub - 1; n >= 0; --n) {
      for (int u = threadIdx.x; u <= Ub; u += blockDim.x) {
        const int t = n - u;
        if (t < 0 || t >= Tb) continue;
        float v;
        if (t == Tb - 1 && u == Ub) v = L[(long)t * U1 + u].x;
        else {
          const float by_blank = t + 1 < Tb ? Bt[(long)(t + 1) * U1 + u] + L[(long)t * U1 + u].x : kNegInf;
          const float by_label = u < Ub ? Bt[(long)t * U1 + u + 1] + L[(long)t * U1 + u].y : kNegInf;
          v = log_add(by_blank, by_label);
        }
        Bt[(long)t * U1 + u] = v;
      }
      __syncthreads();
    }
  }
}

// One 64-lane wave per lattice row; lanes stride over V.
template <typename T>
__global__ void __launch_bounds__(256) rnnt_grad_kernel(const T* __restrict__ logits, const int* __restrict__ labels,
                                                        const int* __restrict__ tlen, const int* __restrict__ ulen,
                                                        const float* __restrict__ lse, const float2* __restrict__ lp,
                                                        const float* __restrict__ alpha, const float* __restrict__ beta,
                                                        const float* __restrict__ loglik,
                                                        const float* __restrict__ gloss, T* __restrict__ grad, int B,
                                                        int Tm, int U1, int V, int blank) {
  const long rows = (long)B * Tm * U1;
  const int lane = threadIdx.x & 63;
  const long wave = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wave; r < rows; r += nwaves) {
    const int u = r % U1, t = (r / U1) % Tm, b = r / ((long)U1 * Tm);
    T* gx = grad + r * V;
    const int Tb = tlen[b], Ub = ulen[b];
    if (t >= Tb || u > Ub) {
      for (int v = lane; v < V; v += 64) gx[v] = from_f<T>(0.f);
      continue;
    }
    const long bu = (long)b * Tm * U1;
    const float ll = loglik[b], g = gloss[b];
    const float a = alpha[r];
    const float occ = __expf(a + beta[r] - ll);                       // node occupancy
    const float2 l2 = lp[r];
    float nb;                                                            // beta after a blank
    if (t + 1 < Tb) nb = beta[bu + (long)(t + 1) * U1 + u];
    else nb = (u == Ub) ? 0.f : kNegInf;                                 // final blank ends the lattice
    const float tb = __expf(a + l2.x + nb - ll);
    const float tl = u < Ub ? __expf(a + l2.y + beta[bu + (long)t * U1 + u + 1] - ll) : 0.f;
    const int y = u < Ub ? labels[(long)b * (U1 - 1) + u] : -1;
    const float m = lse[r];
    const T* x = logits + r * V;
    for (int v = lane; v < V; v += 64) {
      float d = __expf(to_f<T>(x[v]) - m) * occ;
      if (v == blank) d -= tb;
      if (v == y) d -= tl;
      gx[v] = from_f<T>(g * d);
    }
  }
}

inline int waves_grid(long rows) {
  long g = (rows + 3) / 4;                 // 4 waves per 256-thread block
  if (g > 16384) g = 16384;
  return g < 1 ? 1 : (int)g;
}

}  // namespace ct

using namespace ct;

extern "C" int ct_rnnt_fwd(const void* logits, int dt, const int* labels, const int* tlen, const int* ulen,
                           float* lse, float* lp, float* alpha, float* beta, float* loglik, int B, int Tm, int U1,
                           int V, int blank, hipStream_t stream) {
  if (U1 > 4096) return 1;
  const long rows = (long)B * Tm * U1;
  const int g = waves_grid(rows);
  if (dt == 0)
    rnnt_logprob_kernel<float><<<g, 256, 0, stream>>>((const float*)logits, labels, tlen, ulen, lse, (float2*)lp, B,
                                                      Tm, U1, V, blank);
  else
    rnnt_logprob_kernel<bf16_t><<<g, 256, 0, stream>>>((const bf16_t*)logits, labels, tlen, ulen, lse, (float2*)lp,
                                                       B, Tm, U1, V, blank);
  rnnt_alpha_beta_kernel<<<dim3(B, 2), 256, 0, stream>>>((const float2*)lp, tlen, ulen, alpha, beta, loglik, Tm, U1);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int ct_rnnt_bwd(const void* logits, int dt, const int* labels, const int* tlen, const int* ulen,
                           const float* lse, const float* lp, const float* alpha, const float* beta,
                           const float* loglik, const float* gloss, void* grad, int B, int Tm, int U1, int V,
                           int blank, hipStream_t stream) {
  const long rows = (long)B * Tm * U1;
  const int g = waves_grid(rows);
  if (dt == 0)
    rnnt_grad_kernel<float><<<g, 256, 0, stream>>>((const float*)logits, labels, tlen, ulen, lse, (const float2*)lp,
                                                   alpha, beta, loglik, gloss, (float*)grad, B, Tm, U1, V, blank);
  else
    rnnt_grad_kernel<bf16_t><<<g, 256, 0, stream>>>((const bf16_t*)logits, labels, tlen, ulen, lse,
                                                    (const float2*)lp, alpha, beta, loglik, gloss, (bf16_t*)grad, B,
                                                    Tm, U1, V, blank);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
