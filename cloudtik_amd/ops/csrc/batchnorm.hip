// Training BatchNorm for NHWC (channels_last) bf16 activations, fused with the residual
// add and ReLU that follow it in every ResNet bottleneck.  The backward never re-reads the
// BN output for the ReLU mask when there is no residual: the mask is the sign of the
// forward pre-activation, recomputed from x with the saved affine coefficients (one fewer
// activation-sized read in each backward pass).  A one-pass fp64-atomic variant of the
// statistics reduction (last block finalises) was measured 4-6x SLOWER on MI355X: ~1000
// blocks x C same-address device-scope atomics serialise, so block partials + a small
// finalize launch stay.
//
// Reference hot path: torchvision resnet50 trained channels_last + bf16 under DDP
// (applications/ai/quickstart/models/image_recognition/pytorch/common/main.py:276-296) and
// the synthetic ResNet-50 benchmark (examples/runtime/ai/basics/pytorch/
// imagenet-resnet50-synthetic-pytorch-distributed.py).  In PyTorch eager that is three
// memory passes per BN (batch_norm, add, relu); here it is:
//   forward : stats kernel (per-block sum/sumsq -> (mean, M2)), finalize (Chan merge of
//             block partials, running-stat update), apply kernel y = relu(x*a + b + res)
//   backward: reduce kernel (sum dy', sum dy'*xhat with dy' = dy * [y > 0]), finalize
//             (dgamma, dbeta, per-channel affine coefficients), apply kernel
//             dx = a*dy' + c1*x + c0 and d(residual) = dy' in the same pass.
// Channels are the contiguous dimension: a thread owns 8 channels (one 16-byte vector) and
// walks rows, so every load is a full coalesced 16-byte-per-lane access.
#include "common.h"
#include <algorithm>
#include <stdlib.h>

namespace ct {

struct BnLayout { int M, C, CV, RPI, rows_per_blk; };

// reduction kernel block size (1024-thread blocks measured no faster: 3.13 vs 3.04 ms per
// step for the backward reductions, 1.18 vs 1.11 for the statistics)
constexpr int BN_RT = 256;

// sum the RPI row-groups' 8-channel partials of (a, b) in LDS (tree; RPI need not be a power
// of two); the totals end up in the rl == 0 threads' registers
__device__ __forceinline__ void bn_block_sum2(float (&a)[8], float (&b)[8], float* la, float* lb, int RPI, int rl,
                                              int CV) {
#pragma unroll
  for (int j = 0; j < 8; ++j) { la[threadIdx.x * 8 + j] = a[j]; lb[threadIdx.x * 8 + j] = b[j]; }
  __syncthreads();
  int P = 1;
  while (P * 2 <= RPI) P *= 2;
  if (rl < RPI && rl >= P) {                          // fold the non-power-of-two tail
    const int t = (rl - P) * CV + threadIdx.x % CV;
#pragma unroll
    for (int j = 0; j < 8; ++j) { la[t * 8 + j] += a[j]; lb[t * 8 + j] += b[j]; }
  }
  __syncthreads();
  for (int h = P / 2; h >= 1; h /= 2) {
    if (rl < h) {
      const int t = threadIdx.x, u = (rl + h) * CV + threadIdx.x % CV;
#pragma unroll
      for (int j = 0; j < 8; ++j) { la[t * 8 + j] += la[u * 8 + j]; lb[t * 8 + j] += lb[u * 8 + j]; }
    }
    __syncthreads();
  }
  if (rl == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = la[threadIdx.x * 8 + j]; b[j] = lb[threadIdx.x * 8 + j]; }
  }
}

__device__ __forceinline__ void bn_thread(const BnLayout& L, int& cv, int& rl) {
  cv = threadIdx.x % L.CV;
  rl = threadIdx.x / L.CV;
}

// per-block (mean, M2) over rows [b*R, (b+1)*R), 4 rows in flight per thread
template <int U>
__global__ __launch_bounds__(BN_RT) void bn_stats_kernel(const bf16_t* __restrict__ x, BnLayout L,
                                                         float* __restrict__ pmean,
                                                         float* __restrict__ pm2) {
  __shared__ float ls[BN_RT * 8];
  __shared__ float lq[BN_RT * 8];
  int cv, rl;
  bn_thread(L, cv, rl);
  const int r0 = blockIdx.x * L.rows_per_blk;
  const int r1 = min(L.M, r0 + L.rows_per_blk);
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s[j] = 0.f; q[j] = 0.f; }
  if (rl < L.RPI) {
    int r = r0 + rl;
    for (; r + (U - 1) * L.RPI < r1; r += U * L.RPI) {
      u16x8 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = reinterpret_cast<const u16x8*>(x + (size_t)(r + u * L.RPI) * L.C)[cv];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float f = bf2f(v[u][j]); s[j] += f; q[j] += f * f; }
    }
    for (; r < r1; r += L.RPI) {
      const u16x8 v = reinterpret_cast<const u16x8*>(x + (size_t)r * L.C)[cv];
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float f = bf2f(v[j]); s[j] += f; q[j] += f * f; }
    }
  }
  bn_block_sum2(s, q, ls, lq, L.RPI, rl, L.CV);
  if (rl == 0) {
    const float n = (float)max(0, r1 - r0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = cv * 8 + j;
      const float mean = n > 0.f ? s[j] / n : 0.f;
      pmean[(size_t)blockIdx.x * L.C + c] = mean;
      pm2[(size_t)blockIdx.x * L.C + c] = n > 0.f ? fmaxf(q[j] - s[j] * mean, 0.f) : 0.f;
    }
  }
}


// Merge of the block partials (per-block mean and M2 over n_b rows); writes save_mean /
// save_invstd, the affine (a, b) and updates the running statistics.  A 1024-thread block
// owns 64 consecutive channels: lane = channel, so every partial load of a wave is one
// contiguous 256-byte line (partials are [block][C]); the 16 waves split the partial rows and
// combine through LDS.  Two passes instead of a sequential Chan merge (whose dependent
// divisions made a 512-partial merge latency-bound): mean = sum(n_b mean_b) / N, then
// M2 = sum(M2_b + n_b (mean_b - mean)^2) -- the same deviation form, no division in a loop.
// (The first version gave each wave one channel and strided its lanes over the partial rows:
// 64 cache lines per load.)
__global__ __launch_bounds__(1024) void bn_finalize_kernel(
    const float* __restrict__ pmean, const float* __restrict__ pm2, int nblk, BnLayout L,
    const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta, float eps, float momentum,
    float* __restrict__ run_mean, float* __restrict__ run_var, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, float* __restrict__ coef_a, float* __restrict__ coef_b) {
  __shared__ float lsum[16][64], lmean[64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const bool live = c < L.C;
  const float R = (float)L.rows_per_blk;
  // up to 256 partials (the direct case and every merged one) the wave's 16 rows of both
  // arrays are loaded in ONE round before pass 1, so pass 2 needs no second memory round trip
  constexpr int KR = 16;
  const bool inreg = nblk <= 16 * KR;
  float mv[KR], m2v[KR];
  // pass 1: sum of n_b * mean_b (every block but the last has R rows)
  float s = 0.f;
  if (live && inreg) {
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int b = w + 16 * k;
      mv[k] = b < nblk ? pmean[(size_t)b * L.C + c] : 0.f;
      m2v[k] = b < nblk ? pm2[(size_t)b * L.C + c] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int b = w + 16 * k;
      const float nb = b >= nblk ? 0.f : (b == nblk - 1 ? (float)(L.M - b * L.rows_per_blk) : R);
      s += nb * mv[k];
    }
  } else if (live) {
#pragma unroll 8
    for (int b = w; b < nblk; b += 16) {
      const float nb = b == nblk - 1 ? (float)(L.M - b * L.rows_per_blk) : R;
      s += nb * pmean[(size_t)b * L.C + c];
    }
  }
  lsum[w][lane] = s;
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int k = 1; k < 16; ++k) s += lsum[k][lane];
    lmean[lane] = s / (float)L.M;
  }
  __syncthreads();
  const float mean = lmean[lane];
  // pass 2: M2 = sum(M2_b + n_b (mean_b - mean)^2)
  float q = 0.f;
  if (live && inreg) {
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int b = w + 16 * k;
      const float nb = b >= nblk ? 0.f : (b == nblk - 1 ? (float)(L.M - b * L.rows_per_blk) : R);
      const float d = mv[k] - mean;
      q += m2v[k] + nb * d * d;
    }
  } else if (live) {
#pragma unroll 8
    for (int b = w; b < nblk; b += 16) {
      const float nb = b == nblk - 1 ? (float)(L.M - b * L.rows_per_blk) : R;
      const float d = pmean[(size_t)b * L.C + c] - mean;
      q += pm2[(size_t)b * L.C + c] + nb * d * d;
    }
  }
  __syncthreads();                                    // lsum reuse
  lsum[w][lane] = q;
  __syncthreads();
  if (w != 0 || !live) return;
#pragma unroll
  for (int k = 1; k < 16; ++k) q += lsum[k][lane];
  const float n = (float)L.M;
  const float var = fmaxf(q / n, 0.f);
  const float invstd = rsqrtf(var + eps);
  const float g = gamma ? bf2f(gamma[c]) : 1.f, bt = beta ? bf2f(beta[c]) : 0.f;
  save_mean[c] = mean;
  save_invstd[c] = invstd;
  coef_a[c] = g * invstd;
  coef_b[c] = bt - mean * g * invstd;
  if (run_mean) {
    const float unb = n > 1.f ? q / (n - 1.f) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
  }
}

// pre-activation of the fused forward, evaluated identically in forward and backward
__device__ __forceinline__ float bn_pre(float x, float a, float b, float r) { return __builtin_fmaf(x, a, b) + r; }

// 8 per-channel floats (two 16-byte loads) for channel vector cv
__device__ __forceinline__ void bn_load8(const float* __restrict__ p, int cv, float (&o)[8]) {
  const f32x4 lo = reinterpret_cast<const f32x4*>(p)[2 * cv], hi = reinterpret_cast<const f32x4*>(p)[2 * cv + 1];
#pragma unroll
  for (int j = 0; j < 4; ++j) { o[j] = lo[j]; o[4 + j] = hi[j]; }
}

// The element-wise passes are grid-stride loops over 16-byte channel vectors.  When the
// vector count per row (CV = C/8) divides the block size -- every ResNet width -- the grid
// stride is a multiple of CV, so a thread always sees the same channel vector: its
// per-channel coefficients are loaded ONCE, before the loop, and the loop body is the two
// or three streaming loads and the store.  (The first version re-loaded 4-10 coefficient
// vectors per 16 data bytes through the cache and took a 64-bit modulo per vector: 3.6-3.9
// TB/s; unrolling the loop several vectors deep did not help, pmc_resnet50.md.)  Other
// widths take the per-vector path.
__device__ __forceinline__ bool bn_fixed_cv(int CV) { return (blockDim.x % CV) == 0; }

// y = act(x * a[c] + b[c] (+ res))
template <int BN_EW>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* __restrict__ x,
                                                       const bf16_t* __restrict__ res,
                                                       const float* __restrict__ a,
                                                       const float* __restrict__ b,
                                                       bf16_t* __restrict__ y, uint8_t* __restrict__ mask,
                                                       long total_vec, int CV, int relu) {
  const long stride = (long)gridDim.x * blockDim.x;
  const long t0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const bool fixed = bn_fixed_cv(CV);
  float av[8], bv[8];
  if (fixed) { bn_load8(a, threadIdx.x % CV, av); bn_load8(b, threadIdx.x % CV, bv); }
  for (long v0 = t0; v0 < total_vec; v0 += BN_EW * stride) {
    u16x8 xv[BN_EW], rv[BN_EW];
#pragma unroll
    for (int u = 0; u < BN_EW; ++u) {
      const long v = v0 + u * stride;
      xv[u] = v < total_vec ? reinterpret_cast<const u16x8*>(x)[v] : u16x8(0);
      rv[u] = (res && v < total_vec) ? reinterpret_cast<const u16x8*>(res)[v] : u16x8(0);
    }
#pragma unroll
    for (int u = 0; u < BN_EW; ++u) {
      const long v = v0 + u * stride;
      if (v >= total_vec) break;
      if (!fixed) { const int cv = (int)(v % CV); bn_load8(a, cv, av); bn_load8(b, cv, bv); }
      u16x8 o;
      uint32_t bits = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = bn_pre(bf2f(xv[u][j]), av[j], bv[j], bf2f(rv[u][j]));
        if (relu) t = fmaxf(t, 0.f);
        o[j] = f2bf(t);
        bits |= (o[j] != 0 && !(o[j] & 0x8000u) ? 1u : 0u) << j;     // y > 0
      }
      reinterpret_cast<u16x8*>(y)[v] = o;
      if (mask) mask[v] = (uint8_t)bits;
    }
  }
}

// y = relu(x * a[c] + b[c] + bf16(x2 * a2[c] + b2[c])) + the ReLU bitmask: a BatchNorm + residual
// + ReLU whose residual is itself a BatchNorm output (the ResNet downsample branch) -- that
// residual is never written and read back.  Rounds the inner BatchNorm output to bf16 first, so
// y is bit-identical to bn_apply(x2) followed by bn_apply(x, res).
__global__ __launch_bounds__(256) void bn_apply2_kernel(const bf16_t* __restrict__ x, const float* __restrict__ a,
                                                        const float* __restrict__ b, const bf16_t* __restrict__ x2,
                                                        const float* __restrict__ a2, const float* __restrict__ b2,
                                                        bf16_t* __restrict__ y, uint8_t* __restrict__ mask,
                                                        long total_vec, int CV) {
  const long stride = (long)gridDim.x * blockDim.x;
  const bool fixed = bn_fixed_cv(CV);
  float av[8], bv[8], a2v[8], b2v[8];
  if (fixed) {
    const int cv = threadIdx.x % CV;
    bn_load8(a, cv, av); bn_load8(b, cv, bv); bn_load8(a2, cv, a2v); bn_load8(b2, cv, b2v);
  }
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < total_vec; v += stride) {
    const u16x8 xv = reinterpret_cast<const u16x8*>(x)[v];
    const u16x8 x2v = reinterpret_cast<const u16x8*>(x2)[v];
    if (!fixed) {
      const int cv = (int)(v % CV);
      bn_load8(a, cv, av); bn_load8(b, cv, bv); bn_load8(a2, cv, a2v); bn_load8(b2, cv, b2v);
    }
    u16x8 o;
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float r = bf2f(f2bf(bn_pre(bf2f(x2v[j]), a2v[j], b2v[j], 0.f)));
      const float t = fmaxf(bn_pre(bf2f(xv[j]), av[j], bv[j], r), 0.f);
      o[j] = f2bf(t);
      bits |= (o[j] != 0 && !(o[j] & 0x8000u) ? 1u : 0u) << j;
    }
    reinterpret_cast<u16x8*>(y)[v] = o;
    mask[v] = (uint8_t)bits;
  }
}

// ReLU mask source for the backward: mode 0 = no ReLU, 1 = read y (fused residual add),
// 2 = recompute the pre-activation from x and the forward affine (a, b): no y read at all,
// 3 = the forward's bitmask (one byte per 8-channel vector, bit j = y > 0: what a BN +
// residual + ReLU forward writes beside y, 1/16 of y's bytes)
struct BnMask {
  int mode;
  const bf16_t* y;
  const float* fa;
  const float* fb;
  const uint8_t* m;
};

// forward affine of channel vector cv (mode 2 only)
__device__ __forceinline__ void bn_mask_coef(const BnMask& mk, int cv, float (&fa)[8], float (&fb)[8]) {
  if (mk.mode == 2) { bn_load8(mk.fa, cv, fa); bn_load8(mk.fb, cv, fb); }
}

__device__ __forceinline__ void bn_mask8(const BnMask& mk, const u16x8& yv, const u16x8& xv, const float (&fa)[8],
                                         const float (&fb)[8], uint32_t mb, bool (&on)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (mk.mode == 0) on[j] = true;
    else if (mk.mode == 1) on[j] = bf2f(yv[j]) > 0.f;
    else if (mk.mode == 3) on[j] = (mb >> j) & 1u;
    else on[j] = bf2f(f2bf(bn_pre(bf2f(xv[j]), fa[j], fb[j], 0.f))) > 0.f;
  }
}

// per-block sums of dy' and dy'*xhat (dy' = masked dy), 4 rows in flight per thread.
// dmask (optional): dy' is also stored -- for a BN + residual-add + ReLU it IS the residual
// branch's gradient, and the apply pass then reads dy' instead of dy and y.
template <int U>
__global__ __launch_bounds__(BN_RT) void bn_bwd_reduce_kernel(
    const bf16_t* __restrict__ dy, BnMask mk, const bf16_t* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ invstd, BnLayout L, float* __restrict__ p1, float* __restrict__ p2,
    bf16_t* __restrict__ dmask) {
  __shared__ float l1[BN_RT * 8];
  __shared__ float l2[BN_RT * 8];
  int cv, rl;
  bn_thread(L, cv, rl);
  const int r0 = blockIdx.x * L.rows_per_blk;
  const int r1 = min(L.M, r0 + L.rows_per_blk);
  float s1[8], s2[8], mu[8], is[8], fa[8], fb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s1[j] = 0.f; s2[j] = 0.f;
    mu[j] = mean[cv * 8 + j]; is[j] = invstd[cv * 8 + j];
  }
  bn_mask_coef(mk, cv, fa, fb);
  if (rl < L.RPI) {
    int r = r0 + rl;
    for (; r + (U - 1) * L.RPI < r1; r += U * L.RPI) {
      u16x8 g[U], xv[U], yv[U];
      uint32_t mb[U];
      size_t o[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        o[u] = (size_t)(r + u * L.RPI) * L.CV + cv;
        g[u] = reinterpret_cast<const u16x8*>(dy)[o[u]];
        xv[u] = reinterpret_cast<const u16x8*>(x)[o[u]];
        yv[u] = mk.mode == 1 ? reinterpret_cast<const u16x8*>(mk.y)[o[u]] : u16x8(0);
        mb[u] = mk.mode == 3 ? mk.m[o[u]] : 0u;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        bool on[8];
        bn_mask8(mk, yv[u], xv[u], fa, fb, mb[u], on);
        u16x8 od;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = on[j] ? bf2f(g[u][j]) : 0.f;
          od[j] = on[j] ? g[u][j] : (unsigned short)0;
          s1[j] += d;
          s2[j] += d * (bf2f(xv[u][j]) - mu[j]) * is[j];
        }
        if (dmask) reinterpret_cast<u16x8*>(dmask)[o[u]] = od;
      }
    }
    for (; r < r1; r += L.RPI) {
      const size_t o = (size_t)r * L.CV + cv;
      const u16x8 g = reinterpret_cast<const u16x8*>(dy)[o];
      const u16x8 xv = reinterpret_cast<const u16x8*>(x)[o];
      const u16x8 yv = mk.mode == 1 ? reinterpret_cast<const u16x8*>(mk.y)[o] : u16x8(0);
      const uint32_t mb = mk.mode == 3 ? mk.m[o] : 0u;
      bool on[8];
      bn_mask8(mk, yv, xv, fa, fb, mb, on);
      u16x8 od;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = on[j] ? bf2f(g[j]) : 0.f;
        od[j] = on[j] ? g[j] : (unsigned short)0;
        s1[j] += d;
        s2[j] += d * (bf2f(xv[j]) - mu[j]) * is[j];
      }
      if (dmask) reinterpret_cast<u16x8*>(dmask)[o] = od;
    }
  }
  bn_block_sum2(s1, s2, l1, l2, L.RPI, rl, L.CV);
  if (rl == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      p1[(size_t)blockIdx.x * L.C + cv * 8 + j] = s1[j];
      p2[(size_t)blockIdx.x * L.C + cv * 8 + j] = s2[j];
    }
  }
}

// dgamma, dbeta and dx = a*dy' + c1*x + c0 coefficients (64 channels per block, lane =
// channel, waves split the partial rows, as above)
template <typename PT>
__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(
    const float* __restrict__ p1, const float* __restrict__ p2, int nblk, int M, int C,
    const bf16_t* __restrict__ gamma, const float* __restrict__ mean,
    const float* __restrict__ invstd, PT* __restrict__ dgamma, PT* __restrict__ dbeta,
    float* __restrict__ ca, float* __restrict__ c1, float* __restrict__ c0, int acc) {
  __shared__ float l1[16][64], l2[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const bool live = c < C;
  float sdy = 0.f, sdx = 0.f;
  if (live) {
#pragma unroll 4
    for (int b = w; b < nblk; b += 16) { sdy += p1[(size_t)b * C + c]; sdx += p2[(size_t)b * C + c]; }
  }
  l1[w][lane] = sdy;
  l2[w][lane] = sdx;
  __syncthreads();
  if (w != 0 || !live) return;
#pragma unroll
  for (int k = 1; k < 16; ++k) { sdy += l1[k][lane]; sdx += l2[k][lane]; }
  // acc: accumulate into the (flat-buffer) parameter gradients instead of overwriting, so
  // no separate AccumulateGrad kernel runs per BatchNorm parameter
  if (dgamma) dgamma[c] = from_f<PT>(acc ? to_f<PT>(dgamma[c]) + sdx : sdx);
  if (dbeta) dbeta[c] = from_f<PT>(acc ? to_f<PT>(dbeta[c]) + sdy : sdy);
  const float g = gamma ? bf2f(gamma[c]) : 1.f;
  const float is = invstd[c];
  const float a = g * is;
  const float k = -a * sdx / M;  // coefficient of xhat
  ca[c] = a;
  c1[c] = k * is;
  c0[c] = -a * sdy / M - k * is * mean[c];
}

template <int BN_EW>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const bf16_t* __restrict__ dy, BnMask mk, const bf16_t* __restrict__ x,
    const float* __restrict__ ca, const float* __restrict__ c1, const float* __restrict__ c0,
    bf16_t* __restrict__ dx, bf16_t* __restrict__ dres, long total_vec, int CV) {
  const long stride = (long)gridDim.x * blockDim.x;
  const bool fixed = bn_fixed_cv(CV);
  float aa[8], kk[8], zz[8], fa[8], fb[8];
  if (fixed) {
    const int cv = threadIdx.x % CV;
    bn_load8(ca, cv, aa); bn_load8(c1, cv, kk); bn_load8(c0, cv, zz);
    bn_mask_coef(mk, cv, fa, fb);
  }
  for (long v0 = blockIdx.x * (long)blockDim.x + threadIdx.x; v0 < total_vec; v0 += BN_EW * stride) {
    u16x8 g[BN_EW], xv[BN_EW], yv[BN_EW];
    uint32_t mb[BN_EW];
#pragma unroll
    for (int u = 0; u < BN_EW; ++u) {
      const long v = v0 + u * stride;
      const bool in = v < total_vec;
      g[u] = in ? reinterpret_cast<const u16x8*>(dy)[v] : u16x8(0);
      xv[u] = in ? reinterpret_cast<const u16x8*>(x)[v] : u16x8(0);
      yv[u] = (in && mk.mode == 1) ? reinterpret_cast<const u16x8*>(mk.y)[v] : u16x8(0);
      mb[u] = (in && mk.mode == 3) ? mk.m[v] : 0u;
    }
#pragma unroll
    for (int u = 0; u < BN_EW; ++u) {
      const long v = v0 + u * stride;
      if (v >= total_vec) break;
      if (!fixed) {
        const int cv = (int)(v % CV);
        bn_load8(ca, cv, aa); bn_load8(c1, cv, kk); bn_load8(c0, cv, zz);
        bn_mask_coef(mk, cv, fa, fb);
      }
      bool on[8];
      bn_mask8(mk, yv[u], xv[u], fa, fb, mb[u], on);
      u16x8 o, od;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = on[j] ? bf2f(g[u][j]) : 0.f;
        o[j] = f2bf(aa[j] * d + kk[j] * bf2f(xv[u][j]) + zz[j]);
        od[j] = f2bf(d);
      }
      reinterpret_cast<u16x8*>(dx)[v] = o;
      if (dres) reinterpret_cast<u16x8*>(dres)[v] = od;
    }
  }
}

// ResNet stem: y = maxpool3x3/s2/p1(relu(x * a + b)) in one pass over x -- the full-resolution
// BN output is never written (nor read back by the pool): the BN backward recomputes its ReLU
// mask from x (mode 2), and the pool backward needs only the argmax, kept as one byte per
// element (window position kh*3+kw; ties go to the first maximum in row-major window order,
// as PyTorch's kernel does).
// Block = one output row (n, oh); thread = (ow, 8-channel chunk) items of that row.  The item's
// chunk is fixed per thread when CV divides the block (ResNet: CV = 8) and the column advances
// by a constant per iteration: no per-item 64-bit division / modulo (the grid-stride form spent
// its time there, 2.4-2.9 TB/s).
__global__ __launch_bounds__(256) void bn_apply_pool_kernel(const bf16_t* __restrict__ x, const float* __restrict__ a,
                                                            const float* __restrict__ b, bf16_t* __restrict__ y,
                                                            uint8_t* __restrict__ arg, int N, int H, int W, int CV,
                                                            int OH, int OW) {
  const int n = blockIdx.x / OH, oh = blockIdx.x - n * OH;
  const int items = OW * CV;
  const bool fixed = bn_fixed_cv(CV);
  float av[8], bv[8];
  if (fixed) { bn_load8(a, threadIdx.x % CV, av); bn_load8(b, threadIdx.x % CV, bv); }
  const long orow = ((long)n * OH + oh) * OW * CV;
  const int cv0 = threadIdx.x % CV, ow0 = threadIdx.x / CV, ostep = blockDim.x / CV;
  for (int i = threadIdx.x, k = 0; i < items; i += blockDim.x, ++k) {
    int ow = ow0 + k * ostep, cv = cv0;
    if (!fixed) {
      ow = i / CV;
      cv = i - ow * CV;
      bn_load8(a, cv, av);
      bn_load8(b, cv, bv);
    }
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int h = 2 * oh - 1 + kh;
      if (h < 0 || h >= H) continue;
      const long rbase = ((long)n * H + h) * W;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int w = 2 * ow - 1 + kw;
        if (w < 0 || w >= W) continue;
        const u16x8 xv = reinterpret_cast<const u16x8*>(x)[(rbase + w) * CV + cv];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // compare the bf16-rounded activation: the pooled value is the BN output as stored
          const float t8 = bf2f(f2bf(fmaxf(bn_pre(bf2f(xv[j]), av[j], bv[j], 0.f), 0.f)));
          if (t8 > best[j]) { best[j] = t8; bi[j] = (uint8_t)(kh * 3 + kw); }
        }
      }
    }
    u16x8 o;
    uint64_t packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) { o[j] = f2bf(best[j]); packed |= (uint64_t)bi[j] << (8 * j); }
    reinterpret_cast<u16x8*>(y)[orow + i] = o;
    reinterpret_cast<uint64_t*>(arg)[orow + i] = packed;
  }
}

// dx[n,h,w,c] = sum of dy over the (<= 4) pooling windows whose argmax is (h, w): a gather, so
// no zero-fill and no atomics.  Block = one input row (n, h) (its <= 2 window rows are
// block-uniform); thread = (w, 8-channel chunk) items of that row.
__global__ __launch_bounds__(256) void maxpool3s2_bwd_kernel(const bf16_t* __restrict__ dy,
                                                             const uint8_t* __restrict__ arg,
                                                             bf16_t* __restrict__ dx, int N, int H, int W, int CV,
                                                             int OH, int OW) {
  const int n = blockIdx.x / H, h = blockIdx.x - n * H;
  const int items = W * CV;
  // windows o with 2o-1 <= h <= 2o+1
  const int oh0 = h >> 1, oh1 = min((h + 1) >> 1, OH - 1);
  const long xrow = ((long)n * H + h) * W * CV;
  const bool fixed = bn_fixed_cv(CV);
  const int cv0 = threadIdx.x % CV, w0 = threadIdx.x / CV, wstep = blockDim.x / CV;
  for (int i = threadIdx.x, k = 0; i < items; i += blockDim.x, ++k) {
    int w = w0 + k * wstep, cv = cv0;
    if (!fixed) {
      w = i / CV;
      cv = i - w * CV;
    }
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    const int ow0 = w >> 1, ow1 = min((w + 1) >> 1, OW - 1);
    // the (at most 2 x 2) windows containing this pixel: all their argmax / gradient loads are
    // issued before any is used (the nested loop with its early continues waited once per window)
    uint64_t pk[4];
    u16x8 gv[4];
    uint8_t pos[4];
    bool ok[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oh = oh0 + (q >> 1), ow = ow0 + (q & 1);
      const int kh = h - (2 * oh - 1), kw = w - (2 * ow - 1);
      ok[q] = oh <= oh1 && ow <= ow1 && kh >= 0 && kh <= 2 && kw >= 0 && kw <= 2;
      const long o = ok[q] ? (((long)n * OH + oh) * OW + ow) * CV + cv : 0;
      pk[q] = ok[q] ? reinterpret_cast<const uint64_t*>(arg)[o] : 0ull;
      gv[q] = ok[q] ? reinterpret_cast<const u16x8*>(dy)[o] : u16x8(0);
      pos[q] = (uint8_t)(kh * 3 + kw);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!ok[q]) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (((pk[q] >> (8 * j)) & 0xFF) == pos[q]) acc[j] += bf2f(gv[q][j]);
    }
    u16x8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = f2bf(acc[j]);
    reinterpret_cast<u16x8*>(dx)[xrow + i] = out;
  }
}

// The stem backward in one pass over the pool's input grid: the max-pool gradient gather (as
// maxpool3s2_bwd_kernel), the ReLU mask recomputed from the BatchNorm input x (y = relu(a x + b)
// as the forward rounded it), the masked gradient dy' stored, and the BatchNorm-backward sums
// of dy' and dy' * xhat per channel for this block's row -- partial row n * H + h of p1 / p2
// (what bn_bwd_given finalizes).  Replaces the separate reduction pass that re-read dy and x
// (bn_bwd_reduce_kernel over 256 x 112 x 112 x 64).  Requires CV | 256 (fixed chunk per thread).
constexpr int MPB_ROWS = 4;   // input rows per workgroup of maxpool3s2_bwd_bn_kernel
__global__ __launch_bounds__(256) void maxpool3s2_bwd_bn_kernel(const bf16_t* __restrict__ dy,
                                                                const uint8_t* __restrict__ arg,
                                                                const bf16_t* __restrict__ x,
                                                                const float* __restrict__ stat,
                                                                bf16_t* __restrict__ dx, float* __restrict__ p1,
                                                                float* __restrict__ p2, int N, int H, int W, int CV,
                                                                int OH, int OW) {
  __shared__ float r1[4][256], r2[4][256];
  const int HB = (H + MPB_ROWS - 1) / MPB_ROWS;
  const int n = blockIdx.x / HB, h0 = (blockIdx.x - n * HB) * MPB_ROWS;
  const int items = W * CV, C = CV * 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cv0 = threadIdx.x % CV, w0 = threadIdx.x / CV, wstep = blockDim.x / CV;
  float mu[8], is[8], fa[8], fb[8], s1[8], s2[8];
  bn_load8(stat, cv0, mu);
  bn_load8(stat + C, cv0, is);
  bn_load8(stat + 2 * C, cv0, fa);
  bn_load8(stat + 3 * C, cv0, fb);
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  for (int h = h0; h < min(H, h0 + MPB_ROWS); ++h) {
    const int oh0 = h >> 1, oh1 = min((h + 1) >> 1, OH - 1);
    const long xrow = ((long)n * H + h) * W * CV;
    for (int i = threadIdx.x, k = 0; i < items; i += blockDim.x, ++k) {
      const int w = w0 + k * wstep;
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
      const int ow0 = w >> 1, ow1 = min((w + 1) >> 1, OW - 1);
      const u16x8 xv = reinterpret_cast<const u16x8*>(x)[xrow + i];
      // the (at most 2 x 2) windows' loads all issued before use (as maxpool3s2_bwd_kernel)
      uint64_t pk[4];
      u16x8 gv[4];
      uint8_t pos[4];
      bool ok[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int oh = oh0 + (q >> 1), ow = ow0 + (q & 1);
        const int kh = h - (2 * oh - 1), kw = w - (2 * ow - 1);
        ok[q] = oh <= oh1 && ow <= ow1 && kh >= 0 && kh <= 2 && kw >= 0 && kw <= 2;
        const long o = ok[q] ? (((long)n * OH + oh) * OW + ow) * CV + cv0 : 0;
        pk[q] = ok[q] ? reinterpret_cast<const uint64_t*>(arg)[o] : 0ull;
        gv[q] = ok[q] ? reinterpret_cast<const u16x8*>(dy)[o] : u16x8(0);
        pos[q] = (uint8_t)(kh * 3 + kw);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (!ok[q]) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (((pk[q] >> (8 * j)) & 0xFF) == pos[q]) acc[j] += bf2f(gv[q][j]);
      }
      u16x8 out;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xf = bf2f(xv[j]);
        const bool on = bf2f(f2bf(bn_pre(xf, fa[j], fb[j], 0.f))) > 0.f;
        out[j] = on ? f2bf(acc[j]) : (unsigned short)0;
        const float d = bf2f(out[j]);
        s1[j] += d;
        s2[j] += d * (xf - mu[j]) * is[j];
      }
      reinterpret_cast<u16x8*>(dx)[xrow + i] = out;
    }
  }
  // per-channel sums: lanes of one wave holding the same chunk (lane % CV) folded by xor
  // shuffles, then the 4 waves through LDS
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    for (int m = CV; m < 64; m <<= 1) {
      s1[j] += __shfl_xor(s1[j], m, 64);
      s2[j] += __shfl_xor(s2[j], m, 64);
    }
  }
  if (lane < CV) {                                // CV <= 32: every chunk in every wave
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      r1[wave][lane * 8 + j] = s1[j];
      r2[wave][lane * 8 + j] = s2[j];
    }
  }
  __syncthreads();
  const long prow = (long)blockIdx.x * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {   // chunk c >> 3 is lane c >> 3 of every wave
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) { t1 += r1[q][c]; t2 += r2[q][c]; }
    p1[prow + c] = t1;
    p2[prow + c] = t2;
  }
}

inline BnLayout bn_layout(int M, int C, int target_blocks) {
  BnLayout L;
  L.M = M; L.C = C; L.CV = C / 8;
  L.RPI = BN_RT / L.CV;
  if (L.RPI < 1) L.RPI = 1;
  int nblk = target_blocks;
  const int min_rows = L.RPI * 8;
  if ((long)nblk * min_rows > M) nblk = (M + min_rows - 1) / min_rows;
  if (nblk < 1) nblk = 1;
  L.rows_per_blk = (M + nblk - 1) / nblk;
  return L;
}
inline int bn_nblk(const BnLayout& L) { return (L.M + L.rows_per_blk - 1) / L.rows_per_blk; }

inline int ew_grid(long work, int ew) {
  long g = (work + 256L * ew - 1) / (256L * ew);   // >= ew vectors per thread
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace ct

using namespace ct;

namespace ct {
// dx = a dm + k x + z and dx2 = a2 dm + k2 x2 + z2 from ONE read of the (already ReLU-masked)
// gradient dm: the two BatchNorms of a ResNet downsample block's residual sum (bn3, down_bn)
__global__ __launch_bounds__(256) void bn_bwd_apply2_kernel(
    const bf16_t* __restrict__ dm, const bf16_t* __restrict__ x, const float* __restrict__ ca,
    const float* __restrict__ c1, const float* __restrict__ c0, const bf16_t* __restrict__ x2,
    const float* __restrict__ ca2, const float* __restrict__ c12, const float* __restrict__ c02,
    bf16_t* __restrict__ dx, bf16_t* __restrict__ dx2, long total_vec, int CV) {
  const long stride = (long)gridDim.x * blockDim.x;
  const bool fixed = bn_fixed_cv(CV);
  float aa[8], kk[8], zz[8], a2[8], k2[8], z2[8];
  if (fixed) {
    const int cv = threadIdx.x % CV;
    bn_load8(ca, cv, aa); bn_load8(c1, cv, kk); bn_load8(c0, cv, zz);
    bn_load8(ca2, cv, a2); bn_load8(c12, cv, k2); bn_load8(c02, cv, z2);
  }
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < total_vec; v += stride) {
    const u16x8 g = reinterpret_cast<const u16x8*>(dm)[v];
    const u16x8 xv = reinterpret_cast<const u16x8*>(x)[v];
    const u16x8 x2v = reinterpret_cast<const u16x8*>(x2)[v];
    if (!fixed) {
      const int cv = (int)(v % CV);
      bn_load8(ca, cv, aa); bn_load8(c1, cv, kk); bn_load8(c0, cv, zz);
      bn_load8(ca2, cv, a2); bn_load8(c12, cv, k2); bn_load8(c02, cv, z2);
    }
    u16x8 o, o2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = bf2f(g[j]);
      o[j] = f2bf(aa[j] * d + kk[j] * bf2f(xv[j]) + zz[j]);
      o2[j] = f2bf(a2[j] * d + k2[j] * bf2f(x2v[j]) + z2[j]);
    }
    reinterpret_cast<u16x8*>(dx)[v] = o;
    reinterpret_cast<u16x8*>(dx2)[v] = o2;
  }
}
}  // namespace ct

extern "C" int ct_bn_max_blocks() { return 2048; }

// vectors per thread per iteration of the apply kernels (CLOUDTIK_AMD_BN_EW: 1, 2 or 4)
static int bn_ew() {
  static int n = [] {
    const char* e = getenv("CLOUDTIK_AMD_BN_EW");
    int v = e ? atoi(e) : 1;
    return v >= 4 ? 4 : (v >= 2 ? 2 : 1);
  }();
  return n;
}

#define BN_EW_DISPATCH(KERNEL, GRIDWORK, ...)                                              \
  do {                                                                                       \
    const int ew_ = bn_ew();                                                                 \
    if (ew_ == 4) KERNEL<4><<<ew_grid(GRIDWORK, 4), 256, 0, stream>>>(__VA_ARGS__);          \
    else if (ew_ == 2) KERNEL<2><<<ew_grid(GRIDWORK, 2), 256, 0, stream>>>(__VA_ARGS__);     \
    else KERNEL<1><<<ew_grid(GRIDWORK, 1), 256, 0, stream>>>(__VA_ARGS__);                   \
  } while (0)

// rows in flight per thread in the reductions (CLOUDTIK_AMD_BN_UNROLL: 4 or 8)
static int bn_unroll() {
  static int n = [] {
    const char* e = getenv("CLOUDTIK_AMD_BN_UNROLL");
    return (e && atoi(e) >= 8) ? 8 : 4;
  }();
  return n;
}

// partial-block count of the reductions (CLOUDTIK_AMD_BN_BLOCKS, <= 2048; default 512)
static int bn_target_blocks() {
  static int n = [] {
    const char* e = getenv("CLOUDTIK_AMD_BN_BLOCKS");
    int v = e ? atoi(e) : 512;
    return v < 64 ? 64 : (v > 2048 ? 2048 : v);
  }();
  return n;
}

// workspace: part = float[2 * 2048 * C]; stat = float[4 * C] (save_mean, save_invstd, a, b)
extern "C" int ct_bn_fwd_train(const void* x, const void* res, const void* gamma, const void* beta,
                               float* run_mean, float* run_var, void* y, float* part, float* stat,
                               int M, int C, float eps, float momentum, int relu, void* mask,
                               hipStream_t stream) {
  if (C % 8 || C / 8 > BN_RT || M <= 0) return -1;
  BnLayout L = bn_layout(M, C, bn_target_blocks());
  const int nblk = bn_nblk(L);
  if (bn_unroll() == 8) bn_stats_kernel<8><<<nblk, BN_RT, 0, stream>>>((const bf16_t*)x, L, part, part + (size_t)2048 * C);
  else bn_stats_kernel<4><<<nblk, BN_RT, 0, stream>>>((const bf16_t*)x, L, part, part + (size_t)2048 * C);
  bn_finalize_kernel<<<ceil_div(C, 64), 1024, 0, stream>>>(part, part + (size_t)2048 * C, nblk, L,
                                                           (const bf16_t*)gamma, (const bf16_t*)beta,
                                                           eps, momentum, run_mean, run_var, stat,
                                                           stat + C, stat + 2 * C, stat + 3 * C);
  const long tv = (long)M * (C / 8);
  BN_EW_DISPATCH(bn_apply_kernel, tv, (const bf16_t*)x, (const bf16_t*)res, stat + 2 * C, stat + 3 * C,
                 (bf16_t*)y, (uint8_t*)mask, tv, C / 8, relu);
  return 0;
}

// First-level merge of per-block (mean, M2) partials: block (g, cb) merges partials
// [g * GROUP, (g + 1) * GROUP) of channels [64 cb, 64 cb + 64) -- one lane per channel, the 4
// waves take interleaved partials and are combined through LDS -- into one (mean, M2) partial
// of GROUP * rows_per_tile rows.  The conv epilogue emits one partial per 64-row wave block
// (12544 for a ResNet-50 layer-1 conv); the single-block-per-64-channels finalize would read
// them serially.
constexpr int BN_MERGE_GROUP = 64;
// Two passes over the group's partials (they stay in cache) instead of a sequential Chan merge:
// mean_g = sum(n_t mean_t) / sum(n_t), then M2_g = sum(M2_t + n_t (mean_t - mean_g)^2) -- no
// division inside the loop (the dependent divisions of the sequential merge made it
// latency-bound: 52 launches, 0.47 ms per ResNet-50 step).
__global__ __launch_bounds__(256) void bn_partials_merge_kernel(const float* __restrict__ pmean,
                                                               const float* __restrict__ pm2, int tiles,
                                                               int rows_per_tile, int M, int C,
                                                               float* __restrict__ omean, float* __restrict__ om2) {
  __shared__ float sn[4][64], ss[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + lane, g = blockIdx.x;
  const int t0 = g * BN_MERGE_GROUP, t1 = min(tiles, t0 + BN_MERGE_GROUP);
  const bool live = c < C;
  // the thread's BN_MERGE_GROUP / 4 rows of both arrays in one round of loads, kept in registers
  // for the second pass
  constexpr int KR = BN_MERGE_GROUP / 4;
  float mv[KR], m2v[KR];
  float n = 0.f, s = 0.f;
  if (live) {
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int t = t0 + w + 4 * k;
      mv[k] = t < t1 ? pmean[(size_t)t * C + c] : 0.f;
      m2v[k] = t < t1 ? pm2[(size_t)t * C + c] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int t = t0 + w + 4 * k;
      const float nb = t < t1 ? (float)max(0, min(rows_per_tile, M - t * rows_per_tile)) : 0.f;
      n += nb;
      s += nb * mv[k];
    }
  }
  sn[w][lane] = n;
  ss[w][lane] = s;
  __syncthreads();
  const float ng = sn[0][lane] + sn[1][lane] + sn[2][lane] + sn[3][lane];
  const float mg = ng > 0.f ? (ss[0][lane] + ss[1][lane] + ss[2][lane] + ss[3][lane]) / ng : 0.f;
  float q = 0.f;
  if (live) {
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int t = t0 + w + 4 * k;
      const float nb = t < t1 ? (float)max(0, min(rows_per_tile, M - t * rows_per_tile)) : 0.f;
      const float d = mv[k] - mg;
      q += m2v[k] + nb * d * d;
    }
  }
  __syncthreads();                                    // ss reuse
  ss[w][lane] = q;
  __syncthreads();
  if (w != 0 || !live) return;
  omean[(size_t)g * C + c] = mg;
  om2[(size_t)g * C + c] = ss[0][lane] + ss[1][lane] + ss[2][lane] + ss[3][lane];
}

// Training forward whose statistics were produced by the PRODUCER of x: per-tile means
// [tiles][C] and M2 [tiles][C] over rows_per_tile rows each (the implicit-GEMM conv epilogue,
// conv.hip).  Only the finalize and the apply pass run: x is read once instead of twice.
// Up to this many per-tile partials the finalize kernels (16 row lanes x 64 channels, loads 8
// deep) read them directly: a first-level merge / sum launch plus its dependent-launch gap costs
// more than the finalize's few extra loads (the layer-4 BatchNorms of ResNet-50: 196 forward
// partials, 98 backward tiles).  CLOUDTIK_AMD_BN_DIRECT_TILES=0: the merge above 128 partials
// and the backward sum always, as before.
static int bn_direct_tiles() {
  static int n = [] {
    const char* e = getenv("CLOUDTIK_AMD_BN_DIRECT_TILES");
    return e ? atoi(e) : 256;
  }();
  return n;
}

// merge (when many) + finalize of producer partials into stat = float[4C]
static void bn_given_finalize(const float* part, int tiles, int rows_per_tile, const void* gamma, const void* beta,
                              float* run_mean, float* run_var, float* stat, int M, int C, float eps, float momentum,
                              hipStream_t stream) {
  if (tiles > std::max(2 * BN_MERGE_GROUP, bn_direct_tiles())) {
    const int groups = ceil_div(tiles, BN_MERGE_GROUP);
    float* om = const_cast<float*>(part) + (size_t)2 * tiles * C;
    bn_partials_merge_kernel<<<dim3(groups, ceil_div(C, 64)), 256, 0, stream>>>(
        part, part + (size_t)tiles * C, tiles, rows_per_tile, M, C, om, om + (size_t)groups * C);
    part = om;
    tiles = groups;
    rows_per_tile *= BN_MERGE_GROUP;
  }
  BnLayout L{M, C, C / 8, 1, rows_per_tile};
  bn_finalize_kernel<<<ceil_div(C, 64), 1024, 0, stream>>>(part, part + (size_t)tiles * C, tiles, L,
                                                           (const bf16_t*)gamma, (const bf16_t*)beta,
                                                           eps, momentum, run_mean, run_var, stat,
                                                           stat + C, stat + 2 * C, stat + 3 * C);
}

// Two BatchNorms with producer partials, y = relu(bn(x) + bn2(x2)) + bitmask (bn_apply2_kernel)
extern "C" int ct_bn_fwd_train_given2(const void* x, const void* gamma, const void* beta, float* run_mean,
                                      float* run_var, const float* part, int tiles, int rows_per_tile, float* stat,
                                      const void* x2, const void* gamma2, const void* beta2, float* run_mean2,
                                      float* run_var2, const float* part2, int tiles2, int rows_per_tile2,
                                      float* stat2, void* y, void* mask, int M, int C, float eps, float momentum,
                                      hipStream_t stream) {
  if (C % 8 || M <= 0 || tiles <= 0 || tiles2 <= 0 || (long)tiles * rows_per_tile < M ||
      (long)tiles2 * rows_per_tile2 < M || !mask)
    return -1;
  bn_given_finalize(part, tiles, rows_per_tile, gamma, beta, run_mean, run_var, stat, M, C, eps, momentum, stream);
  bn_given_finalize(part2, tiles2, rows_per_tile2, gamma2, beta2, run_mean2, run_var2, stat2, M, C, eps, momentum,
                    stream);
  const long tv = (long)M * (C / 8);
  bn_apply2_kernel<<<ew_grid(tv, 1), 256, 0, stream>>>((const bf16_t*)x, stat + 2 * C, stat + 3 * C,
                                                       (const bf16_t*)x2, stat2 + 2 * C, stat2 + 3 * C, (bf16_t*)y,
                                                       (uint8_t*)mask, tv, C / 8);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

extern "C" int ct_bn_fwd_train_given(const void* x, const void* res, const void* gamma, const void* beta,
                                     float* run_mean, float* run_var, void* y, const float* part, int tiles,
                                     int rows_per_tile, float* stat, int M, int C, float eps, float momentum,
                                     int relu, void* mask, hipStream_t stream) {
  if (C % 8 || M <= 0 || tiles <= 0 || (long)tiles * rows_per_tile < M) return -1;
  if (tiles > std::max(2 * BN_MERGE_GROUP, bn_direct_tiles())) {
    // merge groups of tiles first, into the tail of the partial buffer (means at
    // part + 2 tiles C, then the M2 rows): the finalize then reads at most 2 * GROUP partials
    const int groups = ceil_div(tiles, BN_MERGE_GROUP);
    float* om = const_cast<float*>(part) + (size_t)2 * tiles * C;
    bn_partials_merge_kernel<<<dim3(groups, ceil_div(C, 64)), 256, 0, stream>>>(
        part, part + (size_t)tiles * C, tiles, rows_per_tile, M, C, om, om + (size_t)groups * C);
    part = om;
    tiles = groups;
    rows_per_tile *= BN_MERGE_GROUP;
  }
  BnLayout L{M, C, C / 8, 1, rows_per_tile};
  bn_finalize_kernel<<<ceil_div(C, 64), 1024, 0, stream>>>(part, part + (size_t)tiles * C, tiles, L,
                                                           (const bf16_t*)gamma, (const bf16_t*)beta,
                                                           eps, momentum, run_mean, run_var, stat,
                                                           stat + C, stat + 2 * C, stat + 3 * C);
  const long tv = (long)M * (C / 8);
  BN_EW_DISPATCH(bn_apply_kernel, tv, (const bf16_t*)x, (const bf16_t*)res, stat + 2 * C, stat + 3 * C,
                 (bf16_t*)y, (uint8_t*)mask, tv, C / 8, relu);
  return 0;
}

// ResNet stem: batch statistics of x, then y = maxpool3x3/s2/p1(relu(bn(x))) + byte argmax
// (stat = float[4C] as ct_bn_fwd_train)
extern "C" int ct_bn_fwd_train_pool(const void* x, const void* gamma, const void* beta, float* run_mean,
                                    float* run_var, void* y, void* arg, float* part, float* stat, int N, int H, int W,
                                    int C, int OH, int OW, float eps, float momentum, hipStream_t stream) {
  const int M = N * H * W;
  if (C % 8 || C / 8 > BN_RT || M <= 0 || OH != (H - 1) / 2 + 1 || OW != (W - 1) / 2 + 1) return -1;
  BnLayout L = bn_layout(M, C, bn_target_blocks());
  const int nblk = bn_nblk(L);
  if (bn_unroll() == 8) bn_stats_kernel<8><<<nblk, BN_RT, 0, stream>>>((const bf16_t*)x, L, part, part + (size_t)2048 * C);
  else bn_stats_kernel<4><<<nblk, BN_RT, 0, stream>>>((const bf16_t*)x, L, part, part + (size_t)2048 * C);
  bn_finalize_kernel<<<ceil_div(C, 64), 1024, 0, stream>>>(part, part + (size_t)2048 * C, nblk, L,
                                                           (const bf16_t*)gamma, (const bf16_t*)beta,
                                                           eps, momentum, run_mean, run_var, stat,
                                                           stat + C, stat + 2 * C, stat + 3 * C);
  if ((long)N * OH >= (1L << 31)) return -1;
  bn_apply_pool_kernel<<<N * OH, 256, 0, stream>>>((const bf16_t*)x, stat + 2 * C, stat + 3 * C, (bf16_t*)y,
                                                   (uint8_t*)arg, N, H, W, C / 8, OH, OW);
  return 0;
}

// The same with the statistics from the stem conv's epilogue partials (conv.hip EPI 1): no
// statistics pass over the full-resolution conv output
extern "C" int ct_bn_fwd_train_pool_given(const void* x, const void* gamma, const void* beta, float* run_mean,
                                          float* run_var, void* y, void* arg, const float* part, int tiles,
                                          int rows_per_tile, float* stat, int N, int H, int W, int C, int OH, int OW,
                                          float eps, float momentum, hipStream_t stream) {
  const int M = N * H * W;
  if (C % 8 || M <= 0 || tiles <= 0 || (long)tiles * rows_per_tile < M || OH != (H - 1) / 2 + 1 ||
      OW != (W - 1) / 2 + 1 || (long)N * OH >= (1L << 31))
    return -1;
  bn_given_finalize(part, tiles, rows_per_tile, gamma, beta, run_mean, run_var, stat, M, C, eps, momentum, stream);
  bn_apply_pool_kernel<<<N * OH, 256, 0, stream>>>((const bf16_t*)x, stat + 2 * C, stat + 3 * C, (bf16_t*)y,
                                                   (uint8_t*)arg, N, H, W, C / 8, OH, OW);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

extern "C" int ct_maxpool3s2_bwd(const void* dy, const void* arg, void* dx, int N, int H, int W, int C, int OH,
                                 int OW, hipStream_t stream) {
  if (C % 8 || OH != (H - 1) / 2 + 1 || OW != (W - 1) / 2 + 1) return -1;
  if ((long)N * H >= (1L << 31)) return -1;
  maxpool3s2_bwd_kernel<<<N * H, 256, 0, stream>>>((const bf16_t*)dy, (const uint8_t*)arg, (bf16_t*)dx, N, H, W,
                                                   C / 8, OH, OW);
  return 0;
}

// partial rows (= workgroups) of ct_maxpool3s2_bwd_bn
extern "C" long ct_maxpool3s2_bwd_bn_rows(int N, int H) { return (long)N * ((H + MPB_ROWS - 1) / MPB_ROWS); }

// maxpool3s2_bwd + the stem BatchNorm's backward reduction (maxpool3s2_bwd_bn_kernel): dxm = the
// masked gradient, part = float[2 * N * H * C] (p1 rows then p2 rows), stat = the forward's float[4C]
extern "C" int ct_maxpool3s2_bwd_bn(const void* dy, const void* arg, const void* x, const float* stat, void* dxm,
                                    float* part, int N, int H, int W, int C, int OH, int OW, hipStream_t stream) {
  if (C % 8 || 256 % (C / 8) || OH != (H - 1) / 2 + 1 || OW != (W - 1) / 2 + 1) return -1;
  // one partial row per workgroup (MPB_ROWS input rows); C <= 256 (CV <= 32 chunks, folded
  // inside each wave)
  if (C / 8 > 32) return -1;
  const long rows = (long)N * ((H + MPB_ROWS - 1) / MPB_ROWS);
  if (rows >= (1L << 31)) return -1;
  maxpool3s2_bwd_bn_kernel<<<(int)rows, 256, 0, stream>>>((const bf16_t*)dy, (const uint8_t*)arg,
                                                          (const bf16_t*)x, stat, (bf16_t*)dxm, part,
                                                          part + rows * C, N, H, W, C / 8, OH, OW);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

// inference-mode forward with given affine coefficients a, b (float[C] each)
extern "C" int ct_bn_apply(const void* x, const void* res, const float* a, const float* b, void* y,
                           int M, int C, int relu, hipStream_t stream) {
  if (C % 8) return -1;
  const long tv = (long)M * (C / 8);
  BN_EW_DISPATCH(bn_apply_kernel, tv, (const bf16_t*)x, (const bf16_t*)res, a, b, (bf16_t*)y, (uint8_t*)nullptr, tv,
                 C / 8, relu);
  return 0;
}

// stat = the forward's float[4C] (mean, invstd, a, b).  relu_mode: 0 none, 1 read y,
// 2 recompute from x (no residual in the forward).  part = float[2 * 2048 * C],
// coef = float[3 * C] scratch.
extern "C" int ct_bn_bwd(const void* dy, const void* y, const void* x, const void* gamma, const float* stat,
                         void* dx, void* dres, void* dgamma, void* dbeta, int param_flags, float* part,
                         float* coef, int M, int C, int relu_mode, hipStream_t stream) {
  if (C % 8 || C / 8 > BN_RT || M <= 0 || relu_mode < 0 || relu_mode > 3) return -1;
  if ((relu_mode == 1 || relu_mode == 3) && !y) return -2;
  BnLayout L = bn_layout(M, C, bn_target_blocks());
  const int nblk = bn_nblk(L);
  // relu_mode 3: `y` is the forward's ReLU bitmask
  const BnMask mk{relu_mode, relu_mode == 1 ? (const bf16_t*)y : nullptr, stat + 2 * C, stat + 3 * C,
                  relu_mode == 3 ? (const uint8_t*)y : nullptr};
  // BN + residual add + ReLU: the reduction pass writes the masked gradient (= the residual
  // branch's gradient, returned as dres) and the apply pass reads it back instead of dy and y:
  // 7 instead of 8 activation-sized passes over the biggest ResNet tensors
  bf16_t* dm = ((relu_mode == 1 || relu_mode == 3) && dres) ? (bf16_t*)dres : nullptr;
  if (bn_unroll() == 8)
    bn_bwd_reduce_kernel<8><<<nblk, BN_RT, 0, stream>>>((const bf16_t*)dy, mk, (const bf16_t*)x, stat, stat + C, L,
                                                        part, part + (size_t)2048 * C, dm);
  else
    bn_bwd_reduce_kernel<4><<<nblk, BN_RT, 0, stream>>>((const bf16_t*)dy, mk, (const bf16_t*)x, stat, stat + C, L,
                                                        part, part + (size_t)2048 * C, dm);
  const int acc = (param_flags >> 1) & 1;   // bit 1: accumulate into dgamma / dbeta
  if (param_flags & 1)
    bn_bwd_finalize_kernel<float><<<ceil_div(C, 64), 1024, 0, stream>>>(
        part, part + (size_t)2048 * C, nblk, M, C, (const bf16_t*)gamma, stat, stat + C,
        (float*)dgamma, (float*)dbeta, coef, coef + C, coef + 2 * C, acc);
  else
    bn_bwd_finalize_kernel<bf16_t><<<ceil_div(C, 64), 1024, 0, stream>>>(
        part, part + (size_t)2048 * C, nblk, M, C, (const bf16_t*)gamma, stat, stat + C,
        (bf16_t*)dgamma, (bf16_t*)dbeta, coef, coef + C, coef + 2 * C, acc);
  const long tv = (long)M * (C / 8);
  if (dm) {
    const BnMask none{0, nullptr, nullptr, nullptr, nullptr};
    BN_EW_DISPATCH(bn_bwd_apply_kernel, tv, (const bf16_t*)dm, none, (const bf16_t*)x, coef, coef + C, coef + 2 * C,
                   (bf16_t*)dx, (bf16_t*)nullptr, tv, C / 8);
  } else {
    BN_EW_DISPATCH(bn_bwd_apply_kernel, tv, (const bf16_t*)dy, mk, (const bf16_t*)x, coef, coef + C, coef + 2 * C,
                   (bf16_t*)dx, (bf16_t*)dres, tv, C / 8);
  }
  return 0;
}

// first-level sum of per-tile BatchNorm-backward partials (the conv data-gradient epilogue's,
// conv.hip EPI 2: thousands of tile rows): rows [64 g, 64 g + 64) of p1 / p2 -> row g of
// q1 / q2.  A block covers min(C, 256) channels (coalesced) and R = 256 / that many tile rows
// in parallel, summed through LDS: at 64 channels (ResNet layer 1) a thread loads 16 rows, not
// 64 in eight dependent rounds with three of its four waves idle (10.8 us per call).
__global__ __launch_bounds__(256) void bn_bwd_partials_sum_kernel(const float* __restrict__ p1,
                                                                 const float* __restrict__ p2, int tiles, int C,
                                                                 float* __restrict__ q1, float* __restrict__ q2) {
  __shared__ float sa[256], sb[256];
  const int Cb = C < 256 ? C : 256, R = 256 / Cb;
  const int r = threadIdx.x / Cb, cl = threadIdx.x - r * Cb;
  const int c = blockIdx.y * 256 + cl;
  const bool live = r < R && c < C;
  const int t0 = blockIdx.x * 64, t1 = min(tiles, t0 + 64);
  float a = 0.f, b = 0.f;
  if (live) {
#pragma unroll 8
    for (int t = t0 + r; t < t1; t += R) {
      a += p1[(size_t)t * C + c];
      b += p2[(size_t)t * C + c];
    }
  }
  sa[threadIdx.x] = a;
  sb[threadIdx.x] = b;
  __syncthreads();
  if (r != 0 || !live) return;
  for (int k = 1; k < R; ++k) {
    a += sa[k * Cb + cl];
    b += sb[k * Cb + cl];
  }
  q1[(size_t)blockIdx.x * C + c] = a;
  q2[(size_t)blockIdx.x * C + c] = b;
}

// BatchNorm (+ ReLU) backward whose reduction was done by the producer of dy (conv.hip EPI 2):
// dym = the already-masked gradient, p1 / p2 = per-tile sums [tiles][C] (p2 = p1 + p2off).
// work = float[2 * ceil(tiles / 64) * C + 3 * C] scratch.
// The two BatchNorm backwards of a ResNet downsample block's residual sum relu(bn(x) + bn2(x2)):
// dym = the masked gradient (the conv epilogue's), p1 / p2 = bn's per-tile sums from that epilogue;
// bn2's sums come from its own reduction pass over dym and x2; then ONE apply pass writes dx and
// dx2 (bn_bwd_apply2_kernel).  param_flags as ct_bn_bwd_given (both parameter pairs alike);
// work = float[2 * ceil(tiles / 64) * C + 3 * C], part2 = float[2 * 2048 * C], coef2 = float[3C].
extern "C" int ct_bn_bwd_given_pair(const void* dym, const void* x, const void* gamma, const float* stat,
                                    const float* p1, long p2off, int tiles, const void* x2, const void* gamma2,
                                    const float* stat2, void* dx, void* dx2, void* dgamma, void* dbeta,
                                    void* dgamma2, void* dbeta2, int param_flags, float* work, float* part2,
                                    float* coef2, int M, int C, hipStream_t stream) {
  if (C % 8 || C / 8 > BN_RT || C > 2048 || M <= 0 || tiles <= 0) return -1;
  const int G = (tiles + 63) / 64;
  float* q1 = work;
  float* q2 = work + (size_t)G * C;
  float* coef = q2 + (size_t)G * C;
  int nq = G;
  if (tiles <= bn_direct_tiles()) {
    q1 = const_cast<float*>(p1);
    q2 = const_cast<float*>(p1) + p2off;
    nq = tiles;
  } else {
    bn_bwd_partials_sum_kernel<<<dim3(G, ceil_div(C, 256)), 256, 0, stream>>>(p1, p1 + p2off, tiles, C, q1, q2);
  }
  BnLayout L = bn_layout(M, C, bn_target_blocks());
  const int nblk = bn_nblk(L);
  const BnMask none{0, nullptr, nullptr, nullptr, nullptr};
  if (bn_unroll() == 8)
    bn_bwd_reduce_kernel<8><<<nblk, BN_RT, 0, stream>>>((const bf16_t*)dym, none, (const bf16_t*)x2, stat2,
                                                        stat2 + C, L, part2, part2 + (size_t)2048 * C, nullptr);
  else
    bn_bwd_reduce_kernel<4><<<nblk, BN_RT, 0, stream>>>((const bf16_t*)dym, none, (const bf16_t*)x2, stat2,
                                                        stat2 + C, L, part2, part2 + (size_t)2048 * C, nullptr);
  const int acc = (param_flags >> 1) & 1;
  if (param_flags & 1) {
    bn_bwd_finalize_kernel<float><<<ceil_div(C, 64), 1024, 0, stream>>>(
        q1, q2, nq, M, C, (const bf16_t*)gamma, stat, stat + C, (float*)dgamma, (float*)dbeta, coef, coef + C,
        coef + 2 * C, acc);
    bn_bwd_finalize_kernel<float><<<ceil_div(C, 64), 1024, 0, stream>>>(
        part2, part2 + (size_t)2048 * C, nblk, M, C, (const bf16_t*)gamma2, stat2, stat2 + C, (float*)dgamma2,
        (float*)dbeta2, coef2, coef2 + C, coef2 + 2 * C, acc);
  } else {
    bn_bwd_finalize_kernel<bf16_t><<<ceil_div(C, 64), 1024, 0, stream>>>(
        q1, q2, nq, M, C, (const bf16_t*)gamma, stat, stat + C, (bf16_t*)dgamma, (bf16_t*)dbeta, coef, coef + C,
        coef + 2 * C, acc);
    bn_bwd_finalize_kernel<bf16_t><<<ceil_div(C, 64), 1024, 0, stream>>>(
        part2, part2 + (size_t)2048 * C, nblk, M, C, (const bf16_t*)gamma2, stat2, stat2 + C, (bf16_t*)dgamma2,
        (bf16_t*)dbeta2, coef2, coef2 + C, coef2 + 2 * C, acc);
  }
  const long tv = (long)M * (C / 8);
  bn_bwd_apply2_kernel<<<ew_grid(tv, 1), 256, 0, stream>>>((const bf16_t*)dym, (const bf16_t*)x, coef, coef + C,
                                                           coef + 2 * C, (const bf16_t*)x2, coef2, coef2 + C,
                                                           coef2 + 2 * C, (bf16_t*)dx, (bf16_t*)dx2, tv, C / 8);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

extern "C" int ct_bn_bwd_given(const void* dym, const void* x, const void* gamma, const float* stat, void* dx,
                               void* dgamma, void* dbeta, int param_flags, const float* p1, long p2off, int tiles,
                               float* work, int M, int C, hipStream_t stream) {
  if (C % 8 || C > 2048 || M <= 0 || tiles <= 0) return -1;
  const int G = (tiles + 63) / 64;
  float* q1 = work;
  float* q2 = work + (size_t)G * C;
  float* coef = q2 + (size_t)G * C;
  int nq = G;
  if (tiles <= bn_direct_tiles()) {            // the finalize sums the tile partials itself
    q1 = const_cast<float*>(p1);
    q2 = const_cast<float*>(p1) + p2off;
    nq = tiles;
  } else {
    bn_bwd_partials_sum_kernel<<<dim3(G, ceil_div(C, 256)), 256, 0, stream>>>(p1, p1 + p2off, tiles, C, q1, q2);
  }
  const int acc = (param_flags >> 1) & 1;
  if (param_flags & 1)
    bn_bwd_finalize_kernel<float><<<ceil_div(C, 64), 1024, 0, stream>>>(
        q1, q2, nq, M, C, (const bf16_t*)gamma, stat, stat + C, (float*)dgamma, (float*)dbeta, coef, coef + C,
        coef + 2 * C, acc);
  else
    bn_bwd_finalize_kernel<bf16_t><<<ceil_div(C, 64), 1024, 0, stream>>>(
        q1, q2, nq, M, C, (const bf16_t*)gamma, stat, stat + C, (bf16_t*)dgamma, (bf16_t*)dbeta, coef, coef + C,
        coef + 2 * C, acc);
  if (dx == nullptr) return hipGetLastError() == hipSuccess ? 0 : 7;   // coefficients only (work + 2 G C)
  const long tv = (long)M * (C / 8);
  const BnMask none{0, nullptr, nullptr, nullptr, nullptr};
  BN_EW_DISPATCH(bn_bwd_apply_kernel, tv, (const bf16_t*)dym, none, (const bf16_t*)x, coef, coef + C, coef + 2 * C,
                 (bf16_t*)dx, (bf16_t*)nullptr, tv, C / 8);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}
