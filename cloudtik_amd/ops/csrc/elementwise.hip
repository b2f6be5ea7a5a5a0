// Memory-bound fused elementwise kernels (bf16, 16-byte vectors per lane):
//   * bias + activation (GELU-erf / ReLU / identity) forward, and its backward with the
//     bias gradient column-sum fused in (FFN1 of BERT: the hipBLASLt GEMM runs bias-free,
//     this kernel adds the bias, applies GELU and keeps the pre-activation for backward).
//   * dropout forward/backward with a regenerated Philox mask (nothing stored).
//   * word + position + token-type embedding gather-sum and its atomic backward
//     (HF BertEmbeddings used by the reference BERT-large pretraining,
//     run_pretrain_mlperf.py:449-471).
//   * fp32 <-> bf16 casts, scaled adds.
#include "common.h"

namespace ct {

enum Act { ACT_NONE = 0, ACT_GELU = 1, ACT_RELU = 2 };

__device__ __forceinline__ float act_f(float x, int act) {
  return act == ACT_GELU ? gelu_erf(x) : (act == ACT_RELU ? fmaxf(x, 0.f) : x);
}
__device__ __forceinline__ float act_g(float x, int act) {
  return act == ACT_GELU ? gelu_erf_grad(x) : (act == ACT_RELU ? (x > 0.f ? 1.f : 0.f) : 1.f);
}

// y[m, n] = act(z[m, n] + bias[n]); rows x N, N % 8 == 0.
// 2-D mapping: blockIdx.x / threadIdx.x&63 pick a column vector (its bias lives in
// registers), the 4 waves of the block and blockIdx.y stride over rows, 4 rows per step
// so four independent 16-byte loads are in flight per lane (no 64-bit modulo per element).
constexpr int kBaRows = 4;
__global__ __launch_bounds__(256) void bias_act_fwd_kernel(const bf16_t* __restrict__ z,
                                                           const bf16_t* __restrict__ bias,
                                                           bf16_t* __restrict__ y, long M,
                                                           int nvec_row, int act) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if (c >= nvec_row) return;
  u16x8 bv = u16x8(0);
  if (bias) bv = reinterpret_cast<const u16x8*>(bias)[c];
  float b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = bf2f(bv[j]);
  const long rstride = (long)gridDim.y * 4 * kBaRows;
  const u16x8* zr = reinterpret_cast<const u16x8*>(z);
  u16x8* yr = reinterpret_cast<u16x8*>(y);
  for (long r0 = ((long)blockIdx.y * 4 + (threadIdx.x >> 6)) * kBaRows; r0 < M; r0 += rstride) {
    u16x8 zv[kBaRows];
#pragma unroll
    for (int k = 0; k < kBaRows; ++k) zv[k] = (r0 + k < M) ? zr[(r0 + k) * nvec_row + c] : u16x8(0);
#pragma unroll
    for (int k = 0; k < kBaRows; ++k) {
      if (r0 + k >= M) break;
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(act_f(bf2f(zv[k][j]) + b[j], act));
      yr[(r0 + k) * nvec_row + c] = o;
    }
  }
}

// dz = dy * act'(z + bias); dbias partials [grid, N] (each block owns a fixed set of
// column-vectors so its partial stays in registers across its grid-stride rows).
// Block: 256 threads = (256 / cols_per_block) rows-in-flight x cols_per_block vectors.
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ z, const bf16_t* __restrict__ bias,
    bf16_t* __restrict__ dz, float* __restrict__ part, int M, int nvec_row, int act) {
  // blockIdx.y selects a 64-vector column slice; threads: 64 column vectors x 4 row lanes
  const int cv = blockIdx.y * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  __shared__ float red[4][64 * 8];
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (cv < nvec_row) {
    u16x8 bv = u16x8(0);
    if (bias) bv = reinterpret_cast<const u16x8*>(bias)[cv];
    const int rstep = gridDim.x * 4;
    int row = blockIdx.x * 4 + rl;
    // two rows per step: four independent 16-byte loads in flight per lane
    for (; row + rstep < M; row += 2 * rstep) {
      const long i0 = (long)row * nvec_row + cv, i1 = (long)(row + rstep) * nvec_row + cv;
      const u16x8 g0 = reinterpret_cast<const u16x8*>(dy)[i0], g1 = reinterpret_cast<const u16x8*>(dy)[i1];
      const u16x8 z0 = act != ACT_NONE ? reinterpret_cast<const u16x8*>(z)[i0] : u16x8(0);
      const u16x8 z1 = act != ACT_NONE ? reinterpret_cast<const u16x8*>(z)[i1] : u16x8(0);
      u16x8 o0, o1;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d0 = bf2f(g0[j]) * act_g(bf2f(z0[j]) + bf2f(bv[j]), act);
        const float d1 = bf2f(g1[j]) * act_g(bf2f(z1[j]) + bf2f(bv[j]), act);
        o0[j] = f2bf(d0);
        o1[j] = f2bf(d1);
        acc[j] += d0 + d1;
      }
      if (dz) {
        reinterpret_cast<u16x8*>(dz)[i0] = o0;
        reinterpret_cast<u16x8*>(dz)[i1] = o1;
      }
    }
    for (; row < M; row += rstep) {
      const long idx = (long)row * nvec_row + cv;
      const u16x8 gv = reinterpret_cast<const u16x8*>(dy)[idx];
      const u16x8 zv = act != ACT_NONE ? reinterpret_cast<const u16x8*>(z)[idx] : u16x8(0);
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = bf2f(gv[j]) * act_g(bf2f(zv[j]) + bf2f(bv[j]), act);
        o[j] = f2bf(d);
        acc[j] += d;
      }
      if (dz) reinterpret_cast<u16x8*>(dz)[idx] = o;
    }
  }
  if (!part) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][(threadIdx.x & 63) * 8 + j] = acc[j];
  __syncthreads();
  const int N = nvec_row * 8;
  for (int t = threadIdx.x; t < 64 * 8; t += 256) {
    const int col = blockIdx.y * 512 + t;
    if (col < N) part[(long)blockIdx.x * N + col] = red[0][t] + red[1][t] + red[2][t] + red[3][t];
  }
}

// y = dropout(x) (keep-scale 1/(1-p)), mask from Philox(seed, offset, vector index)
__global__ __launch_bounds__(256) void dropout_kernel(const bf16_t* __restrict__ x,
                                                      bf16_t* __restrict__ y, long total_vec,
                                                      uint32_t thresh, float scale, uint64_t seed,
                                                      uint64_t offset) {
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < total_vec;
       v += (long)gridDim.x * blockDim.x) {
    const u16x8 xv = reinterpret_cast<const u16x8*>(x)[v];
    const uint32_t keep = dropout_bits8(seed, offset, (uint64_t)v, thresh);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = ((keep >> j) & 1u) ? f2bf(bf2f(xv[j]) * scale) : (bf16_t)0;
    reinterpret_cast<u16x8*>(y)[v] = o;
  }
}

// out[t, :] = W[ids[t]] + P[pos(t)] + T[tt[t]]   (pos(t) = t % S), row width N
__global__ __launch_bounds__(256) void embed3_fwd_kernel(
    const int64_t* __restrict__ ids, const int64_t* __restrict__ tt, const bf16_t* __restrict__ W,
    const bf16_t* __restrict__ P, const bf16_t* __restrict__ T, bf16_t* __restrict__ out, int ntok,
    int S, int N) {
  const int nvec = N >> 3;
  const int lane = threadIdx.x & 63;
  for (int t = blockIdx.x * 4 + (threadIdx.x >> 6); t < ntok; t += gridDim.x * 4) {
    const long wi = ids[t];
    const long ti = tt ? tt[t] : 0;
    const int pi = t % S;
    for (int c = lane; c < nvec; c += 64) {
      const u16x8 a = reinterpret_cast<const u16x8*>(W + wi * N)[c];
      u16x8 b = u16x8(0), d = u16x8(0);
      if (P) b = reinterpret_cast<const u16x8*>(P + (long)pi * N)[c];
      if (T) d = reinterpret_cast<const u16x8*>(T + ti * N)[c];
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(a[j]) + bf2f(b[j]) + bf2f(d[j]));
      reinterpret_cast<u16x8*>(out + (long)t * N)[c] = o;
    }
  }
}

// Scatter-add rows of g into fp32 tables with float atomics (chip-wide ~1.3 TB/s of added
// bytes; each wave-instruction adds 256 contiguous bytes of one row: the full-rate shape).
__global__ __launch_bounds__(256) void embed3_bwd_kernel(
    const int64_t* __restrict__ ids, const int64_t* __restrict__ tt, const bf16_t* __restrict__ g,
    float* __restrict__ dW, float* __restrict__ dP, float* __restrict__ dT, int ntok, int S, int N) {
  const int lane = threadIdx.x & 63;
  for (int t = blockIdx.x * 4 + (threadIdx.x >> 6); t < ntok; t += gridDim.x * 4) {
    const long wi = ids[t];
    const long ti = tt ? tt[t] : 0;
    const int pi = t % S;
    const bf16_t* gr = g + (long)t * N;
    for (int c = lane; c < N; c += 64) {
      const float v = bf2f(gr[c]);
      if (dW) atomicAdd(dW + wi * N + c, v);
      if (dP) atomicAdd(dP + (long)pi * N + c, v);
      if (dT) atomicAdd(dT + ti * N + c, v);
    }
  }
}

// Same gradients, one workgroup per (position s, 256 columns): the thread of column c walks
// the batch (tokens b*S + s), scatter-adds into the word table (atomics: rows differ per
// token, little contention) and keeps the position and token-type sums in registers.  The
// per-token kernel above sent every token's row into the SAME position row (B-way
// contention) and into one of two token-type rows (B*S/2-way): 0.76 ms per BERT-large step,
// almost all of it serialised same-address atomics.
__global__ __launch_bounds__(256) void embed3_bwd_seq_kernel(
    const int64_t* __restrict__ ids, const int64_t* __restrict__ tt, const bf16_t* __restrict__ g,
    float* __restrict__ dW, float* __restrict__ dP, float* __restrict__ dT, int B, int S, int N, int nT) {
  const int s = blockIdx.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= N) return;
  float ps = 0.f, t0 = 0.f, t1 = 0.f;
  // consecutive tokens of this position with the same id (every sequence's [CLS] at s = 0, the
  // padding tail) are summed in a register and added once: B same-address atomics serialise at
  // the memory side
  long cur = -1;
  float run = 0.f;
#pragma unroll 8
  for (int b = 0; b < B; ++b) {
    const long t = (long)b * S + s;
    const float v = bf2f(g[t * N + c]);
    if (dW) {
      const long id = ids[t];
      if (id != cur) {
        if (cur >= 0) atomicAdd(dW + cur * N + c, run);
        cur = id;
        run = v;
      } else {
        run += v;
      }
    }
    ps += v;
    if (dT) {
      const long ti = tt ? tt[t] : 0;
      if (nT <= 2) {
        if (ti == 0) t0 += v; else t1 += v;
      } else {
        atomicAdd(dT + ti * N + c, v);
      }
    }
  }
  if (dW && cur >= 0) atomicAdd(dW + cur * N + c, run);
  if (dP) dP[(long)s * N + c] += ps;   // (s, c) belongs to this thread alone
  if (dT && nT <= 2) {
    atomicAdd(dT + c, t0);
    if (nT == 2) atomicAdd(dT + N + c, t1);
  }
}

template <typename IN, typename OUT>
__global__ void cast_kernel(const IN* __restrict__ x, OUT* __restrict__ y, long n, float scale,
                            int accumulate) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float v = to_f<IN>(x[i]) * scale;
    if (accumulate) v += to_f<OUT>(y[i]);
    y[i] = from_f<OUT>(v);
  }
}

inline int grid_for(long work, int block = 256) {
  long g = (work + block - 1) / block;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace ct

using namespace ct;

extern "C" int ct_bias_act_fwd(const void* z, const void* bias, void* y, long M, int N, int act,
                               hipStream_t stream) {
  if (N % 8) return -1;
  const int nvec = N / 8;
  const int gx = (nvec + 63) / 64;
  // enough row blocks for ~8 waves per SIMD over 256 CUs, each wave 4 rows per step
  long gy = (M + 4 * kBaRows - 1) / (4 * kBaRows);
  const long want = (8L * 1024 + gx - 1) / gx;
  if (gy > want) gy = want;
  if (gy < 1) gy = 1;
  bias_act_fwd_kernel<<<dim3(gx, (unsigned)gy), 256, 0, stream>>>((const bf16_t*)z, (const bf16_t*)bias,
                                                                 (bf16_t*)y, M, nvec, act);
  return 0;
}

extern "C" int ct_bias_act_bwd_grid(long M) {
  long g = (M + 3) / 4;
  return (int)(g > 256 ? 256 : g);
}

// part: float[ct_bias_act_bwd_grid(M) * N] workspace (may be null if no dbias wanted)
extern "C" int ct_bias_act_bwd(const void* dy, const void* z, const void* bias, void* dz,
                               float* part, void* dbias, long M, int N, int act, int param_fp32,
                               int accumulate, hipStream_t stream);
extern "C" int ct_colsum(const float* part, void* out, int P, int N, int out_fp32, int accumulate,
                         hipStream_t stream);
extern "C" int ct_bias_act_bwd(const void* dy, const void* z, const void* bias, void* dz,
                               float* part, void* dbias, long M, int N, int act, int param_fp32,
                               int accumulate, hipStream_t stream) {
  if (N % 8) return -1;
  const int gx = ct_bias_act_bwd_grid(M);
  dim3 grid(gx, ceil_div(N / 8, 64));
  bias_act_bwd_kernel<<<grid, 256, 0, stream>>>((const bf16_t*)dy, (const bf16_t*)z,
                                                (const bf16_t*)bias, (bf16_t*)dz,
                                                dbias ? part : nullptr, (int)M, N / 8, act);
  if (dbias) ct_colsum(part, dbias, gx, N, param_fp32, accumulate, stream);
  return 0;
}

extern "C" int ct_dropout(const void* x, void* y, long n, float p, uint64_t seed, uint64_t offset,
                          hipStream_t stream) {
  if (n % 8) return -1;
  const long tv = n / 8;
  dropout_kernel<<<grid_for(tv), 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, tv,
                                                   dropout_threshold(p), 1.f / (1.f - p), seed,
                                                   offset);
  return 0;
}

extern "C" int ct_embed3_fwd(const int64_t* ids, const int64_t* tt, const void* W, const void* P,
                             const void* T, void* out, int ntok, int S, int N, hipStream_t stream) {
  if (N % 8) return -1;
  embed3_fwd_kernel<<<grid_for(ntok, 4), 256, 0, stream>>>(ids, tt, (const bf16_t*)W,
                                                           (const bf16_t*)P, (const bf16_t*)T,
                                                           (bf16_t*)out, ntok, S, N);
  return 0;
}

// nT: rows of the token-type table (0 if none)
extern "C" int ct_embed3_bwd(const int64_t* ids, const int64_t* tt, const void* g, float* dW,
                             float* dP, float* dT, int ntok, int S, int N, int nT, hipStream_t stream) {
  if (S > 0 && ntok % S == 0 && S <= 65535) {
    dim3 grid(S, (N + 255) / 256);
    embed3_bwd_seq_kernel<<<grid, 256, 0, stream>>>(ids, tt, (const bf16_t*)g, dW, dP, dT, ntok / S, S, N, nT);
    return 0;
  }
  embed3_bwd_kernel<<<grid_for(ntok, 4), 256, 0, stream>>>(ids, tt, (const bf16_t*)g, dW, dP, dT,
                                                           ntok, S, N);
  return 0;
}

// ---------------------------------------------------------------- split-K weight-grad reduce
// g[i] = bf16( (accumulate ? g[i] : 0) + sum_s P[s*n + i] ) -- the second half of a split-K
// weight-gradient GEMM (the partials come from one batched hipBLASLt GEMM with fp32 output).
// One pass: 8 elements per thread, S fp32 float4 pairs + one bf16x8 load/store.
// clear: the partials are zeroed after they are read (a persistent fp32 accumulation buffer --
// the fused FFN dgrad's bias-gradient atomics -- is then ready for its next use without a fill
// kernel)
__global__ void __launch_bounds__(256) splitk_reduce_kernel(float* __restrict__ P, int S, long nv,
                                                            bf16_t* __restrict__ g, int accumulate, int clear) {
  const long n = nv * 8;
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < nv; v += (long)gridDim.x * blockDim.x) {
    float acc[8];
    if (accumulate) {
      const u16x8 gv = *reinterpret_cast<const u16x8*>(g + v * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = bf2f(gv[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    }
    // unrolled so several slabs' loads are in flight per thread (a rolled loop waits one
    // memory latency per slab)
#pragma unroll 4
    for (int s = 0; s < S; ++s) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(P + s * n + v * 8);
      const f32x4 b = *reinterpret_cast<const f32x4*>(P + s * n + v * 8 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { acc[j] += a[j]; acc[4 + j] += b[j]; }
      if (clear) {
        *reinterpret_cast<f32x4*>(P + s * n + v * 8) = f32x4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4*>(P + s * n + v * 8 + 4) = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    *reinterpret_cast<u16x8*>(g + v * 8) = o;
  }
}

extern "C" int ct_splitk_reduce(const float* P, int S, long n, void* g, int accumulate, hipStream_t stream) {
  if (n % 8) return -1;
  const long nv = n / 8;
  splitk_reduce_kernel<<<grid_for(nv), 256, 0, stream>>>(const_cast<float*>(P), S, nv, (bf16_t*)g, accumulate, 0);
  return 0;
}

// Two independent reductions in ONE launch (vectors [0, nv) of the first pair, then the second
// pair's): a weight gradient's fp32 slabs and its bias's [S][N] column-sum partials, which were
// two back-to-back launches per weight-gradient site (the bias one a few microseconds of launch
// for a few KB of data).
struct Reduce2 { const float* P[2]; int S[2]; long nv[2]; bf16_t* g[2]; };

__global__ void __launch_bounds__(256) splitk_reduce2_kernel(Reduce2 r, int accumulate) {
  const long nt = r.nv[0] + r.nv[1];
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < nt; t += (long)gridDim.x * blockDim.x) {
    const int k = t < r.nv[0] ? 0 : 1;
    const long v = k ? t - r.nv[0] : t;
    const long n = r.nv[k] * 8;
    const float* P = r.P[k];
    bf16_t* g = r.g[k];
    float acc[8];
    if (accumulate) {
      const u16x8 gv = *reinterpret_cast<const u16x8*>(g + v * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = bf2f(gv[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    }
#pragma unroll 4
    for (int s = 0; s < r.S[k]; ++s) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(P + s * n + v * 8);
      const f32x4 b = *reinterpret_cast<const f32x4*>(P + s * n + v * 8 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { acc[j] += a[j]; acc[4 + j] += b[j]; }
    }
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    *reinterpret_cast<u16x8*>(g + v * 8) = o;
  }
}

extern "C" int ct_splitk_reduce2(const float* P, int S, long n, void* g, const float* P2, int S2, long n2,
                                 void* g2, int accumulate, hipStream_t stream) {
  if (n % 8 || n2 % 8) return -1;
  Reduce2 r{{P, P2}, {S, S2}, {n / 8, n2 / 8}, {(bf16_t*)g, (bf16_t*)g2}};
  splitk_reduce2_kernel<<<grid_for(r.nv[0] + r.nv[1]), 256, 0, stream>>>(r, accumulate);
  return 0;
}

extern "C" int ct_splitk_reduce_clear(float* P, int S, long n, void* g, int accumulate, hipStream_t stream) {
  if (n % 8) return -1;
  const long nv = n / 8;
  splitk_reduce_kernel<<<grid_for(nv), 256, 0, stream>>>(P, S, nv, (bf16_t*)g, accumulate, 1);
  return 0;
}

// ---------------------------------------------------------------- multi-tensor accumulate
// dst_t += src_t for a list of (src, dst, n) chunks in ONE launch (block = chunk): the
// deferred conv-weight gradients of train/optim.py FlatParamSpace land in the flat gradient
// buffer with this instead of one AccumulateGrad add kernel per parameter.  Chunks start at
// 16-byte-aligned element offsets; the tail of a chunk runs element-wise.
template <typename T>
__global__ void __launch_bounds__(256) mt_add_kernel(const int64_t* __restrict__ table) {
  const T* src = reinterpret_cast<const T*>(table[3 * blockIdx.x]);
  T* dst = reinterpret_cast<T*>(table[3 * blockIdx.x + 1]);
  const long n = table[3 * blockIdx.x + 2];
  constexpr int V = 16 / sizeof(T);
  const long nv = n / V;
  for (long i = threadIdx.x; i < nv; i += blockDim.x) {
    if (sizeof(T) == 2) {
      u16x8 a = reinterpret_cast<const u16x8*>(src)[i], b = reinterpret_cast<u16x8*>(dst)[i], o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(b[j]) + bf2f(a[j]));
      reinterpret_cast<u16x8*>(dst)[i] = o;
    } else {
      f32x4 a = reinterpret_cast<const f32x4*>(src)[i], b = reinterpret_cast<f32x4*>(dst)[i];
      reinterpret_cast<f32x4*>(dst)[i] = a + b;
    }
  }
  for (long i = nv * V + threadIdx.x; i < n; i += blockDim.x)
    dst[i] = from_f<T>(to_f<T>(dst[i]) + to_f<T>(src[i]));
}

extern "C" int ct_mt_add(const int64_t* table, int nchunks, int is_f32, hipStream_t stream) {
  if (nchunks <= 0) return 0;
  if (nchunks > 65535 * 32) return -1;
  if (is_f32) mt_add_kernel<float><<<nchunks, 256, 0, stream>>>(table);
  else mt_add_kernel<bf16_t><<<nchunks, 256, 0, stream>>>(table);
  return 0;
}

// ---------------------------------------------------------------- multi-tensor pack / unpack
// Gradient-bucket flatten for collectives (reference SSD distributed.py:13-48 and Horovod
// tensor fusion, SURVEY.md §2.15 "Gradient bucket pack/scale/unpack"): tensor t (ptrs[t],
// sizes[t] elements) <-> flat[offs[t] ...], with a scale and an optional fp32<->bf16 cast
// (compression), for all tensors in ONE launch (blockIdx.y = tensor).
template <typename TS, typename TD>
__global__ void __launch_bounds__(256) mt_copy_kernel(const uint64_t* __restrict__ ptrs, const int64_t* __restrict__ sizes,
                                                      const int64_t* __restrict__ offs, void* flat, float scale, int unpack) {
  const int t = blockIdx.y;
  const long n = sizes[t];
  TS* tp = reinterpret_cast<TS*>(ptrs[t]);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    if (!unpack) reinterpret_cast<TD*>(flat)[offs[t] + i] = from_f<TD>(to_f<TS>(tp[i]) * scale);
    else tp[i] = from_f<TS>(to_f<TD>(reinterpret_cast<const TD*>(flat)[offs[t] + i]) * scale);
  }
}

extern "C" int ct_mt_copy(const uint64_t* ptrs, const int64_t* sizes, const int64_t* offs, int ntensors, long max_numel,
                          void* flat, int tensor_dt, int flat_dt, float scale, int unpack, hipStream_t stream) {
  if (ntensors <= 0) return 0;
  if (ntensors > 65535) return -1;
  long gx = (max_numel + 255) / 256;
  if (gx > 256) gx = 256;
  if (gx < 1) gx = 1;
  const dim3 grid((unsigned)gx, (unsigned)ntensors);
  if (tensor_dt == 0 && flat_dt == 0) mt_copy_kernel<float, float><<<grid, 256, 0, stream>>>(ptrs, sizes, offs, flat, scale, unpack);
  else if (tensor_dt == 0 && flat_dt == 1) mt_copy_kernel<float, bf16_t><<<grid, 256, 0, stream>>>(ptrs, sizes, offs, flat, scale, unpack);
  else if (tensor_dt == 1 && flat_dt == 0) mt_copy_kernel<bf16_t, float><<<grid, 256, 0, stream>>>(ptrs, sizes, offs, flat, scale, unpack);
  else mt_copy_kernel<bf16_t, bf16_t><<<grid, 256, 0, stream>>>(ptrs, sizes, offs, flat, scale, unpack);
  return 0;
}

// dtype codes: 0 = fp32, 1 = bf16
extern "C" int ct_cast(const void* x, int xdt, void* y, int ydt, long n, float scale, int accumulate,
                       hipStream_t stream) {
  const int g = grid_for(n);
  if (xdt == 0 && ydt == 1) cast_kernel<float, bf16_t><<<g, 256, 0, stream>>>((const float*)x, (bf16_t*)y, n, scale, accumulate);
  else if (xdt == 1 && ydt == 0) cast_kernel<bf16_t, float><<<g, 256, 0, stream>>>((const bf16_t*)x, (float*)y, n, scale, accumulate);
  else if (xdt == 0 && ydt == 0) cast_kernel<float, float><<<g, 256, 0, stream>>>((const float*)x, (float*)y, n, scale, accumulate);
  else cast_kernel<bf16_t, bf16_t><<<g, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, n, scale, accumulate);
  return 0;
}
