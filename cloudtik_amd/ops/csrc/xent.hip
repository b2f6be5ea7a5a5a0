// Fused softmax cross-entropy with the gradient produced in the same launch.
//
// For BERT pretraining the masked-LM loss is taken only at the gathered masked positions
// (the reference runs HF BERT with `config.dense_seq_output`, run_pretrain_mlperf.py:462,
// i.e. the 1024x30522 decoder only on <= max_predictions_per_seq=76 rows per sequence).
// The [rows, V] logits are read twice (online max/sum pass, then the gradient pass) and the
// gradient  (softmax - onehot) * scale  is written IN PLACE of the logits, so the biggest
// activation of the step is never materialised twice.  `scale` is read from device memory
// (1 / #valid labels, computed on device) so nothing synchronises with the host.
#include "common.h"
#include <cstdlib>

namespace ct {

__global__ __launch_bounds__(256) void xent_fwd_kernel(
    const bf16_t* __restrict__ logits, bf16_t* __restrict__ dlogits, int ld, int V,
    const int64_t* __restrict__ labels, float* __restrict__ loss_rows, float* __restrict__ lse_rows,
    const float* __restrict__ scale_dev, int R, int ignore_index, float label_smoothing) {
  __shared__ float red[8];
  __shared__ float red2[8];
  const float scale = scale_dev ? *scale_dev : 1.f;
  const int nvec = ld >> 3;
  for (int r = blockIdx.x; r < R; r += gridDim.x) {
    const u16x8* row = reinterpret_cast<const u16x8*>(logits + (size_t)r * ld);
    const int64_t lab = labels[r];
    const bool valid = lab != ignore_index && lab >= 0 && lab < V;
    // read the target logit before any thread of the block starts overwriting the row
    const float xl = (threadIdx.x == 0 && valid) ? bf2f(logits[(size_t)r * ld + lab]) : 0.f;
    // pass 1: online max / sum-exp per thread
    float mx = -INFINITY, sm = 0.f, sum_logit = 0.f;
    for (int c = threadIdx.x; c < nvec; c += blockDim.x) {
      const u16x8 v = row[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = c * 8 + j;
        if (col < V) {
          const float x = bf2f(v[j]);
          sum_logit += x;
          if (x > mx) { sm = sm * __expf(mx - x) + 1.f; mx = x; }
          else sm += __expf(x - mx);
        }
      }
    }
    // combine (max, sum) across the wave then across waves
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float omx = __shfl_xor(mx, o, 64), osm = __shfl_xor(sm, o, 64);
      const float nmx = fmaxf(mx, omx);
      sm = (mx == -INFINITY ? 0.f : sm * __expf(mx - nmx)) + (omx == -INFINITY ? 0.f : osm * __expf(omx - nmx));
      mx = nmx;
    }
    sum_logit = wave_sum(sum_logit);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if (lane == 0) { red[wid] = mx; red2[wid] = sm; }
    __syncthreads();
    float gmx = -INFINITY;
    for (int w = 0; w < nw; ++w) gmx = fmaxf(gmx, red[w]);
    float gsm = 0.f;
    for (int w = 0; w < nw; ++w) gsm += red2[w] * __expf(red[w] - gmx);
    __syncthreads();
    if (lane == 0) red[wid] = sum_logit;
    __syncthreads();
    float gsl = 0.f;
    for (int w = 0; w < nw; ++w) gsl += red[w];
    const float lse = gmx + __logf(gsm);
    if (threadIdx.x == 0) {
      float loss = 0.f;
      if (valid) {
        loss = (1.f - label_smoothing) * (lse - xl) + label_smoothing * (lse - gsl / V);
      }
      loss_rows[r] = loss;
      if (lse_rows) lse_rows[r] = lse;
    }
    // pass 2: gradient (may overwrite the logits in place: every element is read before
    // it is written by the same thread)
    u16x8* drow = reinterpret_cast<u16x8*>(dlogits + (size_t)r * ld);
    const float sv = valid ? scale : 0.f;
    const float smooth = label_smoothing / V;
    for (int c = threadIdx.x; c < nvec; c += blockDim.x) {
      const u16x8 v = row[c];
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = c * 8 + j;
        float gval = 0.f;
        if (col < V) {
          const float p = __expf(bf2f(v[j]) - lse);
          gval = (p - smooth - (col == lab ? (1.f - label_smoothing) : 0.f)) * sv;
        }
        o[j] = f2bf(gval);
      }
      drow[c] = o;
    }
  }
}

// The same with the row held in registers (NV 16-byte vectors per thread, rows up to
// NV * 256 * 8 columns): the row is read from memory ONCE -- the two-pass kernel above re-reads
// it for the gradient, and a 60 KB BERT vocabulary row per block does not stay in L2 across
// the passes (the 1.2 GB of MLM logits went through memory twice).  All NV loads are issued
// together; the max, then the exp-sum, then the gradient run on the registers.
// bf16 halves of a packed 32-bit register as fp32.  The asm keeps each conversion at its use:
// as plain C++ the three passes share the conversions and the compiler keeps 8 NV fp32 values
// live (254 VGPRs at NV = 16, one wave per SIMD) instead of the 4 NV packed registers.
__device__ __forceinline__ float xent_lo(uint32_t w) {
  uint32_t r;
  asm volatile("v_lshlrev_b32 %0, 16, %1" : "=v"(r) : "v"(w));
  return __uint_as_float(r);
}
__device__ __forceinline__ float xent_hi(uint32_t w) {
  uint32_t r;
  asm volatile("v_and_b32 %0, 0xffff0000, %1" : "=v"(r) : "v"(w));
  return __uint_as_float(r);
}
__device__ __forceinline__ float xent_el(const uint4& v, int j) {
  const uint32_t w = j < 2 ? v.x : (j < 4 ? v.y : (j < 6 ? v.z : v.w));
  return (j & 1) ? xent_hi(w) : xent_lo(w);
}

template <int NV>
__global__ __launch_bounds__(256) void xent_fwd_reg_kernel(
    const bf16_t* __restrict__ logits, bf16_t* __restrict__ dlogits, int ld, int V,
    const int64_t* __restrict__ labels, float* __restrict__ loss_rows, float* __restrict__ lse_rows,
    const float* __restrict__ scale_dev, int R, int ignore_index, float label_smoothing) {
  __shared__ float red[3][8];
  const float scale = scale_dev ? *scale_dev : 1.f;
  const int nvec = ld >> 3;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int r = blockIdx.x; r < R; r += gridDim.x) {
    const u16x8* row = reinterpret_cast<const u16x8*>(logits + (size_t)r * ld);
    const int64_t lab64 = labels[r];
    const bool valid = lab64 != ignore_index && lab64 >= 0 && lab64 < V;
    // the label's (thread, register, element): block-uniform, so the one-hot below is a scalar
    // test per register instead of a 64-bit compare per element
    const int lab = valid ? (int)lab64 : -1;
    const int lab_t = valid ? (lab >> 3) & 255 : -1, lab_k = valid ? (lab >> 3) >> 8 : -1, lab_j = lab & 7;
    uint4 v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = threadIdx.x + k * 256;
      v[k] = c < nvec ? reinterpret_cast<const uint4*>(row)[c] : uint4{0u, 0u, 0u, 0u};
    }
    // columns >= V (vocabulary padding, vector slots past the row) become -inf in place, so the
    // passes below need no per-element column masks (kept live across the passes, those masks
    // were what filled the register file); real logits are finite
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c0 = (threadIdx.x + k * 256) * 8;
      if (c0 + 8 > V) {
        uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (c0 + j >= V) w[j >> 1] = (j & 1) ? ((w[j >> 1] & 0xFFFFu) | 0xFF800000u) : ((w[j >> 1] & 0xFFFF0000u) | 0xFF80u);
        v[k] = uint4{w[0], w[1], w[2], w[3]};
      }
    }
    // the target logit, from the register that holds it (no second read of the row)
    float xl = 0.f;
    if (lab_t == (int)threadIdx.x) {
#pragma unroll
      for (int k = 0; k < NV; ++k)
        if (lab_k == k) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (lab_j == j) xl = xent_el(v[k], j);
        }
    }
    float mx = -INFINITY, sum_logit = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = xent_el(v[k], j);
        mx = fmaxf(mx, x);
        sum_logit += x == -INFINITY ? 0.f : x;
      }
    mx = wave_max(mx);
    sum_logit = wave_sum(sum_logit);
    xl = wave_sum(xl);
    if (lane == 0) { red[0][wid] = mx; red[1][wid] = sum_logit; red[2][wid] = xl; }
    __syncthreads();
    float gmx = -INFINITY, gsl = 0.f, gxl = 0.f;
    for (int w = 0; w < nw; ++w) { gmx = fmaxf(gmx, red[0][w]); gsl += red[1][w]; gxl += red[2][w]; }
    float sm = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) sm += __expf(xent_el(v[k], j) - gmx);     // exp(-inf) = 0
    sm = wave_sum(sm);
    __syncthreads();                       // every wave has read red[] above
    if (lane == 0) red[0][wid] = sm;
    __syncthreads();
    float gsm = 0.f;
    for (int w = 0; w < nw; ++w) gsm += red[0][w];
    const float lse = gmx + __logf(gsm);
    if (threadIdx.x == 0) {
      float loss = 0.f;
      if (valid) loss = (1.f - label_smoothing) * (lse - gxl) + label_smoothing * (lse - gsl / V);
      loss_rows[r] = loss;
      if (lse_rows) lse_rows[r] = lse;
    }
    u16x8* drow = reinterpret_cast<u16x8*>(dlogits + (size_t)r * ld);
    const float sv = valid ? scale : 0.f;
    const float smooth = label_smoothing / V;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = threadIdx.x + k * 256;
      if (c < nvec) {
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = xent_el(v[k], j);
          float q = __expf(x - lse) - smooth;
          if (lab_k == k && lab_j == j && lab_t == (int)threadIdx.x) q -= 1.f - label_smoothing;
          o[j] = f2bf(x == -INFINITY ? 0.f : q * sv);
        }
        drow[c] = o;
      }
    }
    __syncthreads();                       // red[] is rewritten by the next row
  }
}

}  // namespace ct

using namespace ct;

extern "C" int ct_xent_fwd(const void* logits, void* dlogits, int ld, int V, const int64_t* labels,
                           float* loss_rows, float* lse_rows, const float* scale_dev, int R,
                           int ignore_index, float label_smoothing, hipStream_t stream) {
  if (ld % 8) return -1;
  int grid = R < 8192 ? R : 8192;
  if (grid < 1) return 0;
  const int nvec = ld / 8;
  static const bool reg_ok = [] {
    const char* e = getenv("CLOUDTIK_AMD_XENT_REG");
    return !(e && atoi(e) == 0);
  }();
  if (reg_ok && nvec <= 16 * 256) {        // row fits the registers of one block (V <= 32768)
    const int nv = (nvec + 255) / 256;
#define CT_XENT_REG(NV_)                                                                          \
    xent_fwd_reg_kernel<NV_><<<grid, 256, 0, stream>>>((const bf16_t*)logits, (bf16_t*)dlogits, ld, V, labels, \
                                                       loss_rows, lse_rows, scale_dev, R, ignore_index,  \
                                                       label_smoothing)
    if (nv <= 4) CT_XENT_REG(4);
    else if (nv <= 8) CT_XENT_REG(8);
    else if (nv <= 12) CT_XENT_REG(12);
    else CT_XENT_REG(16);
#undef CT_XENT_REG
    return 0;
  }
  xent_fwd_kernel<<<grid, 256, 0, stream>>>((const bf16_t*)logits, (bf16_t*)dlogits, ld, V, labels,
                                            loss_rows, lse_rows, scale_dev, R, ignore_index,
                                            label_smoothing);
  return 0;
}
