// Shared device helpers for the cloudtik_amd CDNA4 (gfx950) op library.
//
// Conventions used by every kernel in this directory:
//   * wave = 64 lanes; blocks are multiples of 64 threads.
//   * bf16 tensors are moved as 16-byte vectors (8 x bf16) per lane (Guideline 13:
//     hipcc does not auto-vectorise 16-bit loads).
//   * statistics / reductions are carried in fp32.
//   * every launch function takes an explicit hipStream_t and performs no
//     allocation or synchronisation, so callers may capture it into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

namespace ct {

typedef unsigned short bf16_t;  // raw storage type for bf16
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;   // MFMA operand (8 x bf16)

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// Round-to-nearest-even; a plain __bf16 cast lowers to v_cvt_pk_bf16_f32 on gfx950
// and keeps NaNs NaN (MI355X_MICROARCH.md correctness table).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

template <typename T>
__device__ __forceinline__ float to_f(T v);
template <>
__device__ __forceinline__ float to_f<float>(float v) { return v; }
template <>
__device__ __forceinline__ float to_f<bf16_t>(bf16_t v) { return bf2f(v); }

template <typename T>
__device__ __forceinline__ T from_f(float v);
template <>
__device__ __forceinline__ float from_f<float>(float v) { return v; }
template <>
__device__ __forceinline__ bf16_t from_f<bf16_t>(float v) { return f2bf(v); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Sum over each 16-lane DPP row (lanes 16k .. 16k + 15), broadcast to the row's lanes: four
// VALU adds with DPP operand swizzles (quad_perm 1032, quad_perm 2301, row_half_mirror,
// row_mirror) instead of four LDS-routed __shfl_xor permutes, each waiting on LDS latency.
// The MFMA 16x16 output layout keeps a fragment's 16 rows in one DPP row, so this is the
// column sum of a fragment.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);     // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);     // quad_perm [2,3,0,1]: quad sums
  v += dpp_mov<0x141>(v);    // row_half_mirror: 8-lane sums
  v += dpp_mov<0x140>(v);    // row_mirror: 16-lane sums
  return v;
}

// Block-wide sum; `scratch` must hold blockDim.x/64 floats. Result broadcast to all threads.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

// GELU (exact, erf form) and its derivative without the libm erf: erf(|z|) = 1 - P(t) e^{-z^2}
// with t = 1 / (1 + p |z|) (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7 -- far below the
// bf16 resolution of the tensors these feed).  For z = x / sqrt(2), e^{-z^2} = e^{-x^2/2} is
// the same exponential the normal pdf in the derivative needs: one exp + one rcp + a few FMA
// per element instead of the branchy libm erf plus a second exp.
__device__ __forceinline__ float gelu_cdf_e(float x, float e) {
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, fabsf(x), 1.f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f),
                                      -0.284496736f), 0.254829592f);
  const float erf_abs = fmaf(-poly, e, 1.f);
  return 0.5f + 0.5f * copysignf(erf_abs, x);
}
__device__ __forceinline__ float gelu_erf(float x) {
  return x * gelu_cdf_e(x, __expf(-0.5f * x * x));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float e = __expf(-0.5f * x * x);
  return fmaf(x * 0.3989422804014327f, e, gelu_cdf_e(x, e));
}

// The same GELU / GELU' on element PAIRS, batched over NP pairs, for GEMM epilogues (the
// matrix cores are idle there).  float2 arithmetic lowers to
// v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 (two lanes' worth of fp32 per instruction); the
// batch is computed stage by stage (all arguments, then all v_rcp / v_exp, then the
// polynomials) so the transcendental results are not consumed by the very next instruction
// (the scalar form left ~2 s_nop per element for those hazards).  exp(-x^2/2) is
// exp2(x * (x * -log2(e)/2)).  Same formula and constants as gelu_cdf_e.
typedef __attribute__((ext_vector_type(2))) float f32x2;

template <int NP, bool GRAD>
__device__ __forceinline__ void gelu2_batch(const f32x2 (&x)[NP], f32x2 (&y)[NP]) {
  const float kE = -0.5f * 1.4426950408889634f;
  f32x2 d[NP], e[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const f32x2 ax = {fabsf(x[p][0]), fabsf(x[p][1])};
    d[p] = __builtin_elementwise_fma(ax, (f32x2)(0.3275911f * 0.70710678118654752f), (f32x2)(1.f));
    e[p] = x[p] * (x[p] * kE);
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    d[p] = f32x2{__builtin_amdgcn_rcpf(d[p][0]), __builtin_amdgcn_rcpf(d[p][1])};
    e[p] = f32x2{__builtin_amdgcn_exp2f(e[p][0]), __builtin_amdgcn_exp2f(e[p][1])};
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const f32x2 t = d[p];
    f32x2 q = __builtin_elementwise_fma(t, (f32x2)(1.061405429f), (f32x2)(-1.453152027f));
    q = __builtin_elementwise_fma(q, t, (f32x2)(1.421413741f));
    q = __builtin_elementwise_fma(q, t, (f32x2)(-0.284496736f));
    q = __builtin_elementwise_fma(q, t, (f32x2)(0.254829592f));
    q = q * t;
    const f32x2 ea = __builtin_elementwise_fma(-q, e[p], (f32x2)(1.f));          // erf(|x| / sqrt 2)
    const f32x2 s = {copysignf(ea[0], x[p][0]), copysignf(ea[1], x[p][1])};
    const f32x2 cdf = __builtin_elementwise_fma(s, (f32x2)(0.5f), (f32x2)(0.5f));
    if constexpr (GRAD)
      y[p] = __builtin_elementwise_fma(x[p] * 0.3989422804014327f, e[p], cdf);
    else
      y[p] = x[p] * cdf;
  }
}

// gelu(x) and gelu'(x) of NP packed pairs in one pass: the two share the erf term and the
// Gaussian exp (the derivative adds one FMA per element).  The FFN1 forward epilogue stores
// gelu'(x) instead of x, so the FFN data-gradient epilogue is a multiply (gemm_nt.hip EPI 6/7).
template <int NP>
__device__ __forceinline__ void gelu2_batch_both(const f32x2 (&x)[NP], f32x2 (&y)[NP], f32x2 (&g)[NP]) {
  const float kE = -0.5f * 1.4426950408889634f;
  f32x2 d[NP], e[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const f32x2 ax = {fabsf(x[p][0]), fabsf(x[p][1])};
    d[p] = __builtin_elementwise_fma(ax, (f32x2)(0.3275911f * 0.70710678118654752f), (f32x2)(1.f));
    e[p] = x[p] * (x[p] * kE);
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    d[p] = f32x2{__builtin_amdgcn_rcpf(d[p][0]), __builtin_amdgcn_rcpf(d[p][1])};
    e[p] = f32x2{__builtin_amdgcn_exp2f(e[p][0]), __builtin_amdgcn_exp2f(e[p][1])};
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const f32x2 t = d[p];
    f32x2 q = __builtin_elementwise_fma(t, (f32x2)(1.061405429f), (f32x2)(-1.453152027f));
    q = __builtin_elementwise_fma(q, t, (f32x2)(1.421413741f));
    q = __builtin_elementwise_fma(q, t, (f32x2)(-0.284496736f));
    q = __builtin_elementwise_fma(q, t, (f32x2)(0.254829592f));
    q = q * t;
    const f32x2 ea = __builtin_elementwise_fma(-q, e[p], (f32x2)(1.f));          // erf(|x| / sqrt 2)
    const f32x2 s = {copysignf(ea[0], x[p][0]), copysignf(ea[1], x[p][1])};
    const f32x2 cdf = __builtin_elementwise_fma(s, (f32x2)(0.5f), (f32x2)(0.5f));
    g[p] = __builtin_elementwise_fma(x[p] * 0.3989422804014327f, e[p], cdf);
    y[p] = x[p] * cdf;
  }
}

// Bijective XCD-aware remap of a 1-D grid (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): consecutive logical tiles land on the same XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace ct

#define CT_HIP_CHECK(expr)                                                              \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
    }                                                                                   \
  } while (0)

// ---------------------------------------------------------------------------------------
// Counter-based RNG for dropout: the mask is a pure function of (seed, offset, element
// index), so backward regenerates it instead of storing it.
// ---------------------------------------------------------------------------------------
namespace ct {
// 32-bit integer hash (xorshift-multiply, full avalanche); bijective on uint32
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}
// 32-bit stream key of (seed, offset); kernel-uniform, so it is computed once per thread
__host__ __device__ __forceinline__ uint32_t dropout_key(uint64_t seed, uint64_t offset) {
  uint32_t k = mix32((uint32_t)(offset >> 32) + 0x632BE5ABu);
  k = mix32(k ^ (uint32_t)offset);
  k = mix32(k ^ (uint32_t)(seed >> 32));
  return mix32(k ^ (uint32_t)seed);
}
// 8 keep-bits (bit j set = keep element 8*v+j) for the 8-element vector number `v`
// of a stream identified by (seed, offset).  Four hashes of the element-pair counter give
// one 16-bit uniform per element, compared with the top 16 bits of the 32-bit threshold
// (p = 0.1 -> 6553 / 65536).  The Philox-4x32-7 stream this replaces cost two 7-round
// calls per 8 elements (28 64-bit multiplies); regenerating the mask in the LayerNorm
// backward made that kernel VALU-bound (74 vs 61 us per BERT-large call without dropout).
__device__ __forceinline__ uint32_t dropout_bits8(uint64_t seed, uint64_t offset, uint64_t v,
                                                 uint32_t thresh) {
  const uint32_t key = dropout_key(seed, offset) ^ mix32((uint32_t)(v >> 30));
  const uint32_t t16 = thresh >> 16;
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    // the key enters twice (add before the multiply, xor after it): with a plain
    // mix32(ctr ^ key) two sites whose keys agree above the counter range would draw
    // XOR-permuted copies of one stream
    const uint32_t r = mix32((((uint32_t)v << 2 | (uint32_t)j) + key) * 0x9E3779B1u ^ key);
    bits |= (uint32_t)((r & 0xFFFFu) >= t16) << (2 * j);
    bits |= (uint32_t)((r >> 16) >= t16) << (2 * j + 1);
  }
  return bits;
}
__host__ __device__ inline uint32_t dropout_threshold(float p) {
  double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}
}  // namespace ct
