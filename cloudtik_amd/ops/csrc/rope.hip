// Rotary position embedding (RoPE) forward / backward for gfx950.
//
// Not in the reference (SURVEY.md §2.15 "RoPE fwd/bwd -- north star requires it in the op
// library").  x is [T, H, D] (T = batch*seq tokens, any token/head strides, unit stride in
// D), rotated in place or into y.  cos/sin are fp32 caches [P, D/2] indexed by the token's
// position (positions[t], or t % seq_len when no position ids are given).
//
//   neox style  (rotate halves):    (x[i], x[i + D/2])
//   gptj style  (interleaved pairs): (x[2i], x[2i + 1])
//   y1 = x1 cos - x2 sin,  y2 = x2 cos + x1 sin.
// The backward is the same rotation by -theta (sign = -1): dx1 = dy1 cos + dy2 sin, ...
//
// One thread owns 4 rotation pairs = 8 bf16 values (two 8-byte loads for neox, one
// 16-byte load for gptj); Q and K of the same token are rotated by the same launch
// (heads_q + heads_k "virtual heads"), so the cos/sin row is read once per token from L2.
// Memory bound: 2 x bytes(q,k) per call.
#include "common.h"

namespace ct {

struct RopeArgs {
  const bf16_t* xq; bf16_t* yq; long q_tok, q_head; int hq;
  const bf16_t* xk; bf16_t* yk; long k_tok, k_head; int hk;
  const float* cos; const float* sin;
  const int64_t* pos; int seq_len; long ntok;
  int D; float sign;
};

template <bool NEOX>
__global__ void __launch_bounds__(256) rope_kernel(RopeArgs a) {
  const int half = a.D / 2;
  const int groups = half / 4;                        // 4 pairs per thread
  const int heads = a.hq + a.hk;
  const long total = a.ntok * heads * groups;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int g = (int)(i % groups);
    const long th = i / groups;
    const int h = (int)(th % heads);
    const long t = th / heads;
    const bf16_t* x;
    bf16_t* y;
    if (h < a.hq) { x = a.xq + t * a.q_tok + h * a.q_head; y = a.yq + t * a.q_tok + h * a.q_head; }
    else { const int hh = h - a.hq; x = a.xk + t * a.k_tok + hh * a.k_head; y = a.yk + t * a.k_tok + hh * a.k_head; }
    const long p = a.pos ? a.pos[t] : (t % a.seq_len);
    const f32x4 c = *reinterpret_cast<const f32x4*>(a.cos + p * half + g * 4);
    f32x4 s = *reinterpret_cast<const f32x4*>(a.sin + p * half + g * 4);
    s *= a.sign;
    if (NEOX) {
      const u16x4 v1 = *reinterpret_cast<const u16x4*>(x + g * 4);
      const u16x4 v2 = *reinterpret_cast<const u16x4*>(x + half + g * 4);
      u16x4 o1, o2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x1 = bf2f(v1[j]), x2 = bf2f(v2[j]);
        o1[j] = f2bf(x1 * c[j] - x2 * s[j]);
        o2[j] = f2bf(x2 * c[j] + x1 * s[j]);
      }
      *reinterpret_cast<u16x4*>(y + g * 4) = o1;
      *reinterpret_cast<u16x4*>(y + half + g * 4) = o2;
    } else {
      const u16x8 v = *reinterpret_cast<const u16x8*>(x + g * 8);
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x1 = bf2f(v[2 * j]), x2 = bf2f(v[2 * j + 1]);
        o[2 * j] = f2bf(x1 * c[j] - x2 * s[j]);
        o[2 * j + 1] = f2bf(x2 * c[j] + x1 * s[j]);
      }
      *reinterpret_cast<u16x8*>(y + g * 8) = o;
    }
  }
}

}  // namespace ct

using namespace ct;

extern "C" int ct_rope(const void* xq, void* yq, long q_tok, long q_head, int hq,
                       const void* xk, void* yk, long k_tok, long k_head, int hk,
                       const float* cos, const float* sin, const int64_t* pos, int seq_len, long ntok,
                       int D, int neox, int backward, hipStream_t stream) {
  if (D % 8 != 0 || (hq + hk) == 0) return -1;
  RopeArgs a{(const bf16_t*)xq, (bf16_t*)yq, q_tok, q_head, hq,
             (const bf16_t*)xk, (bf16_t*)yk, k_tok, k_head, hk,
             cos, sin, pos, seq_len, ntok, D, backward ? -1.f : 1.f};
  const long total = ntok * (long)(hq + hk) * (D / 8);
  long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  if (neox) rope_kernel<true><<<(int)g, 256, 0, stream>>>(a);
  else rope_kernel<false><<<(int)g, 256, 0, stream>>>(a);
  return 0;
}
