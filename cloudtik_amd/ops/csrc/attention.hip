// Fused multi-head attention (forward + backward) on CDNA4 MFMA, head_dim 64, bf16 I/O.
//
// Hot op of the reference's BERT-large pretraining: HF BertSelfAttention, 16 heads x 64,
// S = 128 (phase-1 shards) / 512, padding mask + attention-prob dropout 0.1
// (run_pretrain_mlperf.py:449-471).  There is no attention kernel in the reference tree --
// it reaches this through PyTorch/IPEX -- so this is designed for MI355X from scratch:
//
// Forward (flash-style, never materialises S x S):
//   * workgroup = 4 waves = 128 queries of one (batch, head); each wave owns 32 queries.
//   * S^T = K . Q^T with v_mfma_f32_32x32x16_bf16: the query sits on the MFMA lane and the
//     keys in the 16 accumulator registers, so a query's softmax row is lane-local except
//     for one xor-32 shuffle (no LDS round trip for the softmax).
//   * the P^T accumulator feeds the next MFMA directly as its B operand
//     (O^T += V^T . P^T, cdna_hip_programming.md §3 "accumulator as next operand"); V^T
//     fragments come from ds_read_b64_tr_b16 transposed LDS reads of the row-major V tile.
//   * K/V tiles of 64 keys, double-buffered in LDS, register-staged (global loads for tile
//     t+1 issued before the MFMAs of tile t, LDS write after: T14).
//   * every 128-byte LDS row is XOR-swizzled at 16-byte granularity with
//     rev3((row >> 1) & 7): conflict-free for both the ds_read_b128 row reads and the
//     ds_read_b64_tr_b16 column reads (see swz()).
//   * online softmax in the exp2 domain; stores O and the per-row log2-sum-exp.
// Backward (FlashAttention-2 structure, "key on the lane"):
//   * workgroup = 4 waves = 128 keys; each wave keeps K, V fragments of its 32 keys in
//     VGPRs and accumulates dK^T, dV^T in registers over all query tiles.
//   * S = Q.K^T and dP = dO.V^T are computed with the key on the lane, so P and dS are
//     already the B operands of dV^T += dO^T.P and dK^T += Q^T.dS (Q^T, dO^T by
//     transposed LDS reads); only dS crosses LDS (once) for dQ = dS.K.
//   * dQ: each wave owns 16 queries x 32 d of the q-tile and sums over all 128 keys itself
//     (16x16x32 MFMAs on transposed reads of dS^T and K: no cross-wave reduction); the
//     q-tile inputs and dS^T are double-buffered, so each q-tile takes ONE barrier.  Stored
//     directly (bf16, 16-byte stores after a permlane16 swap) when one workgroup covers all
//     keys (S <= 128, the BERT phase-1 case), otherwise accumulated with fp32 atomics and
//     converted by a tiny kernel.
//   * attention-prob dropout regenerated from a counter hash (nothing stored).
#include "common.h"
#include <cstdlib>
#include <type_traits>

namespace ct {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int rev3(int x) { return ((x & 1) << 2) | (x & 2) | ((x >> 2) & 1); }
// byte offset of 16-byte chunk c of `row` inside a [rows][64 x bf16] LDS tile
__device__ __forceinline__ int swz(int row, int c) { return row * 128 + ((c ^ rev3((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int swz_e(int row, int col) { return swz(row, col >> 3) + ((col & 7) << 1); }
// 8-byte chunk XOR of key row `key` in the backward's dS^T image ([keys][32 q], 64-byte rows).
// Writes (ds_write_b64, 16-lane groups over 32 banks): 16 consecutive keys hit distinct
// (parity, chunk) slots.  Transposing reads (32-lane halves over 64 banks, 8 consecutive rows
// 8a .. 8a + 7, 4 chunks each): rows r and r + 4 share a 64-byte window and their chunk sets
// differ in bit 2.
__device__ __forceinline__ int dsw(int key) { return ((key >> 1) & 7) ^ (key & 4); }

__device__ __forceinline__ bf16x8_t lds_b128(const char* p) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8*>(p));
}
__device__ __forceinline__ s16x4 lds_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}
__device__ __forceinline__ bf16x8_t cat_tr(s16x4 lo, s16x4 hi) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}
__device__ __forceinline__ bf16x8_t gload_frag(const bf16_t* p, bool valid) {
  u16x8 v = valid ? *reinterpret_cast<const u16x8*>(p) : u16x8(0);
  return __builtin_bit_cast(bf16x8_t, v);
}
__device__ __forceinline__ f32x16 mfma32(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
typedef __attribute__((address_space(3))) void at_lds_void;
// global_load_lds_dwordx4: lane l's 16 bytes at sbase + voff land at LDS wave_base + 16 l (one
// 1 KB wave instruction, no staging registers).  sbase must be wave-uniform.  The compiler does
// not count these in vmcnt: callers wait with s_waitcnt vmcnt(0) before the barrier.
__device__ __forceinline__ void at_glds16s(const void* sbase, unsigned voff, const char* lds_wave_base) {
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(at_lds_void*)lds_wave_base);
  const uint64_t sb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)sbase) |
                      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)sbase >> 32)) << 32);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sb), "s"(la)
               : "memory", "m0");
}
// Store a 64-wide row held as two 32x32 MFMA accumulators in the "row on the lane" layout:
// lane (r, hh) holds columns d = 8 g + 4 hh .. + 3 of row r (A0: d < 32, A1: d + 32).  A
// v_permlane32_swap of the (g, g + 1) pair between the lane halves leaves each lane 8
// consecutive columns (hh = 0: block g, hh = 1: block g + 1), so the row goes out as 16-byte
// stores, 4 per lane instead of 8 of 8 bytes (the store tail of these short kernels is
// issue-bound).  Every lane must take part (the swap); `valid` only gates the stores.
__device__ __forceinline__ void store_row64(bf16_t* p, const f32x16& A0, const f32x16& A1, float mul, int hh,
                                            bool valid) {
  u16x8 ov[4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) {
      const f32x16& A = t ? A1 : A0;
      const int g0 = 2 * gp, g1 = g0 + 1;
      const u16x4 x = {f2bf(A[4 * g0] * mul), f2bf(A[4 * g0 + 1] * mul), f2bf(A[4 * g0 + 2] * mul),
                       f2bf(A[4 * g0 + 3] * mul)};
      const u16x4 y = {f2bf(A[4 * g1] * mul), f2bf(A[4 * g1 + 1] * mul), f2bf(A[4 * g1 + 2] * mul),
                       f2bf(A[4 * g1 + 3] * mul)};
      const uint2 xv = __builtin_bit_cast(uint2, x), yv = __builtin_bit_cast(uint2, y);
      const auto s0 = __builtin_amdgcn_permlane32_swap(xv.x, yv.x, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(xv.y, yv.y, false, false);
      // s*[0] = the new x (hh = 1 lanes: the partner's y), s*[1] = the new y
      const uint4 v = {s0[0], s1[0], s0[1], s1[1]};
      ov[2 * t + gp] = __builtin_bit_cast(u16x8, v);
    }
  if (!valid) return;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) *reinterpret_cast<u16x8*>(p + 32 * t + 8 * (2 * gp + hh)) = ov[2 * t + gp];
}

__device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}
// 16-bit uniform pair for element pair `pair` (elements 2*pair, 2*pair+1)
__device__ __forceinline__ uint32_t drop_pair(uint32_t base, uint64_t pair) {
  return hash_u32((uint32_t)pair ^ base);
}

struct AttnFwdArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; bf16_t* o;
  long q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh, o_sb, o_ss, o_sh;
  const float* kbias; long kb_sb;  // additive per-key bias [B, Sk] (natural-log units)
  float* lse;                      // [B*H, Sq] log2-domain log-sum-exp
  int B, H, Sq, Sk;
  float scale_log2;                // softmax scale * log2(e)
  uint32_t thr16; float inv_keep; uint32_t hash_base; int causal;
  // relative-position bias (T5): score(q, k) += relb[h][k - q + rel_base] (natural-log units)
  const float* relb; long relb_sh; int relb_len; int rel_base;
};

constexpr int kRelBiasMax = 4096;   // LDS floats for one head's relative-offset bias vector

// WPE: waves per SIMD the register budget must allow (256 threads = 1 wave per SIMD per
// workgroup).  The compiler's default budget (236 VGPR + 32 AGPR) allowed ONE resident
// workgroup per CU, so a workgroup's Q/K/V loads never overlapped another's MFMAs; at 2 the
// kernel fits in ~170 VGPRs without spills.
// GL: K/V tiles go global -> LDS by global_load_lds (at_glds16s) instead of through the
// stK/stV (+ k1/v1) staging registers: wave w DMAs rows 16 w .. 16 w + 15 of the K and the V
// tile (two 1 KB wave instructions each).  Lane l lands at physical chunk l & 7 of row
// 16 w + 8 i + (l >> 3), so it fetches logical chunk (l & 7) ^ rev3(((row >> 1) & 7)) =
// (l & 7) ^ rev3((4 i + (l >> 4)) & 7) -- the same swizzled image the register path writes.
// Keys past Sk read key Sk - 1 (finite data; their -inf key bias zeroes them), so no load is
// out of bounds and no zero fill is needed.
template <bool DROP, bool CAUSAL, bool REL = false, int WPE = 2, bool GL = false>
__global__ __launch_bounds__(256, WPE) void attn_fwd_d64_kernel(AttnFwdArgs a) {
  // [buf][K,V][64 rows][128 B] then [buf][64] fp32 log2-domain key bias (-inf past Sk)
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 64 * 128 + 2 * 64 * 4];
  float* kbias_lds = reinterpret_cast<float*>(smem + 32768);
  // one head's relative-position bias vector, log2-scaled (REL variant only; the first
  // K/V tile's barrier below publishes it)
  __shared__ float relb_lds[REL ? kRelBiasMax : 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int qi = blockIdx.x * 128 + w * 32 + r;
  const bool qvalid = qi < a.Sq;
  const float LOG2E = 1.4426950408889634f;
  if (REL)
    for (int i = tid; i < a.relb_len; i += 256) relb_lds[i] = a.relb[h * a.relb_sh + i] * LOG2E;

  const bf16_t* qp = a.q + b * a.q_sb + h * a.q_sh + (long)qi * a.q_ss;
  bf16x8_t qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = gload_frag(qp + 16 * s + 8 * hh, qvalid);

  const bf16_t* kp = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vp = a.v + b * a.v_sb + h * a.v_sh;
  const float* kbp = a.kbias ? a.kbias + b * a.kb_sb : nullptr;
  const int srow = tid >> 3, sch = tid & 7;
  u16x8 stK[2], stV[2];
  float stB = 0.f;
  // element pair index base of this lane's query row (dropout stream); Sk even
  const uint32_t rb2 = (uint32_t)((((uint64_t)bh * a.Sq + qi) * (uint64_t)a.Sk) >> 1);

  f32x16 O0, O1;
#pragma unroll
  for (int i = 0; i < 16; ++i) { O0[i] = 0.f; O1[i] = 0.f; }
  float m = -INFINITY, l = 0.f;
  const int nt = (a.Sk + 63) / 64;

#define FWD_GLOAD(kt_)                                                               \
  _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_) {                                 \
    const int key_ = (kt_) * 64 + srow + 32 * i_;                                    \
    const bool ok_ = key_ < a.Sk;                                                    \
    stK[i_] = ok_ ? *reinterpret_cast<const u16x8*>(kp + (key_ * (int)a.k_ss + sch * 8)) : u16x8(0); \
    stV[i_] = ok_ ? *reinterpret_cast<const u16x8*>(vp + (key_ * (int)a.v_ss + sch * 8)) : u16x8(0); \
  }                                                                                  \
  if (tid < 64) {                                                                    \
    const int kk_ = (kt_) * 64 + tid;                                                \
    stB = kk_ < a.Sk ? (kbp ? kbp[kk_] * LOG2E : 0.f) : -INFINITY;                   \
  }
#define FWD_SWRITE(buf_)                                                             \
  _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_) {                                 \
    char* kb_ = smem + (buf_) * 16384;                                               \
    *reinterpret_cast<u16x8*>(kb_ + swz(srow + 32 * i_, sch)) = stK[i_];             \
    *reinterpret_cast<u16x8*>(kb_ + 8192 + swz(srow + 32 * i_, sch)) = stV[i_];      \
  }                                                                                  \
  if (tid < 64) kbias_lds[(buf_) * 64 + tid] = stB;

  // Sk <= 128 (BERT phase 1): both K/V tiles are loaded up front (a second staging set; the
  // accumulators are not live yet, so it costs no occupancy) and sit in the two LDS buffers
  // before the first MFMA -- one memory latency per workgroup instead of two in series, and
  // no barrier inside the loop
  const bool resident = nt == 2;
#define FWD_GLDS(kt_, buf_)                                                                    \
  _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_) {                                           \
    const int row_ = 16 * w + 8 * i_ + (lane >> 3);                                            \
    const unsigned key_ = (unsigned)min((kt_) * 64 + row_, a.Sk - 1);                          \
    const unsigned c_ = (unsigned)((lane & 7) ^ rev3((4 * i_ + (lane >> 4)) & 7));             \
    char* dst_ = smem + (buf_) * 16384 + (16 * w + 8 * i_) * 128;                              \
    at_glds16s(kp, (key_ * (unsigned)a.k_ss + c_ * 8u) * 2u, dst_);                            \
    at_glds16s(vp, (key_ * (unsigned)a.v_ss + c_ * 8u) * 2u, dst_ + 8192);                     \
  }
  if constexpr (GL) {
    FWD_GLDS(0, 0);
    if (resident) {
      FWD_GLDS(1, 1);
      if (tid < 128) stB = tid < a.Sk ? (kbp ? kbp[tid] * LOG2E : 0.f) : -INFINITY;
    } else if (tid < 64) {
      stB = tid < a.Sk ? (kbp ? kbp[tid] * LOG2E : 0.f) : -INFINITY;
    }
    if (tid < (resident ? 128 : 64)) kbias_lds[tid] = stB;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
  FWD_GLOAD(0);
  if (resident) {
    u16x8 k1[2], v1[2];
    float b1 = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int key = 64 + srow + 32 * i;
      const bool ok = key < a.Sk;
      k1[i] = ok ? *reinterpret_cast<const u16x8*>(kp + (key * (int)a.k_ss + sch * 8)) : u16x8(0);
      v1[i] = ok ? *reinterpret_cast<const u16x8*>(vp + (key * (int)a.v_ss + sch * 8)) : u16x8(0);
    }
    if (tid < 64) {
      const int kk = 64 + tid;
      b1 = kk < a.Sk ? (kbp ? kbp[kk] * LOG2E : 0.f) : -INFINITY;
    }
    FWD_SWRITE(0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<u16x8*>(smem + 16384 + swz(srow + 32 * i, sch)) = k1[i];
      *reinterpret_cast<u16x8*>(smem + 16384 + 8192 + swz(srow + 32 * i, sch)) = v1[i];
    }
    if (tid < 64) kbias_lds[64 + tid] = b1;
  } else {
    FWD_SWRITE(0);
  }
  }
  __syncthreads();

  const int trow = (lane >> 2) & 3;
  const int tcol = ((lane >> 4) & 1) * 16 + (lane & 3) * 4;

  for (int kt = 0; kt < nt; ++kt) {
    const int buf = kt & 1;
    if (!resident && kt + 1 < nt) {
      if constexpr (GL) {
        // buf ^ 1 was last read in tile kt - 1, which ended with a barrier
        FWD_GLDS(kt + 1, buf ^ 1);
        if (tid < 64) {
          const int kk = (kt + 1) * 64 + tid;
          stB = kk < a.Sk ? (kbp ? kbp[kk] * LOG2E : 0.f) : -INFINITY;
        }
      } else {
        FWD_GLOAD(kt + 1);
      }
    }
    const char* Kb = smem + buf * 16384;
    const char* Vb = Kb + 8192;
    f32x16 S0, S1;
#pragma unroll
    for (int i = 0; i < 16; ++i) { S0[i] = 0.f; S1[i] = 0.f; }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      S0 = mfma32(lds_b128(Kb + swz(r, 2 * s + hh)), qf[s], S0);
      S1 = mfma32(lds_b128(Kb + swz(32 + r, 2 * s + hh)), qf[s], S1);
    }
    // reg i <-> key kt*64 + t*32 + 8(i>>2) + 4hh + (i&3): 4 consecutive keys per group,
    // so the bias comes in as float4 LDS reads; -inf bias masks keys past Sk
    const float* kbt = kbias_lds + buf * 64 + 4 * hh;
    float mx = -INFINITY;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(kbt + 8 * g);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(kbt + 32 + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * g + j;
        float x0 = fmaf(S0[i], a.scale_log2, b0[j]);
        float x1 = fmaf(S1[i], a.scale_log2, b1[j]);
        if (REL) {
          const int ri = kt * 64 + 8 * g + 4 * hh + j - qi + a.rel_base;
          x0 += relb_lds[min(max(ri, 0), a.relb_len - 1)];
          x1 += relb_lds[min(max(ri + 32, 0), a.relb_len - 1)];
        }
        if (CAUSAL) {
          const int key0 = kt * 64 + 8 * g + 4 * hh + j;
          if (key0 > qi) x0 = -INFINITY;
          if (key0 + 32 > qi) x1 = -INFINITY;
        }
        S0[i] = x0; S1[i] = x1;
        mx = fmaxf(mx, fmaxf(x0, x1));
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m, mx);
    const float msub = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = __builtin_amdgcn_exp2f(m - msub);
    m = m_new;
    float ps = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      S0[i] = __builtin_amdgcn_exp2f(S0[i] - msub);
      S1[i] = __builtin_amdgcn_exp2f(S1[i] - msub);
      ps += S0[i] + S1[i];
    }
    l = l * alpha + ps;
#pragma unroll
    for (int i = 0; i < 16; ++i) { O0[i] *= alpha; O1[i] *= alpha; }
    // dropout: one 32-bit hash per (even, odd) key pair, one 16-bit uniform each.  Dropped
    // probabilities are zeroed in place (compare + select); the 1/(1-p) rescale is folded
    // into the final 1/l normalisation (l is the pre-dropout row sum), so no per-element
    // multiply.  (r >> 16) >= t16  <=>  r >= t16 << 16; (r & 0xFFFF) >= t16  <=>
    // (r << 16) >= t16 << 16: one compare per element.
    if (DROP) {
      const uint32_t pbase = rb2 + (uint32_t)(kt * 32 + 2 * hh);
      const uint32_t thi = a.thr16 << 16;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int i = 0; i < 16; i += 2) {  // (i&3) in {0,2}: an even key and its odd partner
          const uint32_t pair = pbase + (uint32_t)(t * 16 + 4 * (i >> 2) + ((i & 3) >> 1));
          const uint32_t rr = hash_u32(pair ^ a.hash_base);
          const bool k0 = (rr << 16) >= thi, k1 = rr >= thi;
          if (t == 0) { S0[i] = k0 ? S0[i] : 0.f; S0[i + 1] = k1 ? S0[i + 1] : 0.f; }
          else { S1[i] = k0 ? S1[i] : 0.f; S1[i + 1] = k1 ? S1[i + 1] : 0.f; }
        }
      }
    }
    // P^T registers -> bf16 B fragments (k-step s2 of tile t = registers 8*s2 .. 8*s2+7)
    bf16x8_t pf[2][2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pf[0][s2][j] = (__bf16)S0[8 * s2 + j];
        pf[1][s2][j] = (__bf16)S1[8 * s2 + j];
      }
    // O^T[d][q] += V^T[d][key] . P^T[key][q]; V^T fragments by transposed LDS reads
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int kb = t * 32 + 16 * s2 + 4 * hh + trow;
        const bf16x8_t a0 = cat_tr(lds_tr(Vb + swz_e(kb, tcol)), lds_tr(Vb + swz_e(kb + 8, tcol)));
        const bf16x8_t a1 = cat_tr(lds_tr(Vb + swz_e(kb, 32 + tcol)), lds_tr(Vb + swz_e(kb + 8, 32 + tcol)));
        O0 = mfma32(a0, pf[t][s2], O0);
        O1 = mfma32(a1, pf[t][s2], O1);
      }
    if (!resident) {
      if constexpr (GL) {
        if (kt + 1 < nt && tid < 64) kbias_lds[(buf ^ 1) * 64 + tid] = stB;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        if (kt + 1 < nt) { FWD_SWRITE(buf ^ 1); }
      }
      __syncthreads();
    }
  }
#undef FWD_GLOAD
#undef FWD_SWRITE
#undef FWD_GLDS
  l += __shfl_xor(l, 32, 64);
  const float inv = l > 0.f ? (DROP ? a.inv_keep : 1.f) / l : 0.f;
  bf16_t* op = a.o + b * a.o_sb + h * a.o_sh + (long)(qvalid ? qi : 0) * a.o_ss;
  store_row64(op, O0, O1, inv, hh, qvalid);
  if (qvalid) {
    if (hh == 0 && a.lse) a.lse[(long)bh * a.Sq + qi] = l > 0.f ? m + log2f(l) : INFINITY;
  }
}


// Pipelined persistent forward (no relative bias): a workgroup walks work items blockIdx.x,
// + gridDim.x, ... (item = q-block + nqb * (batch * H + head)) and runs ONE flat loop over the
// K/V tiles of all of them.  The K/V (+ key bias) of flat tile f + 2 are loaded into one of two
// register staging sets at step f and written to LDS at the end of step f + 1, so every load
// has two tile computations to land (the one-set kernel above gives it one).  Measured SLOWER
// than the one-item kernel (75.5 vs 65.9 us on BERT-large shapes): the hardware dispatcher
// already overlaps one workgroup's loads with another's MFMAs, and the persistent walk only
// adds loop-carried state (199 VGPRs, 2 waves/SIMD).  Kept as an opt-in (CLOUDTIK_AMD_ATTN_FWD_PIPE=1)
// for long sequences, where items have many tiles.  The next item's Q fragments
// are loaded at the first tile of the current item.  The loop is unrolled by two so the
// staging set is a compile-time choice (a runtime index would put the sets in scratch).
template <bool DROP, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void attn_fwd_pipe_kernel(AttnFwdArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 64 * 128 + 2 * 64 * 4];
  float* kbias_lds = reinterpret_cast<float*>(smem + 32768);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int nqb = (a.Sq + 127) / 128;
  const int nitems = nqb * a.B * a.H;
  const int G = gridDim.x;
  if ((int)blockIdx.x >= nitems) return;
  const float LOG2E = 1.4426950408889634f;
  const int srow = tid >> 3, sch = tid & 7;
  const int nt = (a.Sk + 63) / 64;
  const int my_items = (nitems - (int)blockIdx.x + G - 1) / G;
  const int nflat = my_items * nt;
  const int trow = (lane >> 2) & 3;
  const int tcol = ((lane >> 4) & 1) * 16 + (lane & 3) * 4;

  u16x8 k0s[2], v0s[2], k1s[2], v1s[2];
  float b0s = 0.f, b1s = 0.f;
  auto gload = [&](int f, u16x8 (&K)[2], u16x8 (&V)[2], float& Bv) {
    const int it = (int)blockIdx.x + (f / nt) * G, kt = f % nt;
    const int bh = it / nqb, b = bh / a.H, h = bh % a.H;
    const bf16_t* kp = a.k + b * a.k_sb + h * a.k_sh;
    const bf16_t* vp = a.v + b * a.v_sb + h * a.v_sh;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int key = kt * 64 + srow + 32 * i;
      const bool ok = key < a.Sk;
      K[i] = ok ? *reinterpret_cast<const u16x8*>(kp + (key * (int)a.k_ss + sch * 8)) : u16x8(0);
      V[i] = ok ? *reinterpret_cast<const u16x8*>(vp + (key * (int)a.v_ss + sch * 8)) : u16x8(0);
    }
    if (tid < 64) {
      const int kk = kt * 64 + tid;
      Bv = kk < a.Sk ? (a.kbias ? a.kbias[b * a.kb_sb + kk] * LOG2E : 0.f) : -INFINITY;
    }
  };
  auto swrite = [&](int buf, const u16x8 (&K)[2], const u16x8 (&V)[2], float Bv) {
    char* kb = smem + buf * 16384;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<u16x8*>(kb + swz(srow + 32 * i, sch)) = K[i];
      *reinterpret_cast<u16x8*>(kb + 8192 + swz(srow + 32 * i, sch)) = V[i];
    }
    if (tid < 64) kbias_lds[buf * 64 + tid] = Bv;
  };
  auto qload = [&](int it, bf16x8_t (&Q)[4]) {
    const int bh = it / nqb, b = bh / a.H, h = bh % a.H;
    const int qi = (it % nqb) * 128 + w * 32 + r;
    const bf16_t* qp = a.q + b * a.q_sb + h * a.q_sh + (long)qi * a.q_ss;
#pragma unroll
    for (int s = 0; s < 4; ++s) Q[s] = gload_frag(qp + 16 * s + 8 * hh, qi < a.Sq);
  };

  bf16x8_t qf[4], qn[4];
  qload(blockIdx.x, qf);
  gload(0, k0s, v0s, b0s);
  if (nflat > 1) gload(1, k1s, v1s, b1s);
  swrite(0, k0s, v0s, b0s);
  __syncthreads();

  f32x16 O0, O1;
  float m = -INFINITY, l = 0.f;

  // one flat step: compute tile f from LDS buffer P (f % 2 == P), K/V of tile f + 2 into
  // staging set P, tile f + 1 (staging set 1 - P) into buffer 1 - P at the end
  auto step = [&](int f, u16x8 (&Kp)[2], u16x8 (&Vp)[2], float& Bp, const u16x8 (&Kq)[2],
                  const u16x8 (&Vq)[2], const float& Bq, int P) {
    if (f + 2 < nflat) gload(f + 2, Kp, Vp, Bp);
    const int fi = f / nt, kt = f - fi * nt;
    const int item = (int)blockIdx.x + fi * G;
    const int bh = item / nqb;
    const int qi = (item % nqb) * 128 + w * 32 + r;
    if (kt == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) { O0[i] = 0.f; O1[i] = 0.f; }
      m = -INFINITY;
      l = 0.f;
      if (fi + 1 < my_items) qload(item + G, qn);
    }
    const char* Kb = smem + P * 16384;
    const char* Vb = Kb + 8192;
    f32x16 S0, S1;
#pragma unroll
    for (int i = 0; i < 16; ++i) { S0[i] = 0.f; S1[i] = 0.f; }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      S0 = mfma32(lds_b128(Kb + swz(r, 2 * s + hh)), qf[s], S0);
      S1 = mfma32(lds_b128(Kb + swz(32 + r, 2 * s + hh)), qf[s], S1);
    }
    const float* kbt = kbias_lds + P * 64 + 4 * hh;
    float mx = -INFINITY;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 bb0 = *reinterpret_cast<const f32x4*>(kbt + 8 * g);
      const f32x4 bb1 = *reinterpret_cast<const f32x4*>(kbt + 32 + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * g + j;
        float x0 = fmaf(S0[i], a.scale_log2, bb0[j]);
        float x1 = fmaf(S1[i], a.scale_log2, bb1[j]);
        if (CAUSAL) {
          const int key0 = kt * 64 + 8 * g + 4 * hh + j;
          if (key0 > qi) x0 = -INFINITY;
          if (key0 + 32 > qi) x1 = -INFINITY;
        }
        S0[i] = x0; S1[i] = x1;
        mx = fmaxf(mx, fmaxf(x0, x1));
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m, mx);
    const float msub = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = __builtin_amdgcn_exp2f(m - msub);
    m = m_new;
    float ps = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      S0[i] = __builtin_amdgcn_exp2f(S0[i] - msub);
      S1[i] = __builtin_amdgcn_exp2f(S1[i] - msub);
      ps += S0[i] + S1[i];
    }
    l = l * alpha + ps;
#pragma unroll
    for (int i = 0; i < 16; ++i) { O0[i] *= alpha; O1[i] *= alpha; }
    if (DROP) {   // the dropout stream of the one-item kernel above, element for element
      const uint32_t rb2 = (uint32_t)((((uint64_t)bh * a.Sq + qi) * (uint64_t)a.Sk) >> 1);
      const uint32_t pbase = rb2 + (uint32_t)(kt * 32 + 2 * hh);
      const uint32_t thi = a.thr16 << 16;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const uint32_t pair = pbase + (uint32_t)(t * 16 + 4 * (i >> 2) + ((i & 3) >> 1));
          const uint32_t rr = hash_u32(pair ^ a.hash_base);
          const bool k0 = (rr << 16) >= thi, k1 = rr >= thi;
          if (t == 0) { S0[i] = k0 ? S0[i] : 0.f; S0[i + 1] = k1 ? S0[i + 1] : 0.f; }
          else { S1[i] = k0 ? S1[i] : 0.f; S1[i + 1] = k1 ? S1[i + 1] : 0.f; }
        }
      }
    }
    bf16x8_t pf[2][2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pf[0][s2][j] = (__bf16)S0[8 * s2 + j];
        pf[1][s2][j] = (__bf16)S1[8 * s2 + j];
      }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int kb = t * 32 + 16 * s2 + 4 * hh + trow;
        const bf16x8_t a0 = cat_tr(lds_tr(Vb + swz_e(kb, tcol)), lds_tr(Vb + swz_e(kb + 8, tcol)));
        const bf16x8_t a1 = cat_tr(lds_tr(Vb + swz_e(kb, 32 + tcol)), lds_tr(Vb + swz_e(kb + 8, 32 + tcol)));
        O0 = mfma32(a0, pf[t][s2], O0);
        O1 = mfma32(a1, pf[t][s2], O1);
      }
    if (kt == nt - 1) {
      float lt = l + __shfl_xor(l, 32, 64);
      const float inv = lt > 0.f ? (DROP ? a.inv_keep : 1.f) / lt : 0.f;
      if (qi < a.Sq) {
        const int b = bh / a.H, h = bh % a.H;
        bf16_t* op = a.o + b * a.o_sb + h * a.o_sh + (long)qi * a.o_ss;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = 8 * g + 4 * hh;
          u16x4 v0 = {f2bf(O0[4 * g] * inv), f2bf(O0[4 * g + 1] * inv), f2bf(O0[4 * g + 2] * inv), f2bf(O0[4 * g + 3] * inv)};
          u16x4 v1 = {f2bf(O1[4 * g] * inv), f2bf(O1[4 * g + 1] * inv), f2bf(O1[4 * g + 2] * inv), f2bf(O1[4 * g + 3] * inv)};
          *reinterpret_cast<u16x4*>(op + d) = v0;
          *reinterpret_cast<u16x4*>(op + 32 + d) = v1;
        }
        if (hh == 0 && a.lse) a.lse[(long)bh * a.Sq + qi] = lt > 0.f ? m + log2f(lt) : INFINITY;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) qf[s] = qn[s];
    }
    if (f + 1 < nflat) swrite(1 - P, Kq, Vq, Bq);
    __syncthreads();
  };
  for (int f = 0; f < nflat; f += 2) {
    step(f, k0s, v0s, b0s, k1s, v1s, b1s, 0);
    if (f + 1 < nflat) step(f + 1, k1s, v1s, b1s, k0s, v0s, b0s, 1);
  }
}

struct AttnBwdArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; const bf16_t* dO; const bf16_t* o;
  long o_sb, o_ss, o_sh;
  bf16_t* dq; bf16_t* dk; bf16_t* dv; float* dq_acc;
  long q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh, do_sb, do_ss, do_sh;
  long dq_sb, dq_ss, dq_sh, dk_sb, dk_ss, dk_sh, dv_sb, dv_ss, dv_sh;
  const float* kbias; long kb_sb;
  const float* lse; const float* delta;
  int B, H, Sq, Sk;
  float scale_log2, scale;
  uint32_t thr16; float inv_keep; uint32_t hash_base; int causal;
};

// GL (single key block and Sq <= 128 only): every LDS tile arrives by global_load_lds -- K, V
// and the first two Q / dO tiles in the prologue, tile t + 2's Q / dO at the top of tile t into
// a THREE-deep ring (the slot tile t - 1 released at its barrier), waited for by a counted
// vmcnt just before tile t + 1's barrier: one and a half tiles of compute cover each load
// (the register-staged form gives half a tile and stalls on it: 47 % of wave cycles parked in
// s_waitcnt / barrier).  lse and delta = rowsum(dO * O) are computed for all (<= 128) rows
// once in the prologue instead of per tile, so the loop issues no register-destined loads.
template <bool DROP, bool CAUSAL, bool MULTI, bool GL = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_d64_kernel(AttnBwdArgs a) {
  // LDS: Q tiles R x 4K | dO tiles R x 4K | K block 16K | V block 16K | dS^T 2 x 8K | lse, delta
  // (R = 2 register-staged: 2 x 32 rows each; R = 3 with GL: all <= 128 rows each)
  // The per-q-tile inputs (Q, dO, lse, delta) and dS^T are multi-buffered, so one barrier per
  // q-tile orders everything: tile t+2 is staged into the buffers tile t (t - 1 with GL) has
  // released, and dQ needs no cross-wave reduction (each wave owns 16 queries x 32 d of the
  // tile's dQ and sums over all 128 keys itself).
  static_assert(!(GL && MULTI), "GL: single key block only");
  constexpr int QR = GL ? 3 : 2;
  constexpr int QB = QR * 4096;
  __shared__ __attribute__((aligned(16))) char smem[2 * QB + 16384 + 16384 + 16384 + (GL ? 1024 : 512)];
  char* Qs = smem;
  char* dOs = smem + QB;
  char* Ks = smem + 2 * QB;
  char* Vs = Ks + 16384;
  char* dSs = Vs + 16384;
  float* lse_s = reinterpret_cast<float*>(dSs + 16384);       // [2][32] or [128]
  float* delta_s = lse_s + (GL ? 128 : 64);                   // [2][32] or [128]

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int k0 = blockIdx.x * 128;
  const int key_l = k0 + w * 32 + r;  // this lane's key (MFMA column)
  const bool kvalid = key_l < a.Sk;
  const float LOG2E = 1.4426950408889634f;

  const bf16_t* kp = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vp = a.v + b * a.v_sb + h * a.v_sh;
  // K and V blocks (128 keys) into LDS: row reads give the B operands of S = Q K^T and
  // dP = dO V^T (re-read per q-tile instead of pinning 32 VGPRs), transposed reads of K
  // give dQ's operand
  if constexpr (GL) {
    // wave w DMAs rows 32 w + 8 i + (lane >> 3); lane l lands at physical chunk l & 7, so it
    // fetches logical chunk (l & 7) ^ rev3(((row >> 1) & 7)) = (l & 7) ^ rev3((4 i + (l >> 4)) & 7).
    // Rows past Sk read row Sk - 1 (finite; their -inf key bias zeroes them)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 32 * w + 8 * i + (lane >> 3);
      const unsigned key = (unsigned)min(k0 + row, a.Sk - 1);
      const unsigned c = (unsigned)((lane & 7) ^ rev3((4 * i + (lane >> 4)) & 7));
      at_glds16s(kp, (key * (unsigned)a.k_ss + c * 8u) * 2u, Ks + (32 * w + 8 * i) * 128);
      at_glds16s(vp, (key * (unsigned)a.v_ss + c * 8u) * 2u, Vs + (32 * w + 8 * i) * 128);
    }
  } else {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    const int row = c >> 3, ch = c & 7;
    const int key = k0 + row;
    const bool ok = key < a.Sk;
    const u16x8 kv = ok ? *reinterpret_cast<const u16x8*>(kp + (long)key * a.k_ss + ch * 8) : u16x8(0);
    const u16x8 vv = ok ? *reinterpret_cast<const u16x8*>(vp + (long)key * a.v_ss + ch * 8) : u16x8(0);
    *reinterpret_cast<u16x8*>(Ks + swz(row, ch)) = kv;
    *reinterpret_cast<u16x8*>(Vs + swz(row, ch)) = vv;
  }
  }
  const int krow = w * 32 + r;   // this lane's key row inside the block
  float kb2 = 0.f;
  if (a.kbias && kvalid) kb2 = a.kbias[b * a.kb_sb + key_l] * LOG2E;
  if (!kvalid) kb2 = -INFINITY;

  f32x16 dV0, dV1, dK0, dK1;
#pragma unroll
  for (int i = 0; i < 16; ++i) { dV0[i] = 0.f; dV1[i] = 0.f; dK0[i] = 0.f; dK1[i] = 0.f; }

  const bf16_t* qbase = a.q + b * a.q_sb + h * a.q_sh;
  const bf16_t* dobase = a.dO + b * a.do_sb + h * a.do_sh;
  const bf16_t* obase = a.o + b * a.o_sb + h * a.o_sh;
  bf16_t* dqbase = a.dq + b * a.dq_sb + h * a.dq_sh;
  const int trow = (lane >> 2) & 3;
  const int tcol = ((lane >> 4) & 1) * 16 + (lane & 3) * 4;
  const int nq = (a.Sq + 31) / 32;
  // MULTI: Sk > 128, several key blocks per (batch, head) -> dQ summed by fp32 atomics
  constexpr bool single_block = !MULTI;
  // 16-byte dQ stores need 8-element strides and a 16-byte aligned base
  const bool dq16 = ((a.dq_ss | a.dq_sb | a.dq_sh) & 7) == 0 && (((uintptr_t)a.dq) & 15) == 0;
  // this wave's share of the tile's dQ: queries 16 (w & 1) .. +16, d 32 (w >> 1) .. +32
  const int dq_q0 = 16 * (w & 1), dq_d0 = 32 * (w >> 1);
  // 16x16x32 fragment lane roles (transposing reads): g = lane >> 4 picks 8 keys, q4 / p4 a
  // row / 4-column group inside them
  const int fg = lane >> 4, fq = (lane & 15) >> 2, fp = lane & 3;

  // Q / dO / lse / delta tiles are register-prefetched two q-tiles ahead (issued before the
  // tile's MFMAs, written to LDS after its barrier into the buffer it has just released)
  const int prow = tid >> 3, pch = tid & 7;
  // delta = rowsum(dO * O) is computed here (no separate kernel): each thread prefetches
  // the O chunk matching its dO chunk; the 8 threads of a row reduce at staging time
  u16x8 pQ, pdO, pO;
  float pL = INFINITY;
#define BWD_PREFETCH(qb_)                                                                   \
  {                                                                                         \
    const int q_ = (qb_) + prow;                                                            \
    const bool ok_ = q_ < a.Sq;                                                             \
    pQ = ok_ ? *reinterpret_cast<const u16x8*>(qbase + (q_ * (int)a.q_ss + pch * 8)) : u16x8(0); \
    pdO = ok_ ? *reinterpret_cast<const u16x8*>(dobase + (q_ * (int)a.do_ss + pch * 8)) : u16x8(0); \
    pO = ok_ ? *reinterpret_cast<const u16x8*>(obase + (q_ * (int)a.o_ss + pch * 8)) : u16x8(0); \
    if (tid < 32) {                                                                         \
      const bool ok2_ = (qb_) + tid < a.Sq;                                                 \
      pL = ok2_ ? a.lse[(long)bh * a.Sq + (qb_) + tid] : INFINITY;                          \
    }                                                                                       \
  }
#define BWD_STAGE(buf_)                                                                     \
  {                                                                                         \
    *reinterpret_cast<u16x8*>(Qs + (buf_) * 4096 + swz(prow, pch)) = pQ;                    \
    *reinterpret_cast<u16x8*>(dOs + (buf_) * 4096 + swz(prow, pch)) = pdO;                  \
    if (tid < 32) lse_s[(buf_) * 32 + tid] = pL;                                            \
    float dd_ = 0.f;                                                                        \
    _Pragma("unroll") for (int j_ = 0; j_ < 8; ++j_) dd_ += bf2f(pdO[j_]) * bf2f(pO[j_]);  \
    dd_ += __shfl_xor(dd_, 1, 64);                                                          \
    dd_ += __shfl_xor(dd_, 2, 64);                                                          \
    dd_ += __shfl_xor(dd_, 4, 64);                                                          \
    if (pch == 0) delta_s[(buf_) * 32 + prow] = dd_;                                        \
  }
  // GL: Q / dO tile t (32 rows) into ring slot `slot_`: wave w DMAs rows 8 w + (lane >> 3) of
  // each (one 1 KB instruction per operand); rows past Sq read row Sq - 1 (finite; their
  // +inf lse zeroes every product they enter)
#define BWD_GLDS(qb_, slot_)                                                                \
  {                                                                                         \
    const unsigned q_ = (unsigned)min((qb_) + 8 * w + (lane >> 3), a.Sq - 1);               \
    const unsigned c_ = (unsigned)((lane & 7) ^ rev3((4 * w + (lane >> 4)) & 7));           \
    at_glds16s(qbase, (q_ * (unsigned)a.q_ss + c_ * 8u) * 2u, Qs + (slot_) * 4096 + w * 1024); \
    at_glds16s(dobase, (q_ * (unsigned)a.do_ss + c_ * 8u) * 2u, dOs + (slot_) * 4096 + w * 1024); \
  }
  if constexpr (GL) {
    BWD_GLDS(0, 0);
    if (nq > 1) BWD_GLDS(32, 1);
    // lse and delta of all rows: thread (row tid >> 1, half tid & 1) dots 32 d of dO and O
    {
      const int row = tid >> 1, hf = tid & 1;
      float dd = 0.f;
      if (row < a.Sq) {
        const bf16_t* dr = dobase + row * (int)a.do_ss + 32 * hf;
        const bf16_t* orow = obase + row * (int)a.o_ss + 32 * hf;
        u16x8 dv[4], ov[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          dv[j] = *reinterpret_cast<const u16x8*>(dr + 8 * j);
          ov[j] = *reinterpret_cast<const u16x8*>(orow + 8 * j);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) dd += bf2f(dv[j][e]) * bf2f(ov[j][e]);
      }
      dd += __shfl_xor(dd, 1, 64);
      if (hf == 0 && row < 128) delta_s[row] = dd;
      if (tid < 128) lse_s[tid] = tid < a.Sq ? a.lse[(long)bh * a.Sq + tid] : INFINITY;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
  BWD_PREFETCH(0);
  BWD_STAGE(0);
  if (nq > 1) {
    BWD_PREFETCH(32);
    BWD_STAGE(1);
  }
  }
  __syncthreads();

  int slot = 0;      // GL: ring slot of tile qt
  for (int qt = 0; qt < nq; ++qt) {
    const int qb = qt * 32;
    const int buf = qt & 1;
    if constexpr (GL) {
      // slot of tile qt + 2 == slot of tile qt - 1 (released at tile qt - 1's barrier)
      if (qt + 2 < nq) { const int s2 = slot == 0 ? 2 : slot - 1; BWD_GLDS(qb + 64, s2); }
    } else {
      if (qt + 2 < nq) BWD_PREFETCH(qb + 64);
    }
    const char* Qt = Qs + (GL ? slot : buf) * 4096;
    const char* dOt = dOs + (GL ? slot : buf) * 4096;
    const float* lse_t = lse_s + (GL ? qb : buf * 32);
    const float* delta_t = delta_s + (GL ? qb : buf * 32);
    char* dSt = dSs + buf * 8192;
    f32x16 S, dP;
#pragma unroll
    for (int i = 0; i < 16; ++i) { S[i] = 0.f; dP[i] = 0.f; }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      S = mfma32(lds_b128(Qt + swz(r, 2 * s + hh)), lds_b128(Ks + swz(krow, 2 * s + hh)), S);
      dP = mfma32(lds_b128(dOt + swz(r, 2 * s + hh)), lds_b128(Vs + swz(krow, 2 * s + hh)), dP);
    }
    // dropout keep bits: the pair (even key, odd key) shares one hash; the two lanes of a
    // pair (lane ^ 1) each hash 8 of the 16 query rows and swap halves with one DPP move
    // packed into one register: bit i = keep decision of register i
    uint32_t keepbits = 0xFFFFu;
    if (DROP) {
      const uint32_t T0 = (uint32_t)(((uint64_t)bh * a.Sq + qb) * (uint64_t)(a.Sk >> 1));
      const uint32_t half_sk = (uint32_t)(a.Sk >> 1);
      const int hsel = r & 1;                // == key_l & 1 (k0, w*32 even)
      uint32_t mine = 0, theirs = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * hsel + j;
        const int qrow = (i & 3) + 8 * (i >> 2) + 4 * hh;
        const uint32_t rr = hash_u32((T0 + (uint32_t)qrow * half_sk + (uint32_t)(key_l >> 1)) ^ a.hash_base);
        const uint32_t klo = (rr & 0xFFFFu) >= a.thr16, khi = (rr >> 16) >= a.thr16;
        mine |= (hsel ? khi : klo) << i;
        theirs |= (hsel ? klo : khi) << i;
      }
      keepbits = mine | (uint32_t)__builtin_amdgcn_update_dpp(0, (int)theirs, 0xB1, 0xF, 0xF, false);
    }
    // reg i <-> query row qrow(i) = (i&3) + 8(i>>2) + 4hh of this tile; column = key_l
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 L4 = *reinterpret_cast<const f32x4*>(lse_t + 8 * g + 4 * hh);
      const f32x4 D4 = *reinterpret_cast<const f32x4*>(delta_t + 8 * g + 4 * hh);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * g + j;
        float x = fmaf(S[i], a.scale_log2, kb2);
        if (CAUSAL && key_l > qb + 8 * g + 4 * hh + j) x = -INFINITY;
        const float p = __builtin_amdgcn_exp2f(x - L4[j]);
        float pd = p, dpv = dP[i];
        if (DROP) {
          const bool keep = (keepbits >> i) & 1u;
          pd = keep ? p * a.inv_keep : 0.f;
          dpv = keep ? dpv * a.inv_keep : 0.f;
        }
        S[i] = pd;                        // P (after dropout) for dV
        dP[i] = p * (dpv - D4[j]);        // dS (unscaled) for dK, dQ
      }
    }
    bf16x8_t pf[2], dsf[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 8; ++j) { pf[s2][j] = (__bf16)S[8 * s2 + j]; dsf[s2][j] = (__bf16)dP[8 * s2 + j]; }
    // dV^T += dO^T . P ; dK^T += Q^T . dS   (A operands by transposed reads of the tiles)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int qr = 16 * s2 + 4 * hh + trow;
      const bf16x8_t ado0 = cat_tr(lds_tr(dOt + swz_e(qr, tcol)), lds_tr(dOt + swz_e(qr + 8, tcol)));
      const bf16x8_t ado1 = cat_tr(lds_tr(dOt + swz_e(qr, 32 + tcol)), lds_tr(dOt + swz_e(qr + 8, 32 + tcol)));
      const bf16x8_t aq0 = cat_tr(lds_tr(Qt + swz_e(qr, tcol)), lds_tr(Qt + swz_e(qr + 8, tcol)));
      const bf16x8_t aq1 = cat_tr(lds_tr(Qt + swz_e(qr, 32 + tcol)), lds_tr(Qt + swz_e(qr + 8, 32 + tcol)));
      dV0 = mfma32(ado0, pf[s2], dV0);
      dV1 = mfma32(ado1, pf[s2], dV1);
      dK0 = mfma32(aq0, dsf[s2], dK0);
      dK1 = mfma32(aq1, dsf[s2], dK1);
    }
    // dS^T -> LDS [128 keys][32 q] (64-byte rows, 8-byte chunks XOR dsw(key), below):
    // each lane owns one key row and 4 runs of 4 consecutive queries -> 4 ds_write_b64
    {
      const int key = w * 32 + r;
      char* rowp = dSt + key * 64;
      const int sw = dsw(key);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 2 * g + hh;     // 8-byte chunk = queries 8g + 4hh .. +3
        u16x4 v = {f2bf(dP[4 * g]), f2bf(dP[4 * g + 1]), f2bf(dP[4 * g + 2]), f2bf(dP[4 * g + 3])};
        *reinterpret_cast<u16x4*>(rowp + ((c ^ sw) << 3)) = v;
      }
    }
    if constexpr (GL) {
      // tile qt + 1's DMA (issued a tile and a half ago) must have landed before this barrier;
      // only tile qt + 2's two pieces may stay in flight
      if (qt + 2 < nq) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      slot = slot == 2 ? 0 : slot + 1;
    }
    __syncthreads();   // the ONLY barrier of the tile: dS^T complete; this tile's Q / dO / lse /
                       // delta buffers free; tile t+1's staged buffers visible
    // tile qt + 2's inputs into the buffers tile qt released at this barrier (staging after the
    // dQ stores instead measured slower: its vmcnt wait then covers those stores too)
    if constexpr (!GL) {
      if (qt + 2 < nq) BWD_STAGE(buf);
    }
    // dQ[q][d] = sum over the 128 keys of dS[q][key] K[key][d], 16x16x32 MFMAs issued as
    // (K^T fragment, dS fragment): the lane ends up with 4 consecutive d of one query.  Both
    // fragments (8 consecutive keys per lane) come from transposing reads of [key][.] images.
    // The key rows a lane reads are a permutation of the natural 8 fg + 4 j + fq (bits 2 and 3
    // swapped: 16 (fg >> 1) + 8 j + 4 (fg & 1) + fq), the same for both operands, so the sum
    // over keys is unchanged: each 32-lane half of a transposing read then covers 8
    // consecutive rows, whose swizzled chunks of K (swz) and of dS^T (dsw) fill all 64 banks
    // (with the natural order rows r and r + 8 of K shared banks: a 2-way conflict on every
    // K^T read).
    f32x4 dq0 = {0.f, 0.f, 0.f, 0.f}, dq1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kr0 = 32 * ks + 16 * (fg >> 1) + 4 * (fg & 1) + fq, kr1 = kr0 + 8;
      const int qc = (dq_q0 >> 2) + fp;        // 8-byte chunk of queries dq_q0 + 4 fp .. + 3
      const bf16x8_t sf = cat_tr(lds_tr(dSt + kr0 * 64 + ((qc ^ dsw(kr0)) << 3)),
                                 lds_tr(dSt + kr1 * 64 + ((qc ^ dsw(kr1)) << 3)));
      const bf16x8_t kf0 = cat_tr(lds_tr(Ks + swz_e(kr0, dq_d0 + 4 * fp)), lds_tr(Ks + swz_e(kr1, dq_d0 + 4 * fp)));
      const bf16x8_t kf1 = cat_tr(lds_tr(Ks + swz_e(kr0, dq_d0 + 16 + 4 * fp)),
                                  lds_tr(Ks + swz_e(kr1, dq_d0 + 16 + 4 * fp)));
      dq0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf0, sf, dq0, 0, 0, 0);
      dq1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf1, sf, dq1, 0, 0, 0);
    }
    // dq0[rr] = dQ[q = dq_q0 + (lane & 15)][d = dq_d0 + 4 (lane >> 4) + rr], dq1 the same +16
    const int q = qb + dq_q0 + (lane & 15);
    if (single_block && dq16 && qb + 32 <= a.Sq) {
      const u16x4 o0 = {f2bf(dq0[0] * a.scale), f2bf(dq0[1] * a.scale), f2bf(dq0[2] * a.scale), f2bf(dq0[3] * a.scale)};
      const u16x4 o1 = {f2bf(dq1[0] * a.scale), f2bf(dq1[1] * a.scale), f2bf(dq1[2] * a.scale), f2bf(dq1[3] * a.scale)};
      // permlane16 swap of the two d blocks: lane group g gets 8 consecutive d
      const uint2 xv = __builtin_bit_cast(uint2, o0), yv = __builtin_bit_cast(uint2, o1);
      const auto s0 = __builtin_amdgcn_permlane16_swap(xv.x, yv.x, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(xv.y, yv.y, false, false);
      const uint4 v = {s0[0], s1[0], s0[1], s1[1]};
      const int d = dq_d0 + 16 * (fg & 1) + 8 * (fg >> 1);
      *reinterpret_cast<uint4*>(dqbase + q * (int)a.dq_ss + d) = v;
    } else if (!single_block) {
      // Sk > 128: the wave's [16 q][32 d] fp32 share goes through LDS so that each atomic
      // wave-instruction adds two contiguous 128-byte row segments (the memory-side atomic
      // unit's full-rate shape) instead of 16 rows x 4 scattered dwords (~10x slower: the
      // backward took 883 us at B 32, S 512 before, 326 after).  Scratch: this wave's own key
      // rows of the OTHER dS^T buffer (tile qt - 1's, read by every wave's dQ before this
      // tile's barrier; rewritten only by this wave, at tile qt + 1); 128-byte rows, 16-byte
      // chunks XOR (q & 7).  Every lane takes part; rows past Sq only skip their atomics.
      char* xw = dSs + (buf ^ 1) * 8192 + w * 2048;
      const int xq = lane & 15;
      *reinterpret_cast<f32x4*>(xw + xq * 128 + ((fg ^ (xq & 7)) << 4)) = dq0;
      *reinterpret_cast<f32x4*>(xw + xq * 128 + (((4 + fg) ^ (xq & 7)) << 4)) = dq1;
      __builtin_amdgcn_wave_barrier();
      const int xd = lane & 31;
      float* accp = a.dq_acc + ((long)bh * a.Sq + qb + dq_q0) * 64 + dq_d0 + xd;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int qr = 2 * i + (lane >> 5);
        const float val = *reinterpret_cast<const float*>(xw + qr * 128 + (((xd >> 2) ^ (qr & 7)) << 4) + ((xd & 3) << 2)) * a.scale;
        if (qb + dq_q0 + qr < a.Sq) atomicAdd(accp + qr * 64, val);
      }
      __builtin_amdgcn_wave_barrier();
    } else if (q < a.Sq) {
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int d = dq_d0 + 16 * t2 + 4 * fg + rr;
          dqbase[q * (int)a.dq_ss + d] = f2bf((t2 ? dq1[rr] : dq0[rr]) * a.scale);
        }
    }
  }
#undef BWD_PREFETCH
#undef BWD_STAGE
#undef BWD_GLDS
  {
    const long kl = kvalid ? key_l : 0;
    store_row64(a.dk + b * a.dk_sb + h * a.dk_sh + kl * a.dk_ss, dK0, dK1, a.scale, hh, kvalid);
    store_row64(a.dv + b * a.dv_sb + h * a.dv_sh + kl * a.dv_ss, dV0, dV1, 1.f, hh, kvalid);
  }
}

// dq (bf16, strided) = dq_acc (fp32 [B*H, Sq, 64])
__global__ void attn_dq_convert_kernel(const float* __restrict__ acc, bf16_t* __restrict__ dq,
                                       long sb, long ss, long sh, int B, int H, int Sq) {
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (t >= (long)B * H * Sq * 64) return;
  const int d = t & 63;
  const long row = t >> 6;
  const int q = row % Sq;
  const int bh = row / Sq;
  const int b = bh / H, h = bh % H;
  dq[b * sb + h * sh + (long)q * ss + d] = f2bf(acc[t]);
}

}  // namespace ct

using namespace ct;

static uint32_t host_hash_u32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}
static void drop_params(float p, uint64_t seed, uint64_t offset, uint32_t* thr16, float* inv_keep,
                        uint32_t* base) {
  long t = (long)(p * 65536.0f + 0.5f);
  *thr16 = (uint32_t)(t > 65535 ? 65535 : t);
  *inv_keep = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const uint32_t s_lo = (uint32_t)seed, s_hi = (uint32_t)(seed >> 32), o_lo = (uint32_t)offset;
  *base = host_hash_u32(s_lo ^ (s_hi * 0x85EBCA6Bu) ^ (o_lo * 0xC2B2AE35u));
}

// Multiprocessor count of the current device (cached per device id).
static int attn_cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// Persistent grid of a kernel with `per_cu` resident workgroups per CU over `nitems` work
// items: every workgroup takes ceil(nitems / slots) items and the grid is the fewest
// workgroups that need no more rounds than that.  CLOUDTIK_AMD_ATTN_PERSIST=0: one
// workgroup per item.
static int attn_persistent_grid(long nitems, int per_cu) {
  static const int on = [] {
    const char* e = getenv("CLOUDTIK_AMD_ATTN_PERSIST");
    return e ? atoi(e) : 1;
  }();
  if (!on || nitems <= 0) return (int)nitems;
  const long slots = (long)attn_cu_count() * per_cu;
  if (nitems <= slots) return (int)nitems;
  const long rounds = (nitems + slots - 1) / slots;
  return (int)((nitems + rounds - 1) / rounds);
}

// strides: [batch, seq, head] in elements for each tensor; head_dim must be 64 (contiguous)
// the kernels index rows inside one (batch, head) slice with 32-bit offsets
static inline bool fits32(long rows, long row_stride) { return rows * row_stride + 64 < (1L << 31); }

extern "C" int ct_attn_fwd(const void* q, const long* qs, const void* k, const long* ks,
                           const void* v, const long* vs, void* o, const long* os,
                           const float* kbias, long kb_sb, float* lse, int B, int H, int Sq,
                           int Sk, float scale, float p_drop, uint64_t seed, uint64_t offset,
                           int causal, hipStream_t stream) {
  if (B <= 0 || H <= 0 || Sq <= 0 || Sk <= 0) return -1;
  if (p_drop > 0.f && (Sk % 2)) return -2;
  if (!fits32(Sq, qs[1]) || !fits32(Sk, ks[1]) || !fits32(Sk, vs[1]) || !fits32(Sq, os[1])) return -5;
  // 16-byte output stores (attn_fwd_d64_kernel's epilogue)
  if (((uintptr_t)o & 15) || os[0] % 8 || os[1] % 8 || os[2] % 8) return -7;
  AttnFwdArgs a;
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.o = (bf16_t*)o;
  a.q_sb = qs[0]; a.q_ss = qs[1]; a.q_sh = qs[2];
  a.k_sb = ks[0]; a.k_ss = ks[1]; a.k_sh = ks[2];
  a.v_sb = vs[0]; a.v_ss = vs[1]; a.v_sh = vs[2];
  a.o_sb = os[0]; a.o_ss = os[1]; a.o_sh = os[2];
  a.kbias = kbias; a.kb_sb = kb_sb; a.lse = lse;
  a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk;
  a.scale_log2 = scale * 1.4426950408889634f;
  drop_params(p_drop, seed, offset, &a.thr16, &a.inv_keep, &a.hash_base);
  a.causal = causal;
  a.relb = nullptr; a.relb_sh = 0; a.relb_len = 0; a.rel_base = 0;
  dim3 grid((Sq + 127) / 128, B * H);
  const bool drop = p_drop > 0.f;
  // default: 2 waves/SIMD.  (r3: 3 with dropout, 168 VGPRs, 74-75 vs 77-78 us per BERT-large
  // layer; since both K/V tiles of an S <= 128 item load up front the 3-wave build spills one
  // register and the BERT-large step is 0.03-0.06 ms faster at 2 in three interleaved rounds:
  // 72.63 / 72.60 / 72.36 vs 72.57 / 72.55 / 72.34 ms)
  static const int wpe_env = [] {
    const char* e = getenv("CLOUDTIK_AMD_ATTN_FWD_WPE");
    return e ? atoi(e) : 0;
  }();
  static const int gl = [] {
    const char* e = getenv("CLOUDTIK_AMD_ATTN_FWD_GLDS");
    return e ? atoi(e) : 1;
  }();
  const int wpe = (wpe_env >= 1 && wpe_env <= 4) ? wpe_env : (gl ? 3 : 2);
  static const int pipe = [] {
    // opt-in: measured slower than the one-item kernel on BERT-large shapes (B 256, S 128,
    // p 0.1: 75.5 us persistent / 84.9 us one item per workgroup vs 65.9 us;
    // profiles/r3/attention_persistent_ab.md)
    const char* e = getenv("CLOUDTIK_AMD_ATTN_FWD_PIPE");
    return e ? atoi(e) : 0;
  }();
  if (pipe) {
    const long nitems = (long)((Sq + 127) / 128) * B * H;
    if (nitems > (1L << 30)) return -6;
    const int g1 = attn_persistent_grid(nitems, 2);
    if (drop && causal) attn_fwd_pipe_kernel<true, true><<<g1, 256, 0, stream>>>(a);
    else if (drop) attn_fwd_pipe_kernel<true, false><<<g1, 256, 0, stream>>>(a);
    else if (causal) attn_fwd_pipe_kernel<false, true><<<g1, 256, 0, stream>>>(a);
    else attn_fwd_pipe_kernel<false, false><<<g1, 256, 0, stream>>>(a);
    return 0;
  }
#define CT_ATTN_FWD(W, G)                                                                          \
  if (drop && causal) attn_fwd_d64_kernel<true, true, false, W, G><<<grid, 256, 0, stream>>>(a);    \
  else if (drop) attn_fwd_d64_kernel<true, false, false, W, G><<<grid, 256, 0, stream>>>(a);        \
  else if (causal) attn_fwd_d64_kernel<false, true, false, W, G><<<grid, 256, 0, stream>>>(a);      \
  else attn_fwd_d64_kernel<false, false, false, W, G><<<grid, 256, 0, stream>>>(a);
  if (gl) {
    if (wpe == 4) { CT_ATTN_FWD(4, true) } else if (wpe == 3) { CT_ATTN_FWD(3, true) } else { CT_ATTN_FWD(2, true) }
  } else {
    if (wpe == 3) { CT_ATTN_FWD(3, false) } else if (wpe == 1) { CT_ATTN_FWD(1, false) } else { CT_ATTN_FWD(2, false) }
  }
#undef CT_ATTN_FWD
  return 0;
}

// Forward with a per-head relative-position bias vector relb [H, relb_len] (row stride
// relb_sh): score(q, k) += relb[h][k - q + rel_base].  Inference path (no dropout).
extern "C" int ct_attn_fwd_relbias(const void* q, const long* qs, const void* k, const long* ks,
                                   const void* v, const long* vs, void* o, const long* os,
                                   const float* kbias, long kb_sb, const float* relb, long relb_sh,
                                   int relb_len, int rel_base, float* lse, int B, int H, int Sq, int Sk,
                                   float scale, int causal, hipStream_t stream) {
  if (B <= 0 || H <= 0 || Sq <= 0 || Sk <= 0 || relb_len <= 0) return -1;
  if (relb_len > kRelBiasMax) return -4;
  if (!fits32(Sq, qs[1]) || !fits32(Sk, ks[1]) || !fits32(Sk, vs[1]) || !fits32(Sq, os[1])) return -5;
  if (((uintptr_t)o & 15) || os[0] % 8 || os[1] % 8 || os[2] % 8) return -7;   // 16-byte output stores
  AttnFwdArgs a;
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.o = (bf16_t*)o;
  a.q_sb = qs[0]; a.q_ss = qs[1]; a.q_sh = qs[2];
  a.k_sb = ks[0]; a.k_ss = ks[1]; a.k_sh = ks[2];
  a.v_sb = vs[0]; a.v_ss = vs[1]; a.v_sh = vs[2];
  a.o_sb = os[0]; a.o_ss = os[1]; a.o_sh = os[2];
  a.kbias = kbias; a.kb_sb = kb_sb; a.lse = lse;
  a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.thr16 = 0; a.inv_keep = 1.f; a.hash_base = 0;
  a.causal = causal;
  a.relb = relb; a.relb_sh = relb_sh; a.relb_len = relb_len; a.rel_base = rel_base;
  dim3 grid((Sq + 127) / 128, B * H);
  if (causal) attn_fwd_d64_kernel<false, true, true><<<grid, 256, 0, stream>>>(a);
  else attn_fwd_d64_kernel<false, false, true><<<grid, 256, 0, stream>>>(a);
  return 0;
}

// delta workspace: float[B*H*Sq]; dq_acc workspace: float[B*H*Sq*64] zeroed (only used
// when Sk > 128)
extern "C" int ct_attn_bwd(const void* q, const long* qs, const void* k, const long* ks,
                           const void* v, const long* vs, const void* o, const long* os,
                           const void* dO, const long* dos, void* dq, const long* dqs, void* dk,
                           const long* dks, void* dv, const long* dvs, const float* kbias,
                           long kb_sb, const float* lse, float* delta, float* dq_acc, int B, int H,
                           int Sq, int Sk, float scale, float p_drop, uint64_t seed,
                           uint64_t offset, int causal, hipStream_t stream) {
  if (B <= 0 || H <= 0 || Sq <= 0 || Sk <= 0) return -1;
  if (p_drop > 0.f && (Sk % 2)) return -2;
  if (!fits32(Sq, qs[1]) || !fits32(Sk, ks[1]) || !fits32(Sk, vs[1]) || !fits32(Sq, os[1]) ||
      !fits32(Sq, dos[1]) || !fits32(Sq, dqs[1])) return -5;
  // 16-byte dK / dV stores (store_row64)
  if (((uintptr_t)dk & 15) || ((uintptr_t)dv & 15) || dks[0] % 8 || dks[1] % 8 || dks[2] % 8 || dvs[0] % 8 ||
      dvs[1] % 8 || dvs[2] % 8)
    return -7;
  const long rows = (long)B * H * Sq;
  AttnBwdArgs a;
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.dO = (const bf16_t*)dO;
  a.o = (const bf16_t*)o; a.o_sb = os[0]; a.o_ss = os[1]; a.o_sh = os[2];
  a.dq = (bf16_t*)dq; a.dk = (bf16_t*)dk; a.dv = (bf16_t*)dv; a.dq_acc = dq_acc;
  a.q_sb = qs[0]; a.q_ss = qs[1]; a.q_sh = qs[2];
  a.k_sb = ks[0]; a.k_ss = ks[1]; a.k_sh = ks[2];
  a.v_sb = vs[0]; a.v_ss = vs[1]; a.v_sh = vs[2];
  a.do_sb = dos[0]; a.do_ss = dos[1]; a.do_sh = dos[2];
  a.dq_sb = dqs[0]; a.dq_ss = dqs[1]; a.dq_sh = dqs[2];
  a.dk_sb = dks[0]; a.dk_ss = dks[1]; a.dk_sh = dks[2];
  a.dv_sb = dvs[0]; a.dv_ss = dvs[1]; a.dv_sh = dvs[2];
  a.kbias = kbias; a.kb_sb = kb_sb; a.lse = lse; a.delta = delta;
  a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk;
  a.scale = scale; a.scale_log2 = scale * 1.4426950408889634f;
  drop_params(p_drop, seed, offset, &a.thr16, &a.inv_keep, &a.hash_base);
  a.causal = causal;
  const int nkb = (Sk + 127) / 128;
  if (nkb > 1 && !dq_acc) return -3;
  if (nkb > 1) hipMemsetAsync(dq_acc, 0, sizeof(float) * rows * 64, stream);
  dim3 grid(nkb, B * H);
  // causal masking is a template parameter (as in the forward): no per-element test of a
  // runtime flag in the non-causal (BERT) kernel
#define CT_ATTN_BWD(M, G)                                                                \
  if (p_drop > 0.f) {                                                                    \
    if (causal) attn_bwd_d64_kernel<true, true, M, G><<<grid, 256, 0, stream>>>(a);      \
    else attn_bwd_d64_kernel<true, false, M, G><<<grid, 256, 0, stream>>>(a);            \
  } else {                                                                               \
    if (causal) attn_bwd_d64_kernel<false, true, M, G><<<grid, 256, 0, stream>>>(a);     \
    else attn_bwd_d64_kernel<false, false, M, G><<<grid, 256, 0, stream>>>(a);           \
  }
  static const int bwd_gl = [] {
    const char* e = getenv("CLOUDTIK_AMD_ATTN_BWD_GL");
    return e ? atoi(e) : 1;
  }();
  if (nkb > 1) { CT_ATTN_BWD(true, false) }
  else if (bwd_gl && Sq <= 128) { CT_ATTN_BWD(false, true) }
  else { CT_ATTN_BWD(false, false) }
#undef CT_ATTN_BWD
  if (nkb > 1)
    attn_dq_convert_kernel<<<(int)((rows * 64 + 255) / 256), 256, 0, stream>>>(
        dq_acc, (bf16_t*)dq, dqs[0], dqs[1], dqs[2], B, H, Sq);
  return 0;
}

extern "C" uint32_t ct_attn_hash_base(uint64_t seed, uint64_t offset) {
  uint32_t t, b; float f;
  drop_params(0.f, seed, offset, &t, &f, &b);
  return b;
}
