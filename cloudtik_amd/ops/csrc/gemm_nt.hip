// Forward / data-gradient GEMM for gfx950 with fused epilogues:
//     D[M, N] = A[M, K] . B[N, K]^T   (bf16 in, fp32 accumulate; both operands K-contiguous)
// epilogues: plain (optionally D += ...), bias + erf-GELU keeping the pre-activation
// (BERT FFN1 forward), and dGELU + bias-gradient column sums (BERT FFN dgrad).  The point is
// the epilogue: without it the [tokens, 4*hidden] activation makes one extra HBM round trip
// per GEMM through a separate elementwise kernel (bias_act_fwd / bias_act_bwd, ~100-200 us
// per layer on BERT-large).  hipBLASLt on this image offers no GELU_AUX / DGELU epilogue
// kernels for bf16 on gfx950 (bench/lt_epilogue_probe.py), and its GELU is the tanh form.
//
// Structure (256 x 256 x 64 tile, 512 threads = 8 waves as 2 (M) x 4 (N), 128 x 64 per wave):
//   * both operands staged global -> LDS with global_load_lds (16 B per lane, lane-linear
//     LDS side, the 16-B chunk XOR swizzle (row >> 1) & 7 applied on the source address) into
//     two 64 KiB buffers of four 16 KiB half-tile images each (cut by reading phase, below);
//   * every K-tile runs as 4 phases, one per 64 x 32 quadrant of the wave's output; each phase
//     = [ds_read_b128 fragments + LDS-DMA issue] barrier [16 MFMA 16x16x32] barrier;
//   * the two wave groups (M halves) run one barrier apart ("ping-pong"): while one group
//     multiplies, the other reads its fragments and issues the next DMA, so the SIMD sees a
//     steady MFMA stream without register-double-buffered fragments;
//   * exactly one half-tile DMA (2 glds per wave) and one counted vmcnt(8) per phase, four
//     halves in flight; fragment reads 12 / 4 / 8 / 0 per phase (schedule: nt_stage_slot);
//   * the MFMA is issued as B-fragment x A-fragment, so each lane ends up with 4 consecutive
//     output COLUMNS of one row; a permlane16 swap between column blocks turns them into 8
//     consecutive columns for 16-byte stores (nt_pair_swap);
//   * blockIdx -> tile goes through the bijective XCD remap; N-tiles vary fastest so the
//     blocks resident on one XCD share A panels in its L2.
//   * staging through registers (global_load_dwordx4 + ds_write_b128 a few phases later) was
//     measured 10 % slower than the LDS-DMA once the DMA's bases are wave-uniform SGPRs.
// The same kernel runs the weight-gradient layout (TN: both operands token-major, transposing
// LDS reads, split-K into fp32 slabs; ct_gemm_tn2).
// Reference: the BERT encoder FFN (HF BertIntermediate + BertOutput).
#include "common.h"
#include <algorithm>
#include <cstdlib>

namespace ct {

typedef __attribute__((ext_vector_type(8))) short nt_s16x8;
typedef __attribute__((address_space(3))) nt_s16x8 nt_lds_s16x8;
typedef __attribute__((address_space(3))) void nt_lds_void;

constexpr int NT_BM = 256, NT_BN = 256, NT_BK = 64, NT_THREADS = 512;
constexpr int NT_ROWB = NT_BK * 2;        // 128 B per LDS image row
constexpr int NT_HALF = 128 * NT_ROWB;    // 16 KiB: 128 rows of one operand
constexpr int NT_BUF = 4 * NT_HALF;       // 64 KiB per K-tile buffer

// EPI 6 / 7 are the derivative-storing pair: the FFN1 forward keeps gelu'(x W1^T + b1) (bf16) as
// its aux output instead of the pre-activation, and the FFN data gradient multiplies by it --
// the dGELU's transcendental work (exp + rcp per element) moves out of the VALU-bound backward
// epilogue into the forward one, which is store-bound and computes the same exp / erf terms anyway.
enum { NT_EPI_PLAIN = 0, NT_EPI_BIAS_GELU_AUX = 1, NT_EPI_DGELU_BGRAD = 2, NT_EPI_F32_SLAB = 3, NT_EPI_NONE = 4,
       NT_EPI_BIAS = 5, NT_EPI_BIAS_GELU_DAUX = 6, NT_EPI_MUL_AUX_BGRAD = 7 };

struct NtArgs {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* D;
  const bf16_t* bias;   // EPI 1: [N]; EPI 2 (optional): added to aux before gelu'
  bf16_t* aux;          // EPI 1: pre-activation out; EPI 2: pre-activation in
  float* dbias;         // EPI 2: [N] fp32, accumulated with atomics (may be null)
  float* P;             // EPI 3: fp32 split-K slabs [splits][M][N]
  float* biasg;         // TN (BIASG): fp32 [splits][M] column sums of A over this split's K
  long lda, ldb, ldd, ldaux;
  long tsplit;          // TN: number of split-K slices (the K-tiles are dealt out as evenly as
                        // possible: the first (K / 64) % splits slices get one K-tile more)
  int M, N, K;
  int accumulate;       // EPI 0: D += result
  int stagger;          // NT / NN one-tile grid: H column-half tiles at each end (0 = none), below
  int group_m;          // NT / NN: M-tiles walked per N-tile in the XCD tile order (1 = row-major)
  int dbias_rows;       // EPI 2 / 7: dbias is [dbias_rows][N] (a power of two; 0 or 1 = [N]): the
                        //   column sums of row-half h = mrow >> 7 go to row h & (dbias_rows - 1)
};

__device__ __forceinline__ int nt_swz(int r) { return (r >> 1) & 7; }

__device__ __forceinline__ void nt_glds16(const void* g, const char* lds_wave_base) {
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(nt_lds_void*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(la) : "memory", "m0");
}

// same, addressed as a wave-uniform 64-bit base (SGPRs) + a per-lane 32-bit byte offset: no
// per-lane 64-bit address arithmetic and no address VGPR pairs to keep live
__device__ __forceinline__ void nt_glds16s(const void* sbase, unsigned voff, const char* lds_wave_base) {
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(nt_lds_void*)lds_wave_base);
  // (readfirstlane returns int: widen through uint32_t, or a low word >= 2^31 sign-extends
  // into the high word)
  const uint64_t sb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)sbase) |
                      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)sbase >> 32)) << 32);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sb), "s"(la)
               : "memory", "m0");
}

// per-lane byte offset of a staging piece: row (lane >> 3) of the piece's 8, 16-B chunk
// (lane & 7) ^ swizzle; the swizzle of image row piece*8 + (lane >> 3) depends on the piece
// only through its parity
__device__ __forceinline__ unsigned nt_lane_off(long ld, int parity, int lane) {
  const int cc = (lane & 7) ^ ((parity * 4 + (lane >> 4)) & 7);
  return (unsigned)(((lane >> 3) * ld + cc * 8) * 2);
}

// 16 x 32 MFMA operand fragment: rows [r0, r0 + 16), k [32 ks, 32 ks + 32); lane l holds row
// r0 + (l & 15), k 32 ks + 8 (l >> 4) .. + 8.  Conflict-free for ds_read_b128's lane groups.
__device__ __forceinline__ nt_s16x8 nt_frag(const char* img, int r0, int ks, int lane) {
  const int row = r0 + (lane & 15);
  const int kc = ks * 4 + (lane >> 4);
  return *(const nt_lds_s16x8*)(img + row * NT_ROWB + ((kc ^ nt_swz(row)) << 4));
}

// ---- TN layout (weight gradients: D[M, N] = A[K, M]^T B[K, N], K = tokens is the row index of
// both operands).  A half-tile image is 64 k-rows x 128 columns (256 B rows): the same 16 KiB
// and the same column sets per half as the NT images' rows, so the phase schedule, the
// fragment indices and the epilogue are shared; only staging and fragment reads differ.
// Fragments need 8 consecutive k per lane: two ds_read_b64_tr_b16 (gfx950's transposing LDS
// read) per 16 x 32 fragment.  Chunk swizzle of 256-B row r: rows r..r+3 and r+8..r+11 land in
// 8 distinct 32-B bank slots for the transposing reads.
constexpr int TN_ROWB = 256;
__device__ __forceinline__ int tn_swz(int r) { return ((r & 3) << 1) | (((r >> 3) & 1) << 3); }

typedef __attribute__((ext_vector_type(4))) short tn_s16x4;
typedef __attribute__((address_space(3))) tn_s16x4 tn_lds_s16x4;

// fragment of image columns [c0, c0 + 16) x k [32 ks, 32 ks + 32): lane l gets column
// c0 + (l & 15), k 32 ks + 8 (l >> 4) .. + 8 -- the nt_frag lane layout
__device__ __forceinline__ nt_s16x8 tn_frag(const char* img, int c0, int ks, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int r0 = 32 * ks + 8 * g + q, r1 = r0 + 4;
  const int ch = (c0 >> 3) + (p >> 1);
  const char* a0 = img + r0 * TN_ROWB + ((ch ^ tn_swz(r0)) << 4) + ((p & 1) << 3);
  const char* a1 = img + r1 * TN_ROWB + ((ch ^ tn_swz(r1)) << 4) + ((p & 1) << 3);
  const tn_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tn_lds_s16x4*)a0);
  const tn_s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tn_lds_s16x4*)a1);
  return nt_s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// per-lane byte offset of a TN staging piece (4 image rows of 256 B = one glds): lane l fills
// LDS chunk (l & 15) of row 4 piece + (l >> 4) with global chunk (l & 15) ^ swizzle; the
// swizzle depends on the piece only through (piece >> 1) & 1 = wave & 1.  Image chunk c ->
// operand column: A halves hold tile columns {0-63, 128-191} (+64 for A1), B halves the
// first (B0) or second (B1) 32 of each 64-column wave block.
__device__ __forceinline__ unsigned tn_lane_off(long ld, int wave, int lane, bool isA) {
  const int q = lane >> 4;
  const int c = (lane & 15) ^ tn_swz(q + 8 * (wave & 1));
  const int col = isA ? (c < 8 ? c * 8 : 128 + (c - 8) * 8) : (c >> 2) * 64 + (c & 3) * 8;
  return (unsigned)((q * ld + col) * 2);
}

__device__ __forceinline__ void nt_bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void nt_mma_begin() {
  nt_bar();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_setprio(1);
}

__device__ __forceinline__ void nt_mma_end() {
  __builtin_amdgcn_s_setprio(0);
  nt_bar();
}

// Half-tile images (16 KiB each, 128 rows x 64 k) are cut by the phase that reads them, not by
// position: A0 = the first 64 rows of each wave group (tile rows 0-63, 128-191), A1 = the other
// 64 (64-127, 192-255), B0 = the first 32 columns of each wave column (0-31, 64-95, ...), B1 = the
// other 32.  Phase q0 reads A0 + B0, q1 B1, q2 A1, q3 nothing, so every half has its own last
// read and is restaged as soon as that allows: one half per phase, in the order A0 B0 B1 A1,
// virtual index v = 4 * tile - 6 + slot (tile 0 and half of tile 1 in the prologue, then the
// half v = p at phase p).  Every phase waits vmcnt(8): the half issued 4 phases earlier has
// landed, and it is first read 5 phases after its issue (one phase after the wait, as the
// barrier offset between the wave groups requires); a half is restaged >= 2 phases after its
// last read (WAR for the group that runs ahead).
struct NtCtx {
  const bf16_t* A;
  const bf16_t* B;
  long lda, ldb, m0, n0, kbase;   // kbase: first k of this split (TN)
  char* lds;
  int wave, lane, ra, rb;
  unsigned offa0, offa1, offb0, offb1;   // per-lane staging offsets (NT: by piece parity; TN: A / B)
  int biasw;                             // BIASG: this wave owns bias rows 2 wc, 2 wc + 1 (else -1)
  int half;                              // 0 full tile; 1 / 2: only the B0 / B1 column halves
};

// Bias gradient inside the weight-gradient GEMM (TN): db[m] = sum_k A[k][m] is one more MFMA per
// A fragment against a constant all-ones B fragment.  The tn == 0 tile of every split does it;
// its 4 wave columns share the work (wave column wc: A fragments 2 wc, 2 wc + 1, in the phase
// that reads them), 4 extra MFMAs in one of the 4 phases.  Replaces a separate column-sum pass
// over the [tokens, 3 * hidden] QKV gradient (~38 us per BERT-large layer).
template <int Q, int I0>
__device__ __forceinline__ void nt_quad_bias(f32x4 (&accb)[2], const nt_s16x8 (&fa)[4][2], int biasw) {
  if (biasw < 0 || (biasw >> 2) != (I0 >> 2)) return;          // rows 0-3 in q0, 4-7 in q2
  nt_s16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (short)0x3F80;           // bf16 1.0
  // fragment indices must stay compile-time: a runtime index into fa would put the whole
  // fragment array in scratch memory
  if ((biasw & 3) == 0) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        accb[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf16x8_t)ones, (bf16x8_t)fa[t][ks], accb[t], 0, 0, 0);
  } else {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        accb[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf16x8_t)ones, (bf16x8_t)fa[2 + t][ks], accb[t], 0, 0, 0);
  }
}

// operand layouts: LAY 0 = NT (A [M,K], B [N,K]), 1 = TN (A [K,M], B [K,N]; weight gradients),
// 2 = NN (A [M,K], B [K,N]; data gradients straight from the [out, in] weight)
template <int LAY> struct NtLay {
  static constexpr bool AT = LAY == 1;    // A stored k-major (transposing staging / reads)
  static constexpr bool BT = LAY >= 1;    // B stored k-major
};

template <int LAY>
__device__ __forceinline__ void nt_stage_slot(const NtCtx& c, long k0, int slot, char* dst) {
  using Ly = NtLay<LAY>;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = c.wave * 2 + i;
    const long krow = c.kbase + k0 + piece * 4;            // k-major images: rows 4 piece .. + 4
    const bf16_t* base;
    unsigned off;
    if (slot == 0 || slot == 3) {                          // A0 / A1
      if constexpr (!Ly::AT) {                             // image rows piece*8 .. +8
        base = c.A + (c.m0 + ((piece >> 3) << 7) + (slot == 3 ? 64 : 0) + (piece & 7) * 8) * c.lda + k0;
        off = i ? c.offa1 : c.offa0;
      } else {
        base = c.A + krow * c.lda + c.m0 + (slot == 3 ? 64 : 0);
        off = c.offa0;
      }
    } else {                                               // B0 / B1
      if constexpr (!Ly::BT) {
        base = c.B + (c.n0 + ((piece >> 2) << 6) + (slot == 2 ? 32 : 0) + (piece & 3) * 8) * c.ldb + k0;
        off = i ? c.offb1 : c.offb0;
      } else {
        base = c.B + krow * c.ldb + c.n0 + (slot == 2 ? 32 : 0);
        off = c.offb0;
      }
    }
    nt_glds16s(base, off, dst + piece * 1024);
  }
}

template <int N>
__device__ __forceinline__ void nt_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// one 16-MFMA quadrant: acc[I0 + i][J0 + j] += A-frags fa[QM] x B-frags fb[QN]
template <int I0, int J0>
__device__ __forceinline__ void nt_quad(f32x4 (&acc)[8][4], const nt_s16x8 (&fa)[4][2], const nt_s16x8 (&fb)[2][2]) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf16x8_t)fb[j][ks], (bf16x8_t)fa[i][ks],
                                                                       acc[I0 + i][J0 + j], 0, 0, 0);
}

// half with virtual index v (see above) -> its buffer slot
template <int LAY>
__device__ __forceinline__ void nt_stage_v(const NtCtx& c, int v) {
  const int T = (v + 6) >> 2, slot = (v + 6) & 3;
  nt_stage_slot<LAY>(c, (long)T * NT_BK, slot, c.lds + (T & 1) * NT_BUF + slot * NT_HALF);
}

template <bool KMAJOR>
__device__ __forceinline__ nt_s16x8 nt_fragment(const char* img, int r0, int ks, int lane) {
  if constexpr (KMAJOR) return tn_frag(img, r0, ks, lane);
  else return nt_frag(img, r0, ks, lane);
}

// DMA plan of one K-tile t (POS: 0 steady, 1 = K-tile nk-2, 2 = the last K-tile): phase q
// issues half v = 4t + q (virtual index, slot order A0 B0 B1 A1) and waits vmcnt(8) in steady
// state (the half of 4 phases ago has landed).  Measured alternatives that change nothing
// (within 2 %): two halves in each of the read-light phases q1 / q3 only, and DMA issued
// before instead of after the phase's fragment reads.
template <int POS>
struct NtPlan {
  static constexpr bool issue(int q) { return POS == 0 || (POS == 1 && q < 2); }
  static constexpr int wait(int q) {
    return POS == 0 ? 8 : (POS == 1 ? (q < 2 ? 8 : (q == 2 ? 6 : 4)) : (q == 0 ? 2 : 0));
  }
};

template <int POS, int DIAG, int LAY, bool BIASG>
__device__ __forceinline__ void nt_ktile(const NtCtx& c, int t, f32x4 (&acc)[8][4], nt_s16x8 (&fa)[2][4][2],
                                         nt_s16x8 (&fb)[2][2][2], f32x4 (&accb)[2]) {
  const char* buf = c.lds + (t & 1) * NT_BUF;
  constexpr bool WAIT = DIAG == 0, BAR = DIAG != 2;
  constexpr bool DMA = DIAG == 0 || DIAG == 3;
  using P = NtPlan<POS>;
#define NT_PHASE_TAIL(Q, I0, J0, FA, FB)                                             \
  if constexpr (DMA && P::issue(Q)) nt_stage_v<LAY>(c, 4 * t + Q);                   \
  if constexpr (WAIT) nt_vm<P::wait(Q)>();                                           \
  if constexpr (BAR) nt_mma_begin(); else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
  if (c.half != (J0 == 0 ? 2 : 1)) nt_quad<I0, J0>(acc, FA, FB);                     \
  if constexpr (BIASG && (Q == 0 || Q == 2)) nt_quad_bias<Q, I0>(accb, FA, c.biasw); \
  if constexpr (BAR) nt_mma_end(); else __builtin_amdgcn_sched_barrier(0);
  // ---- q0: B0 + A0 fragments
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) fb[0][j][ks] = nt_fragment<NtLay<LAY>::BT>(buf + 1 * NT_HALF, c.rb + j * 16, ks, c.lane);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) fa[0][i][ks] = nt_fragment<NtLay<LAY>::AT>(buf + 0 * NT_HALF, c.ra + i * 16, ks, c.lane);
  NT_PHASE_TAIL(0, 0, 0, fa[0], fb[0])
  // ---- q1: B1 fragments
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) fb[1][j][ks] = nt_fragment<NtLay<LAY>::BT>(buf + 2 * NT_HALF, c.rb + j * 16, ks, c.lane);
  NT_PHASE_TAIL(1, 0, 2, fa[0], fb[1])
  // ---- q2: A1 fragments
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) fa[1][i][ks] = nt_fragment<NtLay<LAY>::AT>(buf + 3 * NT_HALF, c.ra + i * 16, ks, c.lane);
  NT_PHASE_TAIL(2, 4, 2, fa[1], fb[1])
  // ---- q3: no fragment reads
  NT_PHASE_TAIL(3, 4, 0, fa[1], fb[0])
#undef NT_PHASE_TAIL
}

// 16-B stores from the MFMA layout: lane l holds 4 consecutive columns 16 j + 4 (l >> 4) .. + 3
// of row (l & 15) in block j; v_permlane16_swap exchanges the odd 16-lane rows of block j with
// the even rows of block j + 1, after which lane l holds 8 consecutive columns
// 8 ((l >> 4) >> 1) .. + 7 of block j + ((l >> 4) & 1) -- one dwordx4 store instead of two
// dwordx2 (the epilogue store tail is store-issue bound: MI355X_MICROARCH.md, attention epilogue
// row; cdna_hip_programming.md T21).  Each store instruction then writes 16 rows x 64
// contiguous bytes.
__device__ __forceinline__ u16x8 nt_pair_swap(u16x4 x, u16x4 y) {
  const uint2 xv = __builtin_bit_cast(uint2, x), yv = __builtin_bit_cast(uint2, y);
  const auto s0 = __builtin_amdgcn_permlane16_swap(xv.x, yv.x, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(xv.y, yv.y, false, false);
  // after the swap this lane holds (s0[0], s1[0]) = columns c .. c+3, (s0[1], s1[1]) = c+4 .. c+7
  const uint4 v = {s0[0], s1[0], s0[1], s1[1]};
  return __builtin_bit_cast(u16x8, v);
}

// inverse of nt_pair_swap (the lane swap is an involution): 8 consecutive columns loaded in the
// store layout -> this lane's 4 columns of blocks j (x) and j + 1 (y) in the MFMA layout
__device__ __forceinline__ void nt_pair_unswap(u16x8 v, u16x4& x, u16x4& y) {
  const uint4 w = __builtin_bit_cast(uint4, v);
  const auto r0 = __builtin_amdgcn_permlane16_swap(w.x, w.z, false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(w.y, w.w, false, false);
  x = __builtin_bit_cast(u16x4, uint2{r0[0], r1[0]});
  y = __builtin_bit_cast(u16x4, uint2{r0[1], r1[1]});
}

// epilogue over one wave's accumulators: acc[i][j][r] holds D[mrow + 16i][ncol + 16j + r]
// (ncol includes this lane's 4 (lane >> 4)); math in that layout, stores after the swap.
// EPI 3 (fp32 split-K slab, row stride N): the lane's 4 columns are one 16-B store already.
// Epilogue operands loaded ahead of their use: the bias columns before the K loop (the
// epilogue used to open with these loads and wait a full memory latency, once per tile; the
// K loop's counted vmcnt waits stay correct -- the loads are older than the DMA they wait
// for, so they are simply waited for too) and the dGELU pre-activation rows two rows ahead
// inside the epilogue.  Issuing the first two rows before the last K-tile as well measured
// slower (343 vs 338 us per BERT-large FFN dgrad): the last K-tile's waits then cover them.
template <int NJ>
struct NtEpiPre {
  u16x4 bias[NJ];
  u16x4 z[2][NJ];
};

template <int EPI, int NJ>
__device__ __forceinline__ void nt_preload_bias(const NtArgs& a, long ncol, NtEpiPre<NJ>& pre) {
  if constexpr (EPI == NT_EPI_BIAS_GELU_AUX || EPI == NT_EPI_DGELU_BGRAD || EPI == NT_EPI_BIAS ||
                EPI == NT_EPI_BIAS_GELU_DAUX) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) pre.bias[j] = a.bias ? *(const u16x4*)(a.bias + ncol + j * 16) : u16x4(0);
  }
}

template <int EPI, int NJ>
__device__ __forceinline__ void nt_preload_z(const NtArgs& a, long mrow, long ncol, NtEpiPre<NJ>& pre) {
  if constexpr (EPI == NT_EPI_DGELU_BGRAD || EPI == NT_EPI_MUL_AUX_BGRAD) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) pre.z[i][j] = *(const u16x4*)(a.aux + (mrow + i * 16) * a.ldaux + ncol + j * 16);
  }
}

// ACC = false: the caller never accumulates into D (EPI 0), so no old-D registers are reserved
template <int EPI, bool BGRAD, int NJ, bool ACC = true>
__device__ __forceinline__ void nt_epilogue(const NtArgs& a, const f32x4 (&acc)[8][NJ], long mrow, long ncol,
                                            int lane, int split, NtEpiPre<NJ>& pre, int half = 0) {
  static_assert(NJ % 2 == 0, "pairs of 16-column blocks");
  if constexpr (EPI == NT_EPI_NONE) {
    // timing diagnostic (CLOUDTIK_AMD_GEMM_DIAG=4): the K loop without the epilogue's memory
    // traffic; the never-taken store keeps the accumulators live
    f32x4 t = acc[0][0];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) t += acc[i][j];
    if (a.accumulate == 0x5EED) *(f32x4*)(a.P ? a.P : (float*)a.D) = t;
    return;
  }
  if constexpr (EPI == NT_EPI_F32_SLAB) {
    float* P = a.P + (long)split * a.M * a.N;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) *(f32x4*)(P + (mrow + i * 16) * a.N + ncol + j * 16) = acc[i][j];
    return;
  }
  float bv[NJ][4] = {};
  if constexpr (EPI == NT_EPI_BIAS_GELU_AUX || EPI == NT_EPI_DGELU_BGRAD || EPI == NT_EPI_BIAS ||
                EPI == NT_EPI_BIAS_GELU_DAUX) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[j][r] = bf2f(pre.bias[j][r]);
  }
  f32x2 cs[2 * NJ];   // dGELU column sums, packed pairs: (block j, columns 2h, 2h + 1)
#pragma unroll
  for (int p = 0; p < 2 * NJ; ++p) cs[p] = f32x2{0.f, 0.f};
  // column of this lane's 16-B chunk after the swap, relative to block 0 of the pair
  const int g = lane >> 4;
  const long scol = (ncol - 4 * g) + 16 * (g & 1) + 8 * (g >> 1);
  // The tensor the epilogue reads (EPI 2 / 7: aux; EPI 0 accumulating: D itself) is loaded for
  // all 8 row blocks up front, as 16-byte pieces in the store layout (full 64-byte row
  // segments), then turned into the MFMA layout (nt_pair_unswap): one memory latency per tile
  // instead of one per row block (a two-row-ahead ring of 8-byte loads before: the EPI 7
  // epilogue cost 19.6 us per tile-round against 14.6 for EPI 6, profiles/r5/gemm_epilogue_probe.md).
  // The fragment registers of the K loop are dead here, so the 64 VGPRs come free.
  constexpr bool RD = EPI == NT_EPI_DGELU_BGRAD || EPI == NT_EPI_MUL_AUX_BGRAD || (EPI == NT_EPI_PLAIN && ACC);
  u16x8 zin[RD ? 8 : 1][NJ / 2];
  if constexpr (RD) {
    const bool rd = EPI != NT_EPI_PLAIN || a.accumulate;
    const bf16_t* src = EPI == NT_EPI_PLAIN ? a.D : a.aux;
    const long ld = EPI == NT_EPI_PLAIN ? a.ldd : a.ldaux;
    if (rd) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int p = 0; p < NJ / 2; ++p) zin[i][p] = *(const u16x8*)(src + (mrow + i * 16) * ld + scol + p * 32);
    }
  }

#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const long m = mrow + i * 16;
    u16x4 out[NJ], pre[NJ];
    if constexpr (EPI == NT_EPI_BIAS) {
      // D = result + bias (the forward Linear: QKV / attention output / FFN2 projections)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[j][r] = f2bf(acc[i][j][r] + bv[j][r]);
    } else if constexpr (EPI == NT_EPI_PLAIN) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (ACC && a.accumulate) {
          u16x4 old, old2;
          nt_pair_unswap(zin[RD ? i : 0][RD ? (j >> 1) : 0], old, old2);
          if (j & 1) old = old2;
#pragma unroll
          for (int r = 0; r < 4; ++r) out[j][r] = f2bf(acc[i][j][r] + bf2f(old[r]));
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) out[j][r] = f2bf(acc[i][j][r]);
        }
      }
    } else {
      // bias + GELU: the row's 4 NJ elements as 2 NJ packed pairs (gelu2_batch: 1550 instead
      // of 1742 VALU instructions and 6 instead of 260 hazard s_nop per wave epilogue).  Same
      // time measured (301 vs 302 us for BERT-large FFN1): the epilogue writes h and z, 2 x
      // 268 MB, at ~5 TB/s -- it is store-bandwidth bound once every CU reaches it together.
      if constexpr (EPI == NT_EPI_BIAS_GELU_DAUX) {
        // h = gelu(x), aux = gelu'(x), x = acc + bias
        f32x2 xv[2 * NJ], gv[2 * NJ], dv[2 * NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            xv[2 * j + h] = f32x2{acc[i][j][2 * h], acc[i][j][2 * h + 1]} + f32x2{bv[j][2 * h], bv[j][2 * h + 1]};
        gelu2_batch_both<2 * NJ>(xv, gv, dv);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              pre[j][2 * h + e] = f2bf(dv[2 * j + h][e]);
              out[j][2 * h + e] = f2bf(gv[2 * j + h][e]);
            }
      } else if constexpr (EPI == NT_EPI_MUL_AUX_BGRAD) {
        // dz = dh * gelu'(z): the derivative was stored by the forward (EPI 6)
        u16x4 z[NJ];
#pragma unroll
        for (int p = 0; p < NJ / 2; ++p) nt_pair_unswap(zin[i][p], z[2 * p], z[2 * p + 1]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gg = acc[i][j][r] * bf2f(z[j][r]);
            out[j][r] = f2bf(gg);
            if constexpr (BGRAD) cs[2 * j + (r >> 1)][r & 1] += gg;
          }
        }
      } else if constexpr (EPI == NT_EPI_BIAS_GELU_AUX) {
        f32x2 xv[2 * NJ], gv[2 * NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            xv[2 * j + h] = f32x2{acc[i][j][2 * h], acc[i][j][2 * h + 1]} + f32x2{bv[j][2 * h], bv[j][2 * h + 1]};
        gelu2_batch<2 * NJ, false>(xv, gv);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              pre[j][2 * h + e] = f2bf(xv[2 * j + h][e]);
              out[j][2 * h + e] = f2bf(gv[2 * j + h][e]);
            }
      } else {
        // dGELU: scalar form (the packed-pair form measured no faster: 366 vs 349 us per
        // BERT-large FFN dgrad)
        u16x4 z[NJ];
#pragma unroll
        for (int p = 0; p < NJ / 2; ++p) nt_pair_unswap(zin[i][p], z[2 * p], z[2 * p + 1]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gg = acc[i][j][r] * gelu_erf_grad(bf2f(z[j][r]) + bv[j][r]);
            out[j][r] = f2bf(gg);
            if constexpr (BGRAD) cs[2 * j + (r >> 1)][r & 1] += gg;
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; j += 2) {
      const long n = scol + j * 16;
      if (half == (j < NJ / 2 ? 2 : 1)) continue;       // the other WG's column half
      *(u16x8*)(a.D + m * a.ldd + n) = nt_pair_swap(out[j], out[j + 1]);
      if constexpr (EPI == NT_EPI_BIAS_GELU_AUX || EPI == NT_EPI_BIAS_GELU_DAUX)
        *(u16x8*)(a.aux + m * a.ldaux + n) = nt_pair_swap(pre[j], pre[j + 1]);
    }
  }
  if constexpr ((EPI == NT_EPI_DGELU_BGRAD || EPI == NT_EPI_MUL_AUX_BGRAD) && BGRAD) {
    // column sums: reduce the 16 rows held by lanes sharing (lane >> 4), then one atomic per
    // column per wave (vector-memory float atomics).  The atomics of one address serialise at
    // the memory side: all 2 x M/256 row halves adding into ONE [N] vector cost BERT-large's FFN
    // data gradient 52 us per call (367.6 vs 315.4 without the sums, 32768 x 4096); spread over
    // dbias_rows copies (reduced by the caller's split-K reduce) each address sees 1/rows of them.
    float* db = a.dbias + (a.dbias_rows > 1 ? (long)((mrow >> 7) & (a.dbias_rows - 1)) * a.N : 0L);
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (half == (j < NJ / 2 ? 2 : 1)) continue;
        float v = cs[2 * j + (r >> 1)][r & 1];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        if ((lane & 15) == 0) atomicAdd(db + ncol + j * 16 + r, v);
      }
  }
}

// DIAG (timing diagnostics only, wrong results): 1 = no DMA / vmcnt in the K loop (MFMA + LDS
// reads + barriers), 2 = additionally no barriers (MFMA + LDS reads), 3 = DMA issued but never
// waited for in the K loop.  LAY: operand layouts (NtLay); 1 = TN weight gradients with
// blockIdx -> (split, tile).
template <int EPI, bool BGRAD, int DIAG = 0, int LAY = 0, bool BIASG = false>
__global__ void __launch_bounds__(NT_THREADS, 1) gemm_nt_kernel(NtArgs a) {
  using Ly = NtLay<LAY>;
  constexpr bool SPLIT = LAY == 1;
  __shared__ __attribute__((aligned(1024))) char lds[2 * NT_BUF];    // 128 KiB, the only LDS object
  const int tiles_n = a.N / NT_BN;
  const int tiles = (a.M / NT_BM) * tiles_n;
  // Staggered grid (NT / NN, a.stagger = H > 0): the first 2H blocks alternate a full tile and
  // the B0 column half of one of tiles H .. 2H-1, and H blocks at the end do their B1 halves.
  // The half tiles (about half the time of a full one) put half of the CUs of the first round
  // half a tile out of phase with the other half for the rest of the grid, so their epilogues
  // -- store- or VALU-bound with the matrix cores idle -- no longer all hit HBM at once; the
  // total work is unchanged.  Dispatch order only decides how well it staggers, never what
  // is computed.
  int v = blockIdx.x, half = 0;
  if constexpr (!SPLIT) {
    const int H = a.stagger;
    if (H > 0) {
      if (v < 2 * H) {
        half = v & 1;
        v = (v & 1) ? H + (v >> 1) : (v >> 1);
      } else if (v >= tiles) {
        half = 2;
        v = H + (v - tiles);
      }
    }
  }
  int L = xcd_remap(v, SPLIT ? gridDim.x : tiles);
  const int split = SPLIT ? L / tiles : 0;
  L -= split * tiles;
  // tile order of the blocks that share an XCD (consecutive L): a.group_m > 1 walks group_m
  // M-tiles for each N-tile (a group_m x (32 / group_m) block of tiles runs at once per XCD,
  // instead of 2 M-rows x every N-tile), so fewer distinct A / B panels stream into each XCD's
  // 4 MiB L2 per round
  int tm, tn;
  if (!SPLIT && a.group_m > 1) {
    const int gsz = a.group_m * tiles_n;
    const int g = L / gsz, r = L - g * gsz;
    tm = g * a.group_m + r % a.group_m;
    tn = r / a.group_m;
  } else {
    tm = L / tiles_n;
    tn = L % tiles_n;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: staging bases in SGPRs
  const int wr = wave >> 2, wc = wave & 3;
  const long m0 = (long)tm * NT_BM, n0 = (long)tn * NT_BN;
  // split-K (TN): the K / 64 K-tiles dealt out over the slices, so any slice count works (e.g.
  // 5 slices of the 512 K-tiles of a 32768-token weight gradient: 48 tiles x 5 = 240 workgroups,
  // one wave, a third of the fp32 slab traffic of 16 power-of-two slices)
  const int kt_all = a.K / NT_BK;
  const int kt_q = SPLIT ? kt_all / (int)a.tsplit : kt_all, kt_r = SPLIT ? kt_all % (int)a.tsplit : 0;
  const int nk = kt_q + (split < kt_r ? 1 : 0);
  const long kfirst = SPLIT ? (long)(split * kt_q + min(split, kt_r)) * NT_BK : 0L;
  NtCtx c{a.A, a.B, a.lda, a.ldb, m0, n0, kfirst, lds, wave, lane, wr * 64, wc * 32,
          0, 0, 0, 0, (BIASG && tn == 0) ? 2 * wc : -1, half};
  f32x4 accb[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  if constexpr (Ly::AT) {
    c.offa0 = c.offa1 = tn_lane_off(a.lda, wave, lane, true);
  } else {
    c.offa0 = nt_lane_off(a.lda, 0, lane);
    c.offa1 = nt_lane_off(a.lda, 1, lane);
  }
  if constexpr (Ly::BT) {
    c.offb0 = c.offb1 = tn_lane_off(a.ldb, wave, lane, false);
  } else {
    c.offb0 = nt_lane_off(a.ldb, 0, lane);
    c.offb1 = nt_lane_off(a.ldb, 1, lane);
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this lane's epilogue coordinates: rows m0 + wr*128 + 16i + (lane & 15), columns
  // n0 + wc*64 + 16j + 4(lane >> 4) + r
  const long emrow = m0 + wr * 128 + (lane & 15), encol = n0 + wc * 64 + (lane >> 4) * 4;
  NtEpiPre<4> epre;
  nt_preload_bias<EPI, 4>(a, encol, epre);

  nt_s16x8 fa[2][4][2];   // [qm][frag][ks]: A rows wr*128 + qm*64 + 16 frag
  nt_s16x8 fb[2][2][2];   // [qn][frag][ks]: B rows wc*64 + qn*32 + 16 frag

  // prologue: halves -6 .. -1 (all of K-tile 0, A0 + B0 of K-tile 1); wait for tile 0's A0, B0
#pragma unroll
  for (int v = -6; v < -2; ++v) nt_stage_v<LAY>(c, v);
  if (nk > 1) {
    nt_stage_v<LAY>(c, -2);
    nt_stage_v<LAY>(c, -1);
    nt_vm<8>();
  } else {
    nt_vm<4>();
  }
  nt_bar();
  if (wr == 1) nt_bar();                                 // group 1 runs one barrier behind

  // steady state: every phase issues one half and keeps 4 in flight; the last two K-tiles
  // drain (halves beyond 4 nk - 7 do not exist)
  int t = 0;
  for (; t < nk - 2; ++t) nt_ktile<0, DIAG, LAY, BIASG>(c, t, acc, fa, fb, accb);
  if (nk >= 2) {
    nt_ktile<1, DIAG, LAY, BIASG>(c, t, acc, fa, fb, accb);
    ++t;
  }
  nt_ktile<2, DIAG, LAY, BIASG>(c, t, acc, fa, fb, accb);
  if (wr == 0) nt_bar();                                 // equal barrier counts for both groups

  // acc[i][j][r] = D[m0 + wr*128 + 16i + (lane & 15)][n0 + wc*64 + 16j + 4(lane >> 4) + r]
  nt_epilogue<EPI, BGRAD, 4>(a, acc, emrow, encol, lane, split, epre, half);
  if constexpr (BIASG) {
    // accb[t] row block 2 wc + t: every column holds the row sum; lanes 0-15 hold rows 0-15
    if (c.biasw >= 0 && lane < 16) {
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2)
        a.biasg[(long)split * a.M + m0 + wr * 128 + 16 * (c.biasw + t2) + lane] = accb[t2][0];
    }
  }
}

// ---------------------------------------------------------------------------------------
// Streamed persistent variant (forward / data-gradient GEMMs, NT and NN layouts).
//
// One workgroup per CU walks several output tiles (w, w + P, w + 2P, ... in the XCD-remapped
// tile order), and its K-tiles form ONE continuous stream: the half-tile DMAs of the next
// output tile are issued by the last phases of the current one exactly as within a tile, so
// the next tile's operands land while this tile's epilogue stores run (the epilogue of one
// wave group also overlaps the other group's MFMA phase: the groups run one barrier apart).
// Nothing else changes: same phases, same LDS images and swizzles, same counted vmcnt waits
// (epilogue stores / bias loads are younger than the in-flight DMAs, so "all but the N youngest
// vector-memory ops" only ever waits for MORE than the pipeline needs).  The one-tile kernel
// pays a workgroup launch, a cold prologue (first DMA latency) and an idle epilogue per tile:
// at K = 1024 (16 K-tiles) that is a large share of the tile.
struct NtStream {
  int nk;            // K-tiles per output tile
  int total_k;       // K-tiles of this workgroup's whole stream
  int tiles_n, tiles, P, wg, my_tiles;
  __device__ __forceinline__ void tile_origin(int j, long& m0, long& n0) const {
    const int L = xcd_remap(j * P + wg, tiles);
    m0 = (long)(L / tiles_n) * NT_BM;
    n0 = (long)(L % tiles_n) * NT_BN;
  }
};

// K-tile cursor of the stream: output tile j of this workgroup, K-tile k inside it, with the
// tile's operand bases (recomputed only when the cursor crosses into the next tile) and the
// K offsets (A: k0 elements; B: k0 for NT, k0 * ldb for NN).  Wave-uniform: SGPRs.
struct NtKCur {
  int j, k;
  long ka, kb;
  const bf16_t* arow;   // A + m0 * lda
  const bf16_t* brow;   // NT: B + n0 * ldb; NN: B + n0
};

// per-wave staging offsets (elements) of the two pieces a wave stages per half, fixed for the
// whole kernel: A rows of piece i in A0 (A1: + 64 rows), B rows of piece i in B0 (B1: + 32)
struct NtSOff {
  long pa[2], pb[2];
  long a64, b32;
};

template <int LAY>
__device__ __forceinline__ void nt_kcur_set(const NtCtx& c, const NtStream& st, NtKCur& q, int j) {
  q.j = j;
  q.k = 0;
  q.ka = 0;
  q.kb = 0;
  if (j < st.my_tiles) {
    long m0, n0;
    st.tile_origin(j, m0, n0);
    q.arow = c.A + m0 * c.lda;
    q.brow = NtLay<LAY>::BT ? c.B + n0 : c.B + n0 * c.ldb;
  }
}

template <int LAY>
__device__ __forceinline__ void nt_kcur_next(const NtCtx& c, const NtStream& st, NtKCur& q) {
  if (++q.k == st.nk) {
    nt_kcur_set<LAY>(c, st, q, q.j + 1);
  } else {
    q.ka += NT_BK;
    q.kb += NtLay<LAY>::BT ? NT_BK * c.ldb : NT_BK;
  }
}

// stage half SLOT (0 A0, 1 B0, 2 B1, 3 A1) of the K-tile at cursor q into buffer buf
template <int LAY, int SLOT>
__device__ __forceinline__ void nt_stage_kt(const NtCtx& c, const NtSOff& so, const NtKCur& q, char* buf) {
  using Ly = NtLay<LAY>;
  static_assert(!Ly::AT, "streamed kernel: NT / NN layouts only");
  char* dst = buf + SLOT * NT_HALF;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = c.wave * 2 + i;
    const bf16_t* base;
    unsigned off;
    if constexpr (SLOT == 0 || SLOT == 3) {
      base = q.arow + so.pa[i] + (SLOT == 3 ? so.a64 : 0) + q.ka;
      off = i ? c.offa1 : c.offa0;
    } else {
      base = q.brow + so.pb[i] + (SLOT == 2 ? so.b32 : 0) + q.kb;
      off = Ly::BT ? c.offb0 : (i ? c.offb1 : c.offb0);
    }
    nt_glds16s(base, off, dst + piece * 1024);
  }
}

// one K-tile of the stream: phases 0 / 1 stage B1 / A1 of K-tile t + 1 (cursor q1), phases 2 / 3
// A0 / B0 of K-tile t + 2 (cursor q2) -- the one-tile kernel's half order (nt_stage_v), with
// every slot a compile-time constant
template <int POS, int LAY>
__device__ __forceinline__ void nt_ktile_stream(const NtCtx& c, const NtSOff& so, const NtKCur& q1,
                                                const NtKCur& q2, int t, f32x4 (&acc)[8][4],
                                                nt_s16x8 (&fa)[2][4][2], nt_s16x8 (&fb)[2][2][2]) {
  const char* buf = c.lds + (t & 1) * NT_BUF;
  char* nbuf = c.lds + ((t + 1) & 1) * NT_BUF;
  char* cbuf = c.lds + (t & 1) * NT_BUF;
  using P = NtPlan<POS>;
#define NT_SPHASE_TAIL(Q, I0, J0, FA, FB)                                                  \
  if constexpr (P::issue(Q)) {                                                             \
    if constexpr (Q == 0) nt_stage_kt<LAY, 2>(c, so, q1, nbuf);                            \
    else if constexpr (Q == 1) nt_stage_kt<LAY, 3>(c, so, q1, nbuf);                       \
    else if constexpr (Q == 2) nt_stage_kt<LAY, 0>(c, so, q2, cbuf);                       \
    else nt_stage_kt<LAY, 1>(c, so, q2, cbuf);                                             \
  }                                                                                        \
  nt_vm<P::wait(Q)>();                                                                     \
  nt_mma_begin();                                                                          \
  nt_quad<I0, J0>(acc, FA, FB);                                                            \
  nt_mma_end();
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) fb[0][j][ks] = nt_fragment<NtLay<LAY>::BT>(buf + 1 * NT_HALF, c.rb + j * 16, ks, c.lane);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) fa[0][i][ks] = nt_fragment<false>(buf + 0 * NT_HALF, c.ra + i * 16, ks, c.lane);
  NT_SPHASE_TAIL(0, 0, 0, fa[0], fb[0])
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) fb[1][j][ks] = nt_fragment<NtLay<LAY>::BT>(buf + 2 * NT_HALF, c.rb + j * 16, ks, c.lane);
  NT_SPHASE_TAIL(1, 0, 2, fa[0], fb[1])
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) fa[1][i][ks] = nt_fragment<false>(buf + 3 * NT_HALF, c.ra + i * 16, ks, c.lane);
  NT_SPHASE_TAIL(2, 4, 2, fa[1], fb[1])
  NT_SPHASE_TAIL(3, 4, 0, fa[1], fb[0])
#undef NT_SPHASE_TAIL
}

template <int EPI, int LAY>
__global__ void __launch_bounds__(NT_THREADS, 1) gemm_nt_stream_kernel(NtArgs a, int P) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * NT_BUF];    // 128 KiB, the only LDS object
  const int tiles_n = a.N / NT_BN;
  const int tiles = (a.M / NT_BM) * tiles_n;
  const int wg = blockIdx.x;
  const int my_tiles = wg < tiles ? (tiles - wg + P - 1) / P : 0;
  const int nk = a.K / NT_BK;
  NtStream st{nk, my_tiles * nk, tiles_n, tiles, P, wg, my_tiles};
  if (my_tiles == 0) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  NtCtx c{a.A, a.B, a.lda, a.ldb, 0, 0, 0, lds, wave, lane, wr * 64, wc * 32, 0, 0, 0, 0, -1, 0};
  c.offa0 = nt_lane_off(a.lda, 0, lane);
  c.offa1 = nt_lane_off(a.lda, 1, lane);
  if constexpr (NtLay<LAY>::BT) {
    c.offb0 = c.offb1 = tn_lane_off(a.ldb, wave, lane, false);
  } else {
    c.offb0 = nt_lane_off(a.ldb, 0, lane);
    c.offb1 = nt_lane_off(a.ldb, 1, lane);
  }
  NtSOff so;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = wave * 2 + i;
    so.pa[i] = (long)(((piece >> 3) << 7) + (piece & 7) * 8) * a.lda;
    so.pb[i] = NtLay<LAY>::BT ? (long)piece * 4 * a.ldb : (long)(((piece >> 2) << 6) + (piece & 3) * 8) * a.ldb;
  }
  so.a64 = 64 * a.lda;
  so.b32 = NtLay<LAY>::BT ? 32 : 32 * a.ldb;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  long m0, n0;                          // origin of the tile being multiplied
  st.tile_origin(0, m0, n0);
  NtEpiPre<4> epre;
  nt_preload_bias<EPI, 4>(a, n0 + wc * 64 + (lane >> 4) * 4, epre);
  nt_s16x8 fa[2][4][2];
  nt_s16x8 fb[2][2][2];

  // prologue: all of K-tile 0 and A0 + B0 of K-tile 1 (the one-tile kernel's halves -6 .. -1)
  NtKCur q1, q2;
  nt_kcur_set<LAY>(c, st, q1, 0);
  nt_stage_kt<LAY, 0>(c, so, q1, lds);
  nt_stage_kt<LAY, 1>(c, so, q1, lds);
  nt_stage_kt<LAY, 2>(c, so, q1, lds);
  nt_stage_kt<LAY, 3>(c, so, q1, lds);
  nt_kcur_next<LAY>(c, st, q1);                          // K-tile 1
  if (st.total_k > 1) {
    nt_stage_kt<LAY, 0>(c, so, q1, lds + NT_BUF);
    nt_stage_kt<LAY, 1>(c, so, q1, lds + NT_BUF);
    nt_vm<8>();
  } else {
    nt_vm<4>();
  }
  q2 = q1;
  nt_kcur_next<LAY>(c, st, q2);                          // K-tile 2
  nt_bar();
  if (wr == 1) nt_bar();                                 // group 1 runs one barrier behind

  // after each K-tile: when an output tile is complete, store it (the next tile's DMAs are
  // already in flight), clear the accumulators and load the next tile's bias
  int jt = 0, kin = 0;
  auto finish_k = [&]() {
    q1 = q2;
    nt_kcur_next<LAY>(c, st, q2);
    if (++kin != nk) return;
    const long emrow = m0 + wr * 128 + (lane & 15), encol = n0 + wc * 64 + (lane >> 4) * 4;
    nt_epilogue<EPI, false, 4>(a, acc, emrow, encol, lane, 0, epre);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    kin = 0;
    if (++jt < my_tiles) {
      st.tile_origin(jt, m0, n0);
      nt_preload_bias<EPI, 4>(a, n0 + wc * 64 + (lane >> 4) * 4, epre);
    }
  };
  // steady state, then the two draining K-tiles of the whole stream (one ktile variant per
  // loop: branching between variants inside one loop body spills the fragment registers)
  const int T = st.total_k;
  int t = 0;
  for (; t < T - 2; ++t) {
    nt_ktile_stream<0, LAY>(c, so, q1, q2, t, acc, fa, fb);
    finish_k();
  }
  if (T >= 2) {
    nt_ktile_stream<1, LAY>(c, so, q1, q2, t, acc, fa, fb);
    finish_k();
    ++t;
  }
  nt_ktile_stream<2, LAY>(c, so, q1, q2, t, acc, fa, fb);
  finish_k();
  if (wr == 0) nt_bar();                                 // equal barrier counts for both groups
}


// nt_glds16s plus the wait states between v_readfirstlane and a VMEM instruction reading its SGPR
// (s_nop 4, cdna_hip_programming.md §5.7 item 2): in the four-wave kernel hipcc keeps the staging
// bases in VGPRs under SGPR pressure and re-reads them right before each DMA
__device__ __forceinline__ void w4_glds16s(const void* sbase, unsigned voff, const char* lds_wave_base) {
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(nt_lds_void*)lds_wave_base);
  const uint64_t sb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)sbase) |
                      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)sbase >> 32)) << 32);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 4\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sb), "s"(la)
               : "memory", "m0");
}


// ---------------------------------------------------------------------------------------
// Four-wave variant (gemm_w4_kernel): the same 256 x 256 x 64 tile, LDS images, swizzles and
// epilogues, but 4 waves of 128 x 128 each instead of 8 of 128 x 64.  Per K-tile a wave reads
// 32 fragments for 128 MFMAs (0.25 per MFMA) where the 8-wave kernel reads 24 for 64 (0.375):
// a third less LDS read traffic beside the LDS-DMA writes (profiles/r2/gemm_nt.md: the DMA
// issue, not the schedule, is what costs the 8-wave kernel).  The 64 accumulator quads fill
// all 256 AGPRs; through the builtin the register allocator rotated them through v_accvgpr
// moves (92 per 128 MFMAs, r6 probe), so the MFMAs are inline asm with the accumulator bound
// "+a": it stays in one AGPR quad for the whole kernel, dst == srcC.  One wave per SIMD, so
// the wave interleaves its own fragment reads and DMA issue between MFMAs:
//   K-tile t = two 32-deep k-steps; k-step 0 multiplies fragment set 0 while reading set 1
//   (k-step 1 of the same LDS slot); then lgkmcnt(0) + vmcnt(0) + one barrier (stage t + 1 has
//   landed, every wave is done reading slot t & 1); k-step 1 multiplies set 1 while issuing
//   the DMA of stage t + 2 into slot t & 1 (front-loaded, one per MFMA) and reading set 0 of
//   K-tile t + 1.  Two 64 KiB slots, one barrier per K-tile.
// Hazards the compiler cannot see through the asm: the epilogue's AGPR reads wait out the last
// MFMA (3 x s_nop 7 between sched_barriers), and the first k-step writes the accumulators with
// srcC = 0 (a zeroing pass of v_accvgpr_write placed by the compiler next to the first MFMAs
// broke the bias epilogues: profiles/r6/gemm_w4_four_wave.md).
template <bool FIRST>
__device__ __forceinline__ void w4_mfma(f32x4& c, const nt_s16x8& b, const nt_s16x8& a) {
  if constexpr (FIRST)      // srcC = 0: the first k-step writes the accumulator (no zeroing pass)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(b), "v"(a));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
}

struct W4Frags {
  nt_s16x8 a[8], b[8];
};

template <int DIAG, bool RD, bool DMA, bool FIRST = false>
__device__ __forceinline__ void w4_kstep(f32x4 (&acc)[8][8], const W4Frags& cur, W4Frags& nxt, const char* rimg,
                                         int ks, int wm, int wn, int lane, char* dimg,
                                         const bf16_t* abase, const bf16_t* bbase, long lda, long ldb, long k0,
                                         unsigned oa0, unsigned oa1, unsigned ob0, unsigned ob1, int wave) {
  // 64 MFMAs in (i, j) order; DMA pieces after the first 16 (A pieces 0-7, B pieces 0-7), one
  // fragment read after every third of the remaining 48
#pragma unroll
  for (int q = 0; q < 64; ++q) {
    const int i = q >> 3, j = q & 7;
    w4_mfma<FIRST>(acc[i][j], cur.b[j], cur.a[i]);
    if constexpr (DIAG != 1 && DMA) {
      if (q < 16) {
        const int pc = q & 7;
        if (q < 8) w4_glds16s(abase + 8 * pc * lda + k0, (pc & 1) ? oa1 : oa0, dimg + (8 * wave + pc) * 1024);
        else w4_glds16s(bbase + 8 * pc * ldb + k0, (pc & 1) ? ob1 : ob0, dimg + 32768 + (8 * wave + pc) * 1024);
      }
    }
    if (RD && q >= 16 && (q - 16) % 3 == 0 && (q - 16) / 3 < 16) {
      // nt_frag with the row-block stride folded into immediates: the swizzle of row
      // 128 w + 16 f + (lane & 15) does not depend on f
      const int f = (q - 16) / 3;
      const int lo = ((ks * 4 + (lane >> 4)) ^ (((lane & 15) >> 1) & 7)) << 4;
      if (f < 8) nxt.a[f] = *(const nt_lds_s16x8*)(rimg + (wm * 128 + (lane & 15)) * NT_ROWB + lo + f * 16 * NT_ROWB);
      else nxt.b[f - 8] = *(const nt_lds_s16x8*)(rimg + 32768 + (wn * 128 + (lane & 15)) * NT_ROWB + lo +
                                                 (f - 8) * 16 * NT_ROWB);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// DIAG (timing only, wrong results): 1 = no DMA in the K loop, 2 = DMA issued, never waited for
template <int EPI, bool BGRAD, int DIAG = 0>
__global__ void __launch_bounds__(256, 1) gemm_w4_kernel(NtArgs a) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * NT_BUF];    // 2 slots x (A 32 KiB | B 32 KiB)
  const int tiles_n = a.N / NT_BN;
  const int tiles = (a.M / NT_BM) * tiles_n;
  const int L = xcd_remap(blockIdx.x, tiles);
  int tm, tn;
  if (a.group_m > 1) {
    const int gsz = a.group_m * tiles_n;
    const int g = L / gsz, r = L - g * gsz;
    tm = g * a.group_m + r % a.group_m;
    tn = r / a.group_m;
  } else {
    tm = L / tiles_n;
    tn = L % tiles_n;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const long m0 = (long)tm * NT_BM, n0 = (long)tn * NT_BN;
  const int nk = a.K / NT_BK;
  // staging: wave w fills image rows 64 w .. 64 w + 63 of both operands (8 pieces of 8 rows)
  const bf16_t* abase = a.A + (m0 + 64 * wave) * a.lda;
  const bf16_t* bbase = a.B + (n0 + 64 * wave) * a.ldb;
  const unsigned oa0 = nt_lane_off(a.lda, 0, lane), oa1 = nt_lane_off(a.lda, 1, lane);
  const unsigned ob0 = nt_lane_off(a.ldb, 0, lane), ob1 = nt_lane_off(a.ldb, 1, lane);
  auto stage = [&](int kt) {
    char* img = lds + (kt & 1) * NT_BUF;
    const long k0 = (long)kt * NT_BK;
#pragma unroll
    for (int pc = 0; pc < 8; ++pc)
      w4_glds16s(abase + 8 * pc * a.lda + k0, (pc & 1) ? oa1 : oa0, img + (8 * wave + pc) * 1024);
#pragma unroll
    for (int pc = 0; pc < 8; ++pc)
      w4_glds16s(bbase + 8 * pc * a.ldb + k0, (pc & 1) ? ob1 : ob0, img + 32768 + (8 * wave + pc) * 1024);
  };

  f32x4 acc[8][8];                                   // first written by the srcC = 0 k-step
  const long emrow = m0 + wm * 128 + (lane & 15), encol = n0 + wn * 128 + (lane >> 4) * 4;
  NtEpiPre<8> epre;
  nt_preload_bias<EPI, 8>(a, encol, epre);

  W4Frags s0, s1;
  stage(0);
  if (nk > 1) stage(1);
  if (nk > 1) nt_vm<16>(); else nt_vm<0>();
  nt_bar();
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    s0.a[f] = nt_frag(lds, wm * 128 + 16 * f, 0, lane);
    s0.b[f] = nt_frag(lds + 32768, wn * 128 + 16 * f, 0, lane);
  }
  // K-tile t: k-step 0 (set 0, reading set 1 from the same slot), the mid-tile wait + barrier,
  // k-step 1 (set 1, DMA of stage t + 2, reading set 0 of K-tile t + 1).  The first K-tile
  // starts the accumulators (srcC = 0), then the steady state, then the last two K-tiles
  // without the DMA / the next-tile reads.
#define W4_TILE(FIRST0, RD1, DMA1, WAITV)                                                          \
  do {                                                                                               \
    const char* img = lds + (t & 1) * NT_BUF;                                                        \
    w4_kstep<DIAG, true, false, FIRST0>(acc, s0, s1, img, 1, wm, wn, lane, nullptr, abase, bbase,    \
                                        a.lda, a.ldb, 0, oa0, oa1, ob0, ob1, wave);                  \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                               \
    if constexpr (DIAG == 0 && WAITV) nt_vm<0>();                                                    \
    nt_bar();                                                                                        \
    w4_kstep<DIAG, RD1, DMA1>(acc, s1, s0, lds + ((t + 1) & 1) * NT_BUF, 0, wm, wn, lane,            \
                              lds + (t & 1) * NT_BUF, abase, bbase, a.lda, a.ldb, (long)(t + 2) * NT_BK, \
                              oa0, oa1, ob0, ob1, wave);                                             \
  } while (0)
  int t = 0;
  if (nk == 1) {
    W4_TILE(true, false, false, false);
  } else {
    if (nk == 2) W4_TILE(true, true, false, true);
    else W4_TILE(true, true, true, true);
    for (t = 1; t < nk - 2; ++t) W4_TILE(false, true, true, true);
    if (nk >= 3) {
      W4_TILE(false, true, false, true);
      ++t;
    }
    W4_TILE(false, false, false, false);
  }
#undef W4_TILE
  // the last MFMAs -> the epilogue's AGPR reads: the scheduler may not move the reads above
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  nt_epilogue<EPI, BGRAD, 8, false>(a, acc, emrow, encol, lane, 0, epre);
}

}  // namespace ct

using namespace ct;

static int nt_cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    return v;
  }();
  return n;
}

// Streamed persistent GEMM: D[M,N] (+)= A[M,K] . B^T (b_kn = 0: B [N,K]; 1: B [K,N]) with
// epilogue 0 (plain; accumulate: D += result) or 5 (+ bias[N]).  One workgroup per CU (or fewer when
// there are fewer tiles).  Nonzero (nothing launched) when unsupported.
extern "C" int ct_gemm_nt_stream(const void* A, long lda, const void* B, long ldb, void* D, long ldd, int M, int N,
                                 int K, int epi, const void* bias, int b_kn, int wgs, int accumulate,
                                 hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % NT_BM || N % NT_BN || K % NT_BK) return 1;
  if (lda % 8 || ldb % 8 || ldd % 8 || lda < K || ldb < (b_kn ? N : K) || ldd < N) return 2;
  if (((uintptr_t)A & 15) || ((uintptr_t)B & 15) || ((uintptr_t)D & 15)) return 3;
  if (epi != 0 && epi != 5) return 6;
  if (epi == 5 && (!bias || ((uintptr_t)bias & 7))) return 4;
  const long tiles = (long)(M / NT_BM) * (N / NT_BN);
  if (tiles > (1L << 30)) return 5;
  const int P = (int)std::min<long>(tiles, wgs > 0 ? wgs : nt_cu_count());
  if (accumulate && epi != 0) return 6;
  NtArgs a{(const bf16_t*)A, (const bf16_t*)B, (bf16_t*)D, (const bf16_t*)bias, nullptr, nullptr, nullptr,
           nullptr, lda, ldb, ldd, 0, 0, M, N, K, accumulate ? 1 : 0};
  if (epi == 5) {
    if (b_kn) gemm_nt_stream_kernel<NT_EPI_BIAS, 2><<<P, NT_THREADS, 0, stream>>>(a, P);
    else gemm_nt_stream_kernel<NT_EPI_BIAS, 0><<<P, NT_THREADS, 0, stream>>>(a, P);
  } else {
    if (b_kn) gemm_nt_stream_kernel<NT_EPI_PLAIN, 2><<<P, NT_THREADS, 0, stream>>>(a, P);
    else gemm_nt_stream_kernel<NT_EPI_PLAIN, 0><<<P, NT_THREADS, 0, stream>>>(a, P);
  }
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

// D[M,N] = A[M,K] . B[N,K]^T (row-major, K-contiguous operands) with epilogue `epi`:
//   0: plain (accumulate: D += result); 1: aux = result + bias, D = gelu(aux);
//   2: D = result * gelu'(aux [+ bias]), dbias += column sums (bias, dbias may be null);
//   6: D = gelu(result + bias), aux = gelu'(result + bias);
//   7: D = result * aux, dbias += column sums (dbias may be null).
// Returns nonzero (and launches nothing) when the shape / alignment is not supported.
extern "C" int ct_gemm_nt(const void* A, long lda, const void* B, long ldb, void* D, long ldd, int M, int N, int K,
                          int epi, int accumulate, const void* bias, void* aux, long ldaux, float* dbias, int b_kn,
                          hipStream_t stream, int dbias_rows) {
  if (dbias_rows < 1 || (dbias_rows & (dbias_rows - 1))) return 6;
  if (M <= 0 || N <= 0 || K <= 0 || M % NT_BM || N % NT_BN || K % NT_BK) return 1;
  if (lda % 8 || ldb % 8 || ldd % 8 || lda < K || ldb < (b_kn ? N : K) || ldd < N) return 2;
  if (((uintptr_t)A & 15) || ((uintptr_t)B & 15) || ((uintptr_t)D & 15)) return 3;
  if ((epi == 1 || epi == 6) && (!bias || !aux || ((uintptr_t)bias & 7))) return 4;
  if (epi == 5 && (!bias || ((uintptr_t)bias & 7))) return 4;
  if ((epi == 1 || epi == 2 || epi == 6 || epi == 7) && (!aux || ((uintptr_t)aux & 15) || ldaux % 8 || ldaux < N))
    return 4;
  if (bias && ((uintptr_t)bias & 7)) return 4;
  const long tiles = (long)(M / NT_BM) * (N / NT_BN);
  if (tiles > (1L << 30)) return 5;
  // stagger half of the first round's CUs by half a tile when the grid has >= 2 rounds
  // (CLOUDTIK_AMD_GEMM_STAGGER: -1 auto, 0 off (default), H > 0 forces H half-tile pairs).
  // Off by default: BERT-large 73.06 / 72.96 ms/step without it, 77.23 / 77.25 with the auto
  // stagger (same box, interleaved; profiles/r5/SUMMARY.md) -- the half tiles stage every
  // operand and keep every barrier, so they cost nearly a full tile, and the grid grows by H.
  static const int stag_env = [] { const char* e = getenv("CLOUDTIK_AMD_GEMM_STAGGER"); return e ? atoi(e) : 0; }();
  int H = 0;
  if (stag_env > 0) H = (int)std::min<long>(stag_env, tiles / 2);
  else if (stag_env < 0 && tiles >= 2L * nt_cu_count()) H = nt_cu_count() / 2;
  const long blocks = tiles + H;
  // CLOUDTIK_AMD_GEMM_GROUP_M: M-tiles per N-tile in the tile order (must divide M / 256).
  // Default 4: BERT-large 72.68 -> 72.43 ms/step (2 interleaved rounds, one box; 8: 73.08;
  // profiles/r5/SUMMARY.md)
  static const int gm_env = [] { const char* e = getenv("CLOUDTIK_AMD_GEMM_GROUP_M"); return e ? atoi(e) : 4; }();
  const int gm = (gm_env > 1 && (M / NT_BM) % gm_env == 0) ? gm_env : 1;
  NtArgs a{(const bf16_t*)A, (const bf16_t*)B, (bf16_t*)D, (const bf16_t*)bias, (bf16_t*)aux, dbias, nullptr,
           nullptr, lda, ldb, ldd, ldaux, 0, M, N, K, accumulate, H, gm, dbias_rows};
  static const int diag = [] { const char* e = getenv("CLOUDTIK_AMD_GEMM_DIAG"); return e ? atoi(e) : 0; }();
  if (diag == 4) {
    if (b_kn) gemm_nt_kernel<NT_EPI_NONE, false, 0, 2><<<(int)blocks, NT_THREADS, 0, stream>>>(a);
    else gemm_nt_kernel<NT_EPI_NONE, false, 0, 0><<<(int)blocks, NT_THREADS, 0, stream>>>(a);
    return 0;
  }
  if (diag && !b_kn) {
    if (diag == 1) gemm_nt_kernel<0, false, 1><<<(int)blocks, NT_THREADS, 0, stream>>>(a);
    else if (diag == 2) gemm_nt_kernel<0, false, 2><<<(int)blocks, NT_THREADS, 0, stream>>>(a);
    else gemm_nt_kernel<0, false, 3><<<(int)blocks, NT_THREADS, 0, stream>>>(a);
    return 0;
  }
#define NT_LAUNCH(E, BG)                                                                  \
  do {                                                                                    \
    if (b_kn) gemm_nt_kernel<E, BG, 0, 2><<<(int)blocks, NT_THREADS, 0, stream>>>(a);     \
    else gemm_nt_kernel<E, BG, 0, 0><<<(int)blocks, NT_THREADS, 0, stream>>>(a);          \
  } while (0)
  switch (epi) {
    case 0: NT_LAUNCH(0, false); break;
    case 1: NT_LAUNCH(1, false); break;
    case 2:
      if (dbias) NT_LAUNCH(2, true);
      else NT_LAUNCH(2, false);
      break;
    case 5: NT_LAUNCH(5, false); break;
    case 6: NT_LAUNCH(6, false); break;
    case 7:
      if (dbias) NT_LAUNCH(7, true);
      else NT_LAUNCH(7, false);
      break;
    default: return 6;
  }
#undef NT_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

// Weight-gradient layout: D[M,N] = A[K,M]^T . B[K,N] (row-major, K = tokens; lda >= M, ldb >= N;
// K % 64 == 0, any 1 <= splits <= K / 64).
// splits > 1: fp32 partial slabs P[splits][M][N] (reduced by ct_splitk_reduce*); splits == 1:
// bf16 out (+)= result (accumulate), row stride ldo.  biasg (optional, fp32 [splits][M]): the
// column sums of A per split (the bias gradient when A is dY).  Nonzero (nothing launched)
// when the shape / alignment is unsupported.
extern "C" int ct_gemm_tn2(const void* A, long lda, const void* B, long ldb, void* out, long ldo, int M, int N,
                           long K, int splits, int accumulate, float* biasg, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || splits < 1 || M % NT_BM || N % NT_BN) return 1;
  if (K % NT_BK || K / NT_BK < splits || K > (1L << 30)) return 2;
  if (lda % 8 || ldb % 8 || lda < M || ldb < N || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return 3;
  if (((uintptr_t)out & 15) || (splits == 1 && (ldo % 8 || ldo < N))) return 4;
  const long blocks = (long)(M / NT_BM) * (N / NT_BN) * splits;
  if (blocks > (1L << 30)) return 5;
  NtArgs a{(const bf16_t*)A, (const bf16_t*)B, splits == 1 ? (bf16_t*)out : nullptr, nullptr, nullptr, nullptr,
           splits > 1 ? (float*)out : nullptr, biasg, lda, ldb, ldo, 0, (long)splits, M, N, (int)K,
           accumulate};
  static const int diag = [] { const char* e = getenv("CLOUDTIK_AMD_GEMM_DIAG"); return e ? atoi(e) : 0; }();
  if (diag == 4) {
    gemm_nt_kernel<NT_EPI_NONE, false, 0, 1><<<(int)blocks, NT_THREADS, 0, stream>>>(a);
    return 0;
  }
  if (biasg) {
    if (splits > 1) gemm_nt_kernel<NT_EPI_F32_SLAB, false, 0, 1, true><<<(int)blocks, NT_THREADS, 0, stream>>>(a);
    else gemm_nt_kernel<NT_EPI_PLAIN, false, 0, 1, true><<<(int)blocks, NT_THREADS, 0, stream>>>(a);
  } else {
    if (splits > 1) gemm_nt_kernel<NT_EPI_F32_SLAB, false, 0, 1><<<(int)blocks, NT_THREADS, 0, stream>>>(a);
    else gemm_nt_kernel<NT_EPI_PLAIN, false, 0, 1><<<(int)blocks, NT_THREADS, 0, stream>>>(a);
  }
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

// Four-wave GEMM (gemm_w4_kernel): D[M,N] = A[M,K] . B[N,K]^T with epilogue 0 (plain; accumulate:
// D += result), 5 (+ bias) or 6 (D = gelu(. + bias), aux = gelu'(. + bias)).  Nonzero (nothing
// launched) when unsupported.  CLOUDTIK_AMD_GEMM_W4_DIAG=1 / 2: timing diagnostics (no DMA / DMA
// never waited for; wrong results).  Measured slower than gemm_nt_kernel: profiles/r6/gemm_w4_four_wave.md.
extern "C" int ct_gemm_w4(const void* A, long lda, const void* B, long ldb, void* D, long ldd, int M, int N, int K,
                          int epi, int accumulate, const void* bias, void* aux, long ldaux, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % NT_BM || N % NT_BN || K % NT_BK) return 1;
  if (lda % 8 || ldb % 8 || ldd % 8 || lda < K || ldb < K || ldd < N) return 2;
  if (((uintptr_t)A & 15) || ((uintptr_t)B & 15) || ((uintptr_t)D & 15)) return 3;
  if ((epi == 5 || epi == 6) && (!bias || ((uintptr_t)bias & 7))) return 4;
  if (epi == 6 && (!aux || ((uintptr_t)aux & 15) || ldaux % 8 || ldaux < N)) return 4;
  if (epi != 0 && epi != 5 && epi != 6) return 6;
  if (accumulate) return 6;                           // (the accumulating epilogue is not instantiated)
  const long tiles = (long)(M / NT_BM) * (N / NT_BN);
  if (tiles > (1L << 30)) return 5;
  static const int gm_env = [] { const char* e = getenv("CLOUDTIK_AMD_GEMM_GROUP_M"); return e ? atoi(e) : 4; }();
  const int gm = (gm_env > 1 && (M / NT_BM) % gm_env == 0) ? gm_env : 1;
  NtArgs a{(const bf16_t*)A, (const bf16_t*)B, (bf16_t*)D, (const bf16_t*)bias, (bf16_t*)aux, nullptr, nullptr,
           nullptr, lda, ldb, ldd, ldaux, 0, M, N, K, 0, 0, gm, 1};
  static const int diag = [] { const char* e = getenv("CLOUDTIK_AMD_GEMM_W4_DIAG"); return e ? atoi(e) : 0; }();
  if (diag == 1 || diag == 2) {
    if (diag == 1) gemm_w4_kernel<0, false, 1><<<(int)tiles, 256, 0, stream>>>(a);
    else gemm_w4_kernel<0, false, 2><<<(int)tiles, 256, 0, stream>>>(a);
    return 0;
  }
  if (epi == 5) gemm_w4_kernel<NT_EPI_BIAS, false><<<(int)tiles, 256, 0, stream>>>(a);
  else if (epi == 6) gemm_w4_kernel<NT_EPI_BIAS_GELU_DAUX, false><<<(int)tiles, 256, 0, stream>>>(a);
  else gemm_w4_kernel<NT_EPI_PLAIN, false><<<(int)tiles, 256, 0, stream>>>(a);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}
