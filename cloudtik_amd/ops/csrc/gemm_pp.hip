// "Paired-tile" persistent GEMM for gfx950: D[M, N] = A[M, K] . B[N, K]^T (bf16 in, fp32
// accumulate), built so the epilogue of one output tile runs WHILE the matrix cores work on
// another tile of the same CU.
//
// Why (profiles/r6/gemm_ffn1_pmc.md): the one-tile 256 x 256 kernel (gemm_nt.hip) keeps the
// matrix cores ~52 % busy on the BERT-large FFN1 shape.  Per output tile ~10 k cycles go to a
// plain epilogue (and ~25 k to the bias + GELU + gelu' one) with every wave of the CU storing
// and no MFMA issued, because both wave groups of the 8-wave workgroup share one tile and
// finish it together.
//
// Structure (one 512-thread workgroup per CU, 144 KiB LDS):
//   * the two wave GROUPS (waves 0-3, 4-7) own DIFFERENT 128 x 256 output tiles (each wave a
//     128 x 64 slice: the same 128 accumulator registers per lane as gemm_nt), each group with
//     its own 3-slot LDS ring of 32-deep K stages (A 128 x 32 + B 256 x 32 = 24 KiB a slot);
//   * time runs in SLOTS separated by one workgroup barrier; a group alternates a READ slot
//     (ds_read_b128 of the 12 operand fragments of one stage + LDS-DMA issue of the stage two
//     ahead) and an MFMA slot (32 MFMA 16x16x32 on those fragments); the groups are one slot
//     apart, so in every slot one wave per SIMD is in its MFMA slot: 32 MFMAs per barrier (the
//     gemm_nt phases carry 16);
//   * when a group finishes a tile it spends E slots on the epilogue (a share of the row blocks
//     per slot) while the other group keeps alternating -- half of those slots still carry an
//     MFMA phase -- and its next tile's first two stages are already in flight (the K stream
//     of a group is continuous across its tiles);
//   * staging: global_load_lds_dwordx4 pieces of 16 rows x 64 B; the 16-byte chunk c of image
//     row r sits at c ^ g((r >> 2) & 3), g = {0, 2, 3, 1}: the four 16-lane groups of every
//     fragment read then hit 16 distinct 16-B bank slots (conflict-free), the swizzle applied
//     on the per-lane SOURCE address (the LDS side of the DMA is lane-linear);
//   * counted vmcnt waits only (the epilogue's stores are counted in), raw s_barrier, the
//     XCD-aware tile order: the 64 group-tiles one XCD runs at a time form an 8 x 8 block of
//     (M, N) tiles, sharing A and B panels in that XCD's L2.
// Price: B panels are not shared between the two groups (1.5x the L2 -> LDS traffic of the
// one-tile kernel's shared 256 x 256 tile): ~25 TB/s chip-wide at full MFMA rate, inside L2's.
// Reference: the BERT encoder projections (HF BertLayer linears, run_pretrain_mlperf.py:449-471).
#include "common.h"
#include <algorithm>
#include <cstdlib>

namespace ct {

typedef __attribute__((ext_vector_type(8))) short pp_s16x8;
typedef __attribute__((address_space(3))) pp_s16x8 pp_lds_s16x8;
typedef __attribute__((address_space(3))) void pp_lds_void;

constexpr int PP_TM = 128, PP_TN = 256, PP_BK = 32, PP_THREADS = 512, PP_NS = 3;
constexpr int PP_ROWB = PP_BK * 2;               // 64 B per image row
constexpr int PP_AIMG = PP_TM * PP_ROWB;         // 8 KiB
constexpr int PP_BIMG = PP_TN * PP_ROWB;         // 16 KiB
constexpr int PP_STAGE = PP_AIMG + PP_BIMG;      // 24 KiB
constexpr int PP_GROUP = PP_NS * PP_STAGE;       // 72 KiB per wave group
constexpr int PP_DMA = 6;                        // LDS-DMA pieces per wave per stage
constexpr int PP_GM = 8;                         // M-tiles per N-tile walk in the tile order

enum { PP_EPI_PLAIN = 0, PP_EPI_BIAS = 5, PP_EPI_BIAS_GELU_DAUX = 6 };

struct PpArgs {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* D;
  const bf16_t* bias;   // EPI 5 / 6: [N]
  bf16_t* aux;          // EPI 6: gelu'(A B^T + bias) out
  long lda, ldb, ldd, ldaux;
  int M, N, K;
  int tiles_m, tiles_n, T;   // 128 x 256 tiles
  int V;                      // virtual CTAs = 2 x workgroups
};

// chunk swizzle g((r >> 2) & 3) for g = {0, 2, 3, 1}
__device__ __forceinline__ int pp_g(int x) { return (0x78 >> (2 * x)) & 3; }

__device__ __forceinline__ pp_s16x8 pp_frag(const char* img, int r0, int lane) {
  const int row = r0 + (lane & 15);
  const int c = lane >> 4;
  return *(const pp_lds_s16x8*)(img + row * PP_ROWB + ((c ^ pp_g((row >> 2) & 3)) << 4));
}

__device__ __forceinline__ void pp_glds16(const void* sbase, unsigned voff, const char* lds_wave_base) {
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(pp_lds_void*)lds_wave_base);
  const uint64_t sb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)sbase) |
                      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)sbase >> 32)) << 32);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sb), "s"(la)
               : "memory", "m0");
}

// 8-byte load the compiler does not track (its result is consumed only after the hand-counted
// vmcnt waits of the K loop have retired it: a compiler-visible load beside the LDS-DMA stream
// would make hipcc wait vmcnt(0) at its first use, draining the DMA ring)
__device__ __forceinline__ uint2 pp_ld8(const void* p) {
  uint2 v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

__device__ __forceinline__ void pp_bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void pp_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// tile t of the group-tile order -> (row, column) origin: PP_GM M-tiles for each N-tile
__device__ __forceinline__ void pp_tile(const PpArgs& a, int t, long& m0, long& n0) {
  const int gsz = PP_GM * a.tiles_n;
  const int gb = t / gsz, r = t - gb * gsz;
  const int rows_here = min(PP_GM, a.tiles_m - gb * PP_GM);
  const int tm = gb * PP_GM + r % rows_here, tn = r / rows_here;
  m0 = (long)tm * PP_TM;
  n0 = (long)tn * PP_TN;
}

// the j-th tile of virtual CTA (xcd, q, g): workgroup wg = xcd + 8 q runs on XCD `xcd` (blocks
// are dealt round-robin over the 8 XCDs), so step j of all of them on one XCD covers one
// contiguous block of V / 8 tiles of the order
__device__ __forceinline__ int pp_tile_index(const PpArgs& a, int wg, int g, int j) {
  const int xcd = wg & 7, q = wg >> 3;
  return j * a.V + xcd * (a.V >> 3) + 2 * q + g;
}

struct PpStream {
  // the group's tile sequence and the K stage cursor of its DMA stream
  int wg, g, j_tiles, S;   // S = stages per tile
  const bf16_t* arow;      // A + m0 * lda of the tile being staged
  const bf16_t* brow;      // B + n0 * ldb
  int dj, dk;              // DMA cursor: tile index in the sequence, stage in the tile
};

__device__ __forceinline__ void pp_cursor_tile(const PpArgs& a, PpStream& s) {
  if (s.dj < s.j_tiles) {
    long m0, n0;
    pp_tile(a, pp_tile_index(a, s.wg, s.g, s.dj), m0, n0);
    s.arow = a.A + m0 * a.lda;
    s.brow = a.B + n0 * a.ldb;
  }
}

// piece q (0-1: A pieces 2 wc + q; 2-5: B pieces 4 wc + q - 2) of the stage at the cursor into
// ring slot `slot`
template <int Q, bool K0 = false>
__device__ __forceinline__ void pp_dma_piece(const PpArgs& a, const PpStream& s, char* grp_lds, int slot, int wc,
                                             unsigned offa, unsigned offb) {
  char* img = grp_lds + slot * PP_STAGE;
  const long k0 = K0 ? 0 : (long)s.dk * PP_BK;
  if constexpr (Q < 2) {
    const int p = 2 * wc + Q;
    pp_glds16(s.arow + (long)(16 * p) * a.lda + k0, offa, img + p * 1024);
  } else {
    const int p = 4 * wc + Q - 2;
    pp_glds16(s.brow + (long)(16 * p) * a.ldb + k0, offb, img + PP_AIMG + p * 1024);
  }
}

__device__ __forceinline__ void pp_cursor_next(const PpArgs& a, PpStream& s) {
  if (++s.dk == s.S) {
    s.dk = 0;
    ++s.dj;
    pp_cursor_tile(a, s);
  }
}

// issue the group's DMA of the stage at the cursor into ring slot `slot`, advance the cursor
// (K0: timing diagnostic, always the tile's first K block -- same LDS traffic, L2-resident source)
template <bool K0 = false>
__device__ __forceinline__ void pp_stage_dma(const PpArgs& a, PpStream& s, char* grp_lds, int slot, int wc,
                                             unsigned offa, unsigned offb) {
  pp_dma_piece<0, K0>(a, s, grp_lds, slot, wc, offa, offb);
  pp_dma_piece<1, K0>(a, s, grp_lds, slot, wc, offa, offb);
  pp_dma_piece<2, K0>(a, s, grp_lds, slot, wc, offa, offb);
  pp_dma_piece<3, K0>(a, s, grp_lds, slot, wc, offa, offb);
  pp_dma_piece<4, K0>(a, s, grp_lds, slot, wc, offa, offb);
  pp_dma_piece<5, K0>(a, s, grp_lds, slot, wc, offa, offb);
  pp_cursor_next(a, s);
}

__device__ __forceinline__ u16x8 pp_pair_swap(u16x4 x, u16x4 y) {
  const uint2 xv = __builtin_bit_cast(uint2, x), yv = __builtin_bit_cast(uint2, y);
  const auto s0 = __builtin_amdgcn_permlane16_swap(xv.x, yv.x, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(xv.y, yv.y, false, false);
  const uint4 v = {s0[0], s1[0], s0[1], s1[1]};
  return __builtin_bit_cast(u16x8, v);
}

// stores of one epilogue row block i (16 rows x 64 columns of the wave): 2 x 16-B stores per
// lane per output tensor.  acc[i][j][r] = D[mrow + 16 i][ncol + 16 j + r].
template <int EPI>
__device__ __forceinline__ void pp_epi_row(const PpArgs& a, const f32x4 (&acc)[8][4], int i, long mrow, long ncol,
                                           const float (&bv)[4][4], int lane) {
  const long m = mrow + 16 * i;
  const int g = lane >> 4;
  const long scol = (ncol - 4 * g) + 16 * (g & 1) + 8 * (g >> 1);
  u16x4 out[4], dd[4];
  if constexpr (EPI == PP_EPI_BIAS_GELU_DAUX) {
    f32x2 xv[8], gv[8], dv[8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        xv[2 * j + h] = f32x2{acc[i][j][2 * h], acc[i][j][2 * h + 1]} + f32x2{bv[j][2 * h], bv[j][2 * h + 1]};
    gelu2_batch_both<8>(xv, gv, dv);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          out[j][2 * h + e] = f2bf(gv[2 * j + h][e]);
          dd[j][2 * h + e] = f2bf(dv[2 * j + h][e]);
        }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[j][r] = f2bf(acc[i][j][r] + bv[j][r]);
  }
#pragma unroll
  for (int j = 0; j < 4; j += 2) {
    *(u16x8*)(a.D + m * a.ldd + scol + j * 16) = pp_pair_swap(out[j], out[j + 1]);
    if constexpr (EPI == PP_EPI_BIAS_GELU_DAUX)
      *(u16x8*)(a.aux + m * a.ldaux + scol + j * 16) = pp_pair_swap(dd[j], dd[j + 1]);
  }
}

// stores per wave per tile epilogue (counted into the vmcnt of the next tile's first wait)
template <int EPI>
struct PpEpi {
  static constexpr int STORES = EPI == PP_EPI_BIAS_GELU_DAUX ? 32 : 16;
};

// E = epilogue slots per tile (the 8 row blocks split evenly over them)
// DP: 0 = production.  Timing diagnostics (wrong results, CLOUDTIK_AMD_PP_DMA): 3 = no DMA after
// the prologue, 4 = every stage re-reads the tile's first K block (same L2->LDS traffic, L2-resident
// source).  Issuing the DMA inside the MFMA slot instead of the READ slot measured slower (r6f).
template <int EPI, int E, int DP = 0>
__global__ void __launch_bounds__(PP_THREADS, 1) gemm_pp_kernel(PpArgs a) {
  static_assert(8 % E == 0, "row blocks per epilogue slot");
  __shared__ __attribute__((aligned(1024))) char lds[2 * PP_GROUP];   // 144 KiB, the only LDS object
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wave >> 2, wc = wave & 3;
  const int wg = blockIdx.x;
  char* glds = lds + g * PP_GROUP;
  const int S = a.K / PP_BK;

  // tiles of this group / of the other group (their slot counts pad each other)
  auto tiles_of = [&](int gg) {
    // the largest j with pp_tile_index(wg, gg, j) < T, plus one
    const int base = (wg & 7) * (a.V >> 3) + 2 * (wg >> 3) + gg;
    return base < a.T ? (a.T - base + a.V - 1) / a.V : 0;
  };
  const int my_tiles = tiles_of(g), other_tiles = tiles_of(g ^ 1);
  const int my_slots = my_tiles * (2 * S + E), other_slots = other_tiles * (2 * S + E);
  const int total_slots = max(my_slots, other_slots);

  // per-lane source offsets of a 16-row piece: row lane >> 2, logical chunk (lane & 3) ^ g(lane >> 4)
  const int prow = lane >> 2, pch = (lane & 3) ^ pp_g((lane >> 4) & 3);
  const unsigned offa = (unsigned)((prow * a.lda + pch * 8) * 2);
  const unsigned offb = (unsigned)((prow * a.ldb + pch * 8) * 2);

  PpStream st{wg, g, my_tiles, S, a.A, a.B, 0, 0};
  pp_cursor_tile(a, st);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  pp_s16x8 fa[8], fb[4];

  // group 1 runs one slot behind group 0
  if (g == 1) pp_bar();
  int used = 0;                                  // slots this group has spent
  if (my_tiles > 0) {
    const int total_stages = my_tiles * S;
    uint2 braw[4] = {};                          // this lane's bias columns, raw bf16 (EPI 5 / 6)
    {
      long tm0, tn0;
      pp_tile(a, pp_tile_index(a, wg, g, 0), tm0, tn0);
      if constexpr (EPI != PP_EPI_PLAIN) {
#pragma unroll
        for (int j = 0; j < 4; ++j) braw[j] = pp_ld8(a.bias + tn0 + wc * 64 + (lane >> 4) * 4 + j * 16);
      }
    }
    // prologue: stages 0 and 1 of the stream (total_stages >= 2: K >= 64)
    pp_stage_dma(a, st, glds, 0, wc, offa, offb);
    pp_stage_dma(a, st, glds, 1, wc, offa, offb);
    pp_vm<PP_DMA>();
    pp_bar();
    ++used;
    long m0 = 0, n0 = 0;
    pp_tile(a, pp_tile_index(a, wg, g, 0), m0, n0);
    int jt = 0, kk = 0;
    for (int s = 0; s < total_stages; ++s) {
      // ---- READ slot: fragments of stage s, DMA of stage s + 2
      const char* img = glds + (s % PP_NS) * PP_STAGE;
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = pp_frag(img, 16 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = pp_frag(img + PP_AIMG, wc * 64 + 16 * j, lane);
      const bool dma2 = DP != 3 && s + 2 < total_stages;
      if (dma2) pp_stage_dma<DP == 4>(a, st, glds, (s + 2) % PP_NS, wc, offa, offb);
      pp_bar();
      // ---- MFMA slot
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf16x8_t)fb[j], (bf16x8_t)fa[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      // stage s + 1 must have landed before the barrier that precedes its READ slot; younger
      // VMEM ops: the stage s + 2 DMA, and the previous tile's epilogue stores when stage s
      // opened a new tile (issued after stage s + 1's DMA)
      if (s + 1 < total_stages) {
        if (!dma2) pp_vm<0>();
        else if (kk == 0 && jt > 0) pp_vm<PP_DMA + PpEpi<EPI>::STORES>();
        else pp_vm<PP_DMA>();
      }
      pp_bar();
      used += 2;
      if (++kk == S) {
        // ---- epilogue slots: the row blocks of this tile, E slots
        const long mrow = m0 + (lane & 15);
        const long ncl = n0 + wc * 64 + (lane >> 4) * 4;
        float bv[4][4] = {};
        if constexpr (EPI != PP_EPI_PLAIN) {
          // the hand-counted waits of the K loop have retired the asm bias loads by here; naming
          // the registers keeps every consumer below this point (cdna_hip_programming.md §5.7 1(ii))
          asm volatile("" : "+v"(braw[0]), "+v"(braw[1]), "+v"(braw[2]), "+v"(braw[3]));
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const u16x4 b4 = __builtin_bit_cast(u16x4, braw[j]);
#pragma unroll
            for (int r = 0; r < 4; ++r) bv[j][r] = bf2f(b4[r]);
          }
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
#pragma unroll
          for (int i = e * (8 / E); i < (e + 1) * (8 / E); ++i) pp_epi_row<EPI>(a, acc, i, mrow, ncl, bv, lane);
          pp_bar();
        }
        used += E;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        kk = 0;
        if (++jt < my_tiles) {
          pp_tile(a, pp_tile_index(a, wg, g, jt), m0, n0);
          // next tile's bias: issued after this epilogue's stores, retired by the K loop's
          // counted waits long before its own epilogue
          if constexpr (EPI != PP_EPI_PLAIN) {
#pragma unroll
            for (int j = 0; j < 4; ++j) braw[j] = pp_ld8(a.bias + n0 + wc * 64 + (lane >> 4) * 4 + j * 16);
          }
        }
      }
    }
  }
  // equal barrier counts: every wave passes total_slots + 1 barriers (group 1's first one is
  // its offset, so it pads one fewer)
  const int target = total_slots + 1;
  for (int k = used + (g == 1 ? 1 : 0); k < target; ++k) pp_bar();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace ct

using namespace ct;

static int pp_cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    return v;
  }();
  return n;
}

// D[M,N] = A[M,K] . B[N,K]^T with epilogue 0 (plain), 5 (+ bias[N]) or 6 (D = gelu(. + bias),
// aux = gelu'(. + bias)).  `wgs` = workgroups (0: the CU count; must be a multiple of 8);
// `eslots` = epilogue slots per tile (1, 2, 4 or 8).  Nonzero (nothing launched) when the shape
// is not supported: M % 128, N % 256, K % 64, or fewer 128 x 256 tiles than 2 x workgroups.
extern "C" int ct_gemm_pp(const void* A, long lda, const void* B, long ldb, void* D, long ldd, int M, int N, int K,
                          int epi, const void* bias, void* aux, long ldaux, int wgs, int eslots, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % PP_TM || N % PP_TN || K % 64) return 1;
  if (lda % 8 || ldb % 8 || ldd % 8 || lda < K || ldb < K || ldd < N) return 2;
  if (((uintptr_t)A & 15) || ((uintptr_t)B & 15) || ((uintptr_t)D & 15)) return 3;
  if ((epi == 5 || epi == 6) && (!bias || ((uintptr_t)bias & 7))) return 4;
  if (epi == 6 && (!aux || ((uintptr_t)aux & 15) || ldaux % 8 || ldaux < N)) return 4;
  if (epi != 0 && epi != 5 && epi != 6) return 6;
  const int P = wgs > 0 ? wgs : pp_cu_count();
  if (P % 8) return 5;
  PpArgs a{(const bf16_t*)A, (const bf16_t*)B, (bf16_t*)D, (const bf16_t*)bias, (bf16_t*)aux,
           lda, ldb, ldd, ldaux, M, N, K, M / PP_TM, N / PP_TN, (M / PP_TM) * (N / PP_TN), 2 * P};
  if (a.T < a.V || (long)a.tiles_m * a.tiles_n > (1L << 30)) return 5;
  // CLOUDTIK_AMD_PP_DMA: DMA placement (kernel template DP), 0 by default
  static const int dp = [] { const char* e = getenv("CLOUDTIK_AMD_PP_DMA"); return e ? atoi(e) : 0; }();
#define PP_LAUNCH(E_, ES_)                                                              \
  do {                                                                                  \
    if (dp == 3) gemm_pp_kernel<E_, ES_, 3><<<P, PP_THREADS, 0, stream>>>(a);       \
    else if (dp == 4) gemm_pp_kernel<E_, ES_, 4><<<P, PP_THREADS, 0, stream>>>(a);       \
    else gemm_pp_kernel<E_, ES_, 0><<<P, PP_THREADS, 0, stream>>>(a);                    \
  } while (0)
#define PP_BY_E(E_)                            \
  switch (eslots) {                            \
    case 1: PP_LAUNCH(E_, 1); break;           \
    case 2: PP_LAUNCH(E_, 2); break;           \
    case 4: PP_LAUNCH(E_, 4); break;           \
    case 8: PP_LAUNCH(E_, 8); break;           \
    default: return 6;                         \
  }
  if (epi == 0) { PP_BY_E(PP_EPI_PLAIN) }
  else if (epi == 5) { PP_BY_E(PP_EPI_BIAS) }
  else { PP_BY_E(PP_EPI_BIAS_GELU_DAUX) }
#undef PP_BY_E
#undef PP_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 7;
}
