// Weight-gradient GEMM for gfx950: C[M, N] (+)= A[T, M]^T . B[T, N], bf16 in, fp32 accumulate.
//
// Every Linear layer's dW = dY^T X is this shape: the reduction runs over the token dimension
// T, which is the ROW (slow) index of both operands, so neither operand is k-contiguous.
// hipBLASLt runs it at ~0.8-0.9 PF/s on the BERT-large shapes even with split-K
// (profiles/steady_bert_large.md).  Here:
//   * 256 x 256 output tile per 512-thread workgroup (8 waves as 2(M) x 4(N), 128 x 64 per wave,
//     32 MFMA 16x16x32 accumulators per wave), 32 tokens per stage, 1 workgroup per CU.
//   * Operand tiles are staged global -> LDS with global_load_lds (16 B per lane, lane-linear
//     LDS image), through a 4-slot ring: 3 stages are in flight while one is multiplied
//     (one stage in flight is latency-bound at ~25% of MFMA peak); the wait is a counted
//     vmcnt and the barriers are raw s_barrier, so the prefetch spans them.
//   * Both images are stored [token][m] (the global row layout) and the MFMA fragments,
//     which need 8 consecutive tokens per lane, are read with ds_read_b64_tr_b16 (gfx950's
//     transposing LDS read): no transpose pass anywhere.  The 16-byte chunks of a row are
//     XOR-swizzled by the source address (the LDS side of glds is lane-linear) so the 8 rows
//     a 32-lane half reads per instruction land in 8 distinct 32-byte bank slots.
//   * Split-K over T (blockIdx -> (split, tile) after a bijective XCD remap, so the blocks
//     that share A / B panels share an L2); fp32 partial slabs are combined by
//     ct_splitk_reduce, or a single split accumulates straight into the bf16 gradient.
// Reference: the Linear backward of HF BERT under DDP (SURVEY.md §2.15 "GEMMs").
#include "common.h"

namespace ct {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

constexpr int GT_BM = 256, GT_BN = 256, GT_BK = 32, GT_THREADS = 512;
constexpr int GT_STAGES = 4;                       // LDS ring: GT_STAGES - 1 stages in flight
constexpr int GT_ROWB = GT_BM * 2;                 // bytes per LDS image row (256 bf16)
constexpr int GT_TILEB = GT_BK * GT_ROWB;          // 16 KiB per operand stage
constexpr int GT_GLDS = GT_TILEB / (GT_THREADS * 16);   // glds per thread per operand stage (2)

// chunk (16 B) swizzle of image row r: rows r..r+3 and r+8..r+11 -> 8 distinct 32 B slots
__device__ __forceinline__ int gt_swz(int r) { return ((r & 3) << 1) | (((r >> 3) & 1) << 3); }

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef const __attribute__((address_space(1))) void gbl_void;

// one global_load_lds_dwordx4 in inline asm: the compiler never sees the LDS-DMA, so it
// inserts no vmcnt(0) ahead of ds_reads it cannot prove disjoint from it (which would drain
// the prefetch every stage).  Ordering is ours: the counted vmcnt + s_barrier in gt_step.
__device__ __forceinline__ void glds16(const void* g, const char* lds_wave_base) {
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(la) : "memory", "m0");
}

// stage one [BK x 256] tile of a [T x ld] row-major operand (rows t0.., columns c0..)
__device__ __forceinline__ void gt_stage(const bf16_t* __restrict__ src, long ld, long t0, long c0, char* lds_tile,
                                         int wave, int lane) {
#pragma unroll
  for (int i = 0; i < GT_GLDS; ++i) {
    const int pair = wave * GT_GLDS + i;           // this wave-instruction fills rows 2*pair, 2*pair+1
    const int r = 2 * pair + (lane >> 5);
    const int c = (lane & 31) ^ gt_swz(r);         // LDS chunk (lane & 31) holds global chunk c
    glds16(src + (t0 + r) * ld + c0 + c * 8, lds_tile + pair * 1024);
  }
}

// A/B fragment of mfma_f32_16x16x32_bf16 for the 16 columns [col0, col0+16) and tokens
// [k0, k0+32) of an image: lane l gets column (l & 15), tokens k0 + 8(l >> 4) + 0..7
__device__ __forceinline__ s16x8 gt_frag(const char* img, int k0, int col0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int r0 = k0 + 8 * g + q, r1 = r0 + 4;
  const int ch = (col0 >> 3) + (p >> 1);
  const char* a0 = img + r0 * GT_ROWB + ((ch ^ gt_swz(r0)) << 4) + ((p & 1) << 3);
  const char* a1 = img + r1 * GT_ROWB + ((ch ^ gt_swz(r1)) << 4) + ((p & 1) << 3);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// one pipeline step: prefetch stage kt+STAGES-1 into the ring slot freed one step ago, wait
// until stage kt has landed (leaving the younger ones in flight), multiply it
__device__ __forceinline__ void gt_step(const bf16_t* __restrict__ A, long lda, const bf16_t* __restrict__ B,
                                        long ldb, long m0, long n0, long tbeg, int kt, int nk, char* ring,
                                        int wave, int lane, int wm, int wn, f32x4 (&acc)[8][4]) {
  const int pf = kt + GT_STAGES - 1;
  if (pf < nk) {
    char* nxt = ring + (pf % GT_STAGES) * 2 * GT_TILEB;
    gt_stage(A, lda, tbeg + (long)pf * GT_BK, m0, nxt, wave, lane);
    gt_stage(B, ldb, tbeg + (long)pf * GT_BK, n0, nxt + GT_TILEB, wave, lane);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GT_GLDS * (GT_STAGES - 1)) : "memory");
  } else if (pf == nk) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GT_GLDS * (GT_STAGES - 2)) : "memory");
  } else if (pf == nk + 1) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GT_GLDS * (GT_STAGES - 3)) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();                     // every wave's DMA of stage kt is visible
  const char* ia = ring + (kt % GT_STAGES) * 2 * GT_TILEB;
  const char* ib = ia + GT_TILEB;
  s16x8 bf[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bf[j] = gt_frag(ib, 0, wn * 64 + j * 16, lane);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const s16x8 af = gt_frag(ia, 0, wm * 128 + i * 16, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf16x8_t)af, (bf16x8_t)bf[j], acc[i][j], 0, 0, 0);
  }
  // the slot of stage kt is restaged at step kt+1 (as stage kt+STAGES): all of its reads
  // must be done first
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// mode 0: fp32 store into out + split * M * N; 1: bf16 out += C; 2: bf16 out = C
__global__ void __launch_bounds__(GT_THREADS, 1) gemm_tn_kernel(const bf16_t* __restrict__ A, long lda,
                                                                 const bf16_t* __restrict__ B, long ldb,
                                                                 void* __restrict__ out, int M, int N,
                                                                 long t_per_split, int splits, int mode) {
  __shared__ __attribute__((aligned(1024))) char ring[GT_STAGES * 2 * GT_TILEB];   // 128 KiB
  const int tiles_n = N / GT_BN, tiles = (M / GT_BM) * tiles_n;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles, tile = L % tiles;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;          // 2 x 4 waves: 128 x 64 each
  const long m0 = (long)tm * GT_BM, n0 = (long)tn * GT_BN;
  const long tbeg = (long)split * t_per_split;
  const int nk = (int)(t_per_split / GT_BK);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: stages 0 .. STAGES-2 in flight
#pragma unroll
  for (int p = 0; p < GT_STAGES - 1; ++p)
    if (p < nk) {
      gt_stage(A, lda, tbeg + (long)p * GT_BK, m0, ring + p * 2 * GT_TILEB, wave, lane);
      gt_stage(B, ldb, tbeg + (long)p * GT_BK, n0, ring + p * 2 * GT_TILEB + GT_TILEB, wave, lane);
    }
  for (int kt = 0; kt < nk; ++kt) gt_step(A, lda, B, ldb, m0, n0, tbeg, kt, nk, ring, wave, lane, wm, wn, acc);

  // epilogue: acc[i][j] reg r -> C[m0 + wm*128 + i*16 + (lane>>4)*4 + r][n0 + wn*64 + j*16 + (lane&15)]
  const long col_base = n0 + wn * 64 + (lane & 15);
  const long row_base = m0 + wm * 128 + (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long idx = (row_base + i * 16 + r) * N + col_base + j * 16;
        const float v = acc[i][j][r];
        if (mode == 0) reinterpret_cast<float*>(out)[(long)split * M * N + idx] = v;
        else if (mode == 1) {
          bf16_t* o = reinterpret_cast<bf16_t*>(out) + idx;
          *o = f2bf(bf2f(*o) + v);
        } else reinterpret_cast<bf16_t*>(out)[idx] = f2bf(v);
      }
}

}  // namespace ct

using namespace ct;

// C[M,N] (+)= A[T,M]^T B[T,N]; A, B row-major with leading dims lda / ldb (elements).
// splits > 1 (mode 0 only): fp32 partials [splits, M, N] for ct_splitk_reduce.
// Returns nonzero (and launches nothing) when the shape is not supported.
extern "C" int ct_gemm_tn(const void* A, long lda, const void* B, long ldb, void* out, int M, int N, long T,
                          int splits, int mode, hipStream_t stream) {
  if (M <= 0 || N <= 0 || M % GT_BM || N % GT_BN || splits < 1) return 1;
  if (T % ((long)splits * GT_BK)) return 2;
  if (lda % 8 || ldb % 8 || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return 3;
  if (splits > 1 && mode != 0) return 4;
  const long blocks = (long)(M / GT_BM) * (N / GT_BN) * splits;
  if (blocks > (1L << 30)) return 5;
  gemm_tn_kernel<<<(int)blocks, GT_THREADS, 0, stream>>>((const bf16_t*)A, lda, (const bf16_t*)B, ldb, out, M, N,
                                                          T / splits, splits, mode);
  return hipGetLastError() == hipSuccess ? 0 : 6;
}
