// Implicit-GEMM convolution over NHWC bf16 activations for gfx950 (MFMA 16x16x32, fp32 acc).
//
// One kernel family serves every convolution of the ResNet family that is not a plain GEMM:
//     Y[m, n] = sum_{t < T, c < Ci} X[pixel(m) + tap(t), c] * W[n, t * Ci + c]
// where row m walks a "row grid" (b, y, x) and tap t adds a (dy, dx) pixel offset:
//   * forward conv:            row grid = output pixels, pixel = (y*sy, x*sx), taps = (r - pad, s - pad);
//   * data gradient, stride 1: X = dY, taps = (pad - r, pad - s), W = the flipped, transposed filter;
//   * data gradient, stride 2: one launch per output-pixel parity class, row grid = that class,
//                              taps = the filter taps that reach it (ops/conv.py builds the plan).
// Out-of-image taps read a zero page, so padding costs no branch in the K loop.
//
// Structure (MI355X_MICROARCH.md / cdna_hip_programming.md §5):
//   * BM x BN output tile per workgroup, K walked 64 channels of one tap at a time (BK = 64);
//   * both operands staged global -> LDS with global_load_lds_dwordx4 (16 B per lane): each
//     A row is one pixel's 64 channels (128 B) -- a per-lane gathered address, which is what
//     LDS-DMA allows (the LDS side is lane-linear, the global side is per lane); the 16-B
//     chunks of a row are XOR-swizzled on the SOURCE side so ds_read_b128 fragment reads are
//     conflict-free;
//   * an NS-slot LDS ring with NS-1 stages in flight, a counted vmcnt and one raw s_barrier per
//     K-step (the DMA spans the barrier; one stage in flight is latency-bound);
//   * blockIdx -> tile through the bijective XCD remap with N-tiles fastest, so the blocks that
//     share an A panel (the expensive gathered operand) run on one XCD's L2;
//   * epilogue: the bf16 tile is re-laid through LDS so each lane stores 16 contiguous bytes
//     (whole rows per wave), optional accumulate (Y += result), and optionally the per-tile
//     BatchNorm statistics of
//     the bf16 output (mean and M2 per channel over the tile's rows, merged by Chan's formula
//     in ct_bn_partials_finalize) -- the separate statistics pass over the conv output goes away.
// Reference workload: torchvision ResNet-50 training, channels_last bf16
// (applications/ai/quickstart/models/image_recognition/pytorch/common/main.py:276-296).
#include "common.h"
#include <algorithm>
#include <cstdlib>

namespace ct {

typedef __attribute__((ext_vector_type(8))) short cv_s16x8;
typedef __attribute__((address_space(3))) cv_s16x8 cv_lds_s16x8;
typedef __attribute__((address_space(3))) void cv_lds_void;

__device__ __attribute__((aligned(256))) uint32_t cv_zero_page[64];   // zero-initialised: OOB source

constexpr int CV_MAXT = 16;

struct ConvArgs {
  const bf16_t* X;      // gathered operand, NHWC [Nb, Hi, Wi, Ci]
  const bf16_t* W;      // [Co][T * Ci], k contiguous
  bf16_t* Y;            // output
  float* part;          // EPI 1: per-tile means [mtiles][Co], then M2 [mtiles][Co]
  int Hi, Wi, Ci;
  int Hr, Wr;           // row grid: m = (b * Hr + y) * Wr + x
  int sy, sx;           // input pixel = (y * sy + dy_t, x * sx + dx_t)
  int Ho, Wo, oys, oxs, oy0, ox0, ldy;   // output pixel = (y * oys + oy0, x * oxs + ox0), row stride ldy
  int Co, M, T;
  int accumulate;        // 1: Y += result; 2: the 1x1 stride-2 data gradient -- also write the zeros
                         //   of the three odd-parity pixels of each written one (no zero-fill pass)
  unsigned long long tdy, tdx;           // 16 taps x 4 bits, biased by 8
  int cpt;              // K-steps (of 64 weight columns) per tap: Ci / 64, or 1 in pixel-chunk mode
  int pixchunk;         // stem modes: 1 = Ci 8, the 8 chunks of a K-step are 8 consecutive pixels;
                        //   2 = Ci 4, chunk g = pixels (2 (g & 3), + 1) of kernel row (g >> 2): two
                        //   filter rows x 8 pixels per K-step (a 7x7 RGB stem: 4 K-steps, not 7)
  // EPI 2 (data gradient feeding a BatchNorm + ReLU backward, mask recomputed from x):
  const bf16_t* bnx;    // the BatchNorm's input, at the same addresses as Y
  const bf16_t* bny;    // its output (ReLU mask source when it had a residual add), or null:
                        //   mask recomputed from x
  const float* bnstat;  // its forward float[4 Co]: mean, invstd, a, b (y = relu(a x + b))
  float* bnp;           // per-tile sums of dy' and dy' * xhat: rows [bntile0 + tm][Co], the
  long bnp2;            //   second set bnp2 floats further
  int bntile0;
  const uint8_t* bnm;   // EPI 2: the BatchNorm's ReLU bitmask (byte per 8 channels), or null
  int dense_out;        // the output grid IS the row grid (every forward, every stride-1 data
                        //   gradient): output row = m * ldy, no pixel arithmetic
};

__device__ __forceinline__ int cv_swz(int r) { return (r >> 1) & 7; }

// q = n / d, r = n % d for 0 <= n < 2^24, d > 0: the float quotient is within one of the exact
// one; one correction each way makes it exact (~10 VALU instead of a ~40-instruction integer
// division sequence)
__device__ __forceinline__ void cv_divmod(int n, int d, float inv_d, int& q, int& r) {
  q = (int)((float)n * inv_d);
  r = n - q * d;
  if (r >= d) {
    ++q;
    r -= d;
  }
  if (r < 0) {
    --q;
    r += d;
  }
}

__device__ __forceinline__ void cv_glds16(const void* g, const char* lds_wave_base) {
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(cv_lds_void*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(la) : "memory", "m0");
}

// LDS-DMA addressed as a wave-uniform 64-bit base (SGPRs) + a per-lane 32-bit byte offset.
// PAD: 5 wait states between the M0 write and the load instead of 1, which also covers a base
// SGPR that a VALU (v_readfirstlane / v_readlane of a spilled SGPR) wrote just before the
// statement -- hipcc pads nothing inside asm (cdna_hip_programming.md §5.7 item 2).  The r6 audit
// of the compiled kernels (profiles/r6/SUMMARY.md) found that pattern in the streamed kernel only.
template <bool PAD = false>
__device__ __forceinline__ void cv_glds16s(const void* sbase, unsigned voff, const char* lds_wave_base) {
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(cv_lds_void*)lds_wave_base);
  const uint64_t sb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)sbase) |
                      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)sbase >> 32)) << 32);
  if constexpr (PAD)
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 4\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sb), "s"(la)
                 : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sb), "s"(la)
                 : "memory", "m0");
}

// LDS-DMA by buffer load: 32-bit per-lane byte offset into a buffer resource whose range check
// returns zeros past num_records (inline asm: a compiler-visible LDS-DMA makes hipcc wait for it
// before every later LDS read, which drains the ring)
__device__ __forceinline__ void cv_bglds16(__amdgpu_buffer_rsrc_t r, unsigned voff, const char* lds_wave_base) {
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(cv_lds_void*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r), "s"(la)
               : "memory", "m0");
}

__device__ __forceinline__ cv_s16x8 cv_frag(const char* img, int r0, int ks, int lane) {
  const int row = r0 + (lane & 15);
  const int kc = ks * 4 + (lane >> 4);
  return *(const cv_lds_s16x8*)(img + row * 128 + ((kc ^ cv_swz(row)) << 4));
}

// a K-step chunk's element offset from its row's pixel and its pixel / row step (stem modes)
template <class Args>
__device__ __forceinline__ void cv_chunk_geo(const Args& a, int gc, unsigned& gca, int& gpx, int& gpy) {
  if (a.pixchunk == 2) {
    gpx = 2 * (gc & 3);
    gpy = gc >> 2;
    gca = (unsigned)((gpy * a.Wi + gpx) * 4);
  } else {
    gpx = a.pixchunk ? gc : 0;                     // stem: the chunk is a pixel step along x
    gpy = 0;
    gca = (unsigned)gc * 8u;                       // element offset of the chunk
  }
}

__device__ __forceinline__ void cv_bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, never for
// vector memory -- __syncthreads() would emit vmcnt(0) and drain the LDS-DMA stages in flight
__device__ __forceinline__ void cs_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  cv_bar();
}

template <int N>
__device__ __forceinline__ void cv_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `rem` later stages (G glds each) are outstanding
template <int G, int NS>
__device__ __forceinline__ void cv_wait_stage(int rem) {
  if constexpr (NS >= 4) {
    if (rem >= 2) { cv_vm<2 * G>(); return; }
  }
  if constexpr (NS >= 3) {
    if (rem >= 1) { cv_vm<G>(); return; }
  }
  cv_vm<0>();
}

// BatchNorm statistics of one wave's rows (EPI 1): the column mean and M2 (sum of squared
// deviations from that mean, two passes over the registers) of the bf16 outputs in the wave's
// WM rows, written as the partials of a WM-row block: means [blocks][Co] then M2 [blocks][Co],
// block = global row / WM (what bn_finalize / bn_partials_finalize merge with Chan's formula).
// Column sums over a 16-row fragment are DPP row sums: no LDS, no workgroup barrier.
template <int MI, int NJ, int WM>
__device__ __forceinline__ void cv_wave_stats(const ConvArgs& a, const f32x4 (&acc)[MI][NJ], const bool (&rv)[MI],
                                              int row0, int col0, int lane) {
  const int nrows = min(WM, a.M - row0);
  if (nrows <= 0) return;
  const float inv = 1.f / (float)nrows;
  const long blocks = ((long)a.M + WM - 1) / WM, pb = row0 / WM;
  float* pm = a.part + pb * a.Co + col0 + 4 * (lane >> 4);
  float* pq = a.part + (blocks + pb) * a.Co + col0 + 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    f32x4 mv, qv;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i) v += acc[i][j][r];
      const float mean = row16_sum(v) * inv;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const float d = acc[i][j][r] - mean;
        q += rv[i] ? d * d : 0.f;
      }
      mv[r] = mean;
      qv[r] = row16_sum(q);
    }
    if ((lane & 15) == 0) {
      *(f32x4*)(pm + 16 * j) = mv;
      *(f32x4*)(pq + 16 * j) = qv;
    }
  }
}

// ---- copy-out of the epilogue (both conv kernels).  Thread tid owns 16-B chunk cc = tid % CPR
// of rows tid / CPR + k * RPP, k < NR.  cv_out_prefetch computes the rows' output addresses and
// issues every global load the copy-out needs (the old Y of an accumulate, the BatchNorm input /
// output of EPI 2) BEFORE the tile goes through LDS, so their latency overlaps the LDS re-lay
// instead of being paid row by row (the compiler cannot hoist them over the previous row's Y
// store: the pointers may alias).
template <int NR>
struct CvOut {
  long yo[NR];
  bool ok[NR];
  u16x8 old[NR], xv[NR], yv[NR];
  uint32_t mb[NR];
};

template <int BM, int CPR, int RPP, int EPI>
__device__ __forceinline__ void cv_out_prefetch(const ConvArgs& a, CvOut<BM / RPP>& o, int m0, int n0, int tid) {
  constexpr int NR = BM / RPP;
  const int HW = a.Hr * a.Wr;
  const float inv_hw = 1.f / (float)HW, inv_w = 1.f / (float)a.Wr;
  const int cc = tid % CPR;
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    const int m = m0 + tid / CPR + k * RPP;
    o.ok[k] = m < a.M;
    if (a.dense_out) {
      o.yo[k] = (long)(o.ok[k] ? m : m0) * a.ldy + n0 + cc * 8;
    } else {
      int b, rem, y, x;
      cv_divmod(o.ok[k] ? m : m0, HW, inv_hw, b, rem);
      cv_divmod(rem, a.Wr, inv_w, y, x);
      o.yo[k] = ((long)(b * a.Ho + y * a.oys + a.oy0) * a.Wo + x * a.oxs + a.ox0) * a.ldy + n0 + cc * 8;
    }
  }
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    if (!o.ok[k]) continue;
    if (a.accumulate == 1) o.old[k] = *(const u16x8*)(a.Y + o.yo[k]);
    if constexpr (EPI == 2) {
      o.xv[k] = *(const u16x8*)(a.bnx + o.yo[k]);
      if (a.bnm) o.mb[k] = a.bnm[o.yo[k] >> 3];
      else if (a.bny) o.yv[k] = *(const u16x8*)(a.bny + o.yo[k]);
    }
  }
}

// the stores (+ accumulate, + EPI 2 mask and per-thread sums s1 / s2 of its 8 channels);
// chunk(row) = the LDS address of this thread's 16-B chunk of tile row `row`
template <int BM, int CPR, int RPP, int EPI, typename ChunkFn>
__device__ __forceinline__ void cv_out_store(const ConvArgs& a, CvOut<BM / RPP>& o, ChunkFn chunk, int tid,
                                             const float (&bfa)[8], const float (&bfb)[8], const float (&bmu)[8],
                                             const float (&bis)[8], float (&s1)[8], float (&s2)[8]) {
  constexpr int NR = BM / RPP;
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    if (!o.ok[k]) continue;
    u16x8 v = *(const u16x8*)chunk(tid / CPR + k * RPP);
    if (a.accumulate == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + bf2f(o.old[k][e]));
    }
    if constexpr (EPI == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xf = bf2f(o.xv[k][e]);
        const bool on = a.bnm ? ((o.mb[k] >> e) & 1u) != 0
                        : (a.bny ? bf2f(o.yv[k][e]) > 0.f : bf2f(f2bf(__builtin_fmaf(xf, bfa[e], bfb[e]))) > 0.f);
        if (!on) v[e] = 0;
        const float d = bf2f(v[e]);
        s1[e] += d;
        s2[e] += d * (xf - bmu[e]) * bis[e];
      }
    }
    *(u16x8*)(a.Y + o.yo[k]) = v;
    if (a.accumulate == 2) {
      const long ld = a.ldy, ldr = (long)a.Wo * a.ldy;
      *(u16x8*)(a.Y + o.yo[k] + ld) = u16x8(0);
      *(u16x8*)(a.Y + o.yo[k] + ldr) = u16x8(0);
      *(u16x8*)(a.Y + o.yo[k] + ldr + ld) = u16x8(0);
    }
  }
}

// One output tile (L = tile index, N-tiles fastest) of conv_igemm_kernel; also the body of
// conv_igemm_phases_kernel, which runs several launches' tiles in one grid.
template <int BM, int BN, int WGM, int WGN, int NS, int EPI>
__device__ __forceinline__ void conv_igemm_tile(const ConvArgs& a, const int L) {
  constexpr int NW = WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 16, NJ = WN / 16;
  constexpr int STAGE = (BM + BN) * 128;
  constexpr int IA = BM / (8 * NW), IB = BN / (8 * NW), G = IA + IB;
  static_assert(IA * 8 * NW == BM && IB * 8 * NW == BN, "tile / wave mismatch");
  static_assert(NS >= 2 && NS <= 4 && NS * STAGE <= 160 * 1024, "LDS ring");
  __shared__ __attribute__((aligned(1024))) char lds[NS * STAGE];   // the only LDS object

  const int ntn = a.Co / BN;
  const int tm = L / ntn, tn = L % ntn;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: weight bases in SGPRs
  const int wm = wave / WGN, wn = wave % WGN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int HW = a.Hr * a.Wr;

  // ---- per-lane gather descriptors: the A rows this lane stages (fixed for the whole K loop)
  int pix[IA], iy0[IA], ix0[IA], gpx[IA], gpy[IA];
  unsigned gca[IA];
#pragma unroll
  for (int j = 0; j < IA; ++j) {
    const int row = (wave * IA + j) * 8 + (lane >> 3);
    const int m = m0 + row;
    const int gc = (lane & 7) ^ cv_swz(row);
    cv_chunk_geo(a, gc, gca[j], gpx[j], gpy[j]);
    if (m < a.M) {
      int b, rem, y, x;
      cv_divmod(m, HW, 1.f / (float)HW, b, rem);
      cv_divmod(rem, a.Wr, 1.f / (float)a.Wr, y, x);
      iy0[j] = y * a.sy;
      ix0[j] = x * a.sx;
      pix[j] = ((b * a.Hi + iy0[j]) * a.Wi + ix0[j]) * a.Ci;
    } else {
      iy0[j] = -(1 << 20);
      ix0[j] = 0;
      pix[j] = 0;
    }
  }
  const long ldw = (long)a.T * a.cpt * 64;
  // weight rows: the 8-row group g = wave * IB + j of staging instruction j starts at a
  // wave-uniform row; the lane's row q = lane >> 3 inside it and its swizzled chunk are a
  // 32-bit byte offset.  The swizzle of row 8 g + q, (4 g + (q >> 1)) & 7, depends on the group
  // only through its parity.
  const bf16_t* wbase[IB];
  unsigned woff[2];
#pragma unroll
  for (int par = 0; par < 2; ++par)
    woff[par] = (unsigned)(((lane >> 3) * ldw + (((lane & 7) ^ ((4 * par + ((lane >> 3) >> 1)) & 7)) * 8)) * 2);
#pragma unroll
  for (int j = 0; j < IB; ++j) wbase[j] = a.W + (long)(n0 + (wave * IB + j) * 8) * ldw;
  const int cpt = a.cpt;                    // 64-column K-steps per tap
  const int KT = a.T * cpt;

  auto stage = [&](int kt, int slot) {
    const int t = kt / cpt, c0 = (kt - t * cpt) << 6;
    const int dy = (int)((a.tdy >> (4 * t)) & 15) - 8, dx = (int)((a.tdx >> (4 * t)) & 15) - 8;
    const int toff = (dy * a.Wi + dx) * a.Ci + c0;
    char* As = lds + slot * STAGE;
    char* Bs = As + BM * 128;
#pragma unroll
    for (int j = 0; j < IA; ++j) {
      const int iy = iy0[j] + dy + gpy[j], ix = ix0[j] + dx + gpx[j];
      const bool ok = (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
      const void* src = ok ? (const void*)(a.X + (long)(pix[j] + toff) + gca[j]) : (const void*)cv_zero_page;
      cv_glds16(src, As + (wave * IA + j) * 1024);
    }
    const long k0 = (long)t * cpt * 64 + c0;
#pragma unroll
    for (int j = 0; j < IB; ++j) cv_glds16s(wbase[j] + k0, woff[(wave * IB + j) & 1], Bs + (wave * IB + j) * 1024);
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < KT) stage(s, s);

  for (int kt = 0; kt < KT; ++kt) {
    const int ahead = KT - 1 - kt;          // stages issued after kt (capped by the ring)
    cv_wait_stage<G, NS>(ahead < NS - 2 ? ahead : NS - 2);
    cv_bar();
    if (kt + NS - 1 < KT) stage(kt + NS - 1, (kt + NS - 1) % NS);
    const char* As = lds + (kt % NS) * STAGE;
    const char* Bs = As + BM * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      cv_s16x8 fa[MI], fb[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = cv_frag(As, wm * WM + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[j] = cv_frag(Bs, wn * WN + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf16x8_t)fb[j], (bf16x8_t)fa[i], acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue.  acc[i][j][r] = Y[row wm*WM + 16 i + (lane & 15)][col wn*WN + 16 j + 4 (lane >> 4) + r]
  // of the tile.  The bf16 tile goes through LDS so that every lane then stores 16 contiguous
  // bytes and a wave writes whole rows: 8-byte stores of the MFMA layout (4 channels of 16
  // rows per instruction) made the epilogue store-issue-bound.
  constexpr int OROW = BN * 2 + 16;                // padded LDS row: 2-way at most on the b64 writes
  static_assert(BM * OROW <= NS * STAGE, "epilogue LDS");
  constexpr int CPR = BN / 8, RPP = (64 * NW) / CPR;
  const int cc = tid % CPR;
  CvOut<BM / RPP> co;
  cv_out_prefetch<BM, CPR, RPP, EPI>(a, co, m0, n0, tid);
  char* ot = lds;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  cv_bar();                                        // every wave is done reading the ring
  bool rv[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int row = wm * WM + 16 * i + (lane & 15);
    rv[i] = m0 + row < a.M;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      u16x4 out;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        out[r] = f2bf(acc[i][j][r]);
        if constexpr (EPI == 1) acc[i][j][r] = rv[i] ? bf2f(out[r]) : 0.f;   // what BatchNorm will read
      }
      *(u16x4*)(ot + row * OROW + (wn * WN + 16 * j + 4 * (lane >> 4)) * 2) = out;
    }
  }
  if constexpr (EPI == 1) cv_wave_stats<MI, NJ, WM>(a, acc, rv, m0 + wm * WM, n0 + wn * WN, lane);
  __syncthreads();
  // coalesced copy-out: row-major 16-B chunks, BN / 8 lanes per row.
  // EPI 2: the BatchNorm backward's reduction pass rides on the copy-out.  This thread's 8
  // channels are fixed over its rows: it masks dy with the ReLU mask recomputed from the
  // BatchNorm input (what bn_bwd_reduce_kernel mode 2 does), stores the masked dy' and sums
  // dy' and dy' * xhat -- the separate pass re-reading dy and x goes away.
  float bmu[8], bis[8], bfa[8], bfb[8], s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s1[e] = 0.f;
    s2[e] = 0.f;
    if constexpr (EPI == 2) {
      const int c = n0 + cc * 8 + e;
      bmu[e] = a.bnstat[c];
      bis[e] = a.bnstat[a.Co + c];
      bfa[e] = a.bnstat[2 * a.Co + c];
      bfb[e] = a.bnstat[3 * a.Co + c];
    } else {
      bmu[e] = bis[e] = bfa[e] = bfb[e] = 0.f;
    }
  }
  cv_out_store<BM, CPR, RPP, EPI>(a, co, [&](int row) { return ot + row * OROW + cc * 16; }, tid, bfa, bfb, bmu,
                                  bis, s1, s2);
  if constexpr (EPI == 2) {
    // column sums over the tile: [RPP][BN] per set in the (now free) LDS, then one thread per
    // column adds the RPP row slots
    static_assert(2 * RPP * BN * 4 <= NS * STAGE, "EPI 2 reduction LDS");
    float* r1 = (float*)lds;
    float* r2 = r1 + RPP * BN;
    __syncthreads();                               // every lane is done reading ot
    const int slot = tid / CPR;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      r1[slot * BN + cc * 8 + e] = s1[e];
      r2[slot * BN + cc * 8 + e] = s2[e];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += 64 * NW) {
      float t1 = 0.f, t2 = 0.f;
#pragma unroll 8
      for (int q = 0; q < RPP; ++q) {
        t1 += r1[q * BN + c];
        t2 += r2[q * BN + c];
      }
      float* p = a.bnp + (long)(a.bntile0 + tm) * a.Co + n0 + c;
      p[0] = t1;
      p[a.bnp2] = t2;
    }
  }
}

template <int BM, int BN, int WGM, int WGN, int NS, int MINB, int EPI>
__global__ void __launch_bounds__(64 * WGM * WGN, MINB) conv_igemm_kernel(ConvArgs a) {
  conv_igemm_tile<BM, BN, WGM, WGN, NS, EPI>(a, xcd_remap(blockIdx.x, gridDim.x));
}

// Up to four launches of one configuration in ONE grid: the output phases of a strided data
// gradient (4 / 2 / 2 / 1 taps for a 3x3 stride-2 conv), each a short launch of a few hundred
// tiles that left the chip draining between them.  Phase i owns tiles [start[i], start[i+1]);
// its arguments are read from the kernel-argument segment at a wave-uniform index.
constexpr int CV_MAXPH = 4;
struct ConvPhases {
  ConvArgs a[CV_MAXPH];
  int start[CV_MAXPH];
  int n;
};

template <int BM, int BN, int WGM, int WGN, int NS, int MINB, int EPI>
__global__ void __launch_bounds__(64 * WGM * WGN, MINB) conv_igemm_phases_kernel(ConvPhases p) {
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int ph = 0;
#pragma unroll
  for (int i = 1; i < CV_MAXPH; ++i)
    if (i < p.n && L >= p.start[i]) ph = i;
  ph = __builtin_amdgcn_readfirstlane(ph);
  conv_igemm_tile<BM, BN, WGM, WGN, NS, EPI>(p.a[ph], L - p.start[ph]);
}

// ------------------------------------------------------------------------------------------
// Streamed persistent variant of conv_igemm_kernel.  Grid = WPC workgroups per CU (or fewer
// when there are fewer tiles); workgroup w walks the tiles w, w + P, w + 2P, ... of the
// XCD-remapped tile order, and its K-steps form ONE stream over (tile, K-step): the LDS ring
// keeps NS - 1 stages in flight ACROSS tile boundaries, so the next tile's first stages land
// while this tile's epilogue runs.  A 1x1 convolution over 64 channels has ONE K-step per tile
// and the one-tile kernel pays a cold DMA latency plus an idle epilogue for each.
//   * the gather descriptors (pixel bases of the A rows, weight row bases) belong to the tile
//     the DMA cursor is in, recomputed when the cursor crosses a tile boundary;
//   * the epilogue re-lays the bf16 tile through the ring slot the tile's last K-step just
//     read (free until the next step's barrier + issue; 16-B chunks XOR-swizzled by row instead
//     of the padded rows of the one-tile kernel, so the image fits the slot exactly);
//   * epilogue stores and loads are younger than the in-flight DMAs: the counted vmcnt waits
//     of the following K-steps only ever wait for more than they need.
template <int BM, int BN, int WGM, int WGN, int NS, int WPC, int EPI>
__global__ void __launch_bounds__(64 * WGM * WGN, WPC) conv_stream_kernel(ConvArgs a, int P) {
  constexpr int NW = WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 16, NJ = WN / 16;
  constexpr int STAGE = (BM + BN) * 128;
  constexpr int IA = BM / (8 * NW), IB = BN / (8 * NW), G = IA + IB;
  constexpr int CPR = BN / 8, RPP = (64 * NW) / CPR;         // copy-out: 16-B chunks per row, rows per pass
  constexpr int REDB = 16;
  static_assert(IA * 8 * NW == BM && IB * 8 * NW == BN, "tile / wave mismatch");
  static_assert(NS >= 2 && NS <= 4 && WPC * (NS * STAGE + REDB) <= 160 * 1024, "LDS ring");
  static_assert(BM * BN * 2 <= STAGE && (CPR == 8 || CPR == 16), "epilogue image in one ring slot");
  static_assert(EPI != 2 || 2 * RPP * BN * 4 <= STAGE, "EPI 2 reduction in one ring slot");
  __shared__ __attribute__((aligned(1024))) char lds[NS * STAGE + REDB];

  const int ntn = a.Co / BN;
  const int tiles = ((a.M + BM - 1) / BM) * ntn;
  const int wg = blockIdx.x;
  if (wg >= tiles) return;
  const int my_tiles = (tiles - wg + P - 1) / P;
  const int KT = a.T * a.cpt;
  const int total = my_tiles * KT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int HW = a.Hr * a.Wr;
  const long ldw = (long)a.T * a.cpt * 64;
  const int cpt = a.cpt;

  // tile-invariant parts of the gather: the lane's rows inside the tile and their swizzled chunk
  int gpx[IA], gpy[IA];
  unsigned gca[IA];
#pragma unroll
  for (int j = 0; j < IA; ++j) {
    const int row = (wave * IA + j) * 8 + (lane >> 3);
    const int gc = (lane & 7) ^ cv_swz(row);
    cv_chunk_geo(a, gc, gca[j], gpx[j], gpy[j]);
  }
  unsigned woff[2];
#pragma unroll
  for (int par = 0; par < 2; ++par)
    woff[par] = (unsigned)(((lane >> 3) * ldw + (((lane & 7) ^ ((4 * par + ((lane >> 3) >> 1)) & 7)) * 8)) * 2);

  // DMA cursor: tile index cj of this workgroup's sequence, K-step ck inside it, stream index cg
  int cj = 0, ck = 0, cg = 0;
  int pix[IA], iy0[IA], ix0[IA];
  const bf16_t* wbase[IB];
  auto cursor_tile = [&](int j) {
    const int L = xcd_remap(j * P + wg, tiles);
    const int m0 = (L / ntn) * BM, n0 = (L % ntn) * BN;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int m = m0 + (wave * IA + i) * 8 + (lane >> 3);
      if (m < a.M) {
        int b, rem, y, x;
        cv_divmod(m, HW, 1.f / (float)HW, b, rem);
        cv_divmod(rem, a.Wr, 1.f / (float)a.Wr, y, x);
        iy0[i] = y * a.sy;
        ix0[i] = x * a.sx;
        pix[i] = ((b * a.Hi + iy0[i]) * a.Wi + ix0[i]) * a.Ci;
      } else {
        iy0[i] = -(1 << 20);
        ix0[i] = 0;
        pix[i] = 0;
      }
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) wbase[i] = a.W + (long)(n0 + (wave * IB + i) * 8) * ldw;
  };
  auto stage_next = [&]() {
    if (cg >= total) return;
    const int slot = cg % NS;
    const int t = ck / cpt, c0 = (ck - t * cpt) << 6;
    const int dy = (int)((a.tdy >> (4 * t)) & 15) - 8, dx = (int)((a.tdx >> (4 * t)) & 15) - 8;
    const int toff = (dy * a.Wi + dx) * a.Ci + c0;
    char* As = lds + slot * STAGE;
    char* Bs = As + BM * 128;
#pragma unroll
    for (int j = 0; j < IA; ++j) {
      const int iy = iy0[j] + dy + gpy[j], ix = ix0[j] + dx + gpx[j];
      const bool ok = (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
      const void* src = ok ? (const void*)(a.X + (long)(pix[j] + toff) + gca[j]) : (const void*)cv_zero_page;
      cv_glds16(src, As + (wave * IA + j) * 1024);
    }
    const long k0 = (long)t * cpt * 64 + c0;
#pragma unroll
    for (int j = 0; j < IB; ++j) cv_glds16s<true>(wbase[j] + k0, woff[(wave * IB + j) & 1], Bs + (wave * IB + j) * 1024);
    ++cg;
    if (++ck == KT) {
      ck = 0;
      if (++cj < my_tiles) cursor_tile(cj);
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  cursor_tile(0);
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) stage_next();

  int jt = 0, kin = 0;
  for (int g = 0; g < total; ++g) {
    const int ahead = total - 1 - g;
    cv_wait_stage<G, NS>(ahead < NS - 2 ? ahead : NS - 2);
    cv_bar();
    stage_next();
    const char* As = lds + (g % NS) * STAGE;
    const char* Bs = As + BM * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      cv_s16x8 fa[MI], fb[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = cv_frag(As, wm * WM + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[j] = cv_frag(Bs, wn * WN + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf16x8_t)fb[j], (bf16x8_t)fa[i], acc[i][j], 0, 0, 0);
    }
    if (++kin != KT) continue;

    // ---- epilogue of tile jt (same math as conv_igemm_kernel; image in ring slot g % NS)
    kin = 0;
    const int L = xcd_remap(jt * P + wg, tiles);
    const int tm = L / ntn, tn = L % ntn;
    const int m0 = tm * BM, n0 = tn * BN;
    char* ot = lds + (g % NS) * STAGE;
    auto ot_chunk = [&](int row, int chunk) -> char* {
      return ot + row * (BN * 2) + ((chunk ^ ((CPR == 8 ? row >> 1 : row) & (CPR - 1))) << 4);
    };
    CvOut<BM / RPP> co;
    cv_out_prefetch<BM, CPR, RPP, EPI>(a, co, m0, n0, tid);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    cv_bar();                                             // every wave is done reading the slot
    bool rv[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wm * WM + 16 * i + (lane & 15);
      rv[i] = m0 + row < a.M;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        u16x4 out;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          out[r] = f2bf(acc[i][j][r]);
          if constexpr (EPI == 1) acc[i][j][r] = rv[i] ? bf2f(out[r]) : 0.f;
        }
        const int col = wn * WN + 16 * j + 4 * (lane >> 4);
        *(u16x4*)(ot_chunk(row, col >> 3) + (col & 7) * 2) = out;
      }
    }
    if constexpr (EPI == 1) cv_wave_stats<MI, NJ, WM>(a, acc, rv, m0 + wm * WM, n0 + wn * WN, lane);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    cs_sync();
    const int cc = tid % CPR;
    float bmu[8], bis[8], bfa[8], bfb[8], s1[8], s2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] = 0.f;
      s2[e] = 0.f;
      if constexpr (EPI == 2) {
        const int c = n0 + cc * 8 + e;
        bmu[e] = a.bnstat[c];
        bis[e] = a.bnstat[a.Co + c];
        bfa[e] = a.bnstat[2 * a.Co + c];
        bfb[e] = a.bnstat[3 * a.Co + c];
      } else {
        bmu[e] = bis[e] = bfa[e] = bfb[e] = 0.f;
      }
    }
    cv_out_store<BM, CPR, RPP, EPI>(a, co, [&](int row) { return ot_chunk(row, cc); }, tid, bfa, bfb, bmu, bis, s1,
                                    s2);
    if constexpr (EPI == 2) {
      float* r1 = (float*)ot;
      float* r2 = r1 + RPP * BN;
      cs_sync();                                    // every lane is done reading the image
      const int slot = tid / CPR;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        r1[slot * BN + cc * 8 + e] = s1[e];
        r2[slot * BN + cc * 8 + e] = s2[e];
      }
      cs_sync();
      for (int c = tid; c < BN; c += 64 * NW) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll 8
        for (int q = 0; q < RPP; ++q) {
          t1 += r1[q * BN + c];
          t2 += r2[q * BN + c];
        }
        float* pp = a.bnp + (long)(a.bntile0 + tm) * a.Co + n0 + c;
        pp[0] = t1;
        pp[a.bnp2] = t2;
      }
    }
    ++jt;
  }
}

// Workgroups of `kernel` that fit on one CU (registers, LDS), at most `want`.  A persistent grid
// sized for more than fit runs its surplus workgroups only after the first ones have walked all
// their tiles: twice the time (the 8-wave streamed kernel with the BatchNorm-backward epilogue
// needs 157 VGPRs, so 3 waves per SIMD, not the 4 of two 8-wave workgroups per CU).
template <typename K>
static int cs_resident(K kernel, int threads, int want) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, threads, 0) != hipSuccess || n <= 0) return want;
  return std::min(n, want);
}

template <int BM, int BN, int WGM, int WGN, int NS, int WPC, int EPI>
static int cs_go(const ConvArgs& a, long tiles, int cus, hipStream_t s) {
  constexpr int threads = 64 * WGM * WGN;
  static const int per_cu = cs_resident(conv_stream_kernel<BM, BN, WGM, WGN, NS, WPC, EPI>, threads, WPC);
  const int P = (int)std::min<long>(tiles, (long)cus * per_cu);
  conv_stream_kernel<BM, BN, WGM, WGN, NS, WPC, EPI><<<P, threads, 0, s>>>(a, P);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

template <int BM, int BN, int WGM, int WGN, int NS, int WPC, bool WITH_BN = false>
static int cs_launch(const ConvArgs& a, int epi, int cus, hipStream_t s) {
  const long tiles = (long)ceil_div(a.M, BM) * (a.Co / BN);
  if (tiles > (1L << 30)) return 5;
  if (epi == 1) return cs_go<BM, BN, WGM, WGN, NS, WPC, 1>(a, tiles, cus, s);
  if (epi == 2) {
    if constexpr (WITH_BN) return cs_go<BM, BN, WGM, WGN, NS, WPC, 2>(a, tiles, cus, s);
    else return 6;
  }
  return cs_go<BM, BN, WGM, WGN, NS, WPC, 0>(a, tiles, cus, s);
}

// ------------------------------------------------------------------------------------------
// Weight gradient: dW[co][t * Ci + c] = sum_m dY[m][co] * X[pixel(m) + tap_t][c]
// a "TN" GEMM whose reduction runs over the pixels (the row index of both NHWC operands):
//   * BK = 32 pixels per stage; both tiles are staged row-major ([pixel][channel], as in memory)
//     by LDS-DMA and the MFMA fragments, which need 8 consecutive pixels per lane, are read with
//     ds_read_b64_tr_b16 (the transposing LDS read) -- no transpose pass;
//   * the X tile is gathered per 16-byte chunk: the chunk's column fixes its tap, the row fixes
//     the pixel, tracked incrementally per lane (+32 pixels per stage) instead of divided out;
//   * split-K over pixel ranges (the output is small, the reduction is up to 800k pixels deep);
//     fp32 partial slabs [split][co][t * Ci + c] are summed by ct_splitk_reduce.
struct WgradArgs {
  const bf16_t* DY;     // [M][Co]
  const bf16_t* X;      // NHWC [Nb, Hi, Wi, Ci]
  float* P;             // [splits][Co][NN]
  int Hi, Wi, Ci, Hr, Wr, sy, sx;
  int Co, NN, M, T, rows_per_split;
  unsigned long long tdy, tdx;
  int Cw;               // weight columns per tap (= Ci, or 64 in pixel-chunk mode)
  int pixchunk;         // stem: 1 = column c of a tap is pixel step c / 8, channel c % 8 (Ci = 8);
                        //   2 = chunk g = c / 8 is pixels 2 (g & 3), + 1 of kernel row g >> 2 (Ci = 4)
};

template <int LPR>
__device__ __forceinline__ int wg_swz(int r) {
  if constexpr (LPR == 8) return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2);
  else return ((r & 3) << 1) | (((r >> 3) & 1) << 3);
}

typedef __attribute__((ext_vector_type(4))) short wg_s16x4;
typedef __attribute__((address_space(3))) wg_s16x4 wg_lds_s16x4;

// 16 columns [col0, col0 + 16) x 32 pixels of a row-major image with ROWB-byte rows: lane l gets
// column (l & 15), pixels 8 (l >> 4) .. + 8
template <int ROWB>
__device__ __forceinline__ cv_s16x8 wg_frag(const char* img, int col0, int lane) {
  constexpr int LPR = ROWB / 16;
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int r0 = 8 * g + q, r1 = r0 + 4;
  const int ch = (col0 >> 3) + (p >> 1);
  const char* a0 = img + r0 * ROWB + ((ch ^ wg_swz<LPR>(r0)) << 4) + ((p & 1) << 3);
  const char* a1 = img + r1 * ROWB + ((ch ^ wg_swz<LPR>(r1)) << 4) + ((p & 1) << 3);
  const wg_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((wg_lds_s16x4*)a0);
  const wg_s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((wg_lds_s16x4*)a1);
  return cv_s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// LIN: a 1x1 / stride-1 weight gradient, X row = pixel: both operands are linear in the pixel
// index and stream by buffer loads (32-bit offsets, one add per row per stage; rows past the split
// read zeros from the range check) instead of the per-row (b, y, x) gather
template <int BMC, int BNC, int WGM, int WGN, int NS, int BK = 32, bool LIN = false>
__global__ void __launch_bounds__(64 * WGM * WGN, 1) conv_wgrad_kernel(WgradArgs a) {
  // BK pixels per stage (32 or 64: one or two MFMA k-steps per barrier)
  constexpr int NW = WGM * WGN;
  static_assert(BK == 32 || BK == 64, "wgrad stage depth");
  constexpr int ROWA = BMC * 2, ROWB = BNC * 2, LPA = ROWA / 16, LPB = ROWB / 16;
  constexpr int TA = BK * ROWA, TB = BK * ROWB, STG = TA + TB;
  constexpr int GA = TA / (1024 * NW), GB = TB / (1024 * NW), G = GA + GB;
  constexpr int RPA = 64 / LPA, RPB = 64 / LPB;          // rows per DMA instruction
  constexpr int WM = BMC / WGM, WN = BNC / WGN, MI = WM / 16, NJ = WN / 16;
  static_assert(GA * 1024 * NW == TA && GB * 1024 * NW == TB, "wgrad tile / waves");
  static_assert(NS * STG <= 160 * 1024 && NS >= 2 && NS <= 4, "wgrad ring");
  __shared__ __attribute__((aligned(1024))) char lds[NS * STG];

  const int tiles_n = a.NN / BNC, tiles = (a.Co / BMC) * tiles_n;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles, tile = L % tiles;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int c0 = tm * BMC, n0 = tn * BNC;
  const int kbeg = split * a.rows_per_split;
  const int kend = min(a.M, kbeg + a.rows_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;

  // A rows (dY): row r of the stage = pixel kbeg + 32 s + r; fixed column chunk per instruction
  int ra[GA];
  unsigned ga_off[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int r = (wave * GA + j) * RPA + lane / LPA;
    ra[j] = r;
    ga_off[j] = (unsigned)(c0 + (((lane % LPA) ^ wg_swz<LPA>(r)) << 3));
  }
  // B rows (gathered X): per instruction the lane's chunk column -> tap, channel; the pixel
  // (b, y, x) of its row is tracked incrementally
  int rb[GB], bb[GB], yb[GB], xb[GB], dyb[GB], dxb[GB], cib[GB], pxb[GB], pyb[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int r = (wave * GB + j) * RPB + lane / LPB;
    rb[j] = r;
    const int n = n0 + (((lane % LPB) ^ wg_swz<LPB>(r)) << 3);
    const int t = n / a.Cw;
    const int c = n - t * a.Cw;
    cib[j] = a.pixchunk ? (c & 7) : c;
    pxb[j] = a.pixchunk == 2 ? 2 * ((c >> 3) & 3) : (a.pixchunk ? (c >> 3) : 0);
    pyb[j] = a.pixchunk == 2 ? (c >> 5) : 0;
    dyb[j] = (int)((a.tdy >> (4 * t)) & 15) - 8;
    dxb[j] = (int)((a.tdx >> (4 * t)) & 15) - 8;
    const int m = kbeg + r, HW = a.Hr * a.Wr;
    bb[j] = m / HW;
    const int rem = m - bb[j] * HW;
    yb[j] = rem / a.Wr;
    xb[j] = rem - yb[j] * a.Wr;
  }

  // LIN operand streams
  __amdgpu_buffer_rsrc_t rdy, rx;
  unsigned va[GA], vb[GB];
  if constexpr (LIN) {
    rdy = __builtin_amdgcn_make_buffer_rsrc((void*)a.DY, 0, kend * a.Co * 2, 0x00020000);
    rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.X, 0, a.M * a.Ci * 2, 0x00020000);
#pragma unroll
    for (int j = 0; j < GA; ++j) va[j] = (unsigned)((kbeg + ra[j]) * a.Co + (int)ga_off[j]) * 2u;
#pragma unroll
    for (int j = 0; j < GB; ++j) vb[j] = (unsigned)((kbeg + rb[j]) * a.Ci + cib[j]) * 2u;
  }

  auto stage = [&](int s, int slot) {
    char* As = lds + slot * STG;
    char* Bs = As + TA;
    if constexpr (LIN) {
#pragma unroll
      for (int j = 0; j < GA; ++j) {
        cv_bglds16(rdy, va[j], As + (wave * GA + j) * 1024);
        va[j] += BK * a.Co * 2;
      }
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        cv_bglds16(rx, vb[j], Bs + (wave * GB + j) * 1024);
        vb[j] += BK * a.Ci * 2;
      }
      return;
    }
    const int kb = kbeg + s * BK;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int m = kb + ra[j];
      const void* src = m < kend ? (const void*)(a.DY + (long)m * a.Co + ga_off[j]) : (const void*)cv_zero_page;
      cv_glds16(src, As + (wave * GA + j) * 1024);
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int m = kb + rb[j];
      const int iy = yb[j] * a.sy + dyb[j] + pyb[j], ix = xb[j] * a.sx + dxb[j] + pxb[j];
      const bool ok = m < kend && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
      const void* src = ok ? (const void*)(a.X + ((long)(bb[j] * a.Hi + iy) * a.Wi + ix) * a.Ci + cib[j])
                           : (const void*)cv_zero_page;
      cv_glds16(src, Bs + (wave * GB + j) * 1024);
      // advance this row's pixel by one stage (BK pixels)
      int x = xb[j] + BK, y = yb[j], b = bb[j];
      while (x >= a.Wr) { x -= a.Wr; ++y; }
      while (y >= a.Hr) { y -= a.Hr; ++b; }
      xb[j] = x; yb[j] = y; bb[j] = b;
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) stage(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = nk - 1 - kt;
    cv_wait_stage<G, NS>(ahead < NS - 2 ? ahead : NS - 2);
    cv_bar();
    if (kt + NS - 1 < nk) stage(kt + NS - 1, (kt + NS - 1) % NS);
    const char* As = lds + (kt % NS) * STG;
    const char* Bs = As + TA;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      cv_s16x8 fa[MI], fb[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = wg_frag<ROWA>(As + ks * 32 * ROWA, wm * WM + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[j] = wg_frag<ROWB>(Bs + ks * 32 * ROWB, wn * WN + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf16x8_t)fb[j], (bf16x8_t)fa[i], acc[i][j], 0, 0, 0);
    }
  }
  // acc[i][j][r] = dW[c0 + wm*WM + 16 i + (lane & 15)][n0 + wn*WN + 16 j + 4 (lane >> 4) + r]
  float* P = a.P + (long)split * a.Co * a.NN;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const long row = c0 + wm * WM + 16 * i + (lane & 15);
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      *(f32x4*)(P + row * a.NN + n0 + wn * WN + 16 * j + 4 * (lane >> 4)) = acc[i][j];
  }
}

template <int BMC, int BNC, int WGM, int WGN, int NS, int BK = 32, bool LIN = false>
static int wg_launch(const WgradArgs& a, int splits, hipStream_t s) {
  const long blocks = (long)(a.Co / BMC) * (a.NN / BNC) * splits;
  if (blocks > (1L << 30)) return 5;
  conv_wgrad_kernel<BMC, BNC, WGM, WGN, NS, BK, LIN><<<(int)blocks, 64 * WGM * WGN, 0, s>>>(a);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

// Weight gradient of a 3x3 / pad 1 convolution (stride 1 or 2) with ALL NINE TAPS in one workgroup:
// tile = 64 output channels x (9 taps x 64 input channels).  The generic kernel above gives each
// tap its own 64 x 64 tile, so every 32-pixel stage moved 8 KB for 16 MFMAs per workgroup and
// re-fetched dY once per tap: at ResNet-50's 64-channel layer-1 shape (802,816 pixels) it ran
// at ~0.2 PF/s, latency-bound behind one barrier per tiny stage.  Here a stage is dY [32 px][64
// co] (4 KB) + the nine shifted X tiles [32 px][64 ci] (36 KB): 36 MFMAs per wave per barrier,
// dY fetched once.
//   * wave w stages pixel rows 8 w .. 8 w + 7 of every tile (one 1 KB LDS-DMA per tile), so a
//     lane tracks ONE pixel; the loads are buffer loads whose range check supplies the zeros:
//     dY's range ends at the split's last row, X's at the tensor end, and a tap that leaves the
//     image (four border masks per stage) gets an offset past the range.  Per tap that is one
//     add and one select -- the 64-bit gather addressing of the first version spent ~140 VALU
//     per stage and ran at 3,100 wave-cycles per 576-cycle MFMA stage;
//   * for the MFMAs wave w owns input channels 16 w .. 16 w + 15 of all nine taps and all 64
//     output channels: acc[4 co blocks][9 taps] = 144 accumulator registers;
//   * fp32 partial slabs [split][Co][9 * Ci] as the generic kernel (same reduce).
template <int NS>
__global__ void __launch_bounds__(256, 2) conv_wgrad3x3_kernel(WgradArgs a) {
  constexpr int BK = 32, TT = BK * 128, STG = 10 * TT;   // dY + 9 tap tiles, 4 KB each
  static_assert(NS * STG <= 160 * 1024, "wgrad3x3 ring");
  __shared__ __attribute__((aligned(1024))) char lds[NS * STG];
  const int ci_tiles = a.Ci / 64, tiles = (a.Co / 64) * ci_tiles;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles, tile = L % tiles;
  const int c0 = (tile / ci_tiles) * 64, ci0 = (tile % ci_tiles) * 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // output pixel grid Hr x Wr at stride sd (1 or 2) over the Hi x Wi input
  const int Hi = a.Hi, Wi = a.Wi, Hr = a.Hr, Wr = a.Wr, sd = a.sy;
  const int kbeg = split * a.rows_per_split;
  const int kend = min(a.M, kbeg + a.rows_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;

  const int r = wave * 8 + (lane >> 3);
  const int chunk = ((lane & 7) ^ wg_swz<8>(r)) << 3;
  const int nimg = a.M / (Hr * Wr);
  const __amdgpu_buffer_rsrc_t rdy = __builtin_amdgcn_make_buffer_rsrc((void*)a.DY, 0, kend * a.Co * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.X, 0, nimg * Hi * Wi * a.Ci * 2, 0x00020000);
  unsigned vdy = (unsigned)((kbeg + r) * a.Co + c0 + chunk) * 2u;
  const unsigned sdy = BK * a.Co * 2, xcol = (unsigned)(ci0 + chunk) * 2u;
  const int rowb = Wi * a.Ci * 2, colb = a.Ci * 2;
  const int ay = BK / Wr, ax = BK - (BK / Wr) * Wr;   // per-stage pixel advance
  int pb, py, px;
  {
    const int m = kbeg + r;
    pb = m / (Hr * Wr);
    const int rem = m - pb * Hr * Wr;
    py = rem / Wr;
    px = rem - py * Wr;
  }

  auto stage = [&](int slot) {
    char* S = lds + slot * STG + wave * 1024;
    cv_bglds16(rdy, vdy, S);
    const int iy = sd * py, ix = sd * px;               // the centre tap's input pixel
    const unsigned vx = (unsigned)(((pb * Hi + iy) * Wi + ix) * a.Ci) * 2u + xcol;
    const bool top = iy > 0, bot = iy < Hi - 1, lef = ix > 0, rig = ix < Wi - 1;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dy = t / 3 - 1, dx = t % 3 - 1;
      const bool ok = (dy < 0 ? top : (dy > 0 ? bot : true)) && (dx < 0 ? lef : (dx > 0 ? rig : true));
      const unsigned off = vx + (unsigned)(dy * rowb + dx * colb);
      cv_bglds16(rx, ok ? off : 0x80000000u, S + (1 + t) * TT);
    }
    vdy += sdy;
    px += ax;
    py += ay;
    if (px >= Wr) { px -= Wr; ++py; }
    while (py >= Hr) { py -= Hr; ++pb; }
  };

  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) stage(s);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = nk - 1 - kt;
    cv_wait_stage<10, NS>(ahead < NS - 2 ? ahead : NS - 2);
    cv_bar();
    if (kt + NS - 1 < nk) stage((kt + NS - 1) % NS);
    const char* As = lds + (kt % NS) * STG;
    cv_s16x8 fa[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = wg_frag<128>(As, 16 * i, lane);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const cv_s16x8 fb = wg_frag<128>(As + (1 + t) * TT, 16 * wave, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf16x8_t)fb, (bf16x8_t)fa[i], acc[i][t], 0, 0, 0);
    }
  }
  // acc[i][t][q] = dW[c0 + 16 i + (lane & 15)][t * Ci + ci0 + 16 wave + 4 (lane >> 4) + q]
  float* P = a.P + (long)split * a.Co * a.NN;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long row = c0 + 16 * i + (lane & 15);
#pragma unroll
    for (int t = 0; t < 9; ++t)
      *(f32x4*)(P + row * a.NN + t * a.Ci + ci0 + 16 * wave + 4 * (lane >> 4)) = acc[i][t];
  }
}

// Chan merge of per-tile (mean, M2) partials -> per-channel mean and biased variance, in
// fp64 (tiles x channels is small).  One thread per channel.
__global__ void bn_partials_finalize_kernel(const float* __restrict__ part, int tiles, int rows_per_tile, int M,
                                            int C, float* __restrict__ mean_out, float* __restrict__ var_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int t = 0; t < tiles; ++t) {
    const double nb = (double)min(rows_per_tile, M - t * rows_per_tile);
    const double mb = part[(long)t * C + c], qb = part[((long)tiles + t) * C + c];
    const double nn = n + nb, d = mb - mean;
    mean += d * nb / nn;
    m2 += qb + d * d * n * nb / nn;
    n = nn;
  }
  mean_out[c] = (float)mean;
  var_out[c] = (float)(m2 / n);
}

// conv_batch_begin() .. conv_batch_end(): the one-tile launches issued in between are collected
// (same configuration, at most CV_MAXPH) and run as ONE conv_igemm_phases_kernel grid
struct CvBatch {
  bool on = false;
  int n = 0, cfg = -1, epi = -1, bm = 0, bn = 0;
  ConvArgs a[CV_MAXPH];
  int (*launch)(const ConvPhases&, int, long, hipStream_t) = nullptr;
};
static thread_local CvBatch g_cv_batch;

template <int BM, int BN, int WGM, int WGN, int NS, int MINB, bool WITH_BN>
static int cv_phases_launch(const ConvPhases& p, int epi, long tiles, hipStream_t s) {
  if (epi == 2) {
    if constexpr (WITH_BN)
      conv_igemm_phases_kernel<BM, BN, WGM, WGN, NS, MINB, 2><<<(int)tiles, 64 * WGM * WGN, 0, s>>>(p);
    else
      return 6;
  } else if (epi == 0) {
    conv_igemm_phases_kernel<BM, BN, WGM, WGN, NS, MINB, 0><<<(int)tiles, 64 * WGM * WGN, 0, s>>>(p);
  } else {
    return 6;
  }
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

template <int BM, int BN, int WGM, int WGN, int NS, int MINB, bool WITH_BN = false>
static int cv_launch(const ConvArgs& a, int epi, hipStream_t s, int cfg = -1) {
  const long tiles = (long)ceil_div(a.M, BM) * (a.Co / BN);
  if (tiles > (1L << 30)) return 5;
  CvBatch& B = g_cv_batch;
  if (B.on && cfg >= 0 && epi != 1) {
    // queued: validated here, launched by conv_batch_end
    if (B.n == CV_MAXPH || (B.n && (B.cfg != cfg || B.epi != epi))) return 10;
    B.cfg = cfg;
    B.epi = epi;
    B.bm = BM;
    B.bn = BN;
    B.launch = &cv_phases_launch<BM, BN, WGM, WGN, NS, MINB, true>;
    B.a[B.n++] = a;
    return 0;
  }
  if (epi == 1)
    conv_igemm_kernel<BM, BN, WGM, WGN, NS, MINB, 1><<<(int)tiles, 64 * WGM * WGN, 0, s>>>(a);
  else if (epi == 2) {
    if constexpr (WITH_BN) conv_igemm_kernel<BM, BN, WGM, WGN, NS, MINB, 2><<<(int)tiles, 64 * WGM * WGN, 0, s>>>(a);
    else return 6;
  } else
    conv_igemm_kernel<BM, BN, WGM, WGN, NS, MINB, 0><<<(int)tiles, 64 * WGM * WGN, 0, s>>>(a);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

}  // namespace ct

using namespace ct;

// tile configurations (BM x BN, waves, LDS ring slots, workgroups per CU):
//   0: 256x64  4w NS3      1: 256x128 8w NS3      2: 128x128 4w NS4      3: 128x64 4w NS4
//   4: 256x64  4w NS2 x2   5: 128x128 4w NS2 x2   6: 256x64  8w NS3      7: 128x64 4w NS2 x2
//   8: 128x64  4w NS2 x3   9: 64x128  4w NS2 x3
// streamed persistent (conv_stream_kernel; workgroups per CU, ring slots):
//  10: 128x128 4w NS4 x1  11: 128x128 4w NS2 x2  12: 128x64 4w NS3 x2  13: 64x128 4w NS3 x2
// 8 waves (2 x 4, 64 x 32 per wave: twice the waves per CU to hide LDS / memory latency):
//  14: 128x128 8w NS2 x2 (one tile per workgroup)   15: the same, streamed
//  16: 128x64 8w (4 x 2, 32 x 32 per wave) NS2 x2    17: 128x64 8w NS3 x2, streamed (no EPI 2:
//      its reduction scratch does not fit a ring slot)
//  18: 256x128 16w (4 x 4, 64 x 32 per wave) NS2 x1
// -1 = pick by shape: short reductions (<= 4 K-steps of 64) want two workgroups per CU so one
// tile's epilogue overlaps another's loads; long ones want the deeper ring.
extern "C" int ct_conv_igemm_rows(int cfg, int Co, int M, int KT) {
  // measured on MI355X over every ResNet-50 shape at batch 256 (bench/conv_igemm_probe.py,
  // profiles/r3/conv_igemm.md): small tiles with 2-3 workgroups per CU win everywhere; the
  // 1-workgroup configurations (deeper ring) never do
  // r4: the streamed 128 x 128 kernel (cfg 11, two persistent workgroups per CU) wins on the
  // large-M layers (every ResNet-50 launch with M >= 200704 output rows and Co % 128 == 0:
  // l2.c1a fwd 145 -> 128 us, dgrad 197 -> 169; l2.c2 dgrad 96 -> 85) and loses on the
  // 50176-row layer-3/4 launches (profiles/r4/conv_stream_probe.md)
  // r4, later: the 8-wave 128 x 128 tiles (cfg 14 one-tile, 15 streamed: twice the waves per CU
  // to hide LDS and memory latency) beat the 4-wave ones on every Co % 128 == 0 shape: one-tile
  // below 400000 rows (l3.c2 fwd 77 -> 73 us, l4.c2s2 dgrad 127 -> 116), streamed above
  // (l1.c3 fwd 115 -> 112; profiles/r4/conv_cfg_8wave.md).  CLOUDTIK_AMD_CONV_RULE=1: the rule
  // before that.  r6: the 256 x 128 16-wave tiles (cfg 18), fastest alone on several layer-3/4
  // shapes, cost 1 ms in the step (20.45 -> 21.5 ms, profiles/r6/conv_cfg_probe.md): rejected.
  static const int rule = [] {
    const char* e = std::getenv("CLOUDTIK_AMD_CONV_RULE");
    return e ? std::atoi(e) : 2;
  }();
  (void)KT;
  if (cfg < 0) {
    if (rule >= 2 && Co % 128 == 0) return M >= 400000 ? 15 : 14;
    if (Co % 128 == 0 && M >= 150000) return 11;
    cfg = Co % 128 ? 8 : (Co == 128 ? 9 : 5);
  }
  return cfg;
}

// rows per BatchNorm-statistics partial (EPI 1 writes one per wave row block: BM / WGM)
extern "C" int ct_conv_igemm_part_rows(int cfg) {
  return (cfg == 6 || cfg == 16 || cfg == 17) ? 32 : 64;
}

extern "C" int ct_conv_igemm_tile_m(int cfg) {
  return (cfg == 0 || cfg == 1 || cfg == 4 || cfg == 6 || cfg == 18) ? 256 : ((cfg == 9 || cfg == 13) ? 64 : 128);
}

static int g_cv_stream_cus = 0;      // test / probe override of the streamed kernels' CU count

static int cv_cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    return v;
  }();
  return g_cv_stream_cus > 0 ? g_cv_stream_cus : n;
}

// streamed conv kernels: workgroups = cus x (workgroups per CU); 0 restores the device's CU count
extern "C" void ct_conv_stream_set_cus(int cus) { g_cv_stream_cus = cus > 0 ? cus : 0; }

// Y = implicit-GEMM conv (see the file comment).  `taps` = T (dy, dx) pairs in [-8, 7].
// Returns nonzero (launching nothing) on an unsupported shape.
// EPI 2 arguments of ct_conv_igemm_bn (NULL bnx: a plain launch)
struct ConvBnBwd {
  const void* bnx;
  const void* bny;
  const void* bnm;
  const float* bnstat;
  float* bnp;
  long bnp2;
  int tile0;
};

static int conv_igemm_impl(const void* X, int Hi, int Wi, int Ci, const void* W, void* Y, int Hr, int Wr, int sy,
                           int sx, int Ho, int Wo, int oys, int oxs, int oy0, int ox0, int ldy, int Co, int M, int T,
                           const int* taps, int accumulate, float* part, int cfg, const ConvBnBwd* bn,
                           hipStream_t stream);

extern "C" int ct_conv_igemm(const void* X, int Hi, int Wi, int Ci, const void* W, void* Y, int Hr, int Wr, int sy,
                             int sx, int Ho, int Wo, int oys, int oxs, int oy0, int ox0, int ldy, int Co, int M,
                             int T, const int* taps, int accumulate, float* part, int cfg, hipStream_t stream) {
  return conv_igemm_impl(X, Hi, Wi, Ci, W, Y, Hr, Wr, sy, sx, Ho, Wo, oys, oxs, oy0, ox0, ldy, Co, M, T, taps,
                         accumulate, part, cfg, nullptr, stream);
}

// data gradient whose output feeds a BatchNorm + ReLU backward (mask from x): Y = masked dy,
// per-tile sums of dy' and dy' * xhat into bnp rows [tile0, tile0 + tiles) (and bnp + bnp2)
extern "C" int ct_conv_igemm_bn(const void* X, int Hi, int Wi, int Ci, const void* W, void* Y, int Hr, int Wr, int sy,
                                int sx, int Ho, int Wo, int oys, int oxs, int oy0, int ox0, int ldy, int Co, int M,
                                int T, const int* taps, int accumulate, int cfg, const void* bnx, const void* bny,
                                const void* bnm, const float* bnstat, float* bnp, long bnp2, int tile0,
                                hipStream_t stream) {
  if (!bnx || !bnstat || !bnp || ((uintptr_t)bnx & 15) || ((uintptr_t)bny & 15) || ((uintptr_t)Y & 15) || ldy % 8)
    return 8;
  const ConvBnBwd bn{bnx, bny, bnm, bnstat, bnp, bnp2, tile0};
  return conv_igemm_impl(X, Hi, Wi, Ci, W, Y, Hr, Wr, sy, sx, Ho, Wo, oys, oxs, oy0, ox0, ldy, Co, M, T, taps,
                         accumulate, nullptr, cfg, &bn, stream);
}

static int conv_igemm_impl(const void* X, int Hi, int Wi, int Ci, const void* W, void* Y, int Hr, int Wr, int sy,
                           int sx, int Ho, int Wo, int oys, int oxs, int oy0, int ox0, int ldy, int Co, int M, int T,
                           const int* taps, int accumulate, float* part, int cfg, const ConvBnBwd* bn,
                           hipStream_t stream) {
  // (M < 2^24: the epilogue's float-reciprocal row division, cv_divmod)
  if (Ci <= 0 || (Ci % 64 && Ci != 8 && Ci != 4) || Co <= 0 || Co % 64 || M <= 0 || M >= (1 << 24) || T <= 0 ||
      T > CV_MAXT)
    return 1;
  // pair mode: every 16-byte chunk starts at an even pixel of an even-width row
  if (Ci == 4 && (Wi % 2 || sx % 2)) return 1;
  if (((uintptr_t)X & 15) || ((uintptr_t)W & 15) || ((uintptr_t)Y & 7) || ldy % 4) return 3;
  // zero-filling mode: exactly the (even, even) phase of a stride-2 output grid, 16-B rows
  if (accumulate == 2 && (Ho != 2 * Hr || Wo != 2 * Wr || oys != 2 || oxs != 2 || oy0 || ox0 || bn ||
                          ((uintptr_t)Y & 15) || ldy % 8))
    return 9;
  const int pixchunk = Ci == 8 ? 1 : (Ci == 4 ? 2 : 0);   // the stem: NHWC8 / NHWC4 input
  ConvArgs a{(const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, part, Hi, Wi, Ci, Hr, Wr, sy, sx,
             Ho, Wo, oys, oxs, oy0, ox0, ldy, Co, M, T, accumulate, 0ull, 0ull, pixchunk ? 1 : Ci / 64, pixchunk,
             nullptr, nullptr, nullptr, nullptr, 0, 0};
  a.dense_out = (Ho == Hr && Wo == Wr && oys == 1 && oxs == 1 && oy0 == 0 && ox0 == 0) ? 1 : 0;
  if (bn) {
    a.bnx = (const bf16_t*)bn->bnx;
    a.bny = (const bf16_t*)bn->bny;
    a.bnm = (const uint8_t*)bn->bnm;
    a.bnstat = bn->bnstat;
    a.bnp = bn->bnp;
    a.bnp2 = bn->bnp2;
    a.bntile0 = bn->tile0;
  }
  for (int t = 0; t < T; ++t) {
    const int dy = taps[2 * t], dx = taps[2 * t + 1];
    if (dy < -8 || dy > 7 || dx < -8 || dx > 7) return 4;
    a.tdy |= (unsigned long long)(dy + 8) << (4 * t);
    a.tdx |= (unsigned long long)(dx + 8) << (4 * t);
  }
  const int epi = bn ? 2 : (part ? 1 : 0);
  const bool autocfg = cfg < 0;
  cfg = ct_conv_igemm_rows(cfg, Co, M, T * a.cpt);
  // the 8-wave streamed kernel's BatchNorm-backward variant holds one workgroup per CU (157
  // VGPRs): the one-tile kernel at two per CU is faster there (l2.c1a dgrad 521 -> 281 us,
  // profiles/r4/conv_epi2_occupancy.md)
  static const bool epi2_stream = [] {
    const char* e = std::getenv("CLOUDTIK_AMD_CONV_EPI2_STREAM");
    return e && std::atoi(e) == 1;
  }();
  if (autocfg && epi == 2 && cfg == 15 && !epi2_stream) cfg = 14;
  if ((cfg == 1 || cfg == 2 || cfg == 5 || cfg == 9 || cfg == 10 || cfg == 11 || cfg == 13 || cfg == 14 ||
       cfg == 15 || cfg == 18) && Co % 128)
    return 2;
  if (epi == 2) {
    // the default (shape-picked) configurations only: the others are not instantiated with EPI 2
    switch (cfg) {
      case 5: return cv_launch<128, 128, 2, 2, 2, 2, true>(a, epi, stream);
      case 8: return cv_launch<128, 64, 2, 2, 2, 3, true>(a, epi, stream);
      case 9: return cv_launch<64, 128, 1, 4, 2, 3, true>(a, epi, stream);
      case 10: return cs_launch<128, 128, 2, 2, 4, 1, true>(a, epi, cv_cu_count(), stream);
      case 11: return cs_launch<128, 128, 2, 2, 2, 2, true>(a, epi, cv_cu_count(), stream);
      case 12: return cs_launch<128, 64, 2, 2, 3, 2, true>(a, epi, cv_cu_count(), stream);
      case 13: return cs_launch<64, 128, 1, 4, 3, 2, true>(a, epi, cv_cu_count(), stream);
      case 14: return cv_launch<128, 128, 2, 4, 2, 2, true>(a, epi, stream, 14);
      case 15: return cs_launch<128, 128, 2, 4, 2, 2, true>(a, epi, cv_cu_count(), stream);
      case 16: return cv_launch<128, 64, 4, 2, 2, 2, true>(a, epi, stream);
      case 18: return cv_launch<256, 128, 4, 4, 2, 1, true>(a, epi, stream);
      default: return 6;
    }
  }
  switch (cfg) {
    case 0: return cv_launch<256, 64, 4, 1, 3, 1>(a, epi, stream);
    case 1: return cv_launch<256, 128, 4, 2, 3, 1>(a, epi, stream);
    case 2: return cv_launch<128, 128, 2, 2, 4, 1>(a, epi, stream);
    case 3: return cv_launch<128, 64, 2, 2, 4, 1>(a, epi, stream);
    case 4: return cv_launch<256, 64, 4, 1, 2, 2>(a, epi, stream);
    case 5: return cv_launch<128, 128, 2, 2, 2, 2>(a, epi, stream);
    case 6: return cv_launch<256, 64, 8, 1, 3, 1>(a, epi, stream);
    case 7: return cv_launch<128, 64, 2, 2, 2, 2>(a, epi, stream);
    case 8: return cv_launch<128, 64, 2, 2, 2, 3>(a, epi, stream);
    case 9: return cv_launch<64, 128, 1, 4, 2, 3>(a, epi, stream);
    case 10: return cs_launch<128, 128, 2, 2, 4, 1>(a, epi, cv_cu_count(), stream);
    case 11: return cs_launch<128, 128, 2, 2, 2, 2>(a, epi, cv_cu_count(), stream);
    case 12: return cs_launch<128, 64, 2, 2, 3, 2>(a, epi, cv_cu_count(), stream);
    case 13: return cs_launch<64, 128, 1, 4, 3, 2>(a, epi, cv_cu_count(), stream);
    case 14: return cv_launch<128, 128, 2, 4, 2, 2, true>(a, epi, stream, 14);
    case 15: return cs_launch<128, 128, 2, 4, 2, 2>(a, epi, cv_cu_count(), stream);
    case 16: return cv_launch<128, 64, 4, 2, 2, 2>(a, epi, stream);
    case 17: return cs_launch<128, 64, 4, 2, 3, 2>(a, epi, cv_cu_count(), stream);
    case 18: return cv_launch<256, 128, 4, 4, 2, 1>(a, epi, stream);
    default: return 6;
  }
}

// ---- data-gradient weight matrices of many convs in one launch (ops/conv.py _DgradWeights):
// dst[ci][t][co] = src[co][r_t][s_t][ci] (channels_last weights [Co][R][S][Ci] -> the dgrad
// operand [Ci][taps * Co]).  One workgroup = one 64 x 64 (co, ci) tile of one tap of one conv,
// described by 8 ints: src offset (elements), dst offset, Co, Ci, R * S * Ci (src row stride),
// tap source offset (r * S + s) * Ci, tap index t, number of taps T, and its first (co0, ci0).
// Transposed through LDS: 16-B reads along ci, 16-B writes along co (the element gather it
// replaces read one 2-B element per 64-B line, plus an index per element).
__global__ __launch_bounds__(256) void dgrad_wgather_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                            const int* __restrict__ desc) {
  __shared__ unsigned short tile[64][64 + 8];
  const int* d = desc + (long)blockIdx.x * 10;
  const long soff = (long)d[0] * 65536 + d[1];   // offsets as (hi, lo) pairs of 16 bits
  const long doff = (long)d[2] * 65536 + d[3];
  const int Co = d[4], Ci = d[5], srow = d[6], tapoff = d[7], t = d[8], T = d[9] & 0xFFFF;
  const int co0 = (d[9] >> 16) & 0xFF, ci0b = (d[9] >> 24) & 0xFF;
  const int cob = co0 * 64, cib = ci0b * 64;
  const int tid = threadIdx.x;
  // load: 64 co rows x 64 ci (8 chunks of 8 per row): 512 chunks, 2 per thread
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = tid + 256 * k, row = c >> 3, ch = c & 7;
    const u16x8 v = *reinterpret_cast<const u16x8*>(src + soff + (long)(cob + row) * srow + tapoff + cib + ch * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) tile[row][ch * 8 + e] = v[e];
  }
  __syncthreads();
  // store: 64 ci rows x 64 co (8 chunks of 8 per row) at dst[ci][t][co]
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = tid + 256 * k, row = c >> 3, ch = c & 7;
    u16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = tile[ch * 8 + e][row];
    *reinterpret_cast<u16x8*>(dst + doff + ((long)(cib + row) * T + t) * Co + cob + ch * 8) = v;
  }
}

extern "C" int ct_dgrad_wgather(const void* src, void* dst, const int* desc, int ntiles, hipStream_t stream) {
  if (ntiles <= 0) return 0;
  dgrad_wgather_kernel<<<ntiles, 256, 0, stream>>>((const bf16_t*)src, (bf16_t*)dst, desc);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

// ---- stem input: [N, C <= 8, H, W] (NCHW, or any strides) bf16 -> NHWC with the channels
// zero-padded to 8 (16 bytes per pixel), in one pass: one thread per pixel reads its C values
// (pixel-contiguous across the wave for NCHW) and writes one 16-B chunk (the pad-then-copy form
// wrote the 205 MB ResNet-50 batch twice)
template <int CP>
__global__ __launch_bounds__(256) void to_nhwc8_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long npix,
                                                       int C, int H, int W, long sn, long sc, long sh, long sw) {
  typedef __attribute__((ext_vector_type(CP))) unsigned short vec_t;
  const long p = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const long hw = (long)H * W;
  const long n = p / hw, r = p - n * hw;
  const int h = (int)(r / W), w = (int)(r - (long)h * W);
  const bf16_t* src = x + n * sn + h * sh + w * sw;
  vec_t v = vec_t(0);
  for (int c = 0; c < C; ++c) v[c] = reinterpret_cast<const unsigned short*>(src)[c * sc];
  reinterpret_cast<vec_t*>(y)[p] = v;
}

// CP = 8 (16 bytes per pixel) or 4 (8 bytes: the pair-chunk stem mode, C <= 4)
extern "C" int ct_to_nhwc8(const void* x, void* y, int N, int C, int H, int W, long sn, long sc, long sh, long sw,
                           int CP, hipStream_t stream) {
  if (C < 1 || C > CP || (CP != 8 && CP != 4)) return 1;
  const long npix = (long)N * H * W;
  if (npix <= 0) return 0;
  const unsigned grid = (unsigned)((npix + 255) / 256);
  if (CP == 8)
    to_nhwc8_kernel<8><<<grid, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, npix, C, H, W, sn, sc, sh, sw);
  else
    to_nhwc8_kernel<4><<<grid, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, npix, C, H, W, sn, sc, sh, sw);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

// conv_batch_begin / conv_batch_end (see CvBatch).  A configuration the batch cannot hold (not
// a one-tile 8-wave 128 x 128 launch, or a second configuration) is launched directly as usual;
// end returns nonzero if a queued launch failed.
extern "C" void ct_conv_batch_begin() {
  g_cv_batch.on = true;
  g_cv_batch.n = 0;
  g_cv_batch.cfg = g_cv_batch.epi = -1;
}

extern "C" int ct_conv_batch_end(hipStream_t stream) {
  CvBatch& B = g_cv_batch;
  B.on = false;
  if (!B.n) return 0;
  ConvPhases p{};
  // the longest reductions first: their tiles are dispatched early, the short ones fill the tail
  int order[CV_MAXPH];
  for (int i = 0; i < B.n; ++i) order[i] = i;
  for (int i = 1; i < B.n; ++i)
    for (int j = i; j > 0 && B.a[order[j]].T > B.a[order[j - 1]].T; --j) std::swap(order[j], order[j - 1]);
  long tiles = 0;
  for (int i = 0; i < B.n; ++i) {
    p.a[i] = B.a[order[i]];
    p.start[i] = (int)tiles;
    tiles += (long)ceil_div(p.a[i].M, B.bm) * (p.a[i].Co / B.bn);
  }
  for (int i = B.n; i < CV_MAXPH; ++i) p.start[i] = (int)tiles;
  p.n = B.n;
  const int n = B.n;
  B.n = 0;
  if (tiles > (1L << 30)) return 5;
  if (n == 1) {
    // one launch: the plain kernel (same tile code)
    if (B.epi == 2) conv_igemm_kernel<128, 128, 2, 4, 2, 2, 2><<<(int)tiles, 512, 0, stream>>>(p.a[0]);
    else conv_igemm_kernel<128, 128, 2, 4, 2, 2, 0><<<(int)tiles, 512, 0, stream>>>(p.a[0]);
    return hipGetLastError() == hipSuccess ? 0 : 7;
  }
  return B.launch(p, B.epi, tiles, stream);
}

extern "C" int ct_bn_partials_finalize(const float* part, int tiles, int rows_per_tile, int M, int C, float* mean,
                                       float* var, hipStream_t stream) {
  bn_partials_finalize_kernel<<<ceil_div(C, 256), 256, 0, stream>>>(part, tiles, rows_per_tile, M, C, mean, var);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

// Sum of S fp32 slabs [S][n] into a bf16 vector (+= when accumulate), parallel over the slabs
// as well: block (x, y) adds slabs [32 y, 32 y + 32) of elements [1024 x, 1024 x + 1024) into an
// fp32 accumulator with atomics (at most S / 32 adders per address), and the last block of each
// column (arrival ticket) converts that element range to bf16.
__global__ void __launch_bounds__(256) splitk_wide_kernel(const float* __restrict__ P, int S, long n, float* acc,
                                                         unsigned* tickets, bf16_t* __restrict__ out, int accumulate) {
  const long e = (long)blockIdx.x * 1024 + threadIdx.x * 4;
  const int s0 = blockIdx.y * 32, s1 = min(S, s0 + 32);
  if (e + 3 < n) {
    // eight slabs' loads in flight per round (a rolled loop waited one memory latency per slab:
    // ~36 us for 128 slabs of a 64 x 576 gradient)
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    int s = s0;
    for (; s + 8 <= s1; s += 8) {
      f32x4 t[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] = *(const f32x4*)(P + (long)(s + k) * n + e);
#pragma unroll
      for (int k = 0; k < 8; ++k) v += t[k];
    }
    for (; s < s1; ++s) v += *(const f32x4*)(P + (long)s * n + e);
#pragma unroll
    for (int r = 0; r < 4; ++r) atomicAdd(acc + e + r, v[r]);
  } else {
    for (long i = e; i < n && i < e + 4; ++i) {
      float v = 0.f;
      for (int s = s0; s < s1; ++s) v += P[(long)s * n + i];
      atomicAdd(acc + i, v);
    }
  }
  // publish: every wave's atomics are done before the ticket (agent-scope release/acquire)
  __shared__ unsigned last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(tickets + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           gridDim.y - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  for (long i = e; i < n && i < e + 4; ++i) {
    const float v = __hip_atomic_load(acc + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    out[i] = f2bf(accumulate ? v + bf2f(out[i]) : v);
  }
}

// wgrad tile configurations: 0 = 64x64 (4 waves 2x2), 1 = 64x128 (2x2), 2 = 128x128 (2x2),
// 3 = 128x256 (8 waves 2x4); 4 / 5 / 6 = cfg 0 / 1 / 2 with 64-pixel stages (two MFMA k-steps per
// barrier); 7 / 8 = cfg 4 with a 2 / 3-slot ring (more workgroups per CU); 9 / 10 = 128x128 on 8
// waves (2x4), 32-pixel stages x 4 slots / 64-pixel x 2; 11 = 128x256 on 16 waves (4x4), 64-pixel
// stages x 2; 12 / 13 = the nine-tap 3x3 kernel (64 co x 9 x 64 ci) with a 3 / 2-slot ring;
// -1 = the largest that divides (Co, T*Ci)
extern "C" int ct_conv_wgrad_cfg(int cfg, int Co, int NN) {
  if (cfg >= 0) return cfg;
  // per-shape probe over every ResNet-50 conv (profiles/r3/conv_wgrad_cfg.md): the 8-wave
  // 128 x 256 tile wins wherever it divides (l4.c2 357 -> 146 us, l3.c2 183 -> 111 us), then
  // 128 x 128, then 64 x 128 for 64-channel outputs (l1.c1 163 -> 128 us)
  // r4: the 8-wave 128 x 128 tile (cfg 9) beats the 4-wave one everywhere and the 8-wave
  // 128 x 256 one for 128-channel outputs (l2.c2 185 -> 130 us, l2.c3 90 -> 69;
  // profiles/r4/conv_cfg_8wave.md)
  // CLOUDTIK_AMD_WGRAD_RULE=2: the 16-wave 128 x 256 tile with 64-pixel stages (cfg 11) instead
  // of cfg 3.  Faster alone on every 256+-channel shape it divides (l3.c2 110 -> 91 us, l4.c2
  // 146 -> 123, l3.down 101 -> 85) but SLOWER in the ResNet-50 step (22.79 -> 23.06 ms): a
  // 1024-thread workgroup on the gradient side stream cannot share a CU with the data-gradient
  // kernels it is meant to overlap (profiles/r4/conv_wgrad_split.md)
  static const int rule = [] {
    const char* e = std::getenv("CLOUDTIK_AMD_WGRAD_RULE");
    return e ? std::atoi(e) : 1;
  }();
  if (Co % 128 == 0 && NN % 256 == 0 && Co >= 256) return rule >= 2 ? 11 : 3;
  if (Co % 128 == 0 && NN % 128 == 0) return 9;
  // CLOUDTIK_AMD_WGRAD_WIDE=1: 64 x 256 tiles for 64-output-channel gradients with 256+ columns
  // (layer-1 256 -> 64 1x1 convs: dY re-read for 1 column tile instead of 2).  Off: the step
  // measured 20.44 / 20.38 / 20.40 -> 20.46 / 20.41 / 20.43 ms
  static const bool wide = [] {
    const char* e = std::getenv("CLOUDTIK_AMD_WGRAD_WIDE");
    return e && std::atoi(e) != 0;
  }();
  if (wide && NN % 256 == 0) return 15;
  // the 64-wide tiles serve the layer-1 shapes (802816-pixel reductions): 64-pixel stages win
  // there (l1.c2 301 -> 289 us, l1.c3 156 -> 142, l1.c1 128 -> 118; profiles/r4/conv_stream_probe.md)
  if (NN % 128 == 0) return 5;
  // 128 x 64 tiles where the output channels allow (layer-1 64 -> 256 1x1 convs: X re-read for
  // 2 co tiles instead of 4).  Alone SLOWER (l1.c3 108 -> 124 us) but the step is faster beside
  // the data gradients: 20.84 / 20.83 / 20.83 + 20.79 / 20.90 / 20.84 / 20.84 -> 20.80 / 20.76 /
  // 20.73 + 20.77 / 20.78 / 20.76 / 20.75 ms (profiles/r5/SUMMARY.md); CLOUDTIK_AMD_WGRAD_TALL=0
  // restores the 64 x 64 tiles
  static const bool tall = [] {
    const char* e = std::getenv("CLOUDTIK_AMD_WGRAD_TALL");
    return !e || std::atoi(e) != 0;
  }();
  if (tall && Co % 128 == 0) return 14;
  return 8;                        // 64 x 64, 64-pixel stages, 3-slot ring (l1.c3 145 -> 137 us)
}

// workspace: n fp32 + ceil(n / 1024) tickets, zeroed here
extern "C" int ct_splitk_reduce_wide(const float* P, int S, long n, void* out, int accumulate, float* ws,
                                     hipStream_t stream) {
  if (S < 1 || n < 1) return 1;
  const long cols = (n + 1023) / 1024;
  unsigned* tickets = (unsigned*)(ws + n);
  if (hipMemsetAsync(ws, 0, n * sizeof(float) + cols * sizeof(unsigned), stream) != hipSuccess) return 7;
  dim3 grid((unsigned)cols, (unsigned)((S + 31) / 32));
  splitk_wide_kernel<<<grid, 256, 0, stream>>>(P, S, n, ws, tickets, (bf16_t*)out, accumulate);
  return hipGetLastError() == hipSuccess ? 0 : 7;
}

// fp32 partials P[splits][Co][T*Ci] of dW; rows_per_split must be a multiple of 32.
extern "C" int ct_conv_wgrad(const void* DY, const void* X, int Hi, int Wi, int Ci, int Hr, int Wr, int sy, int sx,
                             int Co, int M, int T, const int* taps, float* P, int splits, int rows_per_split, int cfg,
                             hipStream_t stream) {
  if (Ci <= 0 || (Ci % 64 && Ci != 8 && Ci != 4) || Co <= 0 || Co % 64 || M <= 0 || T <= 0 || T > CV_MAXT ||
      splits < 1)
    return 1;
  if (Ci == 4 && (Wi % 2 || sx % 2)) return 1;
  if (rows_per_split % 32 || (long)rows_per_split * splits < M) return 2;
  if (((uintptr_t)DY & 15) || ((uintptr_t)X & 15) || ((uintptr_t)P & 15)) return 3;
  const int pixchunk = Ci == 8 ? 1 : (Ci == 4 ? 2 : 0), Cw = pixchunk ? 64 : Ci;
  WgradArgs a{(const bf16_t*)DY, (const bf16_t*)X, P, Hi, Wi, Ci, Hr, Wr, sy, sx, Co, T * Cw, M, T, rows_per_split,
              0ull, 0ull, Cw, pixchunk};
  for (int t = 0; t < T; ++t) {
    const int dy = taps[2 * t], dx = taps[2 * t + 1];
    if (dy < -8 || dy > 7 || dx < -8 || dx > 7) return 4;
    a.tdy |= (unsigned long long)(dy + 8) << (4 * t);
    a.tdx |= (unsigned long long)(dx + 8) << (4 * t);
  }
  cfg = ct_conv_wgrad_cfg(cfg, Co, a.NN);
  if (cfg == 12 || cfg == 13) {      // 3x3 / stride 1 or 2 / pad 1, all taps per workgroup
    if (T != 9 || sy != sx || (sy != 1 && sy != 2) || Hr != (Hi - 1) / sy + 1 || Wr != (Wi - 1) / sx + 1 || pixchunk ||
        Ci % 64)
      return 2;
    if ((long)M / (Hr * Wr) * Hi * Wi * Ci * 2 >= (1L << 31) || (long)M * Co * 2 >= (1L << 31)) return 5;   // 32-bit buffer offsets
    for (int t = 0; t < 9; ++t)
      if (taps[2 * t] != t / 3 - 1 || taps[2 * t + 1] != t % 3 - 1) return 4;
    const long blocks = (long)(Co / 64) * (Ci / 64) * splits;
    if (blocks > (1L << 30)) return 5;
    if (cfg == 12) conv_wgrad3x3_kernel<3><<<(int)blocks, 256, 0, stream>>>(a);
    else conv_wgrad3x3_kernel<2><<<(int)blocks, 256, 0, stream>>>(a);
    return hipGetLastError() == hipSuccess ? 0 : 7;
  }
  if (cfg == 14) {                   // 128 co x 64 columns (4 waves 2x2, 64-pixel stages x 3)
    if (Co % 128 || rows_per_split % 64) return 2;
  } else if (cfg == 15) {            // 64 co x 256 columns (4 waves 2x2, 64-pixel stages x 2)
    if (a.NN % 256 || rows_per_split % 64) return 2;
  } else {
    const int tile = cfg == 11 ? 3 : (cfg >= 9 ? 2 : (cfg >= 7 ? 0 : (cfg >= 4 ? cfg - 4 : cfg)));
    if ((tile >= 2 && Co % 128) || (tile == 3 && a.NN % 256) || (tile >= 1 && a.NN % 128)) return 2;
    if (cfg >= 4 && cfg != 9 && rows_per_split % 64) return 2;
  }
  static const bool lin_on = [] {
    const char* e = std::getenv("CLOUDTIK_AMD_WGRAD_LIN");
    return !e || std::atoi(e) != 0;
  }();
  const bool lin = lin_on && T == 1 && taps[0] == 0 && taps[1] == 0 && sy == 1 && sx == 1 && Hr == Hi && Wr == Wi &&
                   !pixchunk && (long)M * Co * 2 < (1L << 31) && (long)M * Ci * 2 < (1L << 31);
  if (lin) {
    switch (cfg) {
      case 3: return wg_launch<128, 256, 2, 4, 4, 32, true>(a, splits, stream);
      case 5: return wg_launch<64, 128, 2, 2, 4, 64, true>(a, splits, stream);
      case 8: return wg_launch<64, 64, 2, 2, 3, 64, true>(a, splits, stream);
      case 9: return wg_launch<128, 128, 2, 4, 4, 32, true>(a, splits, stream);
      case 14: return wg_launch<128, 64, 2, 2, 3, 64, true>(a, splits, stream);
      case 15: return wg_launch<64, 256, 2, 2, 2, 64, true>(a, splits, stream);
      default: break;
    }
  }
  switch (cfg) {
    case 0: return wg_launch<64, 64, 2, 2, 4>(a, splits, stream);
    case 1: return wg_launch<64, 128, 2, 2, 4>(a, splits, stream);
    case 2: return wg_launch<128, 128, 2, 2, 4>(a, splits, stream);
    case 3: return wg_launch<128, 256, 2, 4, 4>(a, splits, stream);
    case 4: return wg_launch<64, 64, 2, 2, 4, 64>(a, splits, stream);
    case 5: return wg_launch<64, 128, 2, 2, 4, 64>(a, splits, stream);
    case 6: return wg_launch<128, 128, 2, 2, 3, 64>(a, splits, stream);
    case 7: return wg_launch<64, 64, 2, 2, 2, 64>(a, splits, stream);
    case 8: return wg_launch<64, 64, 2, 2, 3, 64>(a, splits, stream);
    case 9: return wg_launch<128, 128, 2, 4, 4>(a, splits, stream);
    case 10: return wg_launch<128, 128, 2, 4, 2, 64>(a, splits, stream);
    case 11: return wg_launch<128, 256, 4, 4, 2, 64>(a, splits, stream);
    case 14: return wg_launch<128, 64, 2, 2, 3, 64>(a, splits, stream);
    case 15: return wg_launch<64, 256, 2, 2, 2, 64>(a, splits, stream);
    default: return 6;
  }
}
