// LayerNorm / RMSNorm forward + backward with a fused "bias + dropout + residual" prologue:
//
//     s = residual + dropout(x + bias)          (each part optional)
//     y = LN(s) * gamma + beta
//
// This is the post-LN block epilogue of HF BERT (BertSelfOutput / BertOutput) that the
// reference's BERT-large pretraining runs 48x per step
// (applications/ai/quickstart/models/language_modeling/pytorch/bert_large/training/
// run_pretrain_mlperf.py:449-471, hidden 1024).  MI355X design:
//   * one wave64 per row, the row held in VGPRs (N <= 2048), bf16 moved as 16-byte
//     vectors, fp32 statistics from registers -> exactly one HBM read of each input.
//   * the projection GEMM runs WITHOUT bias (plain hipBLASLt); its bias, the dropout and
//     the residual add are folded in here, and backward folds d(bias) = colsum(dx) into
//     the same pass as dgamma/dbeta -> no separate bias-grad reduction kernel.
//   * dropout mask regenerated from Philox(seed, offset, index) in backward: nothing stored.
//   * backward keeps per-lane dgamma/dbeta/dbias partials across a grid-stride row loop;
//     cross-row reduction = [grid x N] fp32 partials + one column-sum kernel (no atomics,
//     bitwise reproducible).
#include "common.h"
#include <cstdlib>

namespace ct {

struct LnFwdArgs {
  const bf16_t* x; const bf16_t* bias; const bf16_t* res;
  const bf16_t* gamma; const bf16_t* beta;
  bf16_t* y; bf16_t* s_out; float* mean_out; float* rstd_out;
  int M, N; float eps; uint32_t thresh; float scale; uint64_t seed, offset;
};

template <int MAXV, bool RMS>
__global__ __launch_bounds__(256) void ln_fwd_kernel(LnFwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int wpb = blockDim.x >> 6;
  const int N = a.N, nvec = N >> 3;
  const bool has_bias = a.bias != nullptr, has_res = a.res != nullptr, drop = a.thresh != 0;
  const bool write_s = a.s_out != nullptr;
  for (int row = blockIdx.x * wpb + (threadIdx.x >> 6); row < a.M; row += gridDim.x * wpb) {
    const u16x8* xr = reinterpret_cast<const u16x8*>(a.x + (size_t)row * N);
    const u16x8* rr = reinterpret_cast<const u16x8*>(a.res + (size_t)row * N);
    const u16x8* br = reinterpret_cast<const u16x8*>(a.bias);
    float v[MAXV][8];
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane + i * 64;
      if (c < nvec) {
        const u16x8 xv = xr[c];
        u16x8 bv = u16x8(0), rv = u16x8(0);
        if (has_bias) bv = br[c];
        if (has_res) rv = rr[c];
        uint32_t keep = 0xFFu;
        if (drop) keep = dropout_bits8(a.seed, a.offset, (uint64_t)row * nvec + c, a.thresh);
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = bf2f(xv[j]) + bf2f(bv[j]);
          if (drop) t = ((keep >> j) & 1u) ? t * a.scale : 0.f;
          t += bf2f(rv[j]);
          o[j] = f2bf(t);
          v[i][j] = bf2f(o[j]);  // normalise the rounded sum: backward sees the same s
          sum += v[i][j];
        }
        if (write_s) reinterpret_cast<u16x8*>(a.s_out + (size_t)row * N)[c] = o;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
      }
    }
    sum = wave_sum(sum);
    const float mean = RMS ? 0.f : sum / N;
    float var = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      if (lane + i * 64 < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; var += d * d; }
      }
    }
    var = wave_sum(var) / N;
    const float rstd = rsqrtf(var + a.eps);
    if (lane == 0) {
      if (a.mean_out) a.mean_out[row] = mean;
      a.rstd_out[row] = rstd;
    }
    u16x8* yr = reinterpret_cast<u16x8*>(a.y + (size_t)row * N);
    const u16x8* g8 = reinterpret_cast<const u16x8*>(a.gamma);
    const u16x8* b8 = reinterpret_cast<const u16x8*>(a.beta);
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane + i * 64;
      if (c < nvec) {
        const u16x8 g = g8[c];
        u16x8 bb = u16x8(0);
        if (!RMS && a.beta) bb = b8[c];
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf((v[i][j] - mean) * rstd * bf2f(g[j]) + bf2f(bb[j]));
        yr[c] = o;
      }
    }
  }
}

struct LnBwdArgs {
  const bf16_t* dy; const bf16_t* s; const bf16_t* gamma; const float* mean; const float* rstd;
  const bf16_t* beta;    // FROMY: s holds the forward's OUTPUT y; xhat = (y - beta) / gamma
  const bf16_t* dextra;  // optional extra gradient added to ds (e.g. a skip path)
  bf16_t* ds;            // grad wrt s (= grad of the residual input)
  bf16_t* dx;            // grad wrt x (after dropout backward); may alias nothing / be null
  float* dg_part; float* db_part; float* dbias_part;
  int M, N; uint32_t thresh; float scale; uint64_t seed, offset;
};

// DBIAS: also the column sums of dx (the gradient of the bias folded into the forward's
// prologue); off when the consumer computes them instead (the projection's weight-gradient
// GEMM sums its dY operand with an all-ones MFMA: ops/transformer.py) -- 16 fewer registers
// and adds per row, a third fewer partials
// 3 waves / SIMD up to N = 1024 (MAXV 2); wider rows (N <= 2048) keep more registers at 2
// (1 with the bias gradient) -- at 3 they spilled 20-550 VGPRs
// FROMY: the backward from the forward's output instead of its input (the "memory-efficient"
// LayerNorm): xhat = (y - beta) / gamma.  The forward then writes no copy of its input sum s --
// y is kept anyway (the next layer's input) -- a quarter of the forward's HBM bytes.  A channel
// whose gamma is exactly 0 gets xhat 0 (its y carries no information about x).
template <int MAXV, bool RMS, bool EXTRA, bool DBIAS, bool FROMY = false, bool PF2 = false>
__global__ __launch_bounds__(256, MAXV <= 2 ? ((FROMY && DBIAS) ? 2 : 3) : (DBIAS ? 1 : 2)) void ln_bwd_kernel(LnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) float red[4][512];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wpb = blockDim.x >> 6;
  const int N = a.N, nvec = N >> 3;
  const bool drop = a.thresh != 0;
  constexpr bool want_dbias = DBIAS;
  float dg[MAXV][8], db[MAXV][8], dbi[DBIAS ? MAXV : 1][8];
  u16x8 gb[MAXV];                    // gamma kept packed (bf16): 4 VGPRs per 8 columns
  // FROMY: beta (bf16) and 1 / gamma (fp32, 0 where gamma is 0) per column in LDS, read per
  // element -- in registers they pushed the kernel into spills at 3 waves / SIMD
  __shared__ __attribute__((aligned(16))) unsigned short ybeta[FROMY ? 2048 : 8];
  __shared__ __attribute__((aligned(16))) float yrg[FROMY ? 2048 : 4];
  if constexpr (FROMY) {
    for (int c = threadIdx.x; c < N; c += blockDim.x) {
      ybeta[c] = a.beta[c];
      const float gf = bf2f(a.gamma[c]);
      yrg[c] = gf != 0.f ? 1.f / gf : 0.f;
    }
    __syncthreads();
  }
  const u16x8* g8 = reinterpret_cast<const u16x8*>(a.gamma);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + i * 64;
    gb[i] = c < nvec ? g8[c] : u16x8(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) { dg[i][j] = 0.f; db[i][j] = 0.f; if (DBIAS) dbi[i][j] = 0.f; }
  }
  // Software pipeline: the s / dy / dextra rows (and mean, rstd) of later rows are in flight
  // while this row's reductions and stores run -- the kernel is latency bound with one row per
  // wave otherwise (measured 3.9 TB/s effective on MI355X before the first prefetch).
  const int stride = gridDim.x * wpb;
  int row = blockIdx.x * wpb + wid;
  // Loads are unconditional (row and column clamped into range; the clamped copies are never
  // used): with a branch around them the compiler's wait-count merge at the join waited for
  // EVERY outstanding load (vmcnt(0)) before the first use, so rows prefetched further ahead
  // were waited for too.
  auto load = [&](u16x8 (&sv)[MAXV], u16x8 (&dv)[MAXV], u16x8 (&ev)[MAXV], float& mn, float& rs, int r) {
    r = min(r, a.M - 1);
    const u16x8* sr = reinterpret_cast<const u16x8*>(a.s + (size_t)r * N);
    const u16x8* dyr = reinterpret_cast<const u16x8*>(a.dy + (size_t)r * N);
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = min(lane + i * 64, nvec - 1);
      sv[i] = sr[c];
      dv[i] = dyr[c];
      if (EXTRA) ev[i] = reinterpret_cast<const u16x8*>(a.dextra + (size_t)r * N)[c];
    }
    mn = (RMS || FROMY) ? 0.f : a.mean[r];
    rs = a.rstd[r];
  };
  auto process = [&](const u16x8 (&csv)[MAXV], const u16x8 (&cdv)[MAXV], const u16x8 (&cev)[MAXV],
                     const float mean, const float rstd, const int row) {
    // pass 1: row sums; xhat and dy*gamma are recomputed in pass 2 from the raw bf16
    // registers instead of being kept live (keeps the kernel at 3 waves / SIMD)
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane + i * 64;
      if (c < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = bf2f(cdv[i][j]);
          const float dgv = d * bf2f(gb[i][j]);
          db[i][j] += d;
          s1 += dgv;
          if constexpr (FROMY) {
            // u = y - beta = gamma * xhat: dy * gamma * xhat = dy * u needs no division, and the
            // dgamma partials (sums of dy * u) are divided by gamma once, when written
            const float u = bf2f(csv[i][j]) - bf2f(ybeta[8 * c + j]);
            dg[i][j] += d * u;
            s2 += d * u;
          } else {
            const float xhat = (bf2f(csv[i][j]) - mean) * rstd;
            dg[i][j] += d * xhat;
            s2 += dgv * xhat;
          }
        }
      }
    }
    s1 = wave_sum(s1) / N;
    s2 = wave_sum(s2) / N;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = lane + i * 64;
      if (c < nvec) {
        const u16x8 ev = EXTRA ? cev[i] : u16x8(0);
        uint32_t keep = 0xFFu;
        if (drop) keep = dropout_bits8(a.seed, a.offset, (uint64_t)row * nvec + c, a.thresh);
        u16x8 o, od;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // FROMY: beta and 1 / gamma read per element (wider LDS reads held 12 more VGPRs)
          const float xhat = FROMY ? (bf2f(csv[i][j]) - bf2f(ybeta[8 * c + j])) * yrg[8 * c + j]
                                   : (bf2f(csv[i][j]) - mean) * rstd;
          const float dgv = bf2f(cdv[i][j]) * bf2f(gb[i][j]);
          float t = RMS ? rstd * (dgv - xhat * s2) : rstd * (dgv - s1 - xhat * s2);
          t += bf2f(ev[j]);
          o[j] = f2bf(t);
          float tx = drop ? (((keep >> j) & 1u) ? t * a.scale : 0.f) : t;
          od[j] = f2bf(tx);
          if constexpr (DBIAS) dbi[i][j] += tx;
        }
        if (a.ds) reinterpret_cast<u16x8*>(a.ds + (size_t)row * N)[c] = o;
        if (a.dx) reinterpret_cast<u16x8*>(a.dx + (size_t)row * N)[c] = od;
      }
    }
  };
  if constexpr (PF2) {
    // two register sets that alternate: while row r is processed, row r + stride's loads are
    // outstanding, and row r + 2 stride's are issued as soon as r's registers are free -- two
    // rows in flight at the wait instead of one, for no more registers than load-then-copy
    u16x8 sA[MAXV], dA[MAXV], eA[MAXV], sB[MAXV], dB[MAXV], eB[MAXV];
    float mA = 0.f, rA = 0.f, mB = 0.f, rB = 0.f;
    load(sA, dA, eA, mA, rA, row);
    load(sB, dB, eB, mB, rB, row + stride);
    while (row < a.M) {
      process(sA, dA, eA, mA, rA, row);
      load(sA, dA, eA, mA, rA, row + 2 * stride);
      row += stride;
      if (row >= a.M) break;
      process(sB, dB, eB, mB, rB, row);
      load(sB, dB, eB, mB, rB, row + 2 * stride);
      row += stride;
    }
  } else {
    u16x8 nsv[MAXV], ndv[MAXV], nev[MAXV];
    float nmean = 0.f, nrstd = 0.f;
    load(nsv, ndv, nev, nmean, nrstd, row);
    for (; row < a.M; row += stride) {
      u16x8 csv[MAXV], cdv[MAXV], cev[MAXV];
#pragma unroll
      for (int i = 0; i < MAXV; ++i) { csv[i] = nsv[i]; cdv[i] = ndv[i]; if (EXTRA) cev[i] = nev[i]; }
      const float mean = nmean, rstd = nrstd;
      load(nsv, ndv, nev, nmean, nrstd, row + stride);
      process(csv, cdv, cev, mean, rstd, row);
    }
  }
  // reduce the block's waves through LDS, 512 columns at a time.  A lane's 8 columns go in as
  // two 16-byte stores whose halves swap when bit 2 of the column group is set: the 8 lanes of
  // a ds_write_b128 group then cover all 32 banks (scalar stores at a 32-byte lane stride were
  // 8-way conflicted: 2.06 M conflict cycles per BERT-large step); the column-order reads
  // undo the swap and stay conflict-free.
  const int nparts = want_dbias ? 3 : 2;
  for (int base = 0; base < N; base += 512) {
    for (int pass = 0; pass < nparts; ++pass) {
#pragma unroll
      for (int i = 0; i < MAXV; ++i) {
        const int c = lane + i * 64;
        const int cl = c - (base >> 3);
        if (c < nvec && cl >= 0 && cl < 64) {
          // select values, not a pointer: a runtime-chosen pointer into the register arrays
          // put dg / db / dbi in scratch memory for the whole kernel (80 B/lane)
          float src[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) src[j] = pass == 0 ? dg[i][j] : (pass == 1 ? db[i][j] : dbi[DBIAS ? i : 0][j]);
          const int hs = (cl >> 2) & 1;
          float* rw = red[wid] + cl * 8;
          *reinterpret_cast<f32x4*>(rw + 4 * hs) = f32x4{src[0], src[1], src[2], src[3]};
          *reinterpret_cast<f32x4*>(rw + 4 * (hs ^ 1)) = f32x4{src[4], src[5], src[6], src[7]};
        }
      }
      __syncthreads();
      float* dst = pass == 0 ? a.dg_part : (pass == 1 ? a.db_part : a.dbias_part);
      for (int col = threadIdx.x; col < 512 && base + col < N; col += blockDim.x) {
        const int cl = col >> 3, j = col & 7;
        const int idx = cl * 8 + 4 * ((j >> 2) ^ ((cl >> 2) & 1)) + (j & 3);
        float t = 0.f;
        for (int w = 0; w < wpb; ++w) t += red[w][idx];
        if (FROMY && pass == 0) t *= yrg[base + col];   // sums of dy * gamma * xhat -> of dy * xhat
        if (dst) dst[(size_t)blockIdx.x * N + base + col] = t;
      }
      __syncthreads();
    }
  }
}

// out[col] (+)= sum_p part[p, col].  Block = 64 columns x 16 row-lanes (1024 threads):
// every wave reads 64 consecutive floats of one partial row (coalesced), 16 waves per CU
// keep enough loads in flight; the 16 lanes per column are merged through LDS.
template <typename OUT>
__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ part,
                                                      OUT* __restrict__ out, int P, int N,
                                                      int accumulate) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  float t = 0.f;
  if (col < N) {
    int p = rl;
    for (; p + 48 < P; p += 64) {
      const float a = part[(size_t)p * N + col], b = part[(size_t)(p + 16) * N + col];
      const float c = part[(size_t)(p + 32) * N + col], d = part[(size_t)(p + 48) * N + col];
      t += (a + b) + (c + d);
    }
    for (; p < P; p += 16) t += part[(size_t)p * N + col];
  }
  red[rl][cl] = t;
  __syncthreads();
  if (rl == 0 && col < N) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][cl];
    if (accumulate) s += to_f<OUT>(out[col]);
    out[col] = from_f<OUT>(s);
  }
}

// Up to three column sums in ONE launch (blockIdx.y picks the (partials, output) pair):
// the LayerNorm backward's dgamma / dbeta / dbias reductions are tiny (a few MB) and were
// three back-to-back launch latencies.  Block = 16 columns x 16 row-lanes (256 threads), so a
// 1024-wide reduction spreads over 3 x 64 workgroups (at 64 columns per 1024-thread block it
// ran on 48 CUs), and each lane keeps 8 independent loads in flight: the kernel is a chain of
// memory latencies, not bandwidth (9 MB per call).
struct Colsum3 { const float* part[3]; void* out[3]; };

template <typename OUT>
__global__ __launch_bounds__(256) void colsum3_kernel(Colsum3 c, int P, int N, int accumulate) {
  __shared__ float red[16][16];
  const float* __restrict__ part = c.part[blockIdx.y];
  OUT* __restrict__ out = reinterpret_cast<OUT*>(c.out[blockIdx.y]);
  const int cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + cl;
  float t[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col < N) {
    int p = rl;
    for (; p + 112 < P; p += 128) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(p + 16 * u) * N + col];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] += v[u];
    }
    for (; p < P; p += 16) t[0] += part[(size_t)p * N + col];
  }
  red[rl][cl] = ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
  __syncthreads();
  if (rl == 0 && col < N) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][cl];
    if (accumulate) s += to_f<OUT>(out[col]);
    out[col] = from_f<OUT>(s);
  }
}

}  // namespace ct

using namespace ct;

static int colsum_multi(const float* const* parts, void* const* outs, int n, int P, int N, int out_fp32,
                        int accumulate, hipStream_t stream) {
  Colsum3 c{};
  for (int i = 0; i < n; ++i) { c.part[i] = parts[i]; c.out[i] = outs[i]; }
  const dim3 grid(ceil_div(N, 16), n);
  if (out_fp32) colsum3_kernel<float><<<grid, 256, 0, stream>>>(c, P, N, accumulate);
  else colsum3_kernel<bf16_t><<<grid, 256, 0, stream>>>(c, P, N, accumulate);
  return 0;
}

extern "C" int ct_colsum(const float* part, void* out, int P, int N, int out_fp32, int accumulate,
                         hipStream_t stream) {
  const int cb = ceil_div(N, 64);
  if (out_fp32) colsum_kernel<float><<<cb, 1024, 0, stream>>>(part, (float*)out, P, N, accumulate);
  else colsum_kernel<bf16_t><<<cb, 1024, 0, stream>>>(part, (bf16_t*)out, P, N, accumulate);
  return 0;
}

extern "C" int ct_layernorm_fwd(const void* x, const void* bias, const void* res, const void* g,
                                const void* b, void* y, void* s_out, float* mean, float* rstd,
                                int M, int N, float eps, int rms, float p_drop, uint64_t seed,
                                uint64_t offset, hipStream_t stream) {
  if (N % 8 != 0 || N > 2048 || M <= 0) return -1;
  LnFwdArgs a;
  a.x = (const bf16_t*)x; a.bias = (const bf16_t*)bias; a.res = (const bf16_t*)res;
  a.gamma = (const bf16_t*)g; a.beta = (const bf16_t*)b; a.y = (bf16_t*)y; a.s_out = (bf16_t*)s_out;
  a.mean_out = mean; a.rstd_out = rstd; a.M = M; a.N = N; a.eps = eps;
  a.thresh = p_drop > 0.f ? dropout_threshold(p_drop) : 0u;
  a.scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.seed = seed; a.offset = offset;
  const int mv = (N / 8 + 63) / 64;
  int grid = ceil_div(M, 4);
  if (grid > 16384) grid = 16384;
#define CT_LNF(MV) case MV: if (rms) ln_fwd_kernel<MV, true><<<grid, 256, 0, stream>>>(a); \
                            else ln_fwd_kernel<MV, false><<<grid, 256, 0, stream>>>(a); break;
  switch (mv) {
    CT_LNF(1) CT_LNF(2) CT_LNF(3) CT_LNF(4)
    default: return -1;
  }
#undef CT_LNF
  return 0;
}

extern "C" int ct_layernorm_bwd_grid(int M, int N) {
  // 768 blocks x 4 waves = 3 waves per SIMD on 256 CUs (the kernel's VGPR budget allows 3
  // for N <= 1024, 2 above)
  const int cap = N > 1024 ? 512 : 768;
  const int grid = ceil_div(M, 4);
  return grid > cap ? cap : grid;
}

// Workspace: part = float[3 * grid * N] (grid = ct_layernorm_bwd_grid(M, N)).
// from_y: `s` is the forward's output y and `beta` its beta (xhat = (y - beta) / gamma; mean unused)
extern "C" int ct_layernorm_bwd2(const void* dy, const void* s, const void* g, const float* mean,
                                 const float* rstd, const void* dextra, void* ds, void* dx,
                                 float* part, void* dgamma, void* dbeta, void* dbias, int M, int N,
                                 int rms, int param_fp32, int accumulate, float p_drop,
                                 uint64_t seed, uint64_t offset, int from_y, const void* beta,
                                 hipStream_t stream) {
  if (N % 8 != 0 || N > 2048 || M <= 0) return -1;
  if (from_y && (rms || !beta)) return -2;        // the output form: LayerNorm with beta only
  const int grid = ct_layernorm_bwd_grid(M, N);
  LnBwdArgs a;
  a.beta = (const bf16_t*)beta;
  a.dy = (const bf16_t*)dy; a.s = (const bf16_t*)s; a.gamma = (const bf16_t*)g; a.mean = mean;
  a.rstd = rstd; a.dextra = (const bf16_t*)dextra; a.ds = (bf16_t*)ds; a.dx = (bf16_t*)dx;
  a.dg_part = part; a.db_part = (rms || !dbeta) ? nullptr : part + (size_t)grid * N;
  a.dbias_part = dbias ? part + (size_t)2 * grid * N : nullptr;
  a.M = M; a.N = N;
  a.thresh = p_drop > 0.f ? dropout_threshold(p_drop) : 0u;
  a.scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.seed = seed; a.offset = offset;
  const int mv = (N / 8 + 63) / 64;
  // two rows in flight per wave (PF2) or one (CLOUDTIK_AMD_LN_BWD_PF2=0)
  static const bool pf2 = [] { const char* e = getenv("CLOUDTIK_AMD_LN_BWD_PF2"); return !e || e[0] != '0'; }();
#define CT_LNB2(MV, DB)                                                                       \
    if (rms) { if (a.dextra) ln_bwd_kernel<MV, true, true, DB><<<grid, 256, 0, stream>>>(a);       \
               else ln_bwd_kernel<MV, true, false, DB><<<grid, 256, 0, stream>>>(a); }               \
    else if (from_y) { if (a.dextra) ln_bwd_kernel<MV, false, true, DB, true><<<grid, 256, 0, stream>>>(a); \
           else ln_bwd_kernel<MV, false, false, DB, true><<<grid, 256, 0, stream>>>(a); }            \
    else if (pf2) { if (a.dextra) ln_bwd_kernel<MV, false, true, DB, false, true><<<grid, 256, 0, stream>>>(a); \
           else ln_bwd_kernel<MV, false, false, DB, false, true><<<grid, 256, 0, stream>>>(a); }     \
    else { if (a.dextra) ln_bwd_kernel<MV, false, true, DB><<<grid, 256, 0, stream>>>(a);          \
           else ln_bwd_kernel<MV, false, false, DB><<<grid, 256, 0, stream>>>(a); }
#define CT_LNB(MV) case MV:                                                                   \
    if (a.dbias_part) { CT_LNB2(MV, true) } else { CT_LNB2(MV, false) }                         \
    break;
  switch (mv) {
    CT_LNB(1) CT_LNB(2) CT_LNB(3) CT_LNB(4)
    default: return -1;
  }
#undef CT_LNB
#undef CT_LNB2
  const float* parts[3];
  void* outs[3];
  int n = 0;
  parts[n] = a.dg_part; outs[n++] = dgamma;
  if (a.db_part) { parts[n] = a.db_part; outs[n++] = dbeta; }
  if (a.dbias_part) { parts[n] = a.dbias_part; outs[n++] = dbias; }
  return colsum_multi(parts, outs, n, grid, N, param_fp32, accumulate, stream);
}

extern "C" int ct_layernorm_bwd(const void* dy, const void* s, const void* g, const float* mean,
                                const float* rstd, const void* dextra, void* ds, void* dx,
                                float* part, void* dgamma, void* dbeta, void* dbias, int M, int N,
                                int rms, int param_fp32, int accumulate, float p_drop,
                                uint64_t seed, uint64_t offset, hipStream_t stream) {
  return ct_layernorm_bwd2(dy, s, g, mean, rstd, dextra, ds, dx, part, dgamma, dbeta, dbias, M, N, rms, param_fp32,
                           accumulate, p_drop, seed, offset, 0, nullptr, stream);
}
