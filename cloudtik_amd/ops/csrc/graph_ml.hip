// Kernels for the classical-ML and graph-ML modeling library:
//
//   * gbdt_hist   -- gradient/hessian histograms for histogram-based gradient boosting
//                    (the work XGBoost's `hist` tree method does; reference
//                    runtime/ai/modeling/classical_ml/.../xgboost/modeling/model/trainer.py).
//   * gbdt_predict -- inference of a whole tree ensemble on binned features.
//   * csr_spmm    -- out[i] = scale_i * sum_e w_e * x[col_e]  (GraphSAGE mean / sum
//                    neighbour aggregation and its transpose for the backward pass;
//                    reference graph_sage/model/homogeneous/*: DGL SAGEConv 'mean').
//
// Layouts are chosen for CDNA4:
//   * binned features are FEATURE-MAJOR uint8 [F, ldb]: a wave reads 64 consecutive rows of
//     one feature as 64 x uint32 (4 rows per lane) -- fully coalesced -- and the per-row
//     node/grad/hess words are loaded once per workgroup and reused for FB features.
//   * histograms accumulate in LDS with native ds_add_f32 (one private histogram per
//     workgroup, <= 64 KB so two workgroups share a CU), then flush with global float
//     atomics (-munsafe-fp-atomics -> global_atomic_add_f32); empty bins are skipped.
//   * SpMM assigns a power-of-two lane group per destination row, 16-byte vector loads of
//     the source rows, fp32 accumulation, 4 edges in flight per group.
#include "common.h"

namespace ct {

// ------------------------------------------------------------------ histogram
// bins  : uint8 [F, ldb] (ldb % 4 == 0, rows >= N are padding)
// node  : int32 [N]  slot of the row's node in this pass, or anything outside
//         [slot_lo, slot_lo + S) to skip the row
// gh    : float2 [N] (gradient, hessian)
// hist  : float [S_total, F, B, 2]  (accumulated; caller zeroes)
template <int FB>
__global__ __launch_bounds__(256) void gbdt_hist_kernel(const uint8_t* __restrict__ bins, long ldb,
                                                        const int* __restrict__ node,
                                                        const float2* __restrict__ gh,
                                                        float* __restrict__ hist, int N, int F, int B,
                                                        int slot_lo, int S, int rows_per_block) {
  extern __shared__ float lh[];  // [FB][S][B][2]
  const int f0 = blockIdx.x * FB;
  const int nf = min(FB, F - f0);
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(N, r0 + rows_per_block);
  const int hsz = FB * S * B * 2;
  for (int i = threadIdx.x; i < hsz; i += 256) lh[i] = 0.f;
  __syncthreads();

  for (int row = r0 + threadIdx.x * 4; row < r1; row += 256 * 4) {
    int nd[4];
    float g[4], h[4];
    if (row + 3 < r1) {
      const int4 n4 = *reinterpret_cast<const int4*>(node + row);
      const float4 a = *reinterpret_cast<const float4*>(gh + row);
      const float4 b = *reinterpret_cast<const float4*>(gh + row + 2);
      nd[0] = n4.x - slot_lo; nd[1] = n4.y - slot_lo; nd[2] = n4.z - slot_lo; nd[3] = n4.w - slot_lo;
      g[0] = a.x; h[0] = a.y; g[1] = a.z; h[1] = a.w; g[2] = b.x; h[2] = b.y; g[3] = b.z; h[3] = b.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = row + k < r1;
        nd[k] = ok ? node[row + k] - slot_lo : -1;
        const float2 v = ok ? gh[row + k] : make_float2(0.f, 0.f);
        g[k] = v.x; h[k] = v.y;
      }
    }
    bool any = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if ((unsigned)nd[k] >= (unsigned)S) nd[k] = -1;
      any |= nd[k] >= 0;
    }
    if (!any) continue;
#pragma unroll
    for (int f = 0; f < FB; ++f) {
      if (f >= nf) break;
      const uint32_t w = *reinterpret_cast<const uint32_t*>(bins + (long)(f0 + f) * ldb + row);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (nd[k] < 0) continue;
        const int b = (w >> (8 * k)) & 0xff;
        float* p = lh + (((f * S + nd[k]) * B + b) << 1);
        atomicAdd(p, g[k]);
        atomicAdd(p + 1, h[k]);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nf * S * B * 2; i += 256) {
    const float v = lh[i];
    if (v == 0.f) continue;
    const int c = i & 1;
    int t = i >> 1;
    const int b = t % B; t /= B;
    const int s = t % S;
    const int f = t / S;
    atomicAdd(hist + ((((long)(slot_lo + s) * F + (f0 + f)) * B + b) << 1) + c, v);
  }
}

// ------------------------------------------------------------------ ensemble predict
// Complete binary trees of M = 2^(depth+1)-1 nodes, node n's children at 2n+1 / 2n+2.
// feat[t, n] < 0 marks a leaf.  A row goes left when its bin is <= thr (bin 0 = missing
// follows dleft).  Tree t contributes to output column t % K.
__global__ __launch_bounds__(256) void gbdt_predict_kernel(const uint8_t* __restrict__ bins, long ldb,
                                                           const int* __restrict__ feat,
                                                           const int* __restrict__ thr,
                                                           const uint8_t* __restrict__ dleft,
                                                           const float* __restrict__ leaf, int T, int M, int K,
                                                           int N, float* __restrict__ out) {
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (long)N * K) return;
  const int row = (int)(gid % N);   // consecutive lanes -> consecutive rows (coalesced bins)
  const int cls = (int)(gid / N);
  float acc = 0.f;
  for (int t = cls; t < T; t += K) {
    const int* ft = feat + (long)t * M;
    const int* th = thr + (long)t * M;
    const uint8_t* dl = dleft + (long)t * M;
    int n = 0;
    int f = ft[0];
    while (f >= 0) {
      const int b = bins[(long)f * ldb + row];
      const bool left = b == 0 ? dl[n] != 0 : b <= th[n];
      n = 2 * n + (left ? 1 : 2);
      f = ft[n];
    }
    acc += leaf[(long)t * M + n];
  }
  out[(long)row * K + cls] += acc;
}

// ------------------------------------------------------------------ CSR SpMM
template <typename T>
struct Vec;
template <>
struct Vec<float> {
  static constexpr int N = 4;
  typedef f32x4 type;
};
template <>
struct Vec<bf16_t> {
  static constexpr int N = 8;
  typedef u16x8 type;
};

template <typename T, int LPR>  // LPR = lanes per destination row (power of two <= 64)
__global__ __launch_bounds__(256) void csr_spmm_kernel(const int64_t* __restrict__ rowptr,
                                                       const int64_t* __restrict__ col,
                                                       const float* __restrict__ w,
                                                       const float* __restrict__ scale, int mean,
                                                       const T* __restrict__ x, long ldx,
                                                       T* __restrict__ out, long ldo, int R, int D) {
  constexpr int V = Vec<T>::N;
  typedef typename Vec<T>::type VT;
  const int lane = threadIdx.x % LPR;
  const long r = ((long)blockIdx.x * 256 + threadIdx.x) / LPR;
  if (r >= R) return;
  const long e0 = rowptr[r], e1 = rowptr[r + 1];
  float s = 1.f;
  if (mean) s = e1 > e0 ? 1.f / (float)(e1 - e0) : 0.f;
  if (scale) s *= scale[r];
  for (int d0 = lane * V; d0 < D; d0 += LPR * V) {
    float acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.f;
    long e = e0;
    for (; e + 3 < e1; e += 4) {
      VT xv[4];
      float we[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        xv[u] = *reinterpret_cast<const VT*>(x + col[e + u] * ldx + d0);
        we[u] = w ? w[e + u] : 1.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] += we[u] * to_f<T>(xv[u][v]);
    }
    for (; e < e1; ++e) {
      const VT xv = *reinterpret_cast<const VT*>(x + col[e] * ldx + d0);
      const float we = w ? w[e] : 1.f;
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] += we * to_f<T>(xv[v]);
    }
    VT o;
#pragma unroll
    for (int v = 0; v < V; ++v) o[v] = from_f<T>(acc[v] * s);
    *reinterpret_cast<VT*>(out + r * ldo + d0) = o;
  }
}

}  // namespace ct

using namespace ct;

extern "C" {

int ct_gbdt_hist(const uint8_t* bins, long ldb, const int* node, const void* gh, float* hist, int N, int F,
                 int B, int slot_lo, int S, hipStream_t st) {
  if (N <= 0 || F <= 0) return 0;
  if (B < 1 || B > 256 || S < 1 || (ldb & 3) || ldb < N) return 1;
  const long per_fb = (long)S * B * 2 * sizeof(float);
  if (per_fb > 64 * 1024) return 2;   // caller splits the slot range
  int fb = 1;
  while (fb < 8 && per_fb * fb * 2 <= 64 * 1024) fb *= 2;
  const int fblocks = (F + fb - 1) / fb;
  // enough workgroups to fill 256 CUs a few times over, row chunks a multiple of 1024
  int rblocks = max(1, 2048 / fblocks);
  int rpb = (N + rblocks - 1) / rblocks;
  rpb = max(1024, (rpb + 1023) / 1024 * 1024);
  rblocks = (N + rpb - 1) / rpb;
  dim3 grid(fblocks, rblocks);
  const size_t lds = per_fb * fb;
  const float2* g = (const float2*)gh;
  switch (fb) {
    case 1: gbdt_hist_kernel<1><<<grid, 256, lds, st>>>(bins, ldb, node, g, hist, N, F, B, slot_lo, S, rpb); break;
    case 2: gbdt_hist_kernel<2><<<grid, 256, lds, st>>>(bins, ldb, node, g, hist, N, F, B, slot_lo, S, rpb); break;
    case 4: gbdt_hist_kernel<4><<<grid, 256, lds, st>>>(bins, ldb, node, g, hist, N, F, B, slot_lo, S, rpb); break;
    default: gbdt_hist_kernel<8><<<grid, 256, lds, st>>>(bins, ldb, node, g, hist, N, F, B, slot_lo, S, rpb); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int ct_gbdt_predict(const uint8_t* bins, long ldb, const int* feat, const int* thr, const uint8_t* dleft,
                    const float* leaf, int T, int M, int K, int N, float* out, hipStream_t st) {
  if (N <= 0 || T <= 0) return 0;
  const long total = (long)N * K;
  gbdt_predict_kernel<<<(unsigned)((total + 255) / 256), 256, 0, st>>>(bins, ldb, feat, thr, dleft, leaf, T, M,
                                                                       K, N, out);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// dtype: 0 fp32, 1 bf16.  D must be a multiple of the vector width (4 fp32 / 8 bf16) and
// ldx / ldo keep 16-byte alignment (checked by the binding).
int ct_csr_spmm(const int64_t* rowptr, const int64_t* col, const float* w, const float* scale, int mean,
                const void* x, long ldx, void* out, long ldo, int R, int D, int dtype, hipStream_t st) {
  if (R <= 0 || D <= 0) return 0;
  const int V = dtype == 0 ? 4 : 8;
  int lpr = 1;
  while (lpr < 64 && lpr * V < D) lpr *= 2;
  const long threads = (long)R * lpr;
  const unsigned grid = (unsigned)((threads + 255) / 256);
#define CT_SPMM(T, L)                                                                                    \
  csr_spmm_kernel<T, L><<<grid, 256, 0, st>>>(rowptr, col, w, scale, mean, (const T*)x, ldx, (T*)out, ldo, \
                                               R, D)
#define CT_SPMM_L(T)                  \
  switch (lpr) {                      \
    case 1: CT_SPMM(T, 1); break;     \
    case 2: CT_SPMM(T, 2); break;     \
    case 4: CT_SPMM(T, 4); break;     \
    case 8: CT_SPMM(T, 8); break;     \
    case 16: CT_SPMM(T, 16); break;   \
    case 32: CT_SPMM(T, 32); break;   \
    default: CT_SPMM(T, 64); break;   \
  }
  if (dtype == 0) {
    CT_SPMM_L(float)
  } else {
    CT_SPMM_L(bf16_t)
  }
#undef CT_SPMM_L
#undef CT_SPMM
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // extern "C"
