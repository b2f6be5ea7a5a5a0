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
                                                        const int* __restrict__ slot_map, int n_nodes,
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
      nd[0] = n4.x; nd[1] = n4.y; nd[2] = n4.z; nd[3] = n4.w;
      g[0] = a.x; h[0] = a.y; g[1] = a.z; h[1] = a.w; g[2] = b.x; h[2] = b.y; g[3] = b.z; h[3] = b.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = row + k < r1;
        nd[k] = ok ? node[row + k] : -1;
        const float2 v = ok ? gh[row + k] : make_float2(0.f, 0.f);
        g[k] = v.x; h[k] = v.y;
      }
    }
    bool any = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // node -> histogram slot (optionally through the level's slot map), then this pass's range
      int sl = nd[k];
      if (slot_map) sl = (unsigned)sl < (unsigned)n_nodes ? slot_map[sl] : -1;
      sl -= slot_lo;
      nd[k] = (unsigned)sl < (unsigned)S ? sl : -1;
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


// ------------------------------------------------------------------ level split search
// One workgroup per (feature f, node s) of the level, one lane per bin (B <= 256).
//  * the node's histogram row is the built child (part[slot]) or, for its sibling,
//    parent - part[sibling slot] (subtraction trick); it is written to hist_cur, which is the
//    parent histogram of the next level.
//  * inclusive scan over bins 1..B-1 (wave shuffles + LDS across the 4 waves) gives the
//    left sums for every threshold, for missing values going left or right; the best
//    (gain, threshold, direction, left hessian) per (s, f) is written out.
struct SplitParams {
  float lambda, alpha, min_child_weight;
};

__device__ __forceinline__ float soft_thr(float g, float a) {
  return a > 0.f ? copysignf(fmaxf(fabsf(g) - a, 0.f), g) : g;
}
__device__ __forceinline__ float leaf_score(float g, float h, const SplitParams& p) {
  const float t = soft_thr(g, p.alpha);
  return t * t / (h + p.lambda);
}

__device__ __forceinline__ float2 block_scan_256(float2 v, float2* lds, float2* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float a = __shfl_up(v.x, o, 64), b = __shfl_up(v.y, o, 64);
    if (lane >= o) { v.x += a; v.y += b; }
  }
  if (lane == 63) lds[wid] = v;
  __syncthreads();
  float2 pre = make_float2(0.f, 0.f);
  for (int w = 0; w < wid; ++w) { pre.x += lds[w].x; pre.y += lds[w].y; }
  *total = make_float2(lds[0].x + lds[1].x + lds[2].x + lds[3].x, lds[0].y + lds[1].y + lds[2].y + lds[3].y);
  return make_float2(v.x + pre.x, v.y + pre.y);
}

__global__ __launch_bounds__(256) void gbdt_split_kernel(const float* __restrict__ part,
                                                         const float* __restrict__ parent,
                                                         const int* __restrict__ slot_map,
                                                         float* __restrict__ hist_cur,
                                                         const uint8_t* __restrict__ feat_mask, int F, int B,
                                                         SplitParams p, float* __restrict__ best_gain,
                                                         int* __restrict__ best_thr, int* __restrict__ best_dir,
                                                         float* __restrict__ best_hl, float* __restrict__ node_gh) {
  __shared__ float2 wsum[4];
  __shared__ float2 miss;
  __shared__ float rg[4];
  __shared__ int ri[4];
  const int f = blockIdx.x, s = blockIdx.y, t = threadIdx.x;
  float2 v = make_float2(0.f, 0.f);
  if (t < B) {
    const long off = (((long)s * F + f) * B + t) * 2;
    if (!slot_map) {
      v = make_float2(part[off], part[off + 1]);
    } else {
      const int sl = slot_map[s];
      if (sl >= 0) {
        const long o = (((long)sl * F + f) * B + t) * 2;
        v = make_float2(part[o], part[o + 1]);
      } else {
        const int sib = slot_map[s ^ 1];
        if (sib >= 0) {
          const long o = (((long)sib * F + f) * B + t) * 2;
          const long po = ((((long)(s >> 1)) * F + f) * B + t) * 2;
          v = make_float2(parent[po] - part[o], parent[po + 1] - part[o + 1]);
        }
      }
    }
    hist_cur[off] = v.x;
    hist_cur[off + 1] = v.y;
  }
  if (t == 0) miss = v;
  const float2 vin = t >= 1 ? v : make_float2(0.f, 0.f);
  float2 tot_nm;
  const float2 cl = block_scan_256(vin, wsum, &tot_nm);   // syncs, so `miss` is visible after
  const float G = tot_nm.x + miss.x, H = tot_nm.y + miss.y;  // every bin incl. missing
  const float parent_score = leaf_score(G, H, p);
  float g_best = -INFINITY, hl_best = 0.f;
  int d_best = 1;
  if (t >= 1 && t <= B - 2 && feat_mask[f]) {
#pragma unroll
    for (int dl = 1; dl >= 0; --dl) {
      const float gl = cl.x + (dl ? miss.x : 0.f), hl = cl.y + (dl ? miss.y : 0.f);
      const float gr = G - gl, hr = H - hl;
      if (hl >= p.min_child_weight && hr >= p.min_child_weight) {
        const float gain = leaf_score(gl, hl, p) + leaf_score(gr, hr, p) - parent_score;
        if (gain > g_best) { g_best = gain; d_best = dl; hl_best = hl; }
      }
    }
  }
  // block argmax, ties -> lower bin
  float bg = g_best;
  int bi = t;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float og = __shfl_xor(bg, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (og > bg || (og == bg && oi < bi)) { bg = og; bi = oi; }
  }
  __shared__ int win;
  if ((t & 63) == 0) { rg[t >> 6] = bg; ri[t >> 6] = bi; }
  __syncthreads();
  if (t == 0) {
    float g0 = rg[0];
    int i0 = ri[0];
    for (int w = 1; w < 4; ++w)
      if (rg[w] > g0 || (rg[w] == g0 && ri[w] < i0)) { g0 = rg[w]; i0 = ri[w]; }
    best_gain[(long)s * F + f] = g0;
    best_thr[(long)s * F + f] = i0;
    win = i0;
    if (f == 0) { node_gh[2 * s] = G; node_gh[2 * s + 1] = H; }
  }
  __syncthreads();
  if (t == win) {                      // the lane owning the winning bin knows its direction
    best_dir[(long)s * F + f] = d_best;
    best_hl[(long)s * F + f] = hl_best;
  }
}

// One workgroup: pick each node's best feature, write the tree arrays and the next level's
// slot map (the child with the smaller hessian is the one whose histogram gets built).
__global__ __launch_bounds__(256) void gbdt_finalize_kernel(const float* __restrict__ best_gain,
                                                            const int* __restrict__ best_thr,
                                                            const int* __restrict__ best_dir,
                                                            const float* __restrict__ best_hl,
                                                            const float* __restrict__ node_gh, int n_level, int F,
                                                            int first, int last_level, SplitParams p, float gamma,
                                                            float eta, float max_delta_step, int* __restrict__ feat,
                                                            int* __restrict__ thr, uint8_t* __restrict__ dleft,
                                                            float* __restrict__ leaf, float* __restrict__ gain,
                                                            float* __restrict__ cover,
                                                            int* __restrict__ slot_next) {
  for (int s = threadIdx.x; s < n_level; s += 256) {
    float g = -INFINITY;
    int bf = 0;
    for (int f = 0; f < F; ++f) {
      const float v = best_gain[(long)s * F + f];
      if (v > g) { g = v; bf = f; }
    }
    const float G = node_gh[2 * s], H = node_gh[2 * s + 1];
    const int n = first + s;
    const bool split = !last_level && isfinite(g) && g > fmaxf(gamma, 1e-12f);
    cover[n] = H;
    if (split) {
      const long k = (long)s * F + bf;
      feat[n] = bf;
      thr[n] = best_thr[k];
      dleft[n] = (uint8_t)best_dir[k];
      gain[n] = g;
      leaf[n] = 0.f;
      const float hl = best_hl[k], hr = H - hl;
      const int small = hr < hl ? 1 : 0;
      slot_next[2 * s + small] = s;
      slot_next[2 * s + 1 - small] = -1;
    } else {
      feat[n] = -1;
      gain[n] = 0.f;
      float w = -soft_thr(G, p.alpha) / (H + p.lambda);
      if (max_delta_step > 0.f) w = fminf(fmaxf(w, -max_delta_step), max_delta_step);
      leaf[n] = w * eta;
      if (!last_level) { slot_next[2 * s] = -1; slot_next[2 * s + 1] = -1; }
    }
  }
}

// Route every active row one level down; rows that reach a leaf add its value to their
// margin (column k of [N, K]) and leave the tree.
__global__ __launch_bounds__(256) void gbdt_partition_kernel(const uint8_t* __restrict__ bins, long ldb,
                                                             int* __restrict__ node, const int* __restrict__ feat,
                                                             const int* __restrict__ thr,
                                                             const uint8_t* __restrict__ dleft,
                                                             const float* __restrict__ leaf, int first, int N,
                                                             float* __restrict__ margin, int K, int k) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= N) return;
  const int s = node[row];
  if (s < 0) return;
  const int n = first + s;
  const int f = feat[n];
  if (f < 0) {
    margin[(long)row * K + k] += leaf[n];
    node[row] = -1;
    return;
  }
  const int b = bins[(long)f * ldb + row];
  const bool left = b == 0 ? dleft[n] != 0 : b <= thr[n];
  node[row] = 2 * s + (left ? 0 : 1);
}

}  // namespace ct

using namespace ct;

extern "C" {

int ct_gbdt_hist(const uint8_t* bins, long ldb, const int* node, const int* slot_map, int n_nodes, const void* gh,
                 float* hist, int N, int F, int B, int slot_lo, int S, hipStream_t st) {
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
    case 1: gbdt_hist_kernel<1><<<grid, 256, lds, st>>>(bins, ldb, node, slot_map, n_nodes, g, hist, N, F, B, slot_lo, S, rpb); break;
    case 2: gbdt_hist_kernel<2><<<grid, 256, lds, st>>>(bins, ldb, node, slot_map, n_nodes, g, hist, N, F, B, slot_lo, S, rpb); break;
    case 4: gbdt_hist_kernel<4><<<grid, 256, lds, st>>>(bins, ldb, node, slot_map, n_nodes, g, hist, N, F, B, slot_lo, S, rpb); break;
    default: gbdt_hist_kernel<8><<<grid, 256, lds, st>>>(bins, ldb, node, slot_map, n_nodes, g, hist, N, F, B, slot_lo, S, rpb); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}


int ct_gbdt_split(const float* part, const float* parent, const int* slot_map, float* hist_cur,
                  const uint8_t* feat_mask, int n_level, int F, int B, float lambda, float alpha, float mcw,
                  float* best_gain, int* best_thr, int* best_dir, float* best_hl, float* node_gh, hipStream_t st) {
  if (B < 3 || B > 256) return 1;
  SplitParams p{lambda, alpha, mcw};
  gbdt_split_kernel<<<dim3(F, n_level), 256, 0, st>>>(part, parent, slot_map, hist_cur, feat_mask, F, B, p, best_gain,
                                                     best_thr, best_dir, best_hl, node_gh);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int ct_gbdt_finalize(const float* best_gain, const int* best_thr, const int* best_dir, const float* best_hl,
                     const float* node_gh, int n_level, int F, int first, int last_level, float lambda, float alpha,
                     float gamma, float eta, float max_delta_step, int* feat, int* thr, uint8_t* dleft, float* leaf,
                     float* gain, float* cover, int* slot_next, hipStream_t st) {
  SplitParams p{lambda, alpha, 0.f};
  gbdt_finalize_kernel<<<1, 256, 0, st>>>(best_gain, best_thr, best_dir, best_hl, node_gh, n_level, F, first,
                                          last_level, p, gamma, eta, max_delta_step, feat, thr, dleft, leaf, gain,
                                          cover, slot_next);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int ct_gbdt_partition(const uint8_t* bins, long ldb, int* node, const int* feat, const int* thr, const uint8_t* dleft,
                      const float* leaf, int first, int N, float* margin, int K, int k, hipStream_t st) {
  if (N <= 0) return 0;
  gbdt_partition_kernel<<<(N + 255) / 256, 256, 0, st>>>(bins, ldb, node, feat, thr, dleft, leaf, first, N, margin,
                                                        K, k);
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
