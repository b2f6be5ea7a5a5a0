// Fused softmax cross-entropy with the gradient produced in the same launch.
//
// For BERT pretraining the masked-LM loss is taken only at the gathered masked positions
// (the reference runs HF BERT with `config.dense_seq_output`, run_pretrain_mlperf.py:462,
// i.e. the 1024x30522 decoder only on <= max_predictions_per_seq=76 rows per sequence).
// The [rows, V] logits are read twice (online max/sum pass, then the gradient pass) and the
// gradient  (softmax - onehot) * scale  is written IN PLACE of the logits, so the biggest
// activation of the step is never materialised twice.  `scale` is read from device memory
// (1 / #valid labels, computed on device) so nothing synchronises with the host.
#include "common.h"

namespace ct {

__global__ __launch_bounds__(256) void xent_fwd_kernel(
    const bf16_t* __restrict__ logits, bf16_t* __restrict__ dlogits, int ld, int V,
    const int64_t* __restrict__ labels, float* __restrict__ loss_rows, float* __restrict__ lse_rows,
    const float* __restrict__ scale_dev, int R, int ignore_index, float label_smoothing) {
  __shared__ float red[8];
  __shared__ float red2[8];
  const float scale = scale_dev ? *scale_dev : 1.f;
  const int nvec = ld >> 3;
  for (int r = blockIdx.x; r < R; r += gridDim.x) {
    const u16x8* row = reinterpret_cast<const u16x8*>(logits + (size_t)r * ld);
    const int64_t lab = labels[r];
    const bool valid = lab != ignore_index && lab >= 0 && lab < V;
    // read the target logit before any thread of the block starts overwriting the row
    const float xl = (threadIdx.x == 0 && valid) ? bf2f(logits[(size_t)r * ld + lab]) : 0.f;
    // pass 1: online max / sum-exp per thread
    float mx = -INFINITY, sm = 0.f, sum_logit = 0.f;
    for (int c = threadIdx.x; c < nvec; c += blockDim.x) {
      const u16x8 v = row[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = c * 8 + j;
        if (col < V) {
          const float x = bf2f(v[j]);
          sum_logit += x;
          if (x > mx) { sm = sm * __expf(mx - x) + 1.f; mx = x; }
          else sm += __expf(x - mx);
        }
      }
    }
    // combine (max, sum) across the wave then across waves
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float omx = __shfl_xor(mx, o, 64), osm = __shfl_xor(sm, o, 64);
      const float nmx = fmaxf(mx, omx);
      sm = (mx == -INFINITY ? 0.f : sm * __expf(mx - nmx)) + (omx == -INFINITY ? 0.f : osm * __expf(omx - nmx));
      mx = nmx;
    }
    sum_logit = wave_sum(sum_logit);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if (lane == 0) { red[wid] = mx; red2[wid] = sm; }
    __syncthreads();
    float gmx = -INFINITY;
    for (int w = 0; w < nw; ++w) gmx = fmaxf(gmx, red[w]);
    float gsm = 0.f;
    for (int w = 0; w < nw; ++w) gsm += red2[w] * __expf(red[w] - gmx);
    __syncthreads();
    if (lane == 0) red[wid] = sum_logit;
    __syncthreads();
    float gsl = 0.f;
    for (int w = 0; w < nw; ++w) gsl += red[w];
    const float lse = gmx + __logf(gsm);
    if (threadIdx.x == 0) {
      float loss = 0.f;
      if (valid) {
        loss = (1.f - label_smoothing) * (lse - xl) + label_smoothing * (lse - gsl / V);
      }
      loss_rows[r] = loss;
      if (lse_rows) lse_rows[r] = lse;
    }
    // pass 2: gradient (may overwrite the logits in place: every element is read before
    // it is written by the same thread)
    u16x8* drow = reinterpret_cast<u16x8*>(dlogits + (size_t)r * ld);
    const float sv = valid ? scale : 0.f;
    const float smooth = label_smoothing / V;
    for (int c = threadIdx.x; c < nvec; c += blockDim.x) {
      const u16x8 v = row[c];
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = c * 8 + j;
        float gval = 0.f;
        if (col < V) {
          const float p = __expf(bf2f(v[j]) - lse);
          gval = (p - smooth - (col == lab ? (1.f - label_smoothing) : 0.f)) * sv;
        }
        o[j] = f2bf(gval);
      }
      drow[c] = o;
    }
  }
}

}  // namespace ct

using namespace ct;

extern "C" int ct_xent_fwd(const void* logits, void* dlogits, int ld, int V, const int64_t* labels,
                           float* loss_rows, float* lse_rows, const float* scale_dev, int R,
                           int ignore_index, float label_smoothing, hipStream_t stream) {
  if (ld % 8) return -1;
  int grid = R < 8192 ? R : 8192;
  if (grid < 1) return 0;
  xent_fwd_kernel<<<grid, 256, 0, stream>>>((const bf16_t*)logits, (bf16_t*)dlogits, ld, V, labels,
                                            loss_rows, lse_rows, scale_dev, R, ignore_index,
                                            label_smoothing);
  return 0;
}
