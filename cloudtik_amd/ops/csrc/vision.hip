// Detection ops for gfx950: NMS, ROIAlign fwd/bwd, ROIPool fwd/bwd, SigmoidFocalLoss
// fwd/bwd -- the MI355X-native replacement of the Mask R-CNN csrc entry points
// (reference maskrcnn_benchmark/csrc/vision.cpp:11-24, cpu/nms_cpu.cpp, cpu/ROIAlign_cpu.cpp;
// SURVEY.md §2.13 N2-N4); deformable conv / PS-RoI pooling live in deform.hip.
//
// NMS is the bitmask formulation: kernel 1 computes, for every box i and 64-box column
// block, a 64-bit word of "box j > i overlaps i above the threshold" (one wave per
// (row block, column block) tile, the column boxes staged in LDS); kernel 2 is one
// workgroup that walks the boxes in score order 64 at a time: wave 0 resolves a chunk's
// diagonal words with scalar bit logic, then all 8 waves OR the kept boxes' rows into the
// removed bitmap in LDS (lanes over column words, waves over kept rows).  No host round trip.
#include "common.h"

namespace ct {

// ------------------------------------------------------------------ NMS
__device__ __forceinline__ float iou(const float* a, const float* b, float offset) {
  const float l = fmaxf(a[0], b[0]), t = fmaxf(a[1], b[1]);
  const float r = fminf(a[2], b[2]), btm = fminf(a[3], b[3]);
  const float w = fmaxf(r - l + offset, 0.f), h = fmaxf(btm - t + offset, 0.f);
  const float inter = w * h;
  const float sa = (a[2] - a[0] + offset) * (a[3] - a[1] + offset);
  const float sb = (b[2] - b[0] + offset) * (b[3] - b[1] + offset);
  return inter / fmaxf(sa + sb - inter, 1e-12f);
}

__global__ void __launch_bounds__(64) nms_mask_kernel(const float* __restrict__ boxes, int n, float thr,
                                                      float offset, uint64_t* __restrict__ mask, int cb) {
  const int rb = blockIdx.y, colb = blockIdx.x;
  if (colb < rb) return;                       // only higher-scored boxes suppress
  __shared__ float cbox[64 * 4];
  const int t = threadIdx.x;
  const int cj = colb * 64 + t;
  if (cj < n) {
#pragma unroll
    for (int k = 0; k < 4; ++k) cbox[t * 4 + k] = boxes[cj * 4 + k];
  }
  __syncthreads();
  const int i = rb * 64 + t;
  if (i >= n) return;
  float me[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) me[k] = boxes[i * 4 + k];
  uint64_t bits = 0;
  const int cols = min(64, n - colb * 64);
  const int start = (colb == rb) ? t + 1 : 0;
  for (int j = start; j < cols; ++j)
    if (iou(me, cbox + j * 4, offset) > thr) bits |= (1ull << j);
  mask[(long)i * cb + colb] = bits;
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = __shfl((uint32_t)v, src, 64), hi = __shfl((uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}

// Sequential-over-chunks reduction of the suppression bitmask.  Wave 0 walks the 64x64
// diagonal block of chunk c in registers (a uniform scalar scan with one shuffle per kept
// box); then ALL waves OR the kept rows into the later words of ``removed`` (LDS, ds_or_b64):
// lanes own words, waves split the kept rows, and each thread keeps NMS_OR_UNROLL row loads
// in flight.  With 8 waves a 5000-box NMS is ~10x faster than a single-wave reduction whose
// OR loop issued one dependent global load at a time.
constexpr int NMS_REDUCE_THREADS = 512;
constexpr int NMS_REDUCE_WAVES = NMS_REDUCE_THREADS / 64;

__global__ void __launch_bounds__(NMS_REDUCE_THREADS) nms_reduce_kernel(const uint64_t* __restrict__ mask, int n,
                                                                        int cb, int64_t* __restrict__ keep,
                                                                        int64_t* __restrict__ nkeep) {
  extern __shared__ uint64_t removed[];
  __shared__ uint64_t kept_s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int d = tid; d < cb; d += NMS_REDUCE_THREADS) removed[d] = 0;
  __syncthreads();
  long count = 0;
  for (int c = 0; c < cb; ++c) {
    if (wave == 0) {
      const int box = c * 64 + lane;
      const uint64_t diag = box < n ? mask[(long)box * cb + c] : 0ull;
      uint64_t word = removed[c];
      const int cols = min(64, n - c * 64);
      uint64_t kept = 0;
      for (int k = 0; k < cols; ++k) {         // uniform scalar walk of the chunk
        if (!((word >> k) & 1ull)) {
          kept |= 1ull << k;
          word |= shfl64(diag, k);
        }
      }
      const bool mine = (kept >> lane) & 1ull;
      const uint64_t below = lane ? (kept & ((1ull << lane) - 1ull)) : 0ull;
      if (mine) keep[count + __popcll(below)] = box;
      if (lane == 0) kept_s = kept;
    }
    __syncthreads();
    const uint64_t kept = kept_s;
    count += __popcll(kept);
    if (c + 1 < cb && kept) {
      // this wave's share of the kept rows: every NMS_REDUCE_WAVES-th set bit
      int rows[64 / NMS_REDUCE_WAVES + 1];
      int nr = 0, r = 0;
      for (uint64_t kk = kept; kk; kk &= kk - 1, ++r)
        if ((r % NMS_REDUCE_WAVES) == wave) rows[nr++] = c * 64 + (__ffsll((unsigned long long)kk) - 1);
      for (int d = c + 1 + lane; d < cb; d += 64) {
        uint64_t acc = 0;
        int i = 0;
        for (; i + 4 <= nr; i += 4) {
          const uint64_t a0 = mask[(long)rows[i] * cb + d], a1 = mask[(long)rows[i + 1] * cb + d];
          const uint64_t a2 = mask[(long)rows[i + 2] * cb + d], a3 = mask[(long)rows[i + 3] * cb + d];
          acc |= (a0 | a1) | (a2 | a3);
        }
        for (; i < nr; ++i) acc |= mask[(long)rows[i] * cb + d];
        if (acc) atomicOr((unsigned long long*)&removed[d], (unsigned long long)acc);
      }
    }
    __syncthreads();
  }
  if (tid == 0) *nkeep = count;
}

// ------------------------------------------------------------------ segmented NMS
// Many independent NMS problems in one launch (RPN: per image x pyramid level; box head: per
// image x class).  Boxes are sorted by (segment, score desc); segment s owns boxes
// [seg[s], seg[s+1]) and its bitmask lives at mask + moff[s].  Mask tiles outside a segment
// exit at once; the reduction runs one 8-wave workgroup per segment, so the serial
// 64-box chunk walk is as long as the LARGEST segment rather than the sum of all of them.
__global__ void __launch_bounds__(64) nms_mask_seg_kernel(const float* __restrict__ boxes,
                                                          const int64_t* __restrict__ seg,
                                                          const int64_t* __restrict__ moff, float thr, float offset,
                                                          uint64_t* __restrict__ mask) {
  const int s = blockIdx.z;
  const long base = seg[s];
  const int n = (int)(seg[s + 1] - base);
  const int cb = (n + 63) / 64;
  const int rb = blockIdx.y, colb = blockIdx.x;
  if (rb >= cb || colb >= cb || colb < rb) return;
  __shared__ float cbox[64 * 4];
  const int t = threadIdx.x;
  const int cj = colb * 64 + t;
  if (cj < n) {
#pragma unroll
    for (int k = 0; k < 4; ++k) cbox[t * 4 + k] = boxes[(base + cj) * 4 + k];
  }
  __syncthreads();
  const int i = rb * 64 + t;
  if (i >= n) return;
  float me[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) me[k] = boxes[(base + i) * 4 + k];
  uint64_t bits = 0;
  const int cols = min(64, n - colb * 64);
  const int start = (colb == rb) ? t + 1 : 0;
  for (int j = start; j < cols; ++j)
    if (iou(me, cbox + j * 4, offset) > thr) bits |= (1ull << j);
  mask[moff[s] + (long)i * cb + colb] = bits;
}

__global__ void __launch_bounds__(NMS_REDUCE_THREADS) nms_reduce_seg_kernel(const uint64_t* __restrict__ mask_all,
                                                                            const int64_t* __restrict__ seg,
                                                                            const int64_t* __restrict__ moff,
                                                                            uint8_t* __restrict__ keep) {
  extern __shared__ uint64_t removed[];
  __shared__ uint64_t kept_s;
  const int s = blockIdx.x;
  const long base = seg[s];
  const int n = (int)(seg[s + 1] - base);
  const int cb = (n + 63) / 64;
  const uint64_t* mask = mask_all + moff[s];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int d = tid; d < cb; d += NMS_REDUCE_THREADS) removed[d] = 0;
  __syncthreads();
  for (int c = 0; c < cb; ++c) {
    if (wave == 0) {
      const int box = c * 64 + lane;
      const uint64_t diag = box < n ? mask[(long)box * cb + c] : 0ull;
      uint64_t word = removed[c];
      const int cols = min(64, n - c * 64);
      uint64_t kept = 0;
      for (int k = 0; k < cols; ++k) {
        if (!((word >> k) & 1ull)) {
          kept |= 1ull << k;
          word |= shfl64(diag, k);
        }
      }
      if (box < n) keep[base + box] = (kept >> lane) & 1ull ? 1 : 0;
      if (lane == 0) kept_s = kept;
    }
    __syncthreads();
    const uint64_t kept = kept_s;
    if (c + 1 < cb && kept) {
      int rows[64 / NMS_REDUCE_WAVES + 1];
      int nr = 0, r = 0;
      for (uint64_t kk = kept; kk; kk &= kk - 1, ++r)
        if ((r % NMS_REDUCE_WAVES) == wave) rows[nr++] = c * 64 + (__ffsll((unsigned long long)kk) - 1);
      for (int d = c + 1 + lane; d < cb; d += 64) {
        uint64_t acc = 0;
        int i = 0;
        for (; i + 4 <= nr; i += 4) {
          const uint64_t a0 = mask[(long)rows[i] * cb + d], a1 = mask[(long)rows[i + 1] * cb + d];
          const uint64_t a2 = mask[(long)rows[i + 2] * cb + d], a3 = mask[(long)rows[i + 3] * cb + d];
          acc |= (a0 | a1) | (a2 | a3);
        }
        for (; i < nr; ++i) acc |= mask[(long)rows[i] * cb + d];
        if (acc) atomicOr((unsigned long long*)&removed[d], (unsigned long long)acc);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ ROIAlign
template <typename T>
__device__ __forceinline__ float bilinear(const T* f, int H, int W, float y, float x) {
  if (y < -1.f || y > H || x < -1.f || x > W) return 0.f;
  y = fmaxf(y, 0.f);
  x = fmaxf(x, 0.f);
  int y0 = (int)y, x0 = (int)x, y1, x1;
  if (y0 >= H - 1) { y1 = y0 = H - 1; y = (float)y0; } else y1 = y0 + 1;
  if (x0 >= W - 1) { x1 = x0 = W - 1; x = (float)x0; } else x1 = x0 + 1;
  const float ly = y - y0, lx = x - x0, hy = 1.f - ly, hx = 1.f - lx;
  return hy * hx * to_f<T>(f[y0 * W + x0]) + hy * lx * to_f<T>(f[y0 * W + x1]) +
         ly * hx * to_f<T>(f[y1 * W + x0]) + ly * lx * to_f<T>(f[y1 * W + x1]);
}

struct RoiGeom { float x0, y0, bw, bh; int gh, gw; };

__device__ __forceinline__ RoiGeom roi_geom(const float* r, float scale, int PH, int PW, int sr, bool aligned) {
  const float off = aligned ? 0.5f : 0.f;
  const float x0 = r[1] * scale - off, y0 = r[2] * scale - off;
  const float x1 = r[3] * scale - off, y1 = r[4] * scale - off;
  float rw = x1 - x0, rh = y1 - y0;
  if (!aligned) { rw = fmaxf(rw, 1.f); rh = fmaxf(rh, 1.f); }
  RoiGeom g;
  g.x0 = x0; g.y0 = y0; g.bw = rw / PW; g.bh = rh / PH;
  g.gh = sr > 0 ? sr : (int)ceilf(rh / PH);
  g.gw = sr > 0 ? sr : (int)ceilf(rw / PW);
  return g;
}

template <typename T>
__global__ void __launch_bounds__(256) roi_align_fwd_kernel(const T* __restrict__ feat, const float* __restrict__ rois,
                                                             T* __restrict__ out, int K, int C, int H, int W, int PH,
                                                             int PW, float scale, int sr, int aligned) {
  const long total = (long)K * C * PH * PW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int pw = i % PW, ph = (i / PW) % PH, c = (i / ((long)PW * PH)) % C;
    const int k = i / ((long)PW * PH * C);
    const float* r = rois + k * 5;
    const int b = (int)r[0];
    const RoiGeom g = roi_geom(r, scale, PH, PW, sr, aligned);
    const T* f = feat + ((long)b * C + c) * H * W;
    float acc = 0.f;
    for (int iy = 0; iy < g.gh; ++iy) {
      const float y = g.y0 + ph * g.bh + (iy + 0.5f) * g.bh / g.gh;
      for (int ix = 0; ix < g.gw; ++ix) {
        const float x = g.x0 + pw * g.bw + (ix + 0.5f) * g.bw / g.gw;
        acc += bilinear(f, H, W, y, x);
      }
    }
    out[i] = from_f<T>(acc / fmaxf((float)(g.gh * g.gw), 1.f));
  }
}

template <typename T>
__global__ void __launch_bounds__(256) roi_align_bwd_kernel(const T* __restrict__ gout, const float* __restrict__ rois,
                                                             float* __restrict__ gfeat, int K, int C, int H, int W, int PH,
                                                             int PW, float scale, int sr, int aligned) {
  const long total = (long)K * C * PH * PW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int pw = i % PW, ph = (i / PW) % PH, c = (i / ((long)PW * PH)) % C;
    const int k = i / ((long)PW * PH * C);
    const float* r = rois + k * 5;
    const int b = (int)r[0];
    const RoiGeom g = roi_geom(r, scale, PH, PW, sr, aligned);
    float* f = gfeat + ((long)b * C + c) * H * W;
    const float go = to_f<T>(gout[i]) / fmaxf((float)(g.gh * g.gw), 1.f);
    for (int iy = 0; iy < g.gh; ++iy) {
      float y = g.y0 + ph * g.bh + (iy + 0.5f) * g.bh / g.gh;
      for (int ix = 0; ix < g.gw; ++ix) {
        float x = g.x0 + pw * g.bw + (ix + 0.5f) * g.bw / g.gw;
        if (y < -1.f || y > H || x < -1.f || x > W) continue;
        y = fmaxf(y, 0.f);
        x = fmaxf(x, 0.f);
        int y0 = (int)y, x0 = (int)x, y1, x1;
        float yy = y, xx = x;
        if (y0 >= H - 1) { y1 = y0 = H - 1; yy = (float)y0; } else y1 = y0 + 1;
        if (x0 >= W - 1) { x1 = x0 = W - 1; xx = (float)x0; } else x1 = x0 + 1;
        const float ly = yy - y0, lx = xx - x0, hy = 1.f - ly, hx = 1.f - lx;
        atomicAdd(f + y0 * W + x0, go * hy * hx);
        atomicAdd(f + y0 * W + x1, go * hy * lx);
        atomicAdd(f + y1 * W + x0, go * ly * hx);
        atomicAdd(f + y1 * W + x1, go * ly * lx);
      }
    }
  }
}

// ------------------------------------------------------------------ ROIAlign, NHWC
// Channels-last variant for the detection models, whose FPN maps are NHWC bf16: one thread
// owns 8 consecutive channels of one output bin, so every bilinear tap is a 16-byte load and
// the 32 threads of a 256-channel bin read one contiguous 512-byte row segment (no NCHW
// transpose of the pyramid, and the [K, PH, PW, C] output is the channels_last layout the
// box / mask head convolutions consume).  Backward scatters with per-channel fp32 atomics
// into an NHWC gradient; neighbouring lanes hit neighbouring addresses (the backward gives
// each lane channels cg, cg + C/8, ... for that).
template <typename T> struct Vec8;
template <> struct Vec8<bf16_t> {
  __device__ static void load(const bf16_t* p, float v[8]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ static void store(bf16_t* p, const float v[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct Vec8<float> {
  __device__ static void load(const float* p, float v[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ static void store(float* p, const float v[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};

struct Tap4 { int o[4]; float w[4]; bool valid; };

// bilinear corner offsets (in pixels of an H x W map) and weights of one sample point
__device__ __forceinline__ Tap4 bilinear_taps(int H, int W, float y, float x) {
  Tap4 t;
  t.valid = !(y < -1.f || y > H || x < -1.f || x > W);
  if (!t.valid) return t;
  y = fmaxf(y, 0.f);
  x = fmaxf(x, 0.f);
  int y0 = (int)y, x0 = (int)x, y1, x1;
  if (y0 >= H - 1) { y1 = y0 = H - 1; y = (float)y0; } else y1 = y0 + 1;
  if (x0 >= W - 1) { x1 = x0 = W - 1; x = (float)x0; } else x1 = x0 + 1;
  const float ly = y - y0, lx = x - x0, hy = 1.f - ly, hx = 1.f - lx;
  t.o[0] = y0 * W + x0; t.o[1] = y0 * W + x1; t.o[2] = y1 * W + x0; t.o[3] = y1 * W + x1;
  t.w[0] = hy * hx; t.w[1] = hy * lx; t.w[2] = ly * hx; t.w[3] = ly * lx;
  return t;
}

// Pyramid levels of one multi-level ROIAlign launch (FPN P2-P5): every RoI carries its level
// (``lvl``, int32; null = level 0), so all levels are pooled by ONE launch with no host-side
// split (the per-level nonzero() + index_copy of a level loop costs a host sync per level).
constexpr int kMaxLevels = 5;
template <typename P> struct Levels {
  P f[kMaxLevels];
  int H[kMaxLevels], W[kMaxLevels];
  float scale[kMaxLevels];
};
// select level l with static indices (v_cndmask), so the descriptor stays in kernel arguments
template <typename P>
__device__ __forceinline__ void pick_level(const Levels<P>& L, int l, P& f, int& H, int& W, float& scale) {
  f = L.f[0]; H = L.H[0]; W = L.W[0]; scale = L.scale[0];
#pragma unroll
  for (int j = 1; j < kMaxLevels; ++j)
    if (l == j) { f = L.f[j]; H = L.H[j]; W = L.W[j]; scale = L.scale[j]; }
}

template <typename T>
__global__ void __launch_bounds__(256) roi_align_nhwc_fwd_kernel(const Levels<const T*> L, const int* __restrict__ lvl,
                                                                  const float* __restrict__ rois, T* __restrict__ out,
                                                                  int K, int C, int PH, int PW, int sr, int aligned) {
  const int CG = C / 8;
  const long total = (long)K * PH * PW * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cg = i % CG;
    const long bin = i / CG;                       // (k, ph, pw)
    const int pw = bin % PW, ph = (bin / PW) % PH, k = bin / ((long)PW * PH);
    const float* r = rois + k * 5;
    const int b = (int)r[0];
    const T* feat;
    int H, W;
    float scale;
    pick_level(L, lvl ? lvl[k] : 0, feat, H, W, scale);
    const RoiGeom g = roi_geom(r, scale, PH, PW, sr, aligned);
    const T* f = feat + (long)b * H * W * C + cg * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int iy = 0; iy < g.gh; ++iy) {
      const float y = g.y0 + ph * g.bh + (iy + 0.5f) * g.bh / g.gh;
      for (int ix = 0; ix < g.gw; ++ix) {
        const float x = g.x0 + pw * g.bw + (ix + 0.5f) * g.bw / g.gw;
        const Tap4 t = bilinear_taps(H, W, y, x);
        if (!t.valid) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v[8];
          Vec8<T>::load(f + (long)t.o[q] * C, v);
#pragma unroll
          for (int c = 0; c < 8; ++c) acc[c] += t.w[q] * v[c];
        }
      }
    }
    const float inv = 1.f / fmaxf((float)(g.gh * g.gw), 1.f);
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] *= inv;
    Vec8<T>::store(out + bin * C + cg * 8, acc);
  }
}

// Backward: atomics, not arithmetic, bound this kernel.  With the detection models' sampling
// ratio 2 the bilinear weights of a bin are separable -- W(row, col) = Wy(row) * Wx(col) with
// Wy / Wx each summed over the bin's 2 sample rows / columns -- and neighbouring samples share
// pixels, so a bin touches ~3 x 3 distinct pixels through its 16 taps.  The per-axis tap
// lists (4 entries, sorted) are merged in registers (static indexing, no scratch) and one
// fp32 atomic is issued per distinct pixel and channel.  Other sampling ratios take the
// direct per-tap path.
__device__ __forceinline__ void axis_taps(float v, int n, float p0, float step, int idx[4], float w[4]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    float y = p0 + (s + 0.5f) * step;
    if (y < -1.f || y > n) { idx[2 * s] = idx[2 * s + 1] = (s ? idx[1] : 0); w[2 * s] = w[2 * s + 1] = 0.f; continue; }
    y = fmaxf(y, 0.f);
    int y0 = (int)y, y1;
    if (y0 >= n - 1) { y1 = y0 = n - 1; y = (float)y0; } else y1 = y0 + 1;
    const float l = y - y0;
    idx[2 * s] = y0; idx[2 * s + 1] = y1;
    w[2 * s] = (1.f - l) * v; w[2 * s + 1] = l * v;
  }
  // merge equal neighbours (the list is non-decreasing): fold into the first occurrence
#pragma unroll
  for (int j = 3; j >= 1; --j)
    if (idx[j] == idx[j - 1]) { w[j - 1] += w[j]; w[j] = 0.f; }
}

template <typename T>
__global__ void __launch_bounds__(256) roi_align_nhwc_bwd_kernel(const T* __restrict__ gout, const Levels<float*> L,
                                                                  const int* __restrict__ lvl,
                                                                  const float* __restrict__ rois, int K, int C, int PH,
                                                                  int PW, int sr, int aligned) {
  const int CG = C / 8;
  const long total = (long)K * PH * PW * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cg = i % CG;
    const long bin = i / CG;
    const int pw = bin % PW, ph = (bin / PW) % PH, k = bin / ((long)PW * PH);
    const float* r = rois + k * 5;
    const int b = (int)r[0];
    float* gfeat;
    int H, W;
    float scale;
    pick_level(L, lvl ? lvl[k] : 0, gfeat, H, W, scale);
    const RoiGeom g = roi_geom(r, scale, PH, PW, sr, aligned);
    // lane-strided channels (cg, cg + CG, ...): consecutive lanes of a wave add into
    // consecutive floats, so every atomic instruction covers whole 128 B lines instead of
    // scattering 4 B per lane over 32 B strides
    float go[8];
    const T* gp = gout + bin * C + cg;
#pragma unroll
    for (int c = 0; c < 8; ++c) go[c] = to_f<T>(gp[c * CG]);
    const float inv = 1.f / fmaxf((float)(g.gh * g.gw), 1.f);
    float* f = gfeat + (long)b * H * W * C + cg;
    if (g.gh == 2 && g.gw == 2) {
      int ry[4], cx[4];
      float wy[4], wx[4];
      axis_taps(inv, H, g.y0 + ph * g.bh, g.bh / 2, ry, wy);
      axis_taps(1.f, W, g.x0 + pw * g.bw, g.bw / 2, cx, wx);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        if (wy[a] == 0.f) continue;
#pragma unroll
        for (int c2 = 0; c2 < 4; ++c2) {
          const float wq = wy[a] * wx[c2];
          if (wq == 0.f) continue;
          float* dst = f + ((long)ry[a] * W + cx[c2]) * C;
#pragma unroll
          for (int c = 0; c < 8; ++c) unsafeAtomicAdd(dst + c * CG, go[c] * wq);
        }
      }
      continue;
    }
    for (int iy = 0; iy < g.gh; ++iy) {
      const float y = g.y0 + ph * g.bh + (iy + 0.5f) * g.bh / g.gh;
      for (int ix = 0; ix < g.gw; ++ix) {
        const float x = g.x0 + pw * g.bw + (ix + 0.5f) * g.bw / g.gw;
        const Tap4 t = bilinear_taps(H, W, y, x);
        if (!t.valid) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float* dst = f + (long)t.o[q] * C;
          const float wq = t.w[q] * inv;
#pragma unroll
          for (int c = 0; c < 8; ++c) unsafeAtomicAdd(dst + c * CG, go[c] * wq);
        }
      }
    }
  }
}

// ------------------------------------------------------------------ ROIPool
template <typename T>
__global__ void __launch_bounds__(256) roi_pool_fwd_kernel(const T* __restrict__ feat, const float* __restrict__ rois,
                                                            T* __restrict__ out, int* __restrict__ argmax, int K, int C,
                                                            int H, int W, int PH, int PW, float scale) {
  const long total = (long)K * C * PH * PW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int pw = i % PW, ph = (i / PW) % PH, c = (i / ((long)PW * PH)) % C;
    const int k = i / ((long)PW * PH * C);
    const float* r = rois + k * 5;
    const int b = (int)r[0];
    const int x0 = (int)roundf(r[1] * scale), y0 = (int)roundf(r[2] * scale);
    const int x1 = (int)roundf(r[3] * scale), y1 = (int)roundf(r[4] * scale);
    const int rw = max(x1 - x0 + 1, 1), rh = max(y1 - y0 + 1, 1);
    const float bw = (float)rw / PW, bh = (float)rh / PH;
    int hs = min(max((int)floorf(ph * bh) + y0, 0), H), he = min(max((int)ceilf((ph + 1) * bh) + y0, 0), H);
    int ws = min(max((int)floorf(pw * bw) + x0, 0), W), we = min(max((int)ceilf((pw + 1) * bw) + x0, 0), W);
    const T* f = feat + ((long)b * C + c) * H * W;
    float best = (he <= hs || we <= ws) ? 0.f : -INFINITY;
    int arg = -1;
    for (int y = hs; y < he; ++y)
      for (int x = ws; x < we; ++x) {
        const float v = to_f<T>(f[y * W + x]);
        if (v > best) { best = v; arg = y * W + x; }
      }
    out[i] = from_f<T>(best);
    argmax[i] = arg;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) roi_pool_bwd_kernel(const T* __restrict__ gout, const float* __restrict__ rois,
                                                            const int* __restrict__ argmax, float* __restrict__ gfeat,
                                                            int K, int C, int H, int W, int PH, int PW) {
  const long total = (long)K * C * PH * PW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int a = argmax[i];
    if (a < 0) continue;
    const int c = (i / ((long)PW * PH)) % C;
    const int k = i / ((long)PW * PH * C);
    const int b = (int)rois[k * 5];
    atomicAdd(gfeat + ((long)b * C + c) * H * W + a, to_f<T>(gout[i]));
  }
}

// ------------------------------------------------------------------ SigmoidFocalLoss
template <typename T>
__global__ void __launch_bounds__(256) focal_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                         float* __restrict__ loss, long N, int C, float gamma, float alpha) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < N * C; i += (long)gridDim.x * blockDim.x) {
    const long n = i / C;
    const int c = (int)(i % C);
    const long t = tgt[n];
    const float c1 = (t == c + 1), c2 = (t >= 0) & (t != c + 1);
    const float x = to_f<T>(logits[i]);
    const float p = 1.f / (1.f + __expf(-x));
    const float term1 = powf(1.f - p, gamma) * __logf(fmaxf(p, 1.17549435e-38f));
    // log(1-p) computed stably: -x*(x>=0) - log(1+exp(-|x|))
    const float log1mp = -x * (x >= 0.f) - __logf(1.f + __expf(x - 2.f * x * (x >= 0.f)));
    const float term2 = powf(p, gamma) * log1mp;
    loss[i] = -c1 * alpha * term1 - c2 * (1.f - alpha) * term2;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) focal_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                         const float* __restrict__ gloss, T* __restrict__ glogits,
                                                         long N, int C, float gamma, float alpha) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < N * C; i += (long)gridDim.x * blockDim.x) {
    const long n = i / C;
    const int c = (int)(i % C);
    const long t = tgt[n];
    const float c1 = (t == c + 1), c2 = (t >= 0) & (t != c + 1);
    const float x = to_f<T>(logits[i]);
    const float p = 1.f / (1.f + __expf(-x));
    const float logp = __logf(fmaxf(p, 1.17549435e-38f));
    const float log1mp = -x * (x >= 0.f) - __logf(1.f + __expf(x - 2.f * x * (x >= 0.f)));
    const float d1 = powf(1.f - p, gamma) * (1.f - p - gamma * p * logp);
    const float d2 = powf(p, gamma) * (gamma * (1.f - p) * log1mp - p);
    glogits[i] = from_f<T>(gloss[i] * (-c1 * alpha * d1 - c2 * (1.f - alpha) * d2));
  }
}

inline int grid1d(long n) {
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  return g < 1 ? 1 : (int)g;
}

}  // namespace ct

using namespace ct;

extern "C" int ct_nms(const float* boxes, int n, float thr, float offset, uint64_t* mask_ws, int64_t* keep,
                      int64_t* nkeep, hipStream_t stream) {
  if (n <= 0) return -1;
  const int cb = (n + 63) / 64;
  if (cb * 8 > 64 * 1024) return -2;               // removed bitmap must fit in LDS (n <= 524288)
  nms_mask_kernel<<<dim3(cb, cb), 64, 0, stream>>>(boxes, n, thr, offset, mask_ws, cb);
  nms_reduce_kernel<<<1, NMS_REDUCE_THREADS, cb * sizeof(uint64_t), stream>>>(mask_ws, n, cb, keep, nkeep);
  return 0;
}

// seg [nseg+1] / moff [nseg] on the device; max_n = largest segment (host-known)
extern "C" int ct_nms_segmented(const float* boxes, const int64_t* seg, const int64_t* moff, int nseg, int max_n,
                                float thr, float offset, uint64_t* mask_ws, uint8_t* keep, hipStream_t stream) {
  if (nseg <= 0 || max_n <= 0) return -1;
  const int cb = (max_n + 63) / 64;
  if (cb * 8 > 64 * 1024 || nseg > 65535) return -2;
  nms_mask_seg_kernel<<<dim3(cb, cb, nseg), 64, 0, stream>>>(boxes, seg, moff, thr, offset, mask_ws);
  nms_reduce_seg_kernel<<<nseg, NMS_REDUCE_THREADS, cb * sizeof(uint64_t), stream>>>(mask_ws, seg, moff, keep);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

extern "C" int ct_roi_align_fwd(const void* feat, const float* rois, void* out, int dt, int K, int C, int H, int W,
                                int PH, int PW, float scale, int sr, int aligned, hipStream_t stream) {
  const int g = grid1d((long)K * C * PH * PW);
  if (dt == 0) roi_align_fwd_kernel<float><<<g, 256, 0, stream>>>((const float*)feat, rois, (float*)out, K, C, H, W, PH, PW, scale, sr, aligned);
  else roi_align_fwd_kernel<bf16_t><<<g, 256, 0, stream>>>((const bf16_t*)feat, rois, (bf16_t*)out, K, C, H, W, PH, PW, scale, sr, aligned);
  return 0;
}

extern "C" int ct_roi_align_bwd(const void* gout, const float* rois, float* gfeat, int dt, int K, int C, int H, int W,
                                int PH, int PW, float scale, int sr, int aligned, hipStream_t stream) {
  const int g = grid1d((long)K * C * PH * PW);
  if (dt == 0) roi_align_bwd_kernel<float><<<g, 256, 0, stream>>>((const float*)gout, rois, gfeat, K, C, H, W, PH, PW, scale, sr, aligned);
  else roi_align_bwd_kernel<bf16_t><<<g, 256, 0, stream>>>((const bf16_t*)gout, rois, gfeat, K, C, H, W, PH, PW, scale, sr, aligned);
  return 0;
}

// nlev levels: feats[l] / gfeats[l] NHWC maps of hw[2l] x hw[2l+1]; lvl [K] int32 on the
// device (null when nlev == 1)
extern "C" int ct_roi_align_nhwc_fwd(const void* const* feats, const int* hw, const float* scales, int nlev,
                                     const int* lvl, const float* rois, void* out, int dt, int K, int C, int PH, int PW,
                                     int sr, int aligned, hipStream_t stream) {
  if (C % 8 || nlev < 1 || nlev > kMaxLevels || (nlev > 1 && !lvl)) return 1;
  const int g = grid1d((long)K * PH * PW * (C / 8));
  if (dt == 0) {
    Levels<const float*> L{};
    for (int l = 0; l < nlev; ++l) { L.f[l] = (const float*)feats[l]; L.H[l] = hw[2 * l]; L.W[l] = hw[2 * l + 1]; L.scale[l] = scales[l]; }
    roi_align_nhwc_fwd_kernel<float><<<g, 256, 0, stream>>>(L, nlev > 1 ? lvl : nullptr, rois, (float*)out, K, C, PH, PW, sr, aligned);
  } else {
    Levels<const bf16_t*> L{};
    for (int l = 0; l < nlev; ++l) { L.f[l] = (const bf16_t*)feats[l]; L.H[l] = hw[2 * l]; L.W[l] = hw[2 * l + 1]; L.scale[l] = scales[l]; }
    roi_align_nhwc_fwd_kernel<bf16_t><<<g, 256, 0, stream>>>(L, nlev > 1 ? lvl : nullptr, rois, (bf16_t*)out, K, C, PH, PW, sr, aligned);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int ct_roi_align_nhwc_bwd(const void* gout, float* const* gfeats, const int* hw, const float* scales,
                                     int nlev, const int* lvl, const float* rois, int dt, int K, int C, int PH, int PW,
                                     int sr, int aligned, hipStream_t stream) {
  if (C % 8 || nlev < 1 || nlev > kMaxLevels || (nlev > 1 && !lvl)) return 1;
  const int g = grid1d((long)K * PH * PW * (C / 8));
  Levels<float*> L{};
  for (int l = 0; l < nlev; ++l) { L.f[l] = gfeats[l]; L.H[l] = hw[2 * l]; L.W[l] = hw[2 * l + 1]; L.scale[l] = scales[l]; }
  if (dt == 0) roi_align_nhwc_bwd_kernel<float><<<g, 256, 0, stream>>>((const float*)gout, L, nlev > 1 ? lvl : nullptr, rois, K, C, PH, PW, sr, aligned);
  else roi_align_nhwc_bwd_kernel<bf16_t><<<g, 256, 0, stream>>>((const bf16_t*)gout, L, nlev > 1 ? lvl : nullptr, rois, K, C, PH, PW, sr, aligned);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int ct_roi_pool_fwd(const void* feat, const float* rois, void* out, int* argmax, int dt, int K, int C, int H,
                               int W, int PH, int PW, float scale, hipStream_t stream) {
  const int g = grid1d((long)K * C * PH * PW);
  if (dt == 0) roi_pool_fwd_kernel<float><<<g, 256, 0, stream>>>((const float*)feat, rois, (float*)out, argmax, K, C, H, W, PH, PW, scale);
  else roi_pool_fwd_kernel<bf16_t><<<g, 256, 0, stream>>>((const bf16_t*)feat, rois, (bf16_t*)out, argmax, K, C, H, W, PH, PW, scale);
  return 0;
}

extern "C" int ct_roi_pool_bwd(const void* gout, const float* rois, const int* argmax, float* gfeat, int dt, int K, int C,
                               int H, int W, int PH, int PW, hipStream_t stream) {
  const int g = grid1d((long)K * C * PH * PW);
  if (dt == 0) roi_pool_bwd_kernel<float><<<g, 256, 0, stream>>>((const float*)gout, rois, argmax, gfeat, K, C, H, W, PH, PW);
  else roi_pool_bwd_kernel<bf16_t><<<g, 256, 0, stream>>>((const bf16_t*)gout, rois, argmax, gfeat, K, C, H, W, PH, PW);
  return 0;
}

extern "C" int ct_focal_fwd(const void* logits, const int64_t* tgt, float* loss, int dt, long N, int C, float gamma,
                            float alpha, hipStream_t stream) {
  const int g = grid1d(N * C);
  if (dt == 0) focal_fwd_kernel<float><<<g, 256, 0, stream>>>((const float*)logits, tgt, loss, N, C, gamma, alpha);
  else focal_fwd_kernel<bf16_t><<<g, 256, 0, stream>>>((const bf16_t*)logits, tgt, loss, N, C, gamma, alpha);
  return 0;
}

extern "C" int ct_focal_bwd(const void* logits, const int64_t* tgt, const float* gloss, void* glogits, int dt, long N,
                            int C, float gamma, float alpha, hipStream_t stream) {
  const int g = grid1d(N * C);
  if (dt == 0) focal_bwd_kernel<float><<<g, 256, 0, stream>>>((const float*)logits, tgt, gloss, (float*)glogits, N, C, gamma, alpha);
  else focal_bwd_kernel<bf16_t><<<g, 256, 0, stream>>>((const bf16_t*)logits, tgt, gloss, (bf16_t*)glogits, N, C, gamma, alpha);
  return 0;
}

// ---------------------------------------------------------------------- image ingest
// uint8 HWC images (as decoded / as stored in Parquet) -> bf16 NHWC (= channels_last NCHW),
// (x / 255 - mean[c]) / std[c], with an optional per-image horizontal flip.  The loader
// ships uint8 over PCIe (half the bytes of bf16); this one pass replaces the
// convert/normalise/permute chain.  Each thread moves 4 pixels: three aligned 32-bit loads
// (12 bytes) and three aligned 64-bit stores (4 x 3 bf16).  Requires W % 4 == 0.
__global__ __launch_bounds__(256) void image_u8_to_bf16_kernel(const uint8_t* __restrict__ in,
                                                               bf16_t* __restrict__ out,
                                                               const uint8_t* __restrict__ flip, long total4,
                                                               int H, int W, float m0, float m1, float m2,
                                                               float s0, float s1, float s2) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;   // quad of output pixels
  if (q >= total4) return;
  const int W4 = W >> 2;
  const long row = q / W4;                               // n * H + h
  const int x4 = (int)(q - row * W4);
  const long n = row / H;
  int src4 = x4;
  const bool f = flip && flip[n];
  if (f) src4 = W4 - 1 - x4;
  const uint32_t* p = reinterpret_cast<const uint32_t*>(in + (row * W + (long)src4 * 4) * 3);
  uint32_t w[3] = {p[0], p[1], p[2]};
  uint8_t px[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) px[i] = (w[i >> 2] >> (8 * (i & 3))) & 0xff;
  const float inv[3] = {1.f / (255.f * s0), 1.f / (255.f * s1), 1.f / (255.f * s2)};
  const float off[3] = {m0 / s0, m1 / s1, m2 / s2};
  bf16_t o[12];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int sp = f ? 3 - k : k;   // mirrored pixel order inside the quad
#pragma unroll
    for (int c = 0; c < 3; ++c) o[k * 3 + c] = f2bf((float)px[sp * 3 + c] * inv[c] - off[c]);
  }
  uint64_t* d = reinterpret_cast<uint64_t*>(out + (row * W + (long)x4 * 4) * 3);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    d[i] = (uint64_t)o[4 * i] | ((uint64_t)o[4 * i + 1] << 16) | ((uint64_t)o[4 * i + 2] << 32) |
           ((uint64_t)o[4 * i + 3] << 48);
  }
}

extern "C" int ct_image_u8_to_bf16(const uint8_t* in, void* out, const uint8_t* flip, int N, int H, int W,
                                   const float* mean, const float* stdv, hipStream_t stream) {
  if (N <= 0) return 0;
  if (W % 4) return 1;
  const long total4 = (long)N * H * (W / 4);
  image_u8_to_bf16_kernel<<<(unsigned)((total4 + 255) / 256), 256, 0, stream>>>(
      in, (bf16_t*)out, flip, total4, H, W, mean[0], mean[1], mean[2], stdv[0], stdv[1], stdv[2]);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
