// hipBLASLt matmul with fused epilogues (bias+GELU with the pre-activation kept, dGELU with the
// bias gradient, bias gradients of the wgrad operands), for the BERT FFN / QKV hot paths where
// the separate elementwise pass costs a full read+write of a [tokens, 4*hidden] activation.
//
// Row-major torch semantics: D[M,N] = alpha * op(A)[M,K] @ op(B)[K,N] + beta * C.  hipBLASLt
// is column-major, so the call is issued as D^T = op(B)^T op(A)^T (operands swapped); the
// "rows" of hipBLASLt's D are then our N (feature) dimension, which is what bias / bias-grad
// vectors are indexed by.  Matmul descriptors and the heuristic's algorithm are cached per
// (shape, strides, ops, epilogue) key; the handle and workspace are PyTorch's own.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/HIPContextLight.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <map>
#include <vector>
#include <mutex>
#include <tuple>

namespace {

#define LT_CHECK(x)                                                                     \
  do {                                                                                  \
    hipblasStatus_t st_ = (x);                                                          \
    TORCH_CHECK(st_ == HIPBLAS_STATUS_SUCCESS, "hipBLASLt: ", #x, " failed: ", (int)st_); \
  } while (0)

using Key = std::tuple<long, long, long, long, long, long, long, long, long, int, int, int, int, int>;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  bool ok = false;
};

std::mutex g_mu;
std::map<Key, Plan> g_plans;

hipDataType dt(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kBFloat16: return HIP_R_16BF;
    case at::kHalf: return HIP_R_16F;
    case at::kFloat: return HIP_R_32F;
    default: TORCH_CHECK(false, "lt_matmul: unsupported dtype");
  }
  return HIP_R_32F;
}

bool rowmajor_ok(const at::Tensor& t) { return t.dim() == 2 && t.stride(1) == 1 && t.stride(0) >= t.size(1); }

}  // namespace

// epilogue: hipblasLtEpilogue_t value.  bias: bias (fwd) or bias-gradient output (BGRAD*,
// DGELU_BGRAD).  aux: pre-activation output (GELU_AUX*) or input (DGELU*).  Returns False when
// hipBLASLt has no algorithm for the combination (caller falls back to separate kernels).
bool lt_matmul(at::Tensor A, at::Tensor B, at::Tensor D, bool trans_a, bool trans_b, double alpha, double beta,
               c10::optional<at::Tensor> C, int64_t epilogue, c10::optional<at::Tensor> bias,
               c10::optional<at::Tensor> aux) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && D.is_cuda(), "lt_matmul: GPU tensors");
  TORCH_CHECK(rowmajor_ok(A) && rowmajor_ok(B) && rowmajor_ok(D), "lt_matmul: 2-D row-major operands");
  const long M = D.size(0), N = D.size(1);
  const long K = trans_a ? A.size(0) : A.size(1);
  TORCH_CHECK((trans_a ? A.size(1) : A.size(0)) == M, "lt_matmul: A rows");
  TORCH_CHECK((trans_b ? B.size(1) : B.size(0)) == K && (trans_b ? B.size(0) : B.size(1)) == N, "lt_matmul: B shape");
  const at::Tensor& Ct = (C.has_value() && C->defined()) ? *C : D;
  TORCH_CHECK(rowmajor_ok(Ct) && Ct.size(0) == M && Ct.size(1) == N, "lt_matmul: C shape");
  const bool has_bias = bias.has_value() && bias->defined();
  const bool has_aux = aux.has_value() && aux->defined();
  if (has_bias) TORCH_CHECK(bias->is_contiguous() && bias->numel() >= N, "lt_matmul: bias length");
  if (has_aux) TORCH_CHECK(rowmajor_ok(*aux) && aux->size(0) == M && aux->size(1) == N, "lt_matmul: aux shape");
  const int bias_dt = has_bias ? (int)dt(*bias) : -1;
  const int aux_dt = has_aux ? (int)dt(*aux) : -1;
  Key key{M, N, K, A.stride(0), B.stride(0), Ct.stride(0), D.stride(0), has_aux ? aux->stride(0) : 0,
          (long)dt(A) * 64 + (long)dt(D), (int)trans_a, (int)trans_b, (int)epilogue, bias_dt, aux_dt};
  const size_t ws_size = at::cuda::getCUDABlasLtWorkspaceSize();
  void* ws = at::cuda::getCUDABlasLtWorkspace();
  hipblasLtHandle_t handle = at::cuda::getCurrentCUDABlasLtHandle();

  Plan* plan;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
      Plan p;
      LT_CHECK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
      // swapped operands: hipBLASLt A := our B, hipBLASLt B := our A
      hipblasOperation_t opa = trans_b ? HIPBLAS_OP_T : HIPBLAS_OP_N;
      hipblasOperation_t opb = trans_a ? HIPBLAS_OP_T : HIPBLAS_OP_N;
      LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
      LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
      hipblasLtEpilogue_t ep = (hipblasLtEpilogue_t)epilogue;
      LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)));
      if (has_bias) {
        hipDataType bt = dt(*bias);
        LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
      }
      if (has_aux) {
        int64_t ld = aux->stride(0);
        hipDataType at_ = dt(*aux);
        LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
        LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at_,
                                                 sizeof(at_)));
      }
      // hipBLASLt A (= our B): stored col-major as [N, K] (no trans) or [K, N] (trans)
      LT_CHECK(hipblasLtMatrixLayoutCreate(&p.a, dt(B), trans_b ? K : N, trans_b ? N : K, B.stride(0)));
      LT_CHECK(hipblasLtMatrixLayoutCreate(&p.b, dt(A), trans_a ? M : K, trans_a ? K : M, A.stride(0)));
      LT_CHECK(hipblasLtMatrixLayoutCreate(&p.c, dt(Ct), N, M, Ct.stride(0)));
      LT_CHECK(hipblasLtMatrixLayoutCreate(&p.d, dt(D), N, M, D.stride(0)));
      hipblasLtMatmulPreference_t pref;
      LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
      uint64_t wsb = ws_size;
      LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb,
                                                     sizeof(wsb)));
      // the epilogue pointers must be set for the heuristic to see a complete problem
      if (has_bias) {
        void* bp = bias->data_ptr();
        LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)));
      }
      if (has_aux) {
        void* ap = aux->data_ptr();
        LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &ap,
                                                 sizeof(ap)));
      }
      hipblasLtMatmulHeuristicResult_t res[8];
      int n = 0;
      hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(handle, p.desc, p.a, p.b, p.c, p.d, pref, 8, res, &n);
      hipblasLtMatmulPreferenceDestroy(pref);
      for (int i = 0; st == HIPBLAS_STATUS_SUCCESS && i < n; ++i) {
        if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= ws_size) {
          p.algo = res[i].algo;
          p.ws = res[i].workspaceSize;
          p.ok = true;
          break;
        }
      }
      it = g_plans.emplace(key, p).first;
    }
    plan = &it->second;
  }
  if (!plan->ok) return false;
  if (has_bias) {
    void* bp = bias->data_ptr();
    LT_CHECK(hipblasLtMatmulDescSetAttribute(plan->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)));
  }
  if (has_aux) {
    void* ap = aux->data_ptr();
    LT_CHECK(hipblasLtMatmulDescSetAttribute(plan->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &ap,
                                             sizeof(ap)));
  }
  const float al = (float)alpha, be = (float)beta;
  LT_CHECK(hipblasLtMatmul(handle, plan->desc, &al, B.data_ptr(), plan->a, A.data_ptr(), plan->b, &be,
                           Ct.data_ptr(), plan->c, D.data_ptr(), plan->d, &plan->algo, ws, plan->ws,
                           at::hip::getCurrentHIPStream().stream()));
  return true;
}

// ---------------------------------------------------------------------------------------
// Strided-batched D[b] = op(A[b]) @ op(B[b]) (beta 0) with the algorithm picked by TIMING every
// solution hipBLASLt has for the problem (hipblaslt_ext::getAllAlgos + matmulIsAlgoSupported),
// once per shape, on the real operands.  Used by the split-K weight-gradient GEMM
// (ops/linear.py): PyTorch's TunableOp does not tune bf16 -> fp32 batched GEMMs, and the
// heuristic's first pick for these transposed-A / fp32-out shapes is a depth-32 tile.
// Candidates slower than 3x the best so far after one run are dropped without more timing.
namespace {
struct BPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  float ms = 0.f;
  int n_tried = 0;
  bool ok = false;
};
std::map<Key, BPlan> g_bplans;

void set_batch(hipblasLtMatrixLayout_t l, int batch, int64_t stride) {
  int32_t bc = batch;
  LT_CHECK(hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc)));
  LT_CHECK(hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &stride,
                                             sizeof(stride)));
}
}  // namespace

// A, B, D: 2-D row-major views of batch 0; batch b's operands start stride_* elements later.
// Returns the tuned algorithm's time in ms (first call) or 0, or -1 when nothing supports it.
double lt_bmm_tuned(at::Tensor A, at::Tensor B, at::Tensor D, bool trans_a, bool trans_b, int64_t batch,
                    int64_t stride_a, int64_t stride_b, int64_t stride_d, int64_t max_timed) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && D.is_cuda(), "lt_bmm_tuned: GPU tensors");
  TORCH_CHECK(rowmajor_ok(A) && rowmajor_ok(B) && rowmajor_ok(D), "lt_bmm_tuned: 2-D row-major operands");
  const long M = D.size(0), N = D.size(1);
  const long K = trans_a ? A.size(0) : A.size(1);
  TORCH_CHECK((trans_a ? A.size(1) : A.size(0)) == M, "lt_bmm_tuned: A rows");
  TORCH_CHECK((trans_b ? B.size(1) : B.size(0)) == K && (trans_b ? B.size(0) : B.size(1)) == N,
              "lt_bmm_tuned: B shape");
  TORCH_CHECK(batch >= 1, "lt_bmm_tuned: batch");
  // the last batch's operands must lie inside the storage the views came from
  auto span_ok = [&](const at::Tensor& t, int64_t stride) {
    const int64_t last = (batch - 1) * stride + (t.size(0) - 1) * t.stride(0) + t.size(1);
    return t.storage_offset() + last <= (int64_t)(t.storage().nbytes() / t.element_size());
  };
  TORCH_CHECK(span_ok(A, stride_a) && span_ok(B, stride_b) && span_ok(D, stride_d), "lt_bmm_tuned: batch span");
  Key key{M, N, K, A.stride(0), B.stride(0), batch, D.stride(0), stride_a * 7 + stride_b * 13 + stride_d,
          (long)dt(A) * 64 + (long)dt(D), (int)trans_a, (int)trans_b, -7, (int)dt(B), 0};
  const size_t ws_size = at::cuda::getCUDABlasLtWorkspaceSize();
  void* ws = at::cuda::getCUDABlasLtWorkspace();
  hipblasLtHandle_t handle = at::cuda::getCurrentCUDABlasLtHandle();
  hipStream_t stream = at::hip::getCurrentHIPStream().stream();
  const float al = 1.f, be = 0.f;
  BPlan* plan;
  double tuned_ms = 0.0;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_bplans.find(key);
    if (it == g_bplans.end()) {
      BPlan p;
      LT_CHECK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
      hipblasOperation_t opa = trans_b ? HIPBLAS_OP_T : HIPBLAS_OP_N;   // swapped operands, as lt_matmul
      hipblasOperation_t opb = trans_a ? HIPBLAS_OP_T : HIPBLAS_OP_N;
      LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
      LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
      LT_CHECK(hipblasLtMatrixLayoutCreate(&p.a, dt(B), trans_b ? K : N, trans_b ? N : K, B.stride(0)));
      LT_CHECK(hipblasLtMatrixLayoutCreate(&p.b, dt(A), trans_a ? M : K, trans_a ? K : M, A.stride(0)));
      LT_CHECK(hipblasLtMatrixLayoutCreate(&p.d, dt(D), N, M, D.stride(0)));
      set_batch(p.a, (int)batch, stride_b);
      set_batch(p.b, (int)batch, stride_a);
      set_batch(p.d, (int)batch, stride_d);
      std::vector<hipblasLtMatmulHeuristicResult_t> all;
      hipblaslt_ext::getAllAlgos(handle, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, opa, opb, dt(B), dt(A), dt(D),
                                 dt(D), HIPBLAS_COMPUTE_32F, all);
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      float best = 1e30f;
      int timed = 0;
      for (auto& r : all) {
        if (max_timed > 0 && timed >= max_timed) break;
        size_t need = 0;
        if (hipblaslt_ext::matmulIsAlgoSupported(handle, p.desc, &al, p.a, p.b, &be, p.d, p.d, r.algo, need) !=
                HIPBLAS_STATUS_SUCCESS || need > ws_size)
          continue;
        auto run = [&]() {
          return hipblasLtMatmul(handle, p.desc, &al, B.data_ptr(), p.a, A.data_ptr(), p.b, &be, D.data_ptr(), p.d,
                                 D.data_ptr(), p.d, &r.algo, ws, need, stream);
        };
        if (run() != HIPBLAS_STATUS_SUCCESS) continue;          // warm-up (and code-object load)
        ++timed;
        hipEventRecord(e0, stream);
        run();
        hipEventRecord(e1, stream);
        hipEventSynchronize(e1);
        float t1 = 0.f;
        hipEventElapsedTime(&t1, e0, e1);
        if (t1 > 3.f * best) continue;
        hipEventRecord(e0, stream);
        for (int i = 0; i < 3; ++i) run();
        hipEventRecord(e1, stream);
        hipEventSynchronize(e1);
        float t3 = 0.f;
        hipEventElapsedTime(&t3, e0, e1);
        const float t = t3 / 3.f;
        if (t < best) {
          best = t;
          p.algo = r.algo;
          p.ws = need;
          p.ok = true;
        }
      }
      hipEventDestroy(e0);
      hipEventDestroy(e1);
      p.ms = p.ok ? best : 0.f;
      p.n_tried = timed;
      tuned_ms = p.ok ? best : -1.0;
      it = g_bplans.emplace(key, p).first;
    }
    plan = &it->second;
  }
  if (!plan->ok) return -1.0;
  LT_CHECK(hipblasLtMatmul(handle, plan->desc, &al, B.data_ptr(), plan->a, A.data_ptr(), plan->b, &be, D.data_ptr(),
                           plan->d, D.data_ptr(), plan->d, &plan->algo, ws, plan->ws, stream));
  return tuned_ms;
}

extern "C" int ct_gemm_nt(const void*, long, const void*, long, void*, long, int, int, int, int, int, const void*,
                          void*, long, float*, int, hipStream_t, int);

// shared checks + launch of gemm_nt / gemm_nn (b_kn: B stored [K, N])
static bool gemm_nt_impl(at::Tensor A, at::Tensor B, at::Tensor D, int64_t epi, bool accumulate,
                         c10::optional<at::Tensor> bias, c10::optional<at::Tensor> aux, c10::optional<at::Tensor> dbias,
                         bool b_kn) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && D.is_cuda(), "gemm_nt: GPU tensors");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16 &&
              D.scalar_type() == at::kBFloat16, "gemm_nt: bf16 operands");
  TORCH_CHECK(rowmajor_ok(A) && rowmajor_ok(B) && rowmajor_ok(D), "gemm_nt: 2-D row-major operands");
  const long M = A.size(0), K = A.size(1), N = b_kn ? B.size(1) : B.size(0);
  TORCH_CHECK((b_kn ? B.size(0) : B.size(1)) == K && D.size(0) == M && D.size(1) == N, "gemm_nt: shape mismatch");
  const bool hb = bias.has_value() && bias->defined(), ha = aux.has_value() && aux->defined(),
             hd = dbias.has_value() && dbias->defined();
  if (hb) TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N,
                      "gemm_nt: bias");
  if (ha) TORCH_CHECK(aux->scalar_type() == at::kBFloat16 && rowmajor_ok(*aux) && aux->size(0) == M &&
                      aux->size(1) == N, "gemm_nt: aux");
  // dbias: [N], or [R][N] with R a power of two (the epilogue spreads its column-sum atomics over
  // the R rows; the caller reduces them)
  const long drows = hd && N > 0 ? dbias->numel() / N : 1;
  if (hd) TORCH_CHECK(dbias->scalar_type() == at::kFloat && dbias->is_contiguous() && dbias->numel() == drows * N &&
                      drows >= 1 && (drows & (drows - 1)) == 0, "gemm_nt: dbias must be [N] or [2^k, N] fp32");
  TORCH_CHECK((epi != 1 && epi != 6) || (hb && ha), "gemm_nt: epilogues 1 / 6 need bias and aux");
  TORCH_CHECK((epi != 2 && epi != 7) || ha, "gemm_nt: epilogues 2 / 7 need aux");
  int rc = ct_gemm_nt(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), D.data_ptr(), D.stride(0), (int)M,
                      (int)N, (int)K, (int)epi, accumulate ? 1 : 0, hb ? bias->data_ptr() : nullptr,
                      ha ? aux->data_ptr() : nullptr, ha ? aux->stride(0) : 0,
                      hd ? dbias->data_ptr<float>() : nullptr, b_kn ? 1 : 0, at::hip::getCurrentHIPStream().stream(),
                      (int)drows);
  return rc == 0;
}

// D[M,N] = A[M,K] @ B[N,K]^T through the hand-written MFMA kernel (csrc/gemm_nt.hip) with
// epilogue 0 plain (accumulate: D +=), 1 bias + GELU keeping aux = pre-activation, 2 dGELU
// with aux = pre-activation and dbias += column sums.  False when the shape is unsupported.
bool gemm_nt(at::Tensor A, at::Tensor B, at::Tensor D, int64_t epi, bool accumulate, c10::optional<at::Tensor> bias,
             c10::optional<at::Tensor> aux, c10::optional<at::Tensor> dbias) {
  return gemm_nt_impl(A, B, D, epi, accumulate, bias, aux, dbias, false);
}

// the same with B stored [K, N] (D = A @ B: a data gradient straight from an [out, in] weight)
bool gemm_nn(at::Tensor A, at::Tensor B, at::Tensor D, int64_t epi, bool accumulate, c10::optional<at::Tensor> bias,
             c10::optional<at::Tensor> aux, c10::optional<at::Tensor> dbias) {
  return gemm_nt_impl(A, B, D, epi, accumulate, bias, aux, dbias, true);
}

extern "C" int ct_gemm_nt_stream(const void*, long, const void*, long, void*, long, int, int, int, int, const void*,
                                 int, int, int, hipStream_t);

// Streamed persistent MFMA GEMM (one workgroup per CU walks its output tiles with one
// continuous K-tile DMA stream): D = A @ B^T (b_kn: B stored [K, N], D = A @ B) [+ bias[N]].
bool gemm_nt_stream(at::Tensor A, at::Tensor B, at::Tensor D, c10::optional<at::Tensor> bias, bool b_kn,
                    int64_t wgs, bool accumulate) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && D.is_cuda(), "gemm_nt_stream: GPU tensors");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16 &&
              D.scalar_type() == at::kBFloat16, "gemm_nt_stream: bf16 operands");
  TORCH_CHECK(rowmajor_ok(A) && rowmajor_ok(B) && rowmajor_ok(D), "gemm_nt_stream: 2-D row-major operands");
  const long M = A.size(0), K = A.size(1), N = b_kn ? B.size(1) : B.size(0);
  TORCH_CHECK((b_kn ? B.size(0) : B.size(1)) == K && D.size(0) == M && D.size(1) == N,
              "gemm_nt_stream: shape mismatch");
  const bool hb = bias.has_value() && bias->defined();
  if (hb) TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N,
                      "gemm_nt_stream: bias");
  int rc = ct_gemm_nt_stream(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), D.data_ptr(), D.stride(0),
                             (int)M, (int)N, (int)K, hb ? 5 : 0, hb ? bias->data_ptr() : nullptr, b_kn ? 1 : 0,
                             (int)wgs, accumulate ? 1 : 0, at::hip::getCurrentHIPStream().stream());
  return rc == 0;
}

extern "C" int ct_gemm_pp(const void*, long, const void*, long, void*, long, int, int, int, int, const void*, void*,
                          long, int, int, hipStream_t);

// Paired-tile persistent MFMA GEMM (gemm_pp.hip): D = A @ B^T with epilogue 0 (plain), 5 (+ bias)
// or 6 (D = gelu(. + bias), aux = gelu'(. + bias)).  False when the shape is unsupported.
bool gemm_pp(at::Tensor A, at::Tensor B, at::Tensor D, int64_t epi, c10::optional<at::Tensor> bias,
             c10::optional<at::Tensor> aux, int64_t wgs, int64_t eslots) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && D.is_cuda(), "gemm_pp: GPU tensors");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16 &&
              D.scalar_type() == at::kBFloat16, "gemm_pp: bf16 operands");
  TORCH_CHECK(rowmajor_ok(A) && rowmajor_ok(B) && rowmajor_ok(D), "gemm_pp: 2-D row-major operands");
  const long M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K && D.size(0) == M && D.size(1) == N, "gemm_pp: shape mismatch");
  const bool hb = bias.has_value() && bias->defined();
  const bool ha = aux.has_value() && aux->defined();
  if (hb) TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N,
                      "gemm_pp: bias");
  if (ha) TORCH_CHECK(aux->scalar_type() == at::kBFloat16 && rowmajor_ok(*aux) && aux->size(0) == M &&
                      aux->size(1) == N, "gemm_pp: aux");
  int rc = ct_gemm_pp(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), D.data_ptr(), D.stride(0), (int)M, (int)N,
                      (int)K, (int)epi, hb ? bias->data_ptr() : nullptr, ha ? aux->data_ptr() : nullptr,
                      ha ? aux->stride(0) : 0, (int)wgs, (int)eslots, at::hip::getCurrentHIPStream().stream());
  return rc == 0;
}

extern "C" int ct_gemm_w4(const void*, long, const void*, long, void*, long, int, int, int, int, int, const void*, void*,
                          long, hipStream_t);

// Four-wave MFMA GEMM (gemm_nt.hip gemm_w4_kernel): D = A @ B^T with epilogue 0 (plain), 5 (+ bias)
// or 6 (D = gelu(. + bias), aux = gelu'(. + bias)).  False when the shape is unsupported.
bool gemm_w4(at::Tensor A, at::Tensor B, at::Tensor D, int64_t epi, c10::optional<at::Tensor> bias,
             c10::optional<at::Tensor> aux) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && D.is_cuda(), "gemm_w4: GPU tensors");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16 &&
              D.scalar_type() == at::kBFloat16, "gemm_w4: bf16 operands");
  TORCH_CHECK(rowmajor_ok(A) && rowmajor_ok(B) && rowmajor_ok(D), "gemm_w4: 2-D row-major operands");
  const long M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K && D.size(0) == M && D.size(1) == N, "gemm_w4: shape mismatch");
  const bool hb = bias.has_value() && bias->defined();
  const bool ha = aux.has_value() && aux->defined();
  if (hb) TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N,
                      "gemm_w4: bias");
  if (ha) TORCH_CHECK(aux->scalar_type() == at::kBFloat16 && rowmajor_ok(*aux) && aux->size(0) == M &&
                      aux->size(1) == N, "gemm_w4: aux");
  int rc = ct_gemm_w4(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), D.data_ptr(), D.stride(0), (int)M, (int)N,
                      (int)K, (int)epi, 0, hb ? bias->data_ptr() : nullptr, ha ? aux->data_ptr() : nullptr,
                      ha ? aux->stride(0) : 0, at::hip::getCurrentHIPStream().stream());
  return rc == 0;
}

extern "C" int ct_gemm_tn2(const void*, long, const void*, long, void*, long, int, int, long, int, int, float*,
                           hipStream_t);

// out[M,N] = A[K,M]^T @ B[K,N] through the MFMA kernel's weight-gradient layout: splits > 1 ->
// out is fp32 [splits, M, N] (partial slabs); splits == 1 -> bf16 [M, N] (+)= result.
static bool gemm_tn2_impl(at::Tensor A, at::Tensor B, at::Tensor out, int64_t splits, bool accumulate,
                          float* biasg) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && out.is_cuda(), "gemm_tn2: GPU tensors");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "gemm_tn2: bf16 operands");
  TORCH_CHECK(rowmajor_ok(A) && rowmajor_ok(B), "gemm_tn2: 2-D row-major operands");
  const long K = A.size(0), M = A.size(1), N = B.size(1);
  TORCH_CHECK(B.size(0) == K, "gemm_tn2: K mismatch");
  long ldo = 0;
  if (splits > 1) {
    TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.dim() == 3 && out.size(0) == splits &&
                out.size(1) == M && out.size(2) == N, "gemm_tn2: fp32 [splits, M, N] slabs");
  } else {
    TORCH_CHECK(out.scalar_type() == at::kBFloat16 && rowmajor_ok(out) && out.size(0) == M && out.size(1) == N,
                "gemm_tn2: bf16 [M, N] out");
    ldo = out.stride(0);
  }
  return ct_gemm_tn2(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), out.data_ptr(), ldo, (int)M, (int)N, K,
                     (int)splits, accumulate ? 1 : 0, biasg, at::hip::getCurrentHIPStream().stream()) == 0;
}

bool gemm_tn2(at::Tensor A, at::Tensor B, at::Tensor out, int64_t splits, bool accumulate) {
  return gemm_tn2_impl(A, B, out, splits, accumulate, nullptr);
}

// the same, also writing biasg[s][m] = sum over split s's K range of A[k][m] (fp32 [splits, M])
bool gemm_tn2_bias(at::Tensor A, at::Tensor B, at::Tensor out, int64_t splits, bool accumulate, at::Tensor biasg) {
  TORCH_CHECK(biasg.is_cuda() && biasg.scalar_type() == at::kFloat && biasg.is_contiguous() &&
              biasg.numel() == splits * A.size(1), "gemm_tn2_bias: fp32 [splits, M] bias partials");
  return gemm_tn2_impl(A, B, out, splits, accumulate, biasg.data_ptr<float>());
}

void register_lt(pybind11::module& m) {
  m.def("gemm_tn2", &gemm_tn2, "weight-gradient GEMM A^T @ B (token-major operands) on the MFMA kernel");
  m.def("gemm_tn2_bias", &gemm_tn2_bias, "gemm_tn2 + per-split column sums of A (bias gradient)");
  m.def("gemm_nt", &gemm_nt, "hand-written MFMA GEMM A @ B^T with fused epilogues");
  m.def("gemm_nt_stream", &gemm_nt_stream, "streamed persistent MFMA GEMM A @ B^T / A @ B (+ bias)",
        pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("D"), pybind11::arg("bias") = pybind11::none(), pybind11::arg("b_kn") = false,
        pybind11::arg("wgs") = 0, pybind11::arg("accumulate") = false);
  m.def("gemm_pp", &gemm_pp, "paired-tile persistent MFMA GEMM A @ B^T (epilogue of one tile beside another's K loop)",
        pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("D"), pybind11::arg("epi") = 0,
        pybind11::arg("bias") = pybind11::none(), pybind11::arg("aux") = pybind11::none(), pybind11::arg("wgs") = 0,
        pybind11::arg("eslots") = 4);
  m.def("gemm_w4", &gemm_w4, "four-wave MFMA GEMM A @ B^T (128 x 128 per wave, AGPR-resident accumulators)",
        pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("D"), pybind11::arg("epi") = 0,
        pybind11::arg("bias") = pybind11::none(), pybind11::arg("aux") = pybind11::none());
  m.def("gemm_nn", &gemm_nn, "hand-written MFMA GEMM A @ B (B stored [K, N]) with fused epilogues");
  m.def("lt_matmul", &lt_matmul, "hipBLASLt matmul with epilogue (row-major semantics)");
  m.def("lt_bmm_tuned", &lt_bmm_tuned, "strided-batched hipBLASLt GEMM, algorithm picked by timing all solutions");
}
