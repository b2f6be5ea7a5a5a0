// Bindings for the GBDT histogram / ensemble-predict kernels and CSR SpMM (graph_ml.hip).
// All shape, dtype and alignment checks are done here, before any launch.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

extern "C" {
int ct_gbdt_hist(const uint8_t*, long, const int*, const int*, int, const void*, float*, int, int, int, int, int,
                 hipStream_t);
int ct_gbdt_split(const float*, const float*, const int*, float*, const uint8_t*, int, int, int, float, float, float,
                  float*, int*, int*, float*, float*, hipStream_t);
int ct_gbdt_finalize(const float*, const int*, const int*, const float*, const float*, int, int, int, int, float, float,
                     float, float, float, int*, int*, uint8_t*, float*, float*, float*, int*, hipStream_t);
int ct_gbdt_partition(const uint8_t*, long, int*, const int*, const int*, const uint8_t*, const float*, int, int,
                      float*, int, int, hipStream_t);
int ct_gbdt_predict(const uint8_t*, long, const int*, const int*, const uint8_t*, const float*, int, int, int, int,
                    float*, hipStream_t);
int ct_csr_spmm(const int64_t*, const int64_t*, const float*, const float*, int, const void*, long, void*, long, int,
                int, int, hipStream_t);
}

namespace {

#define GCHECK(x) TORCH_CHECK((x).is_cuda() && (x).is_contiguous(), #x " must be a contiguous GPU tensor")
#define GDT(x, d) TORCH_CHECK((x).scalar_type() == (d), #x " has the wrong dtype")

hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// bins [F, ldb] uint8 (ldb % 4 == 0), node [N] int32, gh [N, 2] fp32, hist [S_total, F, B, 2] fp32
void gbdt_hist(at::Tensor bins, int64_t n_rows, at::Tensor node, at::Tensor gh, at::Tensor hist, int64_t slot_lo,
               int64_t n_slots, c10::optional<at::Tensor> slot_map) {
  GCHECK(bins); GCHECK(node); GCHECK(gh); GCHECK(hist);
  GDT(bins, at::kByte); GDT(node, at::kInt); GDT(gh, at::kFloat); GDT(hist, at::kFloat);
  TORCH_CHECK(bins.dim() == 2 && hist.dim() == 4 && hist.size(3) == 2, "gbdt_hist: bad ranks");
  const int F = (int)bins.size(0);
  const long ldb = bins.size(1);
  const int N = (int)n_rows;
  TORCH_CHECK(ldb % 4 == 0 && ldb >= N, "gbdt_hist: bins row stride must be >= rows and a multiple of 4");
  TORCH_CHECK(node.numel() >= N && gh.numel() >= 2L * N, "gbdt_hist: node / gh too short");
  TORCH_CHECK(hist.size(1) == F, "gbdt_hist: hist feature dim mismatch");
  const int B = (int)hist.size(2);
  TORCH_CHECK(B >= 1 && B <= 256, "gbdt_hist: at most 256 bins");
  TORCH_CHECK(slot_lo >= 0 && n_slots >= 1 && slot_lo + n_slots <= hist.size(0), "gbdt_hist: slot range");
  TORCH_CHECK((long)n_slots * B * 8 <= 64 * 1024, "gbdt_hist: slot chunk too large for LDS");
  TORCH_CHECK(aligned16(node.data_ptr()) && aligned16(gh.data_ptr()) && aligned16(bins.data_ptr()),
              "gbdt_hist: inputs must be 16-byte aligned");
  const int* sm = nullptr;
  int n_nodes = 0;
  if (slot_map.has_value()) {
    GCHECK(*slot_map); GDT(*slot_map, at::kInt);
    sm = slot_map->data_ptr<int>();
    n_nodes = (int)slot_map->numel();     // slot values must be < hist.size(0) (the kernel range-checks)
  }
  int rc = ct_gbdt_hist(bins.data_ptr<uint8_t>(), ldb, node.data_ptr<int>(), sm, n_nodes, gh.data_ptr(),
                        hist.data_ptr<float>(), N, F, B, (int)slot_lo, (int)n_slots, stream());
  TORCH_CHECK(rc == 0, "ct_gbdt_hist failed: ", rc);
}

// out [N, K] fp32 (accumulated); trees: feat/thr int32 [T, M], dleft uint8 [T, M], leaf fp32 [T, M]
void gbdt_predict(at::Tensor bins, int64_t n_rows, at::Tensor feat, at::Tensor thr, at::Tensor dleft,
                  at::Tensor leaf, at::Tensor out) {
  GCHECK(bins); GCHECK(feat); GCHECK(thr); GCHECK(dleft); GCHECK(leaf); GCHECK(out);
  GDT(bins, at::kByte); GDT(feat, at::kInt); GDT(thr, at::kInt); GDT(dleft, at::kByte); GDT(leaf, at::kFloat);
  GDT(out, at::kFloat);
  TORCH_CHECK(feat.dim() == 2 && thr.sizes() == feat.sizes() && dleft.sizes() == feat.sizes() &&
                  leaf.sizes() == feat.sizes(), "gbdt_predict: tree arrays must all be [T, M]");
  const int T = (int)feat.size(0), M = (int)feat.size(1);
  TORCH_CHECK(((M + 1) & M) == 0, "gbdt_predict: M must be 2^(depth+1)-1");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == n_rows, "gbdt_predict: out must be [N, K]");
  const int K = (int)out.size(1);
  TORCH_CHECK(bins.size(1) >= n_rows, "gbdt_predict: bins too short");
  // every internal node must point at a real feature and children must stay inside the tree
  auto internal = feat.ge(0);
  TORCH_CHECK(feat.lt(bins.size(0)).all().item<bool>(), "gbdt_predict: feature index out of range");
  if (M > 1) {
    auto last_level = internal.narrow(1, M / 2, M - M / 2);
    TORCH_CHECK(!last_level.any().item<bool>(), "gbdt_predict: deepest level must be leaves");
  }
  int rc = ct_gbdt_predict(bins.data_ptr<uint8_t>(), bins.size(1), feat.data_ptr<int>(), thr.data_ptr<int>(),
                           dleft.data_ptr<uint8_t>(), leaf.data_ptr<float>(), T, M, K, (int)n_rows,
                           out.data_ptr<float>(), stream());
  TORCH_CHECK(rc == 0, "ct_gbdt_predict failed: ", rc);
}

// out [R, D] = (mean ? 1/deg : 1) * (scale?) * sum_e w_e x[col_e]; x [*, D] fp32/bf16 rows.
// col values must be in [0, x.size(0)) -- validated here (bounds of a gather on the GPU).
void csr_spmm(at::Tensor rowptr, at::Tensor col, c10::optional<at::Tensor> w, c10::optional<at::Tensor> scale,
              bool mean, at::Tensor x, at::Tensor out, bool check_bounds) {
  GCHECK(rowptr); GCHECK(col); GCHECK(x); GCHECK(out);
  GDT(rowptr, at::kLong); GDT(col, at::kLong);
  TORCH_CHECK(x.scalar_type() == out.scalar_type(), "csr_spmm: x / out dtype mismatch");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "csr_spmm: fp32 or bf16");
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.size(1) == out.size(1), "csr_spmm: x [S, D], out [R, D]");
  const int R = (int)out.size(0), D = (int)x.size(1);
  const int dt = x.scalar_type() == at::kFloat ? 0 : 1;
  const int V = dt == 0 ? 4 : 8;
  TORCH_CHECK(D % V == 0, "csr_spmm: feature dim must be a multiple of ", V);
  TORCH_CHECK(aligned16(x.data_ptr()) && aligned16(out.data_ptr()), "csr_spmm: 16-byte aligned rows");
  TORCH_CHECK(rowptr.numel() == R + 1, "csr_spmm: rowptr must have R + 1 entries");
  const float* wp = nullptr;
  if (w.has_value()) {
    GCHECK(*w); GDT(*w, at::kFloat);
    TORCH_CHECK(w->numel() == col.numel(), "csr_spmm: one weight per edge");
    wp = w->data_ptr<float>();
  }
  const float* sp = nullptr;
  if (scale.has_value()) {
    GCHECK(*scale); GDT(*scale, at::kFloat);
    TORCH_CHECK(scale->numel() == R, "csr_spmm: one scale per row");
    sp = scale->data_ptr<float>();
  }
  if (check_bounds && col.numel() > 0) {
    TORCH_CHECK(rowptr[R].item<int64_t>() <= col.numel() && rowptr[0].item<int64_t>() >= 0,
                "csr_spmm: rowptr exceeds col");
    TORCH_CHECK(col.min().item<int64_t>() >= 0 && col.max().item<int64_t>() < x.size(0),
                "csr_spmm: column index out of range");
  }
  int rc = ct_csr_spmm(rowptr.data_ptr<int64_t>(), col.data_ptr<int64_t>(), wp, sp, mean ? 1 : 0, x.data_ptr(),
                       x.stride(0), out.data_ptr(), out.stride(0), R, D, dt, stream());
  TORCH_CHECK(rc == 0, "ct_csr_spmm failed: ", rc);
}


// One level of tree growth after its histogram is built:
//   part   [P, F, B, 2] built histograms (P = n_level for level 0, else n_level / 2)
//   parent [n_level / 2, F, B, 2] previous level's full histograms (ignored at level 0)
//   slot_map [n_level] node -> built slot or -1 (None at level 0)
// writes hist_cur [n_level, F, B, 2], the tree arrays at [first, first + n_level) and
// slot_next [2 * n_level] (unless last_level).
void gbdt_level(at::Tensor part, c10::optional<at::Tensor> parent, c10::optional<at::Tensor> slot_map,
                at::Tensor hist_cur, at::Tensor feat_mask, int64_t level, bool last_level, double lambda, double alpha,
                double min_child_weight, double gamma, double eta, double max_delta_step, at::Tensor feat,
                at::Tensor thr, at::Tensor dleft, at::Tensor leaf, at::Tensor gain, at::Tensor cover,
                at::Tensor slot_next, at::Tensor ws_gain, at::Tensor ws_thr, at::Tensor ws_dir, at::Tensor ws_hl,
                at::Tensor node_gh) {
  GCHECK(part); GCHECK(hist_cur); GCHECK(feat_mask); GCHECK(feat); GCHECK(thr); GCHECK(dleft); GCHECK(leaf);
  GCHECK(gain); GCHECK(cover); GCHECK(slot_next); GCHECK(ws_gain); GCHECK(ws_thr); GCHECK(ws_dir); GCHECK(ws_hl);
  GCHECK(node_gh);
  const long n_level = 1L << level;
  TORCH_CHECK(hist_cur.dim() == 4 && hist_cur.size(0) == n_level && hist_cur.size(3) == 2, "gbdt_level: hist_cur");
  const int F = (int)hist_cur.size(1), B = (int)hist_cur.size(2);
  TORCH_CHECK(B >= 3 && B <= 256, "gbdt_level: 3..256 bins");
  TORCH_CHECK(part.size(1) == F && part.size(2) == B, "gbdt_level: part shape");
  TORCH_CHECK(feat_mask.numel() == F && feat_mask.scalar_type() == at::kByte, "gbdt_level: feature mask");
  const long first = n_level - 1;
  TORCH_CHECK(feat.numel() >= first + n_level && thr.numel() == feat.numel() && dleft.numel() == feat.numel() &&
                  leaf.numel() == feat.numel() && gain.numel() == feat.numel() && cover.numel() == feat.numel(),
              "gbdt_level: tree arrays too small");
  TORCH_CHECK(ws_gain.numel() >= n_level * F && ws_thr.numel() >= n_level * F && ws_dir.numel() >= n_level * F &&
                  ws_hl.numel() >= n_level * F && node_gh.numel() >= 2 * n_level, "gbdt_level: workspace too small");
  TORCH_CHECK(last_level || slot_next.numel() >= 2 * n_level, "gbdt_level: slot_next too small");
  const float* pp = nullptr;
  const int* sm = nullptr;
  if (level == 0) {
    TORCH_CHECK(part.size(0) >= 1, "gbdt_level: level-0 histogram");
  } else {
    TORCH_CHECK(parent.has_value() && slot_map.has_value(), "gbdt_level: parent and slot_map needed below the root");
    GCHECK(*parent); GCHECK(*slot_map);
    TORCH_CHECK(parent->size(0) == n_level / 2 && slot_map->numel() == n_level && part.size(0) >= n_level / 2,
                "gbdt_level: parent / slot_map / part sizes");
    pp = parent->data_ptr<float>();
    sm = slot_map->data_ptr<int>();
  }
  int rc = ct_gbdt_split(part.data_ptr<float>(), pp, sm, hist_cur.data_ptr<float>(), feat_mask.data_ptr<uint8_t>(),
                         (int)n_level, F, B, (float)lambda, (float)alpha, (float)min_child_weight,
                         ws_gain.data_ptr<float>(), ws_thr.data_ptr<int>(), ws_dir.data_ptr<int>(),
                         ws_hl.data_ptr<float>(), node_gh.data_ptr<float>(), stream());
  TORCH_CHECK(rc == 0, "ct_gbdt_split failed: ", rc);
  rc = ct_gbdt_finalize(ws_gain.data_ptr<float>(), ws_thr.data_ptr<int>(), ws_dir.data_ptr<int>(),
                        ws_hl.data_ptr<float>(), node_gh.data_ptr<float>(), (int)n_level, F, (int)first,
                        last_level ? 1 : 0, (float)lambda, (float)alpha, (float)gamma, (float)eta,
                        (float)max_delta_step, feat.data_ptr<int>(), thr.data_ptr<int>(), dleft.data_ptr<uint8_t>(),
                        leaf.data_ptr<float>(), gain.data_ptr<float>(), cover.data_ptr<float>(),
                        slot_next.data_ptr<int>(), stream());
  TORCH_CHECK(rc == 0, "ct_gbdt_finalize failed: ", rc);
}

// node [N] int32 level-local (-1 = done); margin [N, K] fp32
void gbdt_partition(at::Tensor bins, int64_t n_rows, at::Tensor node, at::Tensor feat, at::Tensor thr,
                    at::Tensor dleft, at::Tensor leaf, int64_t level, at::Tensor margin, int64_t k) {
  GCHECK(bins); GCHECK(node); GCHECK(feat); GCHECK(thr); GCHECK(dleft); GCHECK(leaf); GCHECK(margin);
  GDT(node, at::kInt); GDT(margin, at::kFloat);
  TORCH_CHECK(node.numel() >= n_rows && margin.dim() == 2 && margin.size(0) >= n_rows && k < margin.size(1),
              "gbdt_partition: shapes");
  TORCH_CHECK(bins.size(1) >= n_rows, "gbdt_partition: bins too short");
  const long first = (1L << level) - 1;
  TORCH_CHECK(feat.numel() >= 2 * first + 1, "gbdt_partition: tree arrays");
  int rc = ct_gbdt_partition(bins.data_ptr<uint8_t>(), bins.size(1), node.data_ptr<int>(), feat.data_ptr<int>(),
                             thr.data_ptr<int>(), dleft.data_ptr<uint8_t>(), leaf.data_ptr<float>(), (int)first,
                             (int)n_rows, margin.data_ptr<float>(), (int)margin.size(1), (int)k, stream());
  TORCH_CHECK(rc == 0, "ct_gbdt_partition failed: ", rc);
}

}  // namespace

void register_graph(pybind11::module& m) {
  m.def("gbdt_hist", &gbdt_hist);
  m.def("gbdt_predict", &gbdt_predict);
  m.def("gbdt_level", &gbdt_level);
  m.def("gbdt_partition", &gbdt_partition);
  m.def("csr_spmm", &csr_spmm);
}
