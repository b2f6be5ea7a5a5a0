// Bindings for the one-shot P2P all-reduce (p2p.hip): IPC export / import of staging and
// signal buffers and the launch.  Pointers cross the Python boundary as integers; every
// launch re-checks ranks, sizes, dtype and alignment before anything reaches the GPU.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

extern "C" {
size_t ct_p2p_signal_bytes();
int ct_p2p_alloc_signal(void**);
int ct_p2p_alloc(void**, size_t);
int ct_p2p_free(void*);
int ct_ipc_get(void*, char*);
int ct_ipc_handle_size();
int ct_ipc_open(const char*, void**);
int ct_ipc_close(void*);
int ct_p2p_allreduce(const void* const*, uint32_t* const*, void*, long, int, int, int, uint32_t, uint64_t,
                     uint32_t*, int, hipStream_t);
int ct_p2p_alloc_flag(void**, void**);
int ct_p2p_free_flag(void*);
long ct_p2p_clock_hz();
}

namespace {

int64_t p2p_alloc(int64_t bytes, bool signal) {
  void* p = nullptr;
  int rc = signal ? ct_p2p_alloc_signal(&p) : ct_p2p_alloc(&p, (size_t)bytes);
  TORCH_CHECK(rc == 0 && p, "p2p_alloc failed: ", rc);
  return reinterpret_cast<int64_t>(p);
}

void p2p_free(int64_t ptr) { TORCH_CHECK(ct_p2p_free(reinterpret_cast<void*>(ptr)) == 0, "p2p_free failed"); }

pybind11::bytes ipc_get(int64_t ptr) {
  std::string h(ct_ipc_handle_size(), '\0');
  TORCH_CHECK(ct_ipc_get(reinterpret_cast<void*>(ptr), &h[0]) == 0, "hipIpcGetMemHandle failed");
  return pybind11::bytes(h);
}

int64_t ipc_open(const std::string& h) {
  TORCH_CHECK((int)h.size() == ct_ipc_handle_size(), "ipc_open: bad handle size");
  void* p = nullptr;
  TORCH_CHECK(ct_ipc_open(h.data(), &p) == 0 && p, "hipIpcOpenMemHandle failed");
  return reinterpret_cast<int64_t>(p);
}

void ipc_close(int64_t ptr) { TORCH_CHECK(ct_ipc_close(reinterpret_cast<void*>(ptr)) == 0, "ipc_close failed"); }

// In place on `out`: copies it into this rank's staging buffer data[rank] (capacity
// `cap_bytes`), then one kernel sums every rank's staging buffer into `out`.
void p2p_allreduce(const std::vector<int64_t>& data, const std::vector<int64_t>& sig, at::Tensor out,
                   int64_t cap_bytes, int64_t rank, int64_t world, int64_t epoch, double timeout_s, int64_t err_dev,
                   int64_t blocks) {
  TORCH_CHECK(out.is_cuda() && out.is_contiguous(), "p2p_allreduce: out must be a contiguous GPU tensor");
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16, "p2p_allreduce: fp32 / bf16");
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "p2p_allreduce: bad rank / world");
  TORCH_CHECK((int64_t)data.size() == world && (int64_t)sig.size() == world, "p2p_allreduce: one buffer per rank");
  TORCH_CHECK(out.numel() * (int64_t)out.element_size() <= cap_bytes, "p2p_allreduce: bucket exceeds staging");
  TORCH_CHECK(err_dev != 0 && timeout_s > 0, "p2p_allreduce: error word / timeout");
  static const long hz = ct_p2p_clock_hz();
  TORCH_CHECK(hz > 0, "p2p_allreduce: no device wall clock rate");
  const uint64_t ticks = (uint64_t)(timeout_s * (double)hz);
  std::vector<const void*> d(world);
  std::vector<uint32_t*> s(world);
  for (int64_t r = 0; r < world; ++r) {
    d[r] = reinterpret_cast<const void*>(data[r]);
    s[r] = reinterpret_cast<uint32_t*>(sig[r]);
  }
  hipStream_t st = at::hip::getCurrentHIPStream().stream();
  // stage this rank's input (stream ordered before the kernel's release fence)
  TORCH_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(data[rank]), out.data_ptr(), out.numel() * out.element_size(),
                             hipMemcpyDeviceToDevice, st) == hipSuccess, "p2p_allreduce: staging copy failed");
  int rc = ct_p2p_allreduce(d.data(), s.data(), out.data_ptr(), (long)out.numel(),
                            out.scalar_type() == at::kFloat ? 0 : 1, (int)rank, (int)world, (uint32_t)epoch,
                            ticks, reinterpret_cast<uint32_t*>(err_dev), (int)blocks, st);
  TORCH_CHECK(rc == 0, "ct_p2p_allreduce failed: ", rc);
}

// host-mapped error word: (host pointer, device pointer)
std::vector<int64_t> p2p_alloc_flag() {
  void *h = nullptr, *d = nullptr;
  TORCH_CHECK(ct_p2p_alloc_flag(&h, &d) == 0 && h && d, "p2p_alloc_flag failed");
  return {reinterpret_cast<int64_t>(h), reinterpret_cast<int64_t>(d)};
}

void p2p_free_flag(int64_t host) { TORCH_CHECK(ct_p2p_free_flag(reinterpret_cast<void*>(host)) == 0, "p2p_free_flag"); }

// the error word a timed-out barrier sets (plain host read of coherent pinned memory: no
// device sync; sees every kernel that has already finished)
int64_t p2p_error(int64_t host) {
  return (int64_t)__atomic_load_n(reinterpret_cast<uint32_t*>(host), __ATOMIC_ACQUIRE);
}

}  // namespace

void register_p2p(pybind11::module& m) {
  m.def("p2p_alloc", &p2p_alloc);
  m.def("p2p_free", &p2p_free);
  m.def("ipc_get", &ipc_get);
  m.def("ipc_open", &ipc_open);
  m.def("ipc_close", &ipc_close);
  m.def("p2p_allreduce", &p2p_allreduce);
  m.def("p2p_error", &p2p_error);
  m.def("p2p_alloc_flag", &p2p_alloc_flag);
  m.def("p2p_free_flag", &p2p_free_flag);
}
