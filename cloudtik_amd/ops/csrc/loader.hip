// Native batch loader: worker threads gather shuffled rows of columnar host data into
// pinned host slots; the consumer's next() issues one hipMemcpyAsync per column on a
// dedicated copy stream, records the slot's event and makes the consumer stream wait on it
// (hipStreamWaitEvent) -- host never blocks on the GPU, H2D overlaps compute.  A slot is
// reused only after its event completed (workers hipEventSynchronize before refilling).
//
// Reference behaviour replaced: the AI runtime's Spark -> Parquet -> Petastorm / torch
// DataLoader path (SURVEY.md §2.14 "Spark data parallelism", §5.9; examples
// mnist-pytorch-spark-horovod...py:159,200-214), which copies synchronously from pageable
// memory in the training process.
//
// Columns are fixed-width rows (row_bytes each, e.g. an int64 label, a 3x224x224 uint8
// image, a 128-token int32 sequence).  Sharding: rank r of w gets every w-th batch of the
// epoch's permutation (same permutation on every rank: seed + epoch), so DP ranks read
// disjoint data.  Host-only mode (no GPU, for tests / CPU training) fills caller buffers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <numeric>
#include <random>
#include <thread>
#include <vector>

namespace {

struct Slot {
  std::vector<char*> bufs;   // one per column
  hipEvent_t event = nullptr;
  bool event_pending = false;
  long rows = 0;
  long batch_id = -1;
};

struct Loader {
  std::vector<const char*> cols;
  std::vector<long> row_bytes;
  long nrows = 0;
  int batch = 1;
  bool shuffle = true, drop_last = false, pinned = true;
  uint64_t seed = 0;
  int rank = 0, world = 1;
  std::vector<Slot> slots;

  std::mutex mu;
  std::condition_variable cv_free, cv_ready;
  std::deque<int> free_slots;
  std::map<long, int> ready;          // batch index within this rank's epoch -> slot
  std::vector<long> perm;
  long nbatches = 0;                  // this rank's batches per epoch
  long next_to_fill = 0, next_to_take = 0;
  long epoch_gen = 0;                 // bumps on reset: stale work is dropped
  bool stop = false;
  std::vector<std::thread> workers;
  std::atomic<long> filled{0};

  long global_batches() const {
    return drop_last ? nrows / batch : (nrows + batch - 1) / batch;
  }
  void build_epoch(long epoch) {
    perm.resize(nrows);
    std::iota(perm.begin(), perm.end(), 0L);
    if (shuffle) {
      std::mt19937_64 g(seed * 0x9E3779B97F4A7C15ull + (uint64_t)epoch);
      std::shuffle(perm.begin(), perm.end(), g);
    }
    const long gb = global_batches();
    // drop_last: every rank runs the same number of steps (collectives stay matched);
    // otherwise the first gb % world ranks see one extra batch (evaluation covers all data)
    nbatches = drop_last ? gb / world : gb / world + (rank < gb % world ? 1 : 0);
    next_to_fill = next_to_take = 0;
    ready.clear();
  }

  void worker() {
    for (;;) {
      long bid, gen;
      int slot;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_free.wait(lk, [&] { return stop || (next_to_fill < nbatches && !free_slots.empty()); });
        if (stop) return;
        bid = next_to_fill++;
        slot = free_slots.front();
        free_slots.pop_front();
        gen = epoch_gen;
      }
      Slot& s = slots[slot];
      if (s.event_pending) {               // previous H2D copy from this slot must be done
        hipEventSynchronize(s.event);
        s.event_pending = false;
      }
      const long gbid = bid * world + rank;
      const long start = gbid * batch;
      const long rows = std::min<long>(batch, nrows - start);
      for (size_t c = 0; c < cols.size(); ++c) {
        const long rb = row_bytes[c];
        char* dst = s.bufs[c];
        const char* src = cols[c];
        for (long r = 0; r < rows; ++r) std::memcpy(dst + r * rb, src + perm[start + r] * rb, rb);
      }
      s.rows = rows;
      s.batch_id = bid;
      {
        std::lock_guard<std::mutex> lk(mu);
        if (gen != epoch_gen) { free_slots.push_back(slot); cv_free.notify_one(); continue; }
        ready[bid] = slot;
        filled++;
      }
      cv_ready.notify_all();
    }
  }

  // returns slot index holding batch next_to_take, or -1 at epoch end
  int take() {
    std::unique_lock<std::mutex> lk(mu);
    if (next_to_take >= nbatches) return -1;
    const long want = next_to_take;
    cv_ready.wait(lk, [&] { return stop || ready.count(want); });
    if (stop) return -1;
    const int slot = ready[want];
    ready.erase(want);
    next_to_take++;
    return slot;
  }
  void give_back(int slot) {
    {
      std::lock_guard<std::mutex> lk(mu);
      free_slots.push_back(slot);
    }
    cv_free.notify_one();
  }
};

}  // namespace

extern "C" {

void* ct_loader_create(int ncols, const void* const* col_ptrs, const long* row_bytes, long nrows, int batch,
                       int shuffle, uint64_t seed, int drop_last, int nworkers, int nslots, int rank, int world,
                       int pinned) {
  if (ncols <= 0 || nrows <= 0 || batch <= 0 || nslots <= 0 || world <= 0 || rank < 0 || rank >= world) return nullptr;
  auto* L = new Loader();
  for (int c = 0; c < ncols; ++c) {
    L->cols.push_back((const char*)col_ptrs[c]);
    L->row_bytes.push_back(row_bytes[c]);
  }
  L->nrows = nrows; L->batch = batch; L->shuffle = shuffle; L->seed = seed; L->drop_last = drop_last;
  L->rank = rank; L->world = world; L->pinned = pinned;
  L->slots.resize(nslots);
  for (int i = 0; i < nslots; ++i) {
    for (int c = 0; c < ncols; ++c) {
      char* p = nullptr;
      const size_t bytes = (size_t)row_bytes[c] * batch;
      if (pinned) {
        if (hipHostMalloc((void**)&p, bytes, hipHostMallocDefault) != hipSuccess) p = nullptr;
      } else {
        p = (char*)std::malloc(bytes);
      }
      if (!p) { delete L; return nullptr; }
      L->slots[i].bufs.push_back(p);
    }
    if (pinned) hipEventCreateWithFlags(&L->slots[i].event, hipEventDisableTiming);
    L->free_slots.push_back(i);
  }
  L->build_epoch(0);
  for (int w = 0; w < std::max(1, nworkers); ++w) L->workers.emplace_back([L] { L->worker(); });
  return L;
}

long ct_loader_num_batches(void* h) { return ((Loader*)h)->nbatches; }

void ct_loader_set_epoch(void* h, long epoch) {
  auto* L = (Loader*)h;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    for (auto& kv : L->ready) L->free_slots.push_back(kv.second);
    L->epoch_gen++;
    L->build_epoch(epoch);
  }
  L->cv_free.notify_all();
}

// GPU mode: copy the next batch into dev_ptrs[c] (each >= batch*row_bytes[c] bytes) on
// copy_stream; consumer_stream waits for it.  Returns the batch's row count, 0 at epoch end.
long ct_loader_next_device(void* h, void* const* dev_ptrs, hipStream_t copy_stream, hipStream_t consumer_stream) {
  auto* L = (Loader*)h;
  const int slot = L->take();
  if (slot < 0) return 0;
  Slot& s = L->slots[slot];
  for (size_t c = 0; c < L->cols.size(); ++c)
    hipMemcpyAsync(dev_ptrs[c], s.bufs[c], (size_t)s.rows * L->row_bytes[c], hipMemcpyHostToDevice, copy_stream);
  hipEventRecord(s.event, copy_stream);
  s.event_pending = true;
  if (consumer_stream != copy_stream) hipStreamWaitEvent(consumer_stream, s.event, 0);
  const long rows = s.rows;
  L->give_back(slot);
  return rows;
}

// host mode: memcpy the next batch into host buffers
long ct_loader_next_host(void* h, void* const* host_ptrs) {
  auto* L = (Loader*)h;
  const int slot = L->take();
  if (slot < 0) return 0;
  Slot& s = L->slots[slot];
  for (size_t c = 0; c < L->cols.size(); ++c) std::memcpy(host_ptrs[c], s.bufs[c], (size_t)s.rows * L->row_bytes[c]);
  const long rows = s.rows;
  L->give_back(slot);
  return rows;
}

void ct_loader_destroy(void* h) {
  auto* L = (Loader*)h;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->stop = true;
  }
  L->cv_free.notify_all();
  L->cv_ready.notify_all();
  for (auto& t : L->workers) t.join();
  for (auto& s : L->slots) {
    if (s.event) { hipEventSynchronize(s.event); hipEventDestroy(s.event); }
    for (char* p : s.bufs) {
      if (L->pinned) hipHostFree(p);
      else std::free(p);
    }
  }
  delete L;
}

}  // extern "C"
