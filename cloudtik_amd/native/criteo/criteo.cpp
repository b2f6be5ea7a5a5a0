// Criteo click-log preprocessor (reference: the DLRM quickstart's Cython build of
// data_utils.py, applications/.../dlrm/training/bfloat16/cython/cython_criteo.py; SURVEY.md
// §2.13 N5).  Parses the TSV "label \t 13 integer features \t 26 hex categorical features"
// format into int32 arrays with all cores, then dictionary-encodes every categorical column
// to contiguous ids in first-appearance order (the reference's convertDicts), one column
// per thread.  C ABI for ctypes; no Python objects, no allocation the caller cannot see.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <unordered_map>
#include <vector>

namespace {

constexpr int kInt = 13, kCat = 26;

struct Mapped {
  const char* p = nullptr;
  size_t n = 0;
  int fd = -1;
  bool open(const char* path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0) return false;
    n = (size_t)st.st_size;
    if (n == 0) return true;
    void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) return false;
    madvise(m, n, MADV_SEQUENTIAL);
    p = (const char*)m;
    return true;
  }
  ~Mapped() {
    if (p) munmap((void*)p, n);
    if (fd >= 0) ::close(fd);
  }
};

// [begin, end) byte ranges that start at line starts, one per thread
std::vector<std::pair<size_t, size_t>> split_lines(const Mapped& m, int parts) {
  std::vector<std::pair<size_t, size_t>> out;
  size_t start = 0;
  for (int i = 1; i <= parts && start < m.n; ++i) {
    size_t end = i == parts ? m.n : std::max(start, m.n * (size_t)i / (size_t)parts);
    while (end < m.n && m.p[end - 1] != '\n') ++end;
    if (end > start) out.emplace_back(start, end);
    start = end;
  }
  return out;
}

long count_range(const char* p, size_t a, size_t b) {
  long c = 0;
  for (size_t i = a; i < b; ++i) c += p[i] == '\n';
  if (b > a && p[b - 1] != '\n') ++c;            // last line without newline
  return c;
}

inline const char* parse_int(const char* s, const char* e, int32_t* v) {
  // empty field -> 0; negative values kept (clipped later by the consumer's log transform)
  bool neg = false;
  long x = 0;
  if (s < e && *s == '-') { neg = true; ++s; }
  while (s < e && *s >= '0' && *s <= '9') x = x * 10 + (*s++ - '0');
  *v = (int32_t)(neg ? -x : x);
  while (s < e && *s != '\t' && *s != '\n' && *s != '\r') ++s;
  return s;
}

inline const char* parse_hex(const char* s, const char* e, int64_t* v) {
  uint64_t x = 0;
  while (s < e) {
    const char c = *s;
    int d;
    if (c >= '0' && c <= '9') d = c - '0';
    else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
    else break;
    x = (x << 4) | (uint64_t)d;
    ++s;
  }
  *v = (int64_t)x;
  while (s < e && *s != '\t' && *s != '\n' && *s != '\r') ++s;
  return s;
}

}  // namespace

extern "C" {

long ct_criteo_count_lines(const char* path, int threads) {
  Mapped m;
  if (!m.open(path)) return -1;
  if (m.n == 0) return 0;
  auto parts = split_lines(m, std::max(1, threads));
  std::vector<long> counts(parts.size());
  std::vector<std::thread> ts;
  for (size_t i = 0; i < parts.size(); ++i)
    ts.emplace_back([&, i] { counts[i] = count_range(m.p, parts[i].first, parts[i].second); });
  for (auto& t : ts) t.join();
  long total = 0;
  for (long c : counts) total += c;
  return total;
}

// y [rows], x_int [rows, 13], x_cat [rows, 26] preallocated for `rows` lines (from
// ct_criteo_count_lines); returns the number of rows parsed or < 0 on error.
long ct_criteo_parse(const char* path, long rows, long long max_ind_range, int threads, int32_t* y, int32_t* x_int,
                     int32_t* x_cat) {
  Mapped m;
  if (!m.open(path)) return -1;
  if (m.n == 0) return 0;
  auto parts = split_lines(m, std::max(1, threads));
  std::vector<long> first(parts.size() + 1, 0);
  {
    std::vector<std::thread> ts;
    std::vector<long> counts(parts.size());
    for (size_t i = 0; i < parts.size(); ++i)
      ts.emplace_back([&, i] { counts[i] = count_range(m.p, parts[i].first, parts[i].second); });
    for (auto& t : ts) t.join();
    for (size_t i = 0; i < parts.size(); ++i) first[i + 1] = first[i] + counts[i];
  }
  if (first.back() > rows) return -2;
  std::vector<std::thread> ts;
  for (size_t i = 0; i < parts.size(); ++i) {
    ts.emplace_back([&, i] {
      const char* s = m.p + parts[i].first;
      const char* e = m.p + parts[i].second;
      long r = first[i];
      while (s < e) {
        const char* le = (const char*)memchr(s, '\n', (size_t)(e - s));
        if (!le) le = e;
        if (le > s) {
          const char* q = s;
          int32_t v;
          q = parse_int(q, le, &v);
          y[r] = v;
          for (int j = 0; j < kInt; ++j) {
            if (q < le && *q == '\t') ++q;
            q = parse_int(q, le, &x_int[r * kInt + j]);
          }
          for (int j = 0; j < kCat; ++j) {
            if (q < le && *q == '\t') ++q;
            int64_t h;
            q = parse_hex(q, le, &h);
            if (max_ind_range > 0) h %= max_ind_range;
            x_cat[r * kCat + j] = (int32_t)h;
          }
          ++r;
        }
        s = le + 1;
      }
    });
  }
  for (auto& t : ts) t.join();
  return first.back();
}

// In-place dictionary encoding of every categorical column (first-appearance order);
// counts[j] = number of distinct values of column j.
void ct_criteo_dict_encode(int32_t* x_cat, long rows, int32_t* counts, int threads) {
  std::vector<std::thread> ts;
  const int nt = std::max(1, std::min(threads, kCat));
  for (int w = 0; w < nt; ++w) {
    ts.emplace_back([=] {
      for (int j = w; j < kCat; j += nt) {
        std::unordered_map<int32_t, int32_t> dict;
        dict.reserve(1 << 16);
        for (long r = 0; r < rows; ++r) {
          int32_t& v = x_cat[r * kCat + j];
          auto it = dict.find(v);
          if (it == dict.end()) it = dict.emplace(v, (int32_t)dict.size()).first;
          v = it->second;
        }
        counts[j] = (int32_t)dict.size();
      }
    });
  }
  for (auto& t : ts) t.join();
}

}  // extern "C"
