// gpu_worker_group.cpp -- see gpu_worker_group.hpp.
#include "gpu_worker_group.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <tuple>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <list>
#include <set>
#include <type_traits>
#include <variant>
#include <exception>
#include <stdexcept>
#include <string>

#include "ct_format.hpp"

namespace herdsman_gpu {

using Status = IWorkerGroup::TaskHandle::Status;

// ------------------------------------------------------------- formats
uint64_t moduli_digest(const uint64_t *m, uint32_t count) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint32_t i = 0; i < count; ++i)
    for (int b = 0; b < 8; ++b) {
      h ^= (m[i] >> (8 * b)) & 0xff;
      h *= 0x100000001b3ull;
    }
  return h;
}

std::vector<std::vector<uint8_t>> read_partition(const std::filesystem::path &path) {
  std::ifstream in(path, std::ios::binary);
  if (!in) throw std::runtime_error("cannot open partition " + path.string());
  std::vector<std::vector<uint8_t>> rows;
  while (true) {
    uint32_t len = 0;
    in.read(reinterpret_cast<char *>(&len), sizeof(len));
    if (in.gcount() == 0) break;
    if (in.gcount() != sizeof(len)) throw std::runtime_error("truncated row header");
    std::vector<uint8_t> row(len);
    in.read(reinterpret_cast<char *>(row.data()), len);
    if ((uint32_t)in.gcount() != len) throw std::runtime_error("truncated row");
    rows.push_back(std::move(row));
  }
  return rows;
}

void write_partition(const std::filesystem::path &path, const std::vector<std::vector<uint8_t>> &rows) {
  std::filesystem::create_directories(path.parent_path());
  std::ofstream out(path, std::ios::binary | std::ios::trunc);
  if (!out) throw std::runtime_error("cannot create partition " + path.string());
  for (const auto &r : rows) {
    const uint32_t len = (uint32_t)r.size();
    out.write(reinterpret_cast<const char *>(&len), sizeof(len));
    out.write(reinterpret_cast<const char *>(r.data()), len);
  }
  if (!out) throw std::runtime_error("write failed " + path.string());
}

PartitionView::PartitionView(const std::filesystem::path &path) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("cannot open partition " + path.string());
  struct stat st {};
  if (::fstat(fd, &st) != 0) {
    ::close(fd);
    throw std::runtime_error("cannot stat partition " + path.string());
  }
  bytes_ = (size_t)st.st_size;
  if (bytes_) {
    map_ = ::mmap(nullptr, bytes_, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
    if (map_ == MAP_FAILED) {
      map_ = nullptr;
      ::close(fd);
      throw std::runtime_error("cannot map partition " + path.string());
    }
    (void)::madvise(map_, bytes_, MADV_SEQUENTIAL);
  }
  ::close(fd);
  const uint8_t *p = static_cast<const uint8_t *>(map_), *end = p + bytes_;
  while (p < end) {
    if (end - p < 4) throw std::runtime_error("truncated row header");
    uint32_t len;
    std::memcpy(&len, p, 4);
    p += 4;
    if ((size_t)(end - p) < len) throw std::runtime_error("truncated row");
    rows_.emplace_back(p, len);
    p += len;
  }
}

PartitionView::~PartitionView() {
  if (map_) ::munmap(map_, bytes_);
}

PartitionIndex::PartitionIndex(const std::filesystem::path &path) : path_(path) {
  fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd_ < 0) throw std::runtime_error("cannot open partition " + path.string());
  struct stat st {};
  if (::fstat(fd_, &st) != 0) {
    ::close(fd_);
    throw std::runtime_error("cannot stat partition " + path.string());
  }
  (void)::posix_fadvise(fd_, 0, 0, POSIX_FADV_SEQUENTIAL);
  const uint64_t size = (uint64_t)st.st_size;
  uint64_t pos = 0;
  while (pos < size) {
    uint32_t len = 0;
    if (size - pos < 4 || ::pread(fd_, &len, 4, (off_t)pos) != 4) {
      ::close(fd_);
      throw std::runtime_error("truncated row header in " + path.string());
    }
    if (size - pos - 4 < len) {
      ::close(fd_);
      throw std::runtime_error("truncated row in " + path.string());
    }
    rows_.emplace_back(pos + 4, len);
    pos += 4 + (uint64_t)len;
  }
}

PartitionIndex::~PartitionIndex() {
  if (fd_ >= 0) ::close(fd_);
}

void PartitionIndex::read(size_t i, size_t off, void *dst, size_t len) const {
  if (off + len > rows_[i].second) throw std::runtime_error("row holds fewer ciphertexts than the circuit reads");
  uint8_t *d = static_cast<uint8_t *>(dst);
  uint64_t at = rows_[i].first + off;
  while (len) {
    const ssize_t r = ::pread(fd_, d, len, (off_t)at);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) throw std::runtime_error("short read from " + path_.string());
    d += r;
    at += (uint64_t)r;
    len -= (size_t)r;
  }
}

PartitionWriter::PartitionWriter(const std::filesystem::path &path, bool durable) : path_(path), durable_(durable) {
  std::filesystem::create_directories(path.parent_path());
  tmp_ = path;
  tmp_ += ".tmp-" + std::to_string((unsigned long)::getpid()) + "-" +
          std::to_string(std::hash<std::thread::id>{}(std::this_thread::get_id()));
  fd_ = ::open(tmp_.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd_ < 0) throw std::runtime_error("cannot create partition " + tmp_.string());
}

PartitionWriter::~PartitionWriter() {
  if (fd_ >= 0) ::close(fd_);
  if (!done_) ::unlink(tmp_.c_str());
}

void PartitionWriter::write_row_at(uint64_t off, const std::vector<std::pair<const void *, size_t>> &parts) const {
  uint32_t len = 0;
  for (const auto &pr : parts) len += (uint32_t)pr.second;
  std::vector<iovec> iov;
  iov.push_back(iovec{&len, 4});
  for (const auto &pr : parts) iov.push_back(iovec{const_cast<void *>(pr.first), pr.second});
  size_t todo = 4 + (size_t)len, first = 0;
  while (todo) {
    const ssize_t w = ::pwritev(fd_, iov.data() + first, (int)(iov.size() - first), (off_t)off);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error("write failed " + tmp_.string());
    }
    todo -= (size_t)w;
    off += (uint64_t)w;
    size_t adv = (size_t)w;
    while (adv && first < iov.size()) {  // partial write: skip what went out
      if (adv >= iov[first].iov_len) {
        adv -= iov[first].iov_len;
        ++first;
      } else {
        iov[first].iov_base = static_cast<char *>(iov[first].iov_base) + adv;
        iov[first].iov_len -= adv;
        adv = 0;
      }
    }
  }
}

uint64_t PartitionWriter::claim(uint64_t bytes) {
  const uint64_t at = end_;
  end_ += bytes;
  return at;
}

void PartitionWriter::append(const std::vector<std::pair<const void *, size_t>> &parts) {
  uint64_t len = 4;
  for (const auto &pr : parts) len += pr.second;
  write_row_at(claim(len), parts);
}

void PartitionWriter::commit() {
  if (durable_ && ::fsync(fd_) != 0) throw std::runtime_error("fsync failed " + tmp_.string());
  if (::close(fd_) != 0) {
    fd_ = -1;
    throw std::runtime_error("close failed " + tmp_.string());
  }
  fd_ = -1;
  std::filesystem::rename(tmp_, path_);
  done_ = true;
  if (durable_) {
    const int dfd = ::open(path_.parent_path().c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
    if (dfd >= 0) {
      (void)::fsync(dfd);
      ::close(dfd);
    }
  }
}

// ------------------------------------------------------------- device state
namespace {

// A lane's IO helper threads, started once (per lane thread and size) and
// parked on a condition variable between jobs: the per-batch row reads and
// writes no longer spawn and join threads.  The calling thread takes chunk 0.
class IoPool {
 public:
  explicit IoPool(unsigned threads) : threads_(threads) {
    for (unsigned t = 1; t < threads_; ++t) workers_.emplace_back([this, t] { loop(t); });
  }
  ~IoPool() {
    {
      std::lock_guard lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &w : workers_) w.join();
  }
  IoPool(const IoPool &) = delete;
  IoPool &operator=(const IoPool &) = delete;
  unsigned size() const { return threads_; }

  // f(i) for i in [0, n) in contiguous chunks; the first exception is rethrown
  // after every chunk has finished
  void run(size_t n, const std::function<void(size_t)> &f) {
    {
      std::lock_guard lk(m_);
      job_ = &f;
      n_ = n;
      err_ = nullptr;
      left_ = threads_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    chunk(0);
    std::unique_lock lk(m_);
    done_cv_.wait(lk, [this] { return left_ == 0; });
    job_ = nullptr;
    if (err_) std::rethrow_exception(err_);
  }

 private:
  void chunk(unsigned t) {
    try {
      for (size_t i = n_ * t / threads_; i < n_ * (t + 1) / threads_; ++i) (*job_)(i);
    } catch (...) {
      std::lock_guard lk(m_);
      if (!err_) err_ = std::current_exception();
    }
  }
  void loop(unsigned t) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      chunk(t);
      {
        std::lock_guard lk(m_);
        --left_;
      }
      done_cv_.notify_one();
    }
  }

  const unsigned threads_;
  std::vector<std::thread> workers_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t)> *job_ = nullptr;
  size_t n_ = 0;
  unsigned left_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
  std::exception_ptr err_;
};

// the calling thread's persistent IoPool of `threads` threads: one per lane (or
// flusher) thread, shared by every kind of job it runs (a thread_local inside
// the parallel_for template would be one pool per lambda type)
IoPool &thread_pool(unsigned threads) {
  thread_local std::unique_ptr<IoPool> pool;
  if (!pool || pool->size() != threads) pool = std::make_unique<IoPool>(threads);
  return *pool;
}

// f(i) for i in [0, n) on up to `threads` threads of the calling thread's pool
template <class F>
void parallel_for(size_t n, unsigned threads, F f) {
  threads = std::max(1u, threads);
  if (threads == 1 || n <= 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  thread_pool(threads).run(n, std::function<void(size_t)>(f));
}

void ck(fhe_ctx *c, int rc, const char *what) {
  if (rc != FHE_OK) throw std::runtime_error(std::string(what) + ": " + fhe_last_error(c));
}

struct DevBuf {
  fhe_ctx *ctx = nullptr;
  uint64_t *p = nullptr;
  size_t words = 0;
  DevBuf() = default;
  DevBuf(fhe_ctx *c, size_t w) : ctx(c), words(w) {
    void *q = nullptr;
    ck(c, fhe_dev_alloc(c, w * 8, &q), "alloc");
    p = static_cast<uint64_t *>(q);
  }
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  DevBuf(DevBuf &&o) noexcept { *this = std::move(o); }
  DevBuf &operator=(DevBuf &&o) noexcept {
    std::swap(ctx, o.ctx);
    std::swap(p, o.p);
    std::swap(words, o.words);
    return *this;
  }
  ~DevBuf() {
    if (p) fhe_dev_free(ctx, p);
  }
};

struct SchemaCtx {
  fhe_ctx *ctx = nullptr;
  uint32_t scheme = 0, log_n = 0, L = 0, K = 0, dnum = 0;
  std::vector<uint64_t> moduli;
  uint64_t q_digest = 0, qp_digest = 0;
  std::vector<uint64_t> level_digest;  // [m] = digest of the first m Q moduli (a level-m ciphertext's header)
  size_t ct_words(uint32_t level) const { return (size_t)2 * level << log_n; }
  size_t ct_words() const { return ct_words(L); }
  size_t key_words() const { return (size_t)dnum * 2 * (L + K) << log_n; }
};

struct KeySet {
  DevBuf relin;
  std::map<uint32_t, DevBuf> galois;
};

// Device buffers of one lane, recycled across instructions and batches: a
// buffer handed back is reused by a later op on the SAME stream, which stream
// order makes safe, so the steady state does no hipMalloc / hipFree.
class Arena {
 public:
  explicit Arena(fhe_ctx *c) : ctx_(c) {}
  Arena(const Arena &) = delete;
  Arena &operator=(const Arena &) = delete;
  ~Arena() {
    for (auto &b : free_) fhe_dev_free(ctx_, b.second);
  }
  uint64_t *get(size_t words, size_t *cap) {
    auto it = free_.lower_bound(words);  // best fit
    if (it != free_.end()) {
      *cap = it->first;
      uint64_t *p = it->second;
      free_.erase(it);
      return p;
    }
    void *q = nullptr;
    ck(ctx_, fhe_dev_alloc(ctx_, words * 8, &q), "arena alloc");
    *cap = words;
    return static_cast<uint64_t *>(q);
  }
  void put(uint64_t *p, size_t cap) { free_.emplace(cap, p); }

 private:
  fhe_ctx *ctx_;
  std::multimap<size_t, uint64_t *> free_;
};

struct ArenaBuf {
  Arena *arena = nullptr;
  uint64_t *p = nullptr;
  size_t cap = 0;
  ArenaBuf() = default;
  ArenaBuf(Arena &a, size_t words) : arena(&a) { p = a.get(words, &cap); }
  ArenaBuf(const ArenaBuf &) = delete;
  ArenaBuf &operator=(const ArenaBuf &) = delete;
  ArenaBuf(ArenaBuf &&o) noexcept { *this = std::move(o); }
  ArenaBuf &operator=(ArenaBuf &&o) noexcept {
    std::swap(arena, o.arena);
    std::swap(p, o.p);
    std::swap(cap, o.cap);
    return *this;
  }
  ~ArenaBuf() {
    if (p) arena->put(p, cap);
  }
};

// Pinned host staging buffer (fhe_host_alloc), grown on demand.
struct Pinned {
  fhe_ctx *ctx = nullptr;
  uint8_t *p = nullptr;
  size_t bytes = 0;
  Pinned() = default;
  Pinned(const Pinned &) = delete;
  Pinned &operator=(const Pinned &) = delete;
  ~Pinned() {
    if (p) fhe_host_free(ctx, p);
  }
  uint8_t *reserve(fhe_ctx *c, size_t need) {
    if (need > bytes) {
      if (p) fhe_host_free(ctx, p);
      p = nullptr;
      bytes = 0;
      void *q = nullptr;
      ck(c, fhe_host_alloc(c, need, &q), "pinned host alloc");
      ctx = c;
      p = static_cast<uint8_t *>(q);
      bytes = need;
    }
    return p;
  }
};

// Pinned staging of one batch in flight: one input buffer per PUSH_INPUT and
// the output buffer; a lane alternates between two of them, so batch k+1's
// inputs are read and batch k-1's outputs written while batch k runs.
struct Slot {
  std::vector<std::unique_ptr<Pinned>> in;
  Pinned out;
  size_t r0 = 0, n = 0;
  uint32_t out_level = 0;  // level of the batch's result ciphertexts
};

// one lane's state for one schema: context (own stream), buffers, staging
struct LaneSchema {
  SchemaCtx s;
  std::unique_ptr<Arena> arena;
  Slot slot[2];
};

double secs_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

struct FrameBudget;

// A MapTask's output partition kept in HBM (GpuWorkerGroupConfig::
// resident_frame_bytes): `rows` ciphertexts at one level, row r at p + r cw.
struct ResidentFrame {
  std::string key;  // session / frame / partition
  int device = 0, schema = 0;
  uint32_t level = 0;
  size_t rows = 0, cw = 0;
  fhe_ctx *ctx = nullptr;  // the allocating lane's context (freed through it)
  uint64_t *p = nullptr;
  size_t bytes() const { return rows * cw * 8; }
  // write-behind: where and how the flusher writes the partition file
  std::filesystem::path file;
  CtHeader header{};
  bool durable = false;
  // the device budget this frame's bytes are charged to (cleared when it is
  // evicted; the memory itself goes when the last reader drops the frame)
  FrameBudget *budget = nullptr;
  // identity of the partition file once it is committed (size, mtime): a
  // lookup that finds the file changed under it (rewritten outside this group)
  // drops the HBM copy instead of serving stale rows
  bool file_known = false;
  uintmax_t file_size = 0;
  std::filesystem::file_time_type file_mtime{};
  ~ResidentFrame();
};

// per device: resident frames by key, least recently used last, and the bytes
// charged (frames in the map plus outputs still being produced)
struct FrameBudget {
  std::map<std::string, std::shared_ptr<ResidentFrame>> map;
  std::list<std::string> lru;
  uint64_t bytes = 0;
};

}  // namespace

struct GpuWorkerGroup::Job {
  std::shared_ptr<Handle> handle;
  herd::common::task_t task;
};

struct GpuWorkerGroup::Lane {
  std::thread thread;
  std::map<int, std::unique_ptr<LaneSchema>> schemas;  // schema -> this lane's context
};

struct GpuWorkerGroup::Device {
  int id = 0;
  std::mutex m;
  std::condition_variable cv;
  std::deque<Job> queue;
  bool stop = false;
  std::vector<std::unique_ptr<Lane>> lanes;
  // evaluation keys, shared by the device's lanes: (session, schema) -> keys
  std::mutex keys_m;
  std::map<std::pair<std::string, int>, std::shared_ptr<KeySet>> keys;
};

// Resident frames of every device and the write-behind flusher's queue.  One
// mutex: lookups happen once per task, not per row.
struct GpuWorkerGroup::Frames {
  std::mutex m;
  std::condition_variable cv;  // flush queue changes, files committed
  std::map<int, FrameBudget> dev;
  std::deque<std::shared_ptr<ResidentFrame>> queue;              // waiting for the flusher
  std::map<std::string, std::shared_ptr<ResidentFrame>> pending;  // queued or being written
  bool stop = false, failed = false;
  // write-behind failures: frame key -> error, until the partition is rewritten
  // (every task that reads the key completes with ERROR), and the sessions
  // whose next scheduled task reports the failure (executor.cpp:168-178 then
  // fails the job)
  std::map<std::string, std::string> flush_failed;
  std::set<std::string> failed_sessions;
  std::map<std::tuple<uint32_t, int, int>, fhe_ctx *> flush_ctx;  // (flusher, device, schema) -> its context
  StageStats st;                                      // flushed rows and time

  // charge `need` bytes to the device, evicting least recently used frames
  // (their memory is freed once no task reads them); false if it cannot fit
  FrameBudget *reserve(int device, uint64_t need, uint64_t cap, std::vector<std::shared_ptr<ResidentFrame>> &evicted) {
    std::lock_guard lk(m);
    FrameBudget &b = dev[device];
    if (need > cap) return nullptr;
    // bytes reserved for outputs still being produced cannot be evicted: evict
    // only when the published frames free enough for the reservation to fit
    uint64_t evictable = 0;
    for (const auto &kv : b.map) evictable += kv.second->bytes();
    if (b.bytes - evictable + need > cap) return nullptr;
    while (b.bytes + need > cap && !b.lru.empty()) {
      auto it = b.map.find(b.lru.back());
      b.lru.pop_back();
      if (it == b.map.end()) continue;
      b.bytes -= it->second->bytes();
      it->second->budget = nullptr;
      evicted.push_back(std::move(it->second));
      b.map.erase(it);
    }
    if (b.bytes + need > cap) return nullptr;
    b.bytes += need;
    return &b;
  }
  void publish(const std::shared_ptr<ResidentFrame> &f, std::vector<std::shared_ptr<ResidentFrame>> &dropped) {
    std::lock_guard lk(m);
    FrameBudget &b = dev[f->device];
    auto it = b.map.find(f->key);
    if (it != b.map.end()) {
      b.bytes -= it->second->bytes();
      it->second->budget = nullptr;
      dropped.push_back(std::move(it->second));
      b.lru.remove(f->key);
    }
    b.map[f->key] = f;
    b.lru.push_front(f->key);
  }
  // the partition is being rewritten: no device may serve its old contents
  // (a failed write-behind of the old contents no longer matters)
  void drop(const std::string &key, std::vector<std::shared_ptr<ResidentFrame>> &dropped) {
    std::lock_guard lk(m);
    flush_failed.erase(key);
    drop_locked(key, dropped);
  }
  void drop_locked(const std::string &key, std::vector<std::shared_ptr<ResidentFrame>> &dropped) {
    for (auto &kv : dev) {
      FrameBudget &b = kv.second;
      auto it = b.map.find(key);
      if (it == b.map.end()) continue;
      b.bytes -= it->second->bytes();
      it->second->budget = nullptr;
      dropped.push_back(std::move(it->second));
      b.map.erase(it);
      b.lru.remove(key);
    }
  }
  // every frame whose key starts with `prefix` (a session's or a data frame's
  // partitions): herdsman deleted them
  void drop_prefix(const std::string &prefix, std::vector<std::shared_ptr<ResidentFrame>> &dropped) {
    std::lock_guard lk(m);
    std::set<std::string> keys;
    for (auto &kv : dev)
      for (auto &f : kv.second.map)
        if (f.first.compare(0, prefix.size(), prefix) == 0) keys.insert(f.first);
    for (const auto &k : keys) drop_locked(k, dropped);
    for (auto it = flush_failed.begin(); it != flush_failed.end();)
      it = it->first.compare(0, prefix.size(), prefix) == 0 ? flush_failed.erase(it) : std::next(it);
  }
  // free every published frame of the device (a device allocation failed)
  void evict_all(int device, std::vector<std::shared_ptr<ResidentFrame>> &evicted) {
    std::lock_guard lk(m);
    FrameBudget &b = dev[device];
    std::vector<std::string> keys(b.lru.begin(), b.lru.end());
    for (const auto &k : keys) drop_locked(k, evicted);
  }
  std::shared_ptr<ResidentFrame> lookup(int device, const std::string &key, int schema) {
    std::vector<std::shared_ptr<ResidentFrame>> stale;  // freed after the lock is released
    std::lock_guard lk(m);
    FrameBudget &b = dev[device];
    auto it = b.map.find(key);
    if (it == b.map.end() || it->second->schema != schema) return nullptr;
    if (it->second->file_known) {  // the committed file must still be the one this frame holds
      std::error_code ec;
      const uintmax_t sz = std::filesystem::file_size(it->second->file, ec);
      const auto mt = ec ? std::filesystem::file_time_type{} : std::filesystem::last_write_time(it->second->file, ec);
      if (ec || sz != it->second->file_size || mt != it->second->file_mtime) {
        drop_locked(key, stale);
        return nullptr;
      }
    }
    b.lru.remove(key);
    b.lru.push_front(key);
    return it->second;
  }
  // a file still being written behind is read only once it is committed
  void wait_file(const std::string &key) {
    std::unique_lock lk(m);
    cv.wait(lk, [&] { return !pending.count(key); });
  }
  // the error of a failed write-behind of `key`, or empty
  std::string flush_error(const std::string &key) {
    std::lock_guard lk(m);
    auto it = flush_failed.find(key);
    return it == flush_failed.end() ? std::string() : it->second;
  }
  // true once per failed write-behind of the session: its next task reports it
  bool take_session_failure(const std::string &session) {
    std::lock_guard lk(m);
    return failed_sessions.erase(session) > 0;
  }
};

namespace {
// the committed file's identity, recorded in a frame that holds its contents
void note_file(ResidentFrame &f) {
  std::error_code ec;
  const uintmax_t sz = std::filesystem::file_size(f.file, ec);
  if (ec) return;
  const auto mt = std::filesystem::last_write_time(f.file, ec);
  if (ec) return;
  f.file_size = sz;
  f.file_mtime = mt;
  f.file_known = true;
}
}  // namespace

ResidentFrame::~ResidentFrame() {
  if (p) fhe_dev_free(ctx, p);
}

namespace {
// release the bytes of a frame that never reached the map (a failed task)
void unreserve(std::mutex &m, FrameBudget &b, ResidentFrame &f) {
  std::lock_guard lk(m);
  if (f.budget) b.bytes -= f.bytes();
  f.budget = nullptr;
}

std::string frame_key(const herd::common::UUID &session, const herd::common::DataFramePtr &p) {
  return session.as_string() + "/" + p.uuid.as_string() + "/" + std::to_string(p.partition);
}
}  // namespace

GpuWorkerGroup::GpuWorkerGroup(GpuWorkerGroupConfig config) : config_(std::move(config)), frames_(new Frames) {
  if (config_.devices.empty()) throw std::invalid_argument("GpuWorkerGroup needs at least one device");
  if (!circuits_lowerable())
    std::fprintf(stderr,
                 "GpuWorkerGroup: herd_common's Circuit has no lowering to backend ops (INTEGRATION.md §2); "
                 "every task will complete with ERROR\n");
  if (config_.lanes_per_device == 0) config_.lanes_per_device = 1;
  if (config_.max_batch == 0) config_.max_batch = 1;
  for (int d : config_.devices) {
    auto dev = std::make_unique<Device>();
    dev->id = d;
    for (uint32_t l = 0; l < config_.lanes_per_device; ++l) dev->lanes.push_back(std::make_unique<Lane>());
    devices_.push_back(std::move(dev));
  }
  for (auto &d : devices_)
    for (auto &l : d->lanes) l->thread = std::thread([this, dp = d.get(), lp = l.get()] { lane_loop(*dp, *lp); });
  completion_thread_ = std::thread([this] { completion_loop(); });
  if (config_.write_behind)
    for (uint32_t i = 0; i < std::max(1u, config_.flush_threads); ++i)
      flush_threads_.emplace_back([this, i] { flush_loop(i); });
}

GpuWorkerGroup::~GpuWorkerGroup() {
  for (auto &d : devices_) {
    {
      std::lock_guard lk(d->m);
      d->stop = true;
    }
    d->cv.notify_all();
  }
  for (auto &d : devices_)
    for (auto &l : d->lanes) l->thread.join();
  // files written behind are committed before the group goes
  if (!flush_threads_.empty()) {
    flush_frames();
    {
      std::lock_guard lk(frames_->m);
      frames_->stop = true;
    }
    frames_->cv.notify_all();
    for (auto &t : flush_threads_) t.join();
  }
  // teardown order: resident frames, keys and lane buffers are freed through
  // their contexts, so they go before the contexts
  {
    std::map<int, FrameBudget> gone;
    {
      std::lock_guard lk(frames_->m);
      gone.swap(frames_->dev);
      for (auto &kv : gone)
        for (auto &f : kv.second.map) f.second->budget = nullptr;
    }
  }
  for (auto &kv : frames_->flush_ctx) fhe_ctx_destroy(kv.second);
  frames_->flush_ctx.clear();
  for (auto &d : devices_) {
    d->keys.clear();
    for (auto &l : d->lanes) {
      for (auto &kv : l->schemas) {
        LaneSchema &ls = *kv.second;
        ls.arena.reset();
        for (Slot &sl : ls.slot) {
          sl.in.clear();
          if (sl.out.p) fhe_host_free(sl.out.ctx, sl.out.p);
          sl.out.p = nullptr;
        }
        fhe_ctx_destroy(ls.s.ctx);
      }
      l->schemas.clear();
    }
  }
  {
    std::lock_guard lk(done_mutex_);
    stopping_ = true;
  }
  done_cv_.notify_one();
  completion_thread_.join();
}

StageStats GpuWorkerGroup::stage_stats() {
  StageStats st;
  {
    std::lock_guard lk(stats_m_);
    st = stats_;
  }
  std::lock_guard lk(frames_->m);
  st.flushed_rows += frames_->st.flushed_rows;
  st.flush_s += frames_->st.flush_s;
  return st;
}

void GpuWorkerGroup::reset_stage_stats() {
  {
    std::lock_guard lk(stats_m_);
    stats_ = StageStats{};
  }
  std::lock_guard lk(frames_->m);
  frames_->st = StageStats{};
}

void GpuWorkerGroup::drop_frames(const herd::common::UUID &session, const herd::common::UUID *frame) {
  std::vector<std::shared_ptr<ResidentFrame>> dropped;
  frames_->drop_prefix(session.as_string() + "/" + (frame ? frame->as_string() + "/" : std::string()), dropped);
}

bool GpuWorkerGroup::flush_frames() {
  std::unique_lock lk(frames_->m);
  frames_->cv.wait(lk, [&] { return frames_->queue.empty() && frames_->pending.empty(); });
  const bool ok = !frames_->failed;
  frames_->failed = false;
  return ok;
}

std::size_t GpuWorkerGroup::concurrent_workers() const noexcept {
  return devices_.size() * config_.lanes_per_device;
}

std::shared_ptr<IWorkerGroup::TaskHandle> GpuWorkerGroup::schedule_task(const herd::common::task_t &task) {
  auto h = std::make_shared<Handle>();
  if (std::holds_alternative<std::monostate>(task) || !circuits_lowerable()) {
    complete(h, Status::ERROR);  // delivered once the executor attaches its callback
    return h;
  }
  const std::string session =
      std::visit([](const auto &t) -> std::string {
        if constexpr (std::is_same_v<std::decay_t<decltype(t)>, std::monostate>) return std::string();
        else return t.session_uuid.as_string();
      }, task);
  if (frames_->take_session_failure(session)) {
    std::fprintf(stderr, "GpuWorkerGroup: session %s: a partition written behind failed to commit; task fails\n",
                 session.c_str());
    complete(h, Status::ERROR);
    return h;
  }
  Device &d = *devices_[next_device_.fetch_add(1) % devices_.size()];  // round robin, like grpc_worker_group.cpp:102
  {
    std::lock_guard lk(d.m);
    d.queue.push_back(Job{h, task});
  }
  d.cv.notify_one();
  return h;
}

void GpuWorkerGroup::complete(const std::shared_ptr<Handle> &h, Status st) {
  h->status_.store(st);
  {
    std::lock_guard lk(done_mutex_);
    done_.push_back(h);
  }
  done_cv_.notify_one();
}

void GpuWorkerGroup::completion_loop() {
  std::vector<std::shared_ptr<Handle>> waiting;  // completed, callback not attached yet
  // poll interval for undelivered handles: 50 us right after a completion
  // (the executor attaches its callback within microseconds), backing off to
  // 5 ms while nothing is delivered
  auto poll = std::chrono::microseconds(50);
  std::unique_lock lk(done_mutex_);
  while (true) {
    done_cv_.wait_for(lk, waiting.empty() ? std::chrono::microseconds(100000) : poll,
                      [&] { return stopping_ || !done_.empty(); });
    const bool fresh = !done_.empty();
    while (!done_.empty()) {
      waiting.push_back(std::move(done_.front()));
      done_.pop_front();
    }
    const bool stop = stopping_;
    lk.unlock();
    size_t delivered = 0;
    for (size_t i = 0; i < waiting.size();) {
      if (waiting[i]->try_deliver()) {
        waiting[i] = std::move(waiting.back());
        waiting.pop_back();
        ++delivered;
      } else {
        ++i;
      }
    }
    poll = (fresh || delivered) ? std::chrono::microseconds(50) : std::min(poll * 2, std::chrono::microseconds(5000));
    lk.lock();
    if (stop && done_.empty()) return;  // handles never picked up by a callback are dropped here
  }
}

// ------------------------------------------------------------- evaluation
namespace {

enum class Op : uint32_t { PUSH_INPUT = 0, ADD = 1, SUB = 2, MUL_RELIN = 3, ROTATE = 4, RESCALE = 5, ROTSUM = 6 };
struct Instr {
  Op op;
  int32_t arg;
};

// herd_common's Circuit -> the backend's stack program.  The stand-in circuit
// (herd_common_standin.hpp) IS such a program; a herd_common Circuit with
// another shape compiles and fails its tasks loudly until its gates are
// mapped here (circuit interpretation, SURVEY.md §8f-4, is blocked on the
// absent herd_common).
template <class C>
std::vector<Instr> lower_circuit(const C &c) {
  if constexpr (requires { c.program.begin()->op; c.program.begin()->arg; }) {
    std::vector<Instr> out;
    for (const auto &i : c.program) {
      const uint32_t op = static_cast<uint32_t>(i.op);
      if (op > static_cast<uint32_t>(Op::ROTSUM)) throw std::runtime_error("unknown circuit op");
      out.push_back(Instr{static_cast<Op>(op), static_cast<int32_t>(i.arg)});
    }
    return out;
  } else {
    throw std::runtime_error("no lowering from this herd_common Circuit to backend ops (INTEGRATION.md §2)");
  }
}

template <class C>
constexpr bool lowerable_v = requires(const C &c) {
  c.program.begin()->op;
  c.program.begin()->arg;
};

template <class T>
int schema_id(T v) {
  return static_cast<int>(v);  // herd_common's SchemaType is an enum (key_service.cpp:28)
}

LaneSchema &lane_schema(std::map<int, std::unique_ptr<LaneSchema>> &m, const GpuWorkerGroupConfig &cfg, int device,
                        int schema) {
  auto it = m.find(schema);
  if (it != m.end()) return *it->second;
  const SchemaParams *sp = nullptr;
  for (const auto &s : cfg.schemas)
    if (s.schema_type == schema) sp = &s;
  if (!sp) throw std::runtime_error("no backend parameters for schema " + std::to_string(schema));
  fhe_params p = sp->params;
  p.moduli = sp->moduli.empty() ? nullptr : sp->moduli.data();
  auto ls = std::make_unique<LaneSchema>();
  SchemaCtx &s = ls->s;
  if (fhe_ctx_create(&p, device, &s.ctx) != FHE_OK)
    throw std::runtime_error(std::string("fhe_ctx_create: ") + fhe_last_error(nullptr));
  ls->arena = std::make_unique<Arena>(s.ctx);
  s.scheme = p.scheme;
  s.log_n = p.log_n;
  s.L = p.num_q;
  s.K = p.num_p;
  s.dnum = p.dnum;
  uint32_t cnt = 0;
  fhe_ctx_moduli(s.ctx, nullptr, 0, &cnt);
  s.moduli.resize(cnt);
  fhe_ctx_moduli(s.ctx, s.moduli.data(), cnt, nullptr);
  s.q_digest = moduli_digest(s.moduli.data(), s.L);
  s.qp_digest = moduli_digest(s.moduli.data(), s.L + s.K);
  s.level_digest.resize(s.L + 1);
  for (uint32_t lv = 1; lv <= s.L; ++lv) s.level_digest[lv] = moduli_digest(s.moduli.data(), lv);
  auto &slot = m[schema];
  slot = std::move(ls);
  // the lane's own stream: lanes of one device run concurrently
  ck(slot->s.ctx, fhe_use_own_stream(slot->s.ctx), "own stream");
  return *slot;
}

std::shared_ptr<KeySet> load_keys(const SchemaCtx &s, const std::filesystem::path &file) {
  std::ifstream in(file, std::ios::binary);
  if (!in) throw std::runtime_error("cannot open key file " + file.string());
  KeyFileHeader h;
  in.read(reinterpret_cast<char *>(&h), sizeof(h));
  if (!in || h.magic != kKeyMagic || h.version != 1) throw std::runtime_error("bad key file header");
  if (h.scheme != s.scheme || h.log_n != s.log_n || h.L != s.L || h.K != s.K || h.dnum != s.dnum ||
      h.moduli_digest != s.qp_digest)
    throw std::runtime_error("key file parameters do not match the schema context");
  auto ks = std::make_shared<KeySet>();
  std::vector<uint64_t> host(s.key_words());
  for (uint32_t i = 0; i < h.n_keys; ++i) {
    KeyEntryHeader e;
    in.read(reinterpret_cast<char *>(&e), sizeof(e));
    in.read(reinterpret_cast<char *>(host.data()), host.size() * 8);
    if (!in) throw std::runtime_error("truncated key file");
    DevBuf d(s.ctx, host.size());
    ck(s.ctx, fhe_memcpy_h2d(s.ctx, d.p, host.data(), host.size() * 8), "key upload");
    if (e.kind == 0) ks->relin = std::move(d);
    else ks->galois.emplace(e.galois_elt, std::move(d));
  }
  ck(s.ctx, fhe_synchronize(s.ctx), "key upload sync");  // visible to every lane's stream from here on
  return ks;
}

// the device's keys for (session, schema), loaded once through the asking lane
std::shared_ptr<KeySet> device_keys(std::mutex &m, std::map<std::pair<std::string, int>, std::shared_ptr<KeySet>> &keys,
                                    const SchemaCtx &s, const std::filesystem::path &key_dir,
                                    const std::string &session, int schema) {
  std::lock_guard lk(m);
  auto &k = keys[std::make_pair(session, schema)];
  if (!k) k = load_keys(s, key_dir / session / (std::to_string(schema) + ".key"));
  return k;
}

// the ciphertext's level (its limb count): 1..L for CKKS, L for BFV
uint32_t check_ct_header(const SchemaCtx &s, const CtHeader &h) {
  const bool level_ok = s.scheme == FHE_SCHEME_CKKS ? (h.n_limbs >= 1 && h.n_limbs <= s.L) : h.n_limbs == s.L;
  if (h.magic != kCtMagic || h.version != 1 || h.scheme != s.scheme || h.log_n != s.log_n || !level_ok ||
      h.moduli_digest != s.level_digest[h.n_limbs])
    throw std::runtime_error("ciphertext header does not match the schema context");
  return h.n_limbs;
}

CtHeader ct_header(const SchemaCtx &s, uint32_t level) {
  CtHeader h;
  h.scheme = (uint8_t)s.scheme;
  h.domain = s.scheme == FHE_SCHEME_CKKS ? 1 : 0;
  h.log_n = s.log_n;
  h.n_limbs = level;
  h.moduli_digest = s.level_digest[level];
  return h;
}

const DevBuf &galois_key(const SchemaCtx &s, const KeySet &ks, int32_t steps, uint32_t *g) {
  ck(s.ctx, fhe_galois_elt(s.ctx, steps, g), "galois_elt");
  auto it = ks.galois.find(*g);
  if (it == ks.galois.end()) throw std::runtime_error("no Galois key for element " + std::to_string(*g));
  return it->second;
}

// Batch k of a MapTask, first half: read the rows' ciphertexts straight from
// the partition file into slot k % 2's pinned buffers (pread), then enqueue
// H2D, the program's ops and D2H on the lane's stream and mark the slot.
// Nothing waits for the GPU here.
// One operand of the stack program: a batch of n ciphertexts at one level,
// in an arena buffer or (view) in a resident frame, which no op writes to.
struct StackCt {
  ArenaBuf buf;
  uint32_t level = 0;
  const uint64_t *view = nullptr;
  const uint64_t *ptr() const { return view ? view : buf.p; }
};

// The level-m copy of a (the first m limbs of each poly), or a itself
StackCt at_level(LaneSchema &ls, StackCt a, uint32_t m, size_t n) {
  if (a.level == m) return a;
  const SchemaCtx &s = ls.s;
  StackCt o{ArenaBuf(*ls.arena, s.ct_words(m) * n), m};
  ck(s.ctx, fhe_level_reduce(s.ctx, a.ptr(), o.buf.p, (uint32_t)n, a.level, m), "level_reduce");
  return o;
}

// Where a MapTask's rows come from and where its results go.
struct MapIo {
  const PartitionIndex *rows = nullptr;  // the input partition file, or
  std::shared_ptr<ResidentFrame> in;     // the input partition resident in HBM (one ciphertext per row)
  std::shared_ptr<ResidentFrame> out;    // this task's output kept resident (null: not kept)
  bool write_file = true;                // the lane copies results back and writes the file
  size_t row_count() const { return in ? in->rows : rows->size(); }
};

// byte offset and level of every input index the program pushes, from row r0
// (a resident row is one ciphertext at the frame's level)
void input_layout(const SchemaCtx &s, const MapIo &io, int32_t max_in, size_t r0, std::vector<size_t> &off,
                  std::vector<uint32_t> &level) {
  off.clear();
  level.clear();
  if (io.in) {
    if (max_in > 0) throw std::runtime_error("row holds fewer ciphertexts than the circuit reads");
    off.push_back(0);
    level.push_back(io.in->level);
    return;
  }
  for (size_t o = 0; (int32_t)off.size() <= max_in;) {
    CtHeader h;
    io.rows->read(r0, o, &h, sizeof(h));
    const uint32_t m = check_ct_header(s, h);
    off.push_back(o);
    level.push_back(m);
    o += sizeof(h) + s.ct_words(m) * 8;
  }
}

int32_t max_input(const std::vector<Instr> &prog) {
  int32_t max_in = -1;
  for (const auto &ins : prog)
    if (ins.op == Op::PUSH_INPUT) max_in = std::max(max_in, ins.arg);
  return max_in;
}

// the level of the program's result for inputs at these levels (the ops'
// level rules below), or 0 if the program is malformed (the batch then fails
// where it runs)
uint32_t program_level(const std::vector<Instr> &prog, const std::vector<uint32_t> &in_level) {
  std::vector<uint32_t> st;
  for (const auto &ins : prog) {
    switch (ins.op) {
      case Op::PUSH_INPUT:
        if (ins.arg < 0 || (size_t)ins.arg >= in_level.size()) return 0;
        st.push_back(in_level[ins.arg]);
        break;
      case Op::ADD:
      case Op::SUB:
      case Op::MUL_RELIN: {
        if (st.size() < 2) return 0;
        const uint32_t b = st.back();
        st.pop_back();
        st.back() = std::min(st.back(), b);
        break;
      }
      case Op::RESCALE:
        if (st.empty() || st.back() < 2) return 0;
        st.back() -= 1;
        break;
      default:
        if (st.empty()) return 0;
    }
  }
  return st.size() == 1 ? st.back() : 0;
}

// Batch k of a MapTask, first half: read the rows' ciphertexts straight from
// the partition file into slot k % 2's pinned buffers (pread), then enqueue
// H2D, the program's ops and D2H on the lane's stream and mark the slot.
// Nothing waits for the GPU here.  A row holds its ciphertexts back to back,
// each CtHeader + 2 m N words at its own level m (CKKS); the batch's first
// row fixes each input's level, and every row must match it.
void enqueue_map_batch(LaneSchema &ls, int si, const KeySet &ks, const std::vector<Instr> &prog, const MapIo &io,
                       size_t r0, size_t n, unsigned io_threads, StageStats &st) {
  const SchemaCtx &s = ls.s;
  Slot &sl = ls.slot[si];
  sl.r0 = r0;
  sl.n = n;
  std::vector<size_t> in_off;
  std::vector<uint32_t> in_level;
  input_layout(s, io, max_input(prog), r0, in_off, in_level);
  std::vector<StackCt> stack;
  size_t push = 0;
  double read_s = 0;
  const auto t_enq = std::chrono::steady_clock::now();
  if (io.in) st.resident_rows += n;
  for (const auto &ins : prog) {
    switch (ins.op) {
      case Op::PUSH_INPUT: {
        if (ins.arg < 0) throw std::runtime_error("negative input index");
        const uint32_t m = in_level[ins.arg];
        const size_t cw = s.ct_words(m), off = in_off[ins.arg];
        if (io.in) {  // resident: the rows are already in HBM, in batch order
          StackCt d;
          d.level = m;
          d.view = io.in->p + r0 * io.in->cw;
          stack.push_back(std::move(d));
          break;
        }
        if (sl.in.size() <= push) sl.in.push_back(std::make_unique<Pinned>());
        uint64_t *host = reinterpret_cast<uint64_t *>(sl.in[push++]->reserve(s.ctx, cw * n * 8));
        const auto t_r = std::chrono::steady_clock::now();
        const PartitionIndex &rows = *io.rows;
        // every row's header is checked on the way (the first row fixed the
        // offsets: a row whose earlier ciphertexts sit at other levels fails
        // here, at the first input whose header does not match)
        parallel_for(n, io_threads, [&](size_t r) {
          CtHeader h;
          rows.read(r0 + r, off, &h, sizeof(h));
          if (h.magic != kCtMagic || h.n_limbs != m)
            throw std::runtime_error("rows of a batch differ in ciphertext level (input " + std::to_string(ins.arg) +
                                     " of row " + std::to_string(r0 + r) + ")");
          check_ct_header(s, h);
          rows.read(r0 + r, off + sizeof(h), host + r * cw, cw * 8);
        });
        read_s += secs_since(t_r);
        StackCt d{ArenaBuf(*ls.arena, cw * n), m};
        ck(s.ctx, fhe_memcpy_h2d_async(s.ctx, d.buf.p, host, cw * n * 8), "h2d");
        stack.push_back(std::move(d));
        break;
      }
      case Op::ADD:
      case Op::SUB:
      case Op::MUL_RELIN: {
        if (stack.size() < 2) throw std::runtime_error("circuit stack underflow");
        StackCt b = std::move(stack.back());
        stack.pop_back();
        StackCt a = std::move(stack.back());
        stack.pop_back();
        const uint32_t m = std::min(a.level, b.level);
        a = at_level(ls, std::move(a), m, n);
        b = at_level(ls, std::move(b), m, n);
        StackCt o{ArenaBuf(*ls.arena, s.ct_words(m) * n), m};
        if (ins.op == Op::ADD) ck(s.ctx, fhe_add_at(s.ctx, a.ptr(), b.ptr(), o.buf.p, (uint32_t)n, m), "add");
        else if (ins.op == Op::SUB) ck(s.ctx, fhe_sub_at(s.ctx, a.ptr(), b.ptr(), o.buf.p, (uint32_t)n, m), "sub");
        else {
          if (!ks.relin.p) throw std::runtime_error("no relinearisation key");
          ck(s.ctx, fhe_mul_relin_at(s.ctx, a.ptr(), b.ptr(), ks.relin.p, o.buf.p, (uint32_t)n, m), "mul_relin");
        }
        stack.push_back(std::move(o));
        break;
      }
      case Op::ROTATE: {
        if (stack.empty()) throw std::runtime_error("circuit stack underflow");
        uint32_t g = 0;
        const DevBuf &gk = galois_key(s, ks, ins.arg, &g);
        const uint32_t m = stack.back().level;
        StackCt o{ArenaBuf(*ls.arena, s.ct_words(m) * n), m};
        ck(s.ctx, fhe_rotate_at(s.ctx, stack.back().ptr(), g, gk.p, o.buf.p, (uint32_t)n, m), "rotate");
        stack.back() = std::move(o);
        break;
      }
      case Op::ROTSUM: {
        // sum of rotations by the steps in the mask, double-hoisted: one ModUp
        // of c1 and ONE ModDown for all of them (fhe_rotate_sum_hoisted_at); bit 0
        // adds the input itself
        if (stack.empty()) throw std::runtime_error("circuit stack underflow");
        const uint32_t mask = (uint32_t)ins.arg;
        if (mask == 0 || (mask >> 31)) throw std::runtime_error("rotsum step mask must be in [1, 2^31)");
        const uint32_t m = stack.back().level;
        std::vector<uint32_t> gs;
        std::vector<const uint64_t *> gks;
        for (int32_t k = 1; k < 31; ++k) {
          if (!((mask >> k) & 1)) continue;
          uint32_t g = 0;
          gks.push_back(galois_key(s, ks, k, &g).p);
          gs.push_back(g);
        }
        if (gs.empty()) break;  // mask 1: the input itself
        const uint64_t *top = stack.back().ptr();
        StackCt o{ArenaBuf(*ls.arena, s.ct_words(m) * n), m};
        ck(s.ctx, fhe_rotate_sum_hoisted_at(s.ctx, top, (uint32_t)gs.size(), gs.data(), gks.data(), o.buf.p,
                                            (uint32_t)n, m), "rotate_sum_hoisted");
        if (mask & 1) ck(s.ctx, fhe_add_at(s.ctx, o.buf.p, top, o.buf.p, (uint32_t)n, m), "rotsum add");
        stack.back() = std::move(o);
        break;
      }
      case Op::RESCALE: {
        if (stack.empty()) throw std::runtime_error("circuit stack underflow");
        const uint32_t m = stack.back().level;
        if (m < 2) throw std::runtime_error("rescale of a level-1 ciphertext");
        StackCt o{ArenaBuf(*ls.arena, s.ct_words(m - 1) * n), m - 1};
        ck(s.ctx, fhe_rescale(s.ctx, stack.back().ptr(), o.buf.p, (uint32_t)n, m), "rescale");
        stack.back() = std::move(o);
        break;
      }
      default:
        throw std::runtime_error("unknown circuit op");
    }
  }
  if (stack.size() != 1) throw std::runtime_error("circuit must leave exactly one ciphertext");
  sl.out_level = stack.back().level;
  const size_t cw = s.ct_words(sl.out_level);
  if (io.out) {  // kept resident for the stage that reads this partition
    if (io.out->level != sl.out_level) throw std::runtime_error("resident frame level mismatch");
    ck(s.ctx, fhe_memcpy_d2d_async(s.ctx, io.out->p + r0 * io.out->cw, stack.back().ptr(), cw * n * 8), "d2d");
  }
  if (io.write_file) {
    uint64_t *host = reinterpret_cast<uint64_t *>(sl.out.reserve(s.ctx, cw * n * 8));
    ck(s.ctx, fhe_memcpy_d2h_async(s.ctx, host, stack.back().ptr(), cw * n * 8), "d2h");
  }
  // the device buffers go back to the arena now: later ops that reuse them are
  // ordered after this batch's copies by the stream
  ck(s.ctx, fhe_mark(s.ctx, (uint32_t)si), "mark");
  st.read_s += read_s;
  st.enqueue_s += secs_since(t_enq) - read_s;
}

// Second half: wait for the slot's mark (its D2H has landed, its H2D sources
// are free again) and append the batch's rows to the output partition.
void finish_map_batch(LaneSchema &ls, int si, PartitionWriter *out, unsigned io_threads, StageStats &st) {
  const SchemaCtx &s = ls.s;
  Slot &sl = ls.slot[si];
  auto t0 = std::chrono::steady_clock::now();
  ck(s.ctx, fhe_wait_mark(s.ctx, (uint32_t)si), "batch wait");
  st.wait_s += secs_since(t0);
  st.batches += 1;
  st.rows += sl.n;
  if (!out) return;  // write-behind: the flusher writes the file from the resident frame
  t0 = std::chrono::steady_clock::now();
  const size_t cw = s.ct_words(sl.out_level);
  const uint64_t *host = reinterpret_cast<const uint64_t *>(sl.out.p);
  const CtHeader h = ct_header(s, sl.out_level);
  const uint64_t row_bytes = 4 + sizeof(h) + cw * 8;
  const uint64_t base = out->claim(row_bytes * sl.n);
  parallel_for(sl.n, io_threads,
               [&](size_t r) { out->write_row_at(base + r * row_bytes, {{&h, sizeof(h)}, {host + r * cw, cw * 8}}); });
  st.write_s += secs_since(t0);
}

std::filesystem::path frame_path(const std::filesystem::path &root, const herd::common::UUID &session,
                                 const herd::common::DataFramePtr &p) {
  return root / session.as_string() / p.uuid.as_string() / std::to_string(p.partition);
}

}  // namespace

bool GpuWorkerGroup::circuits_lowerable() noexcept { return lowerable_v<herd::common::Circuit>; }

// write-behind: the flusher copies each queued resident frame back in chunks
// (two pinned buffers, the next chunk's D2H under the current chunk's file
// writes) on a context and stream of its own, and commits the partition file
void GpuWorkerGroup::flush_loop(uint32_t id) {
  constexpr size_t kRows = 16;
  Pinned stage[2];
  for (;;) {
    std::shared_ptr<ResidentFrame> f;
    {
      std::unique_lock lk(frames_->m);
      frames_->cv.wait(lk, [&] { return frames_->stop || !frames_->queue.empty(); });
      if (frames_->queue.empty()) return;
      f = frames_->queue.front();
      frames_->queue.pop_front();
    }
    const auto t0 = std::chrono::steady_clock::now();
    std::string err;
    try {
      fhe_ctx *c = nullptr;
      {
        std::lock_guard lk(frames_->m);
        c = frames_->flush_ctx[std::make_tuple(id, f->device, f->schema)];
      }
      if (!c) {
        const SchemaParams *sp = nullptr;
        for (const auto &x : config_.schemas)
          if (x.schema_type == f->schema) sp = &x;
        if (!sp) throw std::runtime_error("no parameters for schema " + std::to_string(f->schema));
        fhe_params p = sp->params;
        p.moduli = sp->moduli.empty() ? nullptr : sp->moduli.data();
        if (fhe_ctx_create(&p, f->device, &c) != FHE_OK)
          throw std::runtime_error(std::string("flusher fhe_ctx_create: ") + fhe_last_error(nullptr));
        {
          std::lock_guard lk(frames_->m);
          frames_->flush_ctx[std::make_tuple(id, f->device, f->schema)] = c;
        }
        ck(c, fhe_use_own_stream(c), "flusher stream");
      }
      PartitionWriter out(f->file, f->durable);
      const uint64_t row_bytes = 4 + sizeof(CtHeader) + f->cw * 8;
      const size_t chunks = (f->rows + kRows - 1) / kRows;
      const auto enqueue = [&](size_t ci) {
        const size_t r0 = ci * kRows, n = std::min(kRows, f->rows - r0);
        uint8_t *h = stage[ci & 1].reserve(c, kRows * f->cw * 8);
        ck(c, fhe_memcpy_d2h_async(c, h, f->p + r0 * f->cw, n * f->cw * 8), "flush d2h");
        ck(c, fhe_mark(c, (uint32_t)(ci & 1)), "flush mark");
      };
      if (chunks) enqueue(0);
      for (size_t ci = 0; ci < chunks; ++ci) {
        ck(c, fhe_wait_mark(c, (uint32_t)(ci & 1)), "flush wait");
        if (ci + 1 < chunks) enqueue(ci + 1);
        const size_t r0 = ci * kRows, n = std::min(kRows, f->rows - r0);
        const uint64_t *host = reinterpret_cast<const uint64_t *>(stage[ci & 1].p);
        const uint64_t base = out.claim(row_bytes * n);
        parallel_for(n, config_.io_threads, [&](size_t r) {
          out.write_row_at(base + r * row_bytes, {{&f->header, sizeof(CtHeader)}, {host + r * f->cw, f->cw * 8}});
        });
      }
      out.commit();
    } catch (const std::exception &e) {
      err = e.what();
    }
    {
      std::lock_guard lk(frames_->m);
      auto it = frames_->pending.find(f->key);
      if (it != frames_->pending.end() && it->second == f) frames_->pending.erase(it);
      frames_->st.flush_s += secs_since(t0);
      if (err.empty()) {
        frames_->st.flushed_rows += f->rows;
        note_file(*f);
      } else {
        frames_->failed = true;
        frames_->flush_failed[f->key] = err;
        frames_->failed_sessions.insert(f->key.substr(0, f->key.find('/')));
        std::fprintf(stderr, "GpuWorkerGroup: write-behind of %s failed: %s\n", f->file.c_str(), err.c_str());
      }
    }
    frames_->cv.notify_all();
  }
}

void GpuWorkerGroup::lane_loop(Device &dev, Lane &lane) {
  while (true) {
    Job job;
    {
      std::unique_lock lk(dev.m);
      dev.cv.wait(lk, [&] { return dev.stop || !dev.queue.empty(); });
      if (dev.queue.empty()) break;  // stopping and drained
      job = std::move(dev.queue.front());
      dev.queue.pop_front();
    }
    Status st = Status::COMPLETED;
    LaneSchema *cur = nullptr;
    StageStats stats;
    const auto t_task = std::chrono::steady_clock::now();
    try {
      if (std::holds_alternative<herd::common::MapTask>(job.task)) {
        const auto &t = std::get<herd::common::MapTask>(job.task);
        const int schema = schema_id(t.crypto_key_ptr.schema_type);
        const std::vector<Instr> prog = lower_circuit(t.circuit);
        LaneSchema &ls = lane_schema(lane.schemas, config_, dev.id, schema);
        cur = &ls;
        const SchemaCtx &s = ls.s;
        auto ks = device_keys(dev.keys_m, dev.keys, s, config_.key_dir, t.session_uuid.as_string(), schema);
        const std::string in_key = frame_key(t.session_uuid, t.input_data_frame_ptr.pointer);
        const std::string out_key = frame_key(t.session_uuid, t.output_data_frame_ptr);
        const auto out_path = frame_path(config_.storage_dir, t.session_uuid, t.output_data_frame_ptr);
        std::vector<std::shared_ptr<ResidentFrame>> released;  // freed outside the frames lock
        frames_->drop(out_key, released);  // the output partition is rewritten: no stale copy stays
        frames_->wait_file(out_key);       // nor may an older flush of it commit after this task's file
        MapIo io;
        std::unique_ptr<PartitionIndex> in_file;
        io.in = frames_->lookup(dev.id, in_key, schema);
        if (!io.in) {
          frames_->wait_file(in_key);  // a file still being written behind
        }
        if (const std::string e = frames_->flush_error(in_key); !e.empty())
          throw std::runtime_error("input partition " + in_key + " was never committed (write-behind failed: " + e + ")");
        if (!io.in) {
          in_file = std::make_unique<PartitionIndex>(
              frame_path(config_.storage_dir, t.session_uuid, t.input_data_frame_ptr.pointer));
          io.rows = in_file.get();
        }
        const size_t nrows = io.row_count();
        // keep the output resident when every batch's result has one level
        if (config_.resident_frame_bytes && nrows) {
          uint32_t lvl = 0;
          bool one = true;
          std::vector<size_t> off;
          std::vector<uint32_t> lv;
          for (size_t r0 = 0; r0 < nrows && one; r0 += config_.max_batch) {
            input_layout(s, io, max_input(prog), r0, off, lv);
            const uint32_t l = program_level(prog, lv);
            one = l != 0 && (r0 == 0 || l == lvl);
            lvl = l;
          }
          const size_t cw = s.ct_words(lvl);
          FrameBudget *budget = nullptr;
          if (one) budget = frames_->reserve(dev.id, (uint64_t)nrows * cw * 8, config_.resident_frame_bytes, released);
          if (budget) {
            auto f = std::make_shared<ResidentFrame>();
            f->key = out_key;
            f->device = dev.id;
            f->schema = schema;
            f->level = lvl;
            f->rows = nrows;
            f->cw = cw;
            f->ctx = s.ctx;
            f->budget = budget;
            f->file = out_path;
            f->header = ct_header(s, lvl);
            f->durable = config_.durable_outputs;
            void *q = nullptr;
            int arc = fhe_dev_alloc(s.ctx, f->bytes(), &q);
            if (arc == FHE_ERR_OOM) {  // idle frames give way before the output falls back to its file
              std::vector<std::shared_ptr<ResidentFrame>> evicted;
              frames_->evict_all(dev.id, evicted);
              evicted.clear();
              arc = fhe_dev_alloc(s.ctx, f->bytes(), &q);
            }
            if (arc == FHE_OK) {
              f->p = static_cast<uint64_t *>(q);
              io.out = std::move(f);
            } else {
              unreserve(frames_->m, *f->budget, *f);  // no room in HBM: the file path alone
            }
          }
        }
        released.clear();
        io.write_file = !(config_.write_behind && io.out);
        struct Unreserve {  // a failed task's resident output never reaches the map
          Frames &fr;
          std::shared_ptr<ResidentFrame> &f;
          ~Unreserve() {
            if (!f) return;
            (void)fhe_synchronize(f->ctx);  // no copy into it is still in flight when it is freed
            if (f->budget) unreserve(fr.m, *f->budget, *f);
          }
        } unreserve_on_failure{*frames_, io.out};
        std::unique_ptr<PartitionWriter> out;
        if (io.write_file) out = std::make_unique<PartitionWriter>(out_path, config_.durable_outputs);
        // two-deep software pipeline over the batches: enqueue batch k, then
        // write batch k-1 while batch k runs on the GPU, then read batch k+1
        int pending = -1;  // slot of the batch enqueued but not yet written
        size_t k = 0;
        for (size_t r0 = 0; r0 < nrows; r0 += config_.max_batch, ++k) {
          const size_t n = std::min<size_t>(config_.max_batch, nrows - r0);
          const int si = (int)(k & 1);
          enqueue_map_batch(ls, si, *ks, prog, io, r0, n, config_.io_threads, stats);
          if (pending >= 0) finish_map_batch(ls, pending, out.get(), config_.io_threads, stats);
          pending = si;
        }
        if (pending >= 0) finish_map_batch(ls, pending, out.get(), config_.io_threads, stats);
        if (out) out->commit();
        if (io.out && io.write_file) note_file(*io.out);
        if (io.out) {
          // every batch's copy into the frame has completed (the last mark);
          // from here a task on any lane of this device reads it from HBM
          frames_->publish(io.out, released);
          if (!io.write_file) {
            {
              std::lock_guard lk(frames_->m);
              frames_->pending[out_key] = io.out;
              frames_->queue.push_back(io.out);
            }
            frames_->cv.notify_all();
          }
          io.out.reset();
        }
      } else {
        // ReduceTask: combine every row of every input partition into one
        // ciphertext with a balanced tree of batched ADDs (MUL_RELIN if the
        // circuit's first op says so), on the GPU.
        const auto &t = std::get<herd::common::ReduceTask>(job.task);
        const int schema = schema_id(t.crypto_key_ptr.schema_type);
        const std::vector<Instr> prog = lower_circuit(t.circuit);
        LaneSchema &ls = lane_schema(lane.schemas, config_, dev.id, schema);
        cur = &ls;
        const SchemaCtx &s = ls.s;
        const bool mul = !prog.empty() && prog.front().op == Op::MUL_RELIN;
        std::shared_ptr<KeySet> ks;
        if (mul) ks = device_keys(dev.keys_m, dev.keys, s, config_.key_dir, t.session_uuid.as_string(), schema);
        {
          std::vector<std::shared_ptr<ResidentFrame>> released;
          const std::string out_key = frame_key(t.session_uuid, t.output_data_frame_ptr);
          frames_->drop(out_key, released);
          frames_->wait_file(out_key);
        }
        // each input partition from HBM when a Map stage on this device left it
        // resident, else from its file
        struct Input {
          std::unique_ptr<PartitionIndex> file;
          std::shared_ptr<ResidentFrame> res;
          size_t size() const { return res ? res->rows : file->size(); }
        };
        std::vector<Input> parts;
        size_t count = 0;
        for (const auto &in : t.input_data_frame_ptrs) {
          Input pi;
          const std::string key = frame_key(t.session_uuid, in.pointer);
          pi.res = frames_->lookup(dev.id, key, schema);
          if (!pi.res) frames_->wait_file(key);
          if (const std::string e = frames_->flush_error(key); !e.empty())
            throw std::runtime_error("input partition " + key + " was never committed (write-behind failed: " + e + ")");
          if (!pi.res)
            pi.file = std::make_unique<PartitionIndex>(frame_path(config_.storage_dir, t.session_uuid, in.pointer));
          count += pi.size();
          parts.push_back(std::move(pi));
        }
        if (count == 0) throw std::runtime_error("reduce over no rows");
        // every row's first ciphertext, all at one level (the first row's)
        uint32_t level = 0;
        for (const auto &pv : parts)
          if (pv.size()) {
            if (pv.res) {
              level = pv.res->level;
            } else {
              CtHeader h;
              pv.file->read(0, 0, &h, sizeof(h));
              level = check_ct_header(s, h);
            }
            break;
          }
        const size_t cw = s.ct_words(level);
        const uint32_t op = mul ? FHE_REDUCE_MUL_RELIN : FHE_REDUCE_ADD;
        const uint64_t *rlk = mul ? ks->relin.p : nullptr;
        // Rows are staged max_batch at a time (two pinned slots, reused after
        // their mark), so host and device memory stay bounded by the batch
        // whatever the partitions hold.  Each chunk is reduced by the balanced
        // tree of fhe_reduce_at; the chunk results merge like a binary counter
        // (two partials of the same height combine, older one first), so at
        // most log2(chunks) + 1 partials are alive.  A single chunk is the
        // plain balanced tree.
        const size_t C = std::max<uint32_t>(1, config_.max_batch);
        struct Partial {
          ArenaBuf buf;
          uint32_t height;
        };
        std::vector<Partial> pend;
        const auto combine = [&](const ArenaBuf &older, ArenaBuf &newer) {
          if (mul) ck(s.ctx, fhe_mul_relin_at(s.ctx, older.p, newer.p, rlk, newer.p, 1, level), "reduce merge");
          else ck(s.ctx, fhe_add_at(s.ctx, older.p, newer.p, newer.p, 1, level), "reduce merge");
        };
        ArenaBuf stage[2] = {ArenaBuf(*ls.arena, C * cw), ArenaBuf(*ls.arena, C * cw)};
        bool used[2] = {false, false};
        size_t pi = 0, ri = 0, k = 0;
        while (pi < parts.size() && parts[pi].size() == 0) ++pi;
        while (pi < parts.size()) {
          const int si = (int)(k++ & 1);
          Slot &sl = ls.slot[si];
          if (used[si]) ck(s.ctx, fhe_wait_mark(s.ctx, (uint32_t)si), "reduce slot wait");
          if (sl.in.empty()) sl.in.push_back(std::make_unique<Pinned>());
          uint64_t *host = reinterpret_cast<uint64_t *>(sl.in[0]->reserve(s.ctx, C * cw * 8));
          // the chunk's rows in partition order (the same tree whatever is
          // resident): file rows staged through pinned memory, resident rows
          // copied on the device
          size_t m = 0, h0 = 0;  // h0: first chunk row of the current host run
          const auto flush_host = [&](size_t upto) {
            if (upto > h0)
              ck(s.ctx, fhe_memcpy_h2d_async(s.ctx, stage[si].p + h0 * cw, host + h0 * cw, (upto - h0) * cw * 8), "h2d");
          };
          for (; m < C && pi < parts.size(); ++m) {
            Input &in = parts[pi];
            if (in.res) {
              if (in.res->level != level) throw std::runtime_error("reduce inputs differ in ciphertext level");
              flush_host(m);
              h0 = m + 1;
              ck(s.ctx, fhe_memcpy_d2d_async(s.ctx, stage[si].p + m * cw, in.res->p + ri * in.res->cw, cw * 8), "d2d");
              stats.resident_rows += 1;
            } else {
              CtHeader h;
              in.file->read(ri, 0, &h, sizeof(h));
              if (check_ct_header(s, h) != level) throw std::runtime_error("reduce inputs differ in ciphertext level");
              in.file->read(ri, sizeof(h), host + m * cw, cw * 8);
            }
            if (++ri == in.size()) {
              ri = 0;
              ++pi;
              while (pi < parts.size() && parts[pi].size() == 0) ++pi;
            }
          }
          flush_host(m);
          ck(s.ctx, fhe_mark(s.ctx, (uint32_t)si), "reduce slot mark");
          used[si] = true;
          Partial p{ArenaBuf(*ls.arena, cw), 0};
          ck(s.ctx, fhe_reduce_at(s.ctx, stage[si].p, (uint32_t)m, op, rlk, p.buf.p, level), "reduce");
          while (!pend.empty() && pend.back().height == p.height) {
            combine(pend.back().buf, p.buf);
            p.height += 1;
            pend.pop_back();
          }
          pend.push_back(std::move(p));
        }
        while (pend.size() > 1) {  // fold the leftover partials, newest first
          Partial p = std::move(pend.back());
          pend.pop_back();
          combine(pend.back().buf, p.buf);
          pend.back().buf = std::move(p.buf);
        }
        Slot &sl = ls.slot[0];
        sl.out_level = level;
        uint64_t *res = reinterpret_cast<uint64_t *>(sl.out.reserve(s.ctx, cw * 8));
        ck(s.ctx, fhe_memcpy_d2h_async(s.ctx, res, pend.back().buf.p, cw * 8), "d2h");
        ck(s.ctx, fhe_synchronize(s.ctx), "reduce sync");
        PartitionWriter out(frame_path(config_.storage_dir, t.session_uuid, t.output_data_frame_ptr),
                            config_.durable_outputs);
        const CtHeader h = ct_header(s, level);
        out.append({{&h, sizeof(h)}, {res, cw * 8}});
        out.commit();
      }
    } catch (const std::exception &e) {
      st = Status::ERROR;  // no exception crosses the seam (executor.cpp:168-178 fails the job)
      std::fprintf(stderr, "GpuWorkerGroup: task failed: %s\n", e.what());
      // copies of this task may still be reading or filling the lane's pinned
      // buffers: let them finish before the next task reuses (or regrows) them
      if (cur) (void)fhe_synchronize(cur->s.ctx);
    }
    stats.task_s = secs_since(t_task);
    stats.tasks = 1;
    {
      std::lock_guard lk(stats_m_);
      stats_ += stats;
    }
    complete(job.handle, st);
  }
}

}  // namespace herdsman_gpu
