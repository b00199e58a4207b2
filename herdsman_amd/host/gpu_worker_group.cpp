// gpu_worker_group.cpp -- see gpu_worker_group.hpp.
#include "gpu_worker_group.hpp"

#include <chrono>
#include <cstring>
#include <fstream>
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

// ------------------------------------------------------------- device state
namespace {

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
  size_t ct_words() const { return (size_t)2 * L << log_n; }
  size_t key_words() const { return (size_t)dnum * 2 * (L + K) << log_n; }
};

struct KeySet {
  DevBuf relin;
  std::map<uint32_t, DevBuf> galois;
};

}  // namespace

struct GpuWorkerGroup::Device {
  int id = 0;
  std::thread thread;
  std::mutex m;
  std::condition_variable cv;
  std::deque<Job> queue;
  std::map<int, SchemaCtx> ctx;                                 // schema -> context
  std::map<std::pair<std::string, int>, std::shared_ptr<KeySet>> keys;  // (session, schema)
};

GpuWorkerGroup::GpuWorkerGroup(GpuWorkerGroupConfig config) : config_(std::move(config)) {
  if (config_.devices.empty()) throw std::invalid_argument("GpuWorkerGroup needs at least one device");
  for (int d : config_.devices) {
    auto dev = std::make_unique<Device>();
    dev->id = d;
    devices_.push_back(std::move(dev));
  }
  for (auto &d : devices_) d->thread = std::thread([this, p = d.get()] { device_loop(*p); });
  completion_thread_ = std::thread([this] { completion_loop(); });
}

GpuWorkerGroup::~GpuWorkerGroup() {
  for (auto &d : devices_) {
    {
      std::lock_guard lk(d->m);
      d->queue.push_back(Job{nullptr, {}});  // stop marker
    }
    d->cv.notify_one();
  }
  for (auto &d : devices_) d->thread.join();
  {
    std::lock_guard lk(done_mutex_);
    stopping_ = true;
  }
  done_cv_.notify_one();
  completion_thread_.join();
}

std::size_t GpuWorkerGroup::concurrent_workers() const noexcept {
  return devices_.size() * config_.tasks_per_device;
}

std::shared_ptr<IWorkerGroup::TaskHandle> GpuWorkerGroup::schedule_task(const herd::common::task_t &task) {
  auto h = std::make_shared<Handle>();
  if (std::holds_alternative<std::monostate>(task)) {
    complete(h, Status::ERROR);  // delivered once the executor attaches its callback
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
  std::unique_lock lk(done_mutex_);
  while (true) {
    done_cv_.wait_for(lk, std::chrono::microseconds(waiting.empty() ? 100000 : 50),
                      [&] { return stopping_ || !done_.empty(); });
    while (!done_.empty()) {
      waiting.push_back(std::move(done_.front()));
      done_.pop_front();
    }
    const bool stop = stopping_;
    lk.unlock();
    for (size_t i = 0; i < waiting.size();) {
      if (waiting[i]->try_deliver()) {
        waiting[i] = std::move(waiting.back());
        waiting.pop_back();
      } else {
        ++i;
      }
    }
    lk.lock();
    if (stop && done_.empty()) return;
  }
}

// ------------------------------------------------------------- evaluation
namespace {

SchemaCtx &schema_ctx(std::map<int, SchemaCtx> &m, const GpuWorkerGroupConfig &cfg, int device, int schema) {
  auto it = m.find(schema);
  if (it != m.end()) return it->second;
  const SchemaParams *sp = nullptr;
  for (const auto &s : cfg.schemas)
    if (s.schema_type == schema) sp = &s;
  if (!sp) throw std::runtime_error("no backend parameters for schema " + std::to_string(schema));
  fhe_params p = sp->params;
  p.moduli = sp->moduli.empty() ? nullptr : sp->moduli.data();
  SchemaCtx s;
  if (fhe_ctx_create(&p, device, &s.ctx) != FHE_OK)
    throw std::runtime_error(std::string("fhe_ctx_create: ") + fhe_last_error(nullptr));
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
  return m.emplace(schema, s).first->second;
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
  ck(s.ctx, fhe_synchronize(s.ctx), "key upload sync");
  return ks;
}

// parse ciphertext k of a row
const uint64_t *row_ct(const SchemaCtx &s, const std::vector<uint8_t> &row, uint32_t k) {
  const size_t one = sizeof(CtHeader) + s.ct_words() * 8;
  if (row.size() < (k + 1) * one) throw std::runtime_error("row holds fewer ciphertexts than the circuit reads");
  CtHeader h;
  std::memcpy(&h, row.data() + k * one, sizeof(h));
  if (h.magic != kCtMagic || h.version != 1 || h.scheme != s.scheme || h.log_n != s.log_n || h.n_limbs != s.L ||
      h.moduli_digest != s.q_digest)
    throw std::runtime_error("ciphertext header does not match the schema context");
  return reinterpret_cast<const uint64_t *>(row.data() + k * one + sizeof(CtHeader));
}

std::vector<uint8_t> make_row(const SchemaCtx &s, const uint64_t *words) {
  CtHeader h;
  h.scheme = (uint8_t)s.scheme;
  h.domain = s.scheme == FHE_SCHEME_CKKS ? 1 : 0;
  h.log_n = s.log_n;
  h.n_limbs = s.L;
  h.moduli_digest = s.q_digest;
  std::vector<uint8_t> row(sizeof(h) + s.ct_words() * 8);
  std::memcpy(row.data(), &h, sizeof(h));
  std::memcpy(row.data() + sizeof(h), words, s.ct_words() * 8);
  return row;
}

const DevBuf &galois_key(const SchemaCtx &s, const KeySet &ks, int32_t steps, uint32_t *g) {
  ck(s.ctx, fhe_galois_elt(s.ctx, steps, g), "galois_elt");
  auto it = ks.galois.find(*g);
  if (it == ks.galois.end()) throw std::runtime_error("no Galois key for element " + std::to_string(*g));
  return it->second;
}

// evaluate the circuit program on `n` rows at once; rows[r] ciphertexts are the inputs
void eval_map_batch(const SchemaCtx &s, const KeySet &ks, const herd::common::Circuit &circ,
                    const std::vector<std::vector<uint8_t>> &rows, size_t r0, size_t n,
                    std::vector<std::vector<uint8_t>> &out_rows) {
  const size_t cw = s.ct_words();
  std::vector<DevBuf> stack;
  std::vector<uint64_t> host(cw * n);
  for (const auto &ins : circ.program) {
    switch (ins.op) {
      case herd::common::CtOp::PUSH_INPUT: {
        for (size_t r = 0; r < n; ++r) std::memcpy(host.data() + r * cw, row_ct(s, rows[r0 + r], ins.arg), cw * 8);
        DevBuf d(s.ctx, cw * n);
        ck(s.ctx, fhe_memcpy_h2d(s.ctx, d.p, host.data(), cw * n * 8), "h2d");
        stack.push_back(std::move(d));
        break;
      }
      case herd::common::CtOp::ADD:
      case herd::common::CtOp::SUB:
      case herd::common::CtOp::MUL_RELIN: {
        if (stack.size() < 2) throw std::runtime_error("circuit stack underflow");
        DevBuf b = std::move(stack.back());
        stack.pop_back();
        DevBuf a = std::move(stack.back());
        stack.pop_back();
        DevBuf o(s.ctx, cw * n);
        if (ins.op == herd::common::CtOp::ADD) ck(s.ctx, fhe_add(s.ctx, a.p, b.p, o.p, (uint32_t)n), "add");
        else if (ins.op == herd::common::CtOp::SUB) ck(s.ctx, fhe_sub(s.ctx, a.p, b.p, o.p, (uint32_t)n), "sub");
        else {
          if (!ks.relin.p) throw std::runtime_error("no relinearisation key");
          ck(s.ctx, fhe_mul_relin(s.ctx, a.p, b.p, ks.relin.p, o.p, (uint32_t)n), "mul_relin");
        }
        stack.push_back(std::move(o));
        break;
      }
      case herd::common::CtOp::ROTATE: {
        if (stack.empty()) throw std::runtime_error("circuit stack underflow");
        uint32_t g = 0;
        const DevBuf &gk = galois_key(s, ks, ins.arg, &g);
        DevBuf o(s.ctx, cw * n);
        ck(s.ctx, fhe_rotate(s.ctx, stack.back().p, g, gk.p, o.p, (uint32_t)n), "rotate");
        stack.back() = std::move(o);
        break;
      }
      default:
        throw std::runtime_error("unknown circuit op");
    }
  }
  if (stack.size() != 1) throw std::runtime_error("circuit must leave exactly one ciphertext");
  ck(s.ctx, fhe_memcpy_d2h(s.ctx, host.data(), stack.back().p, cw * n * 8), "d2h");
  for (size_t r = 0; r < n; ++r) out_rows.push_back(make_row(s, host.data() + r * cw));
}

std::filesystem::path frame_path(const std::filesystem::path &root, const herd::common::UUID &session,
                                 const herd::common::DataFramePtr &p) {
  return root / session.as_string() / p.uuid.as_string() / std::to_string(p.partition);
}

}  // namespace

void GpuWorkerGroup::device_loop(Device &dev) {
  while (true) {
    Job job;
    {
      std::unique_lock lk(dev.m);
      dev.cv.wait(lk, [&] { return !dev.queue.empty(); });
      job = std::move(dev.queue.front());
      dev.queue.pop_front();
    }
    if (!job.handle) break;
    Status st = Status::COMPLETED;
    try {
      if (std::holds_alternative<herd::common::MapTask>(job.task)) {
        const auto &t = std::get<herd::common::MapTask>(job.task);
        SchemaCtx &s = schema_ctx(dev.ctx, config_, dev.id, t.crypto_key_ptr.schema_type);
        auto key_id = std::make_pair(t.session_uuid.as_string(), t.crypto_key_ptr.schema_type);
        auto &ks = dev.keys[key_id];
        if (!ks)
          ks = load_keys(s, config_.key_dir / t.session_uuid.as_string() /
                                (std::to_string(t.crypto_key_ptr.schema_type) + ".key"));
        const auto rows = read_partition(frame_path(config_.storage_dir, t.session_uuid, t.input_data_frame_ptr.pointer));
        std::vector<std::vector<uint8_t>> out;
        out.reserve(rows.size());
        for (size_t r0 = 0; r0 < rows.size(); r0 += config_.max_batch) {
          const size_t n = std::min<size_t>(config_.max_batch, rows.size() - r0);
          eval_map_batch(s, *ks, t.circuit, rows, r0, n, out);
        }
        write_partition(frame_path(config_.storage_dir, t.session_uuid, t.output_data_frame_ptr), out);
      } else {
        // ReduceTask: combine every row of every input partition into one
        // ciphertext with a balanced tree of batched ADDs (MUL_RELIN if the
        // circuit's first op says so), on the GPU.
        const auto &t = std::get<herd::common::ReduceTask>(job.task);
        SchemaCtx &s = schema_ctx(dev.ctx, config_, dev.id, t.crypto_key_ptr.schema_type);
        const bool mul = !t.circuit.program.empty() && t.circuit.program.front().op == herd::common::CtOp::MUL_RELIN;
        std::shared_ptr<KeySet> ks;
        if (mul) {
          auto &k = dev.keys[std::make_pair(t.session_uuid.as_string(), t.crypto_key_ptr.schema_type)];
          if (!k)
            k = load_keys(s, config_.key_dir / t.session_uuid.as_string() /
                                 (std::to_string(t.crypto_key_ptr.schema_type) + ".key"));
          ks = k;
        }
        std::vector<uint64_t> host;
        size_t count = 0;
        const size_t cw = s.ct_words();
        for (const auto &in : t.input_data_frame_ptrs) {
          for (const auto &row : read_partition(frame_path(config_.storage_dir, t.session_uuid, in.pointer))) {
            host.resize((count + 1) * cw);
            std::memcpy(host.data() + count * cw, row_ct(s, row, 0), cw * 8);
            ++count;
          }
        }
        if (count == 0) throw std::runtime_error("reduce over no rows");
        DevBuf a(s.ctx, count * cw);
        ck(s.ctx, fhe_memcpy_h2d(s.ctx, a.p, host.data(), count * cw * 8), "h2d");
        // balanced tree, one batched add / mul+relin per level (fhe_reduce)
        ck(s.ctx, fhe_reduce(s.ctx, a.p, (uint32_t)count, mul ? FHE_REDUCE_MUL_RELIN : FHE_REDUCE_ADD,
                             mul ? ks->relin.p : nullptr, a.p), "reduce");
        std::vector<uint64_t> res(cw);
        ck(s.ctx, fhe_memcpy_d2h(s.ctx, res.data(), a.p, cw * 8), "d2h");
        write_partition(frame_path(config_.storage_dir, t.session_uuid, t.output_data_frame_ptr), {make_row(s, res.data())});
      }
    } catch (const std::exception &) {
      st = Status::ERROR;  // no exception crosses the seam (executor.cpp:168-178 fails the job)
    }
    complete(job.handle, st);
  }
  dev.keys.clear();  // key buffers are freed through their context: before it goes
  for (auto &kv : dev.ctx) fhe_ctx_destroy(kv.second.ctx);
}

}  // namespace herdsman_gpu
