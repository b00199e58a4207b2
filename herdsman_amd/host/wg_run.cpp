// wg_run -- drive GpuWorkerGroup exactly the way herdsman's Executor does
// (/root/reference/src/execution/executor/executor.cpp:82-94: schedule_task,
// THEN set_completion_callback) and report the task status.  Used by the
// tests and usable by hand to run one Map/Reduce task over partition files.
//
//   wg_run map    STORAGE KEYS SESSION SCHEMA PARAMS IN_FRAME PART OUT_FRAME PROGRAM...
//   wg_run reduce STORAGE KEYS SESSION SCHEMA PARAMS OUT_FRAME OUT_PART IN_FRAME:PART... [-- mul]
//   wg_run race   N            (seam test: N malformed tasks, callback attached late)
//   wg_run chain  STORAGE KEYS SESSION SCHEMA PARAMS IN_FRAME PARTS MID_FRAME OUT_FRAME PROG1... -- PROG2...
//                 two chained Map stages over PARTS partitions (stage 2 reads stage 1's
//                 output frame, from HBM when it is resident)
//   wg_run bench  DIR PARAMS PARTS ROWS [LANES [MAX_BATCH [REPS]]]
//                 MapTask throughput: writes PARTS partitions of ROWS rows
//                 (two ciphertexts each, uniform residues made on the GPU) and a
//                 relinearisation key under DIR, then keeps concurrent_workers()
//                 MapTasks "in0 in1 mul" in flight, as the Executor does
//                 (executor.cpp:96-113), and reports ct-mult+relin/s end to end
//                 (partition read, PCIe both ways, GPU, partition write): the
//                 mean and spread of REPS (default 5) warm repetitions after one
//                 warm-up, and where the lanes' time went (GpuWorkerGroup::stage_stats).
//   wg_run chainbench DIR PARAMS PARTS ROWS [LANES [MAX_BATCH [REPS]]]
//                 the same inputs; stage 1 "in0 in1 mul" into a fresh frame, then stage 2
//                 "in0 in0 mul" over that frame, each timed (stage 2 with and without
//                 waiting for write-behind files)
// Group knobs from the environment: WG_DEVICE, WG_LANES, WG_MAX_BATCH, WG_IO_THREADS,
// WG_RESIDENT_BYTES (0 = no resident frames), WG_WRITE_BEHIND=1
// PARAMS = scheme,log_n,L,K,dnum,t[,moduli_file[,behz|hps]]   PROGRAM tokens: in<i> add sub mul rot:<k> rescale
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <future>
#include <iostream>
#include <sstream>
#include <string>
#include <thread>

#include "ct_format.hpp"
#include "gpu_worker_group.hpp"

using herdsman_gpu::GpuWorkerGroup;
using herdsman_gpu::GpuWorkerGroupConfig;
using Status = IWorkerGroup::TaskHandle::Status;

static const char *name(Status s) {
  switch (s) {
    case Status::COMPLETED: return "COMPLETED";
    case Status::PENDING: return "PENDING";
    case Status::TIME_OUT: return "TIME_OUT";
    default: return "ERROR";
  }
}

static herdsman_gpu::SchemaParams parse_params(int schema, const std::string &spec) {
  herdsman_gpu::SchemaParams sp;
  sp.schema_type = schema;
  std::stringstream ss(spec);
  std::string tok;
  std::vector<std::string> v;
  while (std::getline(ss, tok, ',')) v.push_back(tok);
  if (v.size() < 6) throw std::runtime_error("PARAMS = scheme,log_n,L,K,dnum,t[,moduli_file[,behz|hps]]");
  sp.params.scheme = std::stoul(v[0]);
  sp.params.log_n = std::stoul(v[1]);
  sp.params.num_q = std::stoul(v[2]);
  sp.params.num_p = std::stoul(v[3]);
  sp.params.dnum = std::stoul(v[4]);
  sp.params.plain_modulus = std::stoull(v[5]);
  sp.params.q_bits = 60;
  sp.params.p_bits = 61;
  if (v.size() > 6 && !v[6].empty()) {
    std::ifstream in(v[6]);
    uint64_t q;
    while (in >> q) sp.moduli.push_back(q);
  }
  if (v.size() > 7) {  // BFV multiplication technique
    if (v[7] == "hps") sp.params.flags |= FHE_FLAG_BFV_HPS;
    else if (v[7] != "behz") throw std::runtime_error("PARAMS mult must be behz or hps");
  }
  return sp;
}

static herd::common::Circuit parse_program(int argc, char **argv, int first) {
  herd::common::Circuit c;
  for (int i = first; i < argc; ++i) {
    const std::string t = argv[i];
    using herd::common::CtOp;
    if (t.rfind("in", 0) == 0) c.program.push_back({CtOp::PUSH_INPUT, std::stoi(t.substr(2))});
    else if (t == "add") c.program.push_back({CtOp::ADD, 0});
    else if (t == "sub") c.program.push_back({CtOp::SUB, 0});
    else if (t == "mul") c.program.push_back({CtOp::MUL_RELIN, 0});
    else if (t.rfind("rot:", 0) == 0) c.program.push_back({CtOp::ROTATE, std::stoi(t.substr(4))});
    else if (t == "rescale") c.program.push_back({CtOp::RESCALE, 0});
    else if (t.rfind("rotsum:", 0) == 0) {  // rotsum:0,1,2,4 -> step mask
      int32_t mask = 0;
      std::string v = t.substr(7);
      for (size_t p0 = 0; p0 < v.size();) {
        size_t p1 = v.find(',', p0);
        if (p1 == std::string::npos) p1 = v.size();
        const int k = std::stoi(v.substr(p0, p1 - p0));
        if (k < 0 || k > 30) throw std::runtime_error("rotsum steps must be in [0, 30]");
        mask |= 1 << k;
        p0 = p1 + 1;
      }
      c.program.push_back({CtOp::ROTSUM, mask});
    }
    else throw std::runtime_error("unknown program token " + t);
  }
  return c;
}

// schedule like the Executor: callback attached after schedule_task returns
static Status run(GpuWorkerGroup &g, const herd::common::task_t &task, int delay_us = 0) {
  auto h = g.schedule_task(task);
  if (delay_us) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
  std::promise<Status> p;
  auto f = p.get_future();
  h->set_completion_callback([&p](Status s) { p.set_value(s); });
  if (f.wait_for(std::chrono::seconds(600)) != std::future_status::ready) return Status::TIME_OUT;
  return f.get();
}

static void ckb(fhe_ctx *c, int rc, const char *what) {
  if (rc != FHE_OK) throw std::runtime_error(std::string(what) + ": " + fhe_last_error(c));
}

// group knobs from the environment (every mode): WG_DEVICE, WG_LANES, WG_MAX_BATCH,
// WG_IO_THREADS, WG_RESIDENT_BYTES (0: no resident frames), WG_WRITE_BEHIND=1
static void env_config(GpuWorkerGroupConfig &cfg) {
  cfg.resident_frame_bytes = 16ull << 30;  // this driver opts in (the library's default is off)
  if (const char *d = std::getenv("WG_DEVICE")) cfg.devices = {std::atoi(d)};
  if (const char *v = std::getenv("WG_LANES")) cfg.lanes_per_device = (uint32_t)std::atoi(v);
  if (const char *v = std::getenv("WG_MAX_BATCH")) cfg.max_batch = (uint32_t)std::atoi(v);
  if (const char *t = std::getenv("WG_IO_THREADS")) cfg.io_threads = (uint32_t)std::max(1, std::atoi(t));
  if (const char *v = std::getenv("WG_RESIDENT_BYTES")) cfg.resident_frame_bytes = std::strtoull(v, nullptr, 10);
  if (const char *v = std::getenv("WG_WRITE_BEHIND")) cfg.write_behind = v[0] == '1';
  if (const char *v = std::getenv("WG_FLUSH_THREADS")) cfg.flush_threads = (uint32_t)std::atoi(v);
}

// Keep concurrent_workers() tasks in flight, as the Executor does
// (executor.cpp:96-113); returns the wall time until the last completion.
// statuses != nullptr: record each task's status instead of throwing on errors
template <class Make>
static double run_all(GpuWorkerGroup &g, int count, Make make, std::vector<Status> *statuses = nullptr) {
  if (statuses) statuses->assign(count, Status::PENDING);
  std::mutex m;
  std::condition_variable cv;
  int done = 0, errors = 0, next = 0, inflight = 0;
  const auto t0 = std::chrono::steady_clock::now();
  std::unique_lock lk(m);
  while (done < count) {
    while (next < count && inflight < (int)g.concurrent_workers()) {
      lk.unlock();
      auto h = g.schedule_task(make(next));
      h->set_completion_callback([&, i = next](Status s) {
        std::lock_guard l2(m);
        if (statuses) (*statuses)[i] = s;
        ++done;
        --inflight;
        if (s != Status::COMPLETED) ++errors;
        cv.notify_one();
      });
      lk.lock();
      ++next;
      ++inflight;
    }
    cv.wait(lk);
  }
  if (errors && !statuses) throw std::runtime_error("tasks failed");
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

static void print_stages(const herdsman_gpu::StageStats &st) {
  const double lane_s = st.read_s + st.enqueue_s + st.wait_s + st.write_s;
  std::printf("stages (summed over lanes, warm reps): %llu tasks, %llu batches, %llu rows (%llu read from HBM-resident "
              "frames); task time %.3f s (%.1f ms per task, of which the stages below %.1f ms)\n",
              (unsigned long long)st.tasks, (unsigned long long)st.batches, (unsigned long long)st.rows,
              (unsigned long long)st.resident_rows, st.task_s, st.tasks ? 1e3 * st.task_s / st.tasks : 0.0,
              st.tasks ? 1e3 * lane_s / st.tasks : 0.0);
  const std::pair<const char *, double> rowsv[] = {{"read rows -> pinned (pread)", st.read_s},
                                                   {"enqueue H2D + kernels + D2H", st.enqueue_s},
                                                   {"wait for the batch's GPU work", st.wait_s},
                                                   {"write output rows", st.write_s}};
  for (const auto &r : rowsv)
    std::printf("  %-32s %8.3f s  %5.1f%%  %8.2f ms/batch\n", r.first, r.second, lane_s > 0 ? 100 * r.second / lane_s : 0.0,
                st.batches ? 1e3 * r.second / st.batches : 0.0);
  if (st.flushed_rows)
    std::printf("  write-behind flusher (off the lanes): %llu rows in %.3f s\n", (unsigned long long)st.flushed_rows,
                st.flush_s);
}

static int bench(int argc, char **argv) {
  const std::string mode = argv[1];
  if (argc < 6)
    throw std::runtime_error("usage: wg_run bench|chainbench DIR PARAMS PARTS ROWS [LANES [MAX_BATCH [REPS]]]");
  const std::filesystem::path dir = argv[2];
  const herdsman_gpu::SchemaParams sp = parse_params(0, argv[3]);
  const int parts = std::atoi(argv[4]), rows = std::atoi(argv[5]);
  GpuWorkerGroupConfig cfg;
  cfg.storage_dir = dir / "storage";
  cfg.key_dir = dir / "keys";
  cfg.schemas = {sp};
  if (argc > 6) cfg.lanes_per_device = (uint32_t)std::atoi(argv[6]);
  if (argc > 7) cfg.max_batch = (uint32_t)std::atoi(argv[7]);
  const int reps = argc > 8 ? std::max(1, std::atoi(argv[8])) : 5;
  env_config(cfg);
  // ---- synthetic inputs, made on the device with the backend's uniform fill
  fhe_params p = sp.params;
  p.moduli = sp.moduli.empty() ? nullptr : sp.moduli.data();
  fhe_ctx *c = nullptr;
  if (fhe_ctx_create(&p, cfg.devices[0], &c) != FHE_OK) throw std::runtime_error(fhe_last_error(nullptr));
  uint32_t nm = 0;
  fhe_ctx_moduli(c, nullptr, 0, &nm);
  std::vector<uint64_t> mods(nm);
  fhe_ctx_moduli(c, mods.data(), nm, nullptr);
  const uint32_t L = p.num_q, K = p.num_p, dnum = p.dnum;
  const size_t n = (size_t)1 << p.log_n, cw = 2 * L * n, kw = (size_t)dnum * 2 * (L + K) * n;
  void *dbuf = nullptr;
  ckb(c, fhe_dev_alloc(c, std::max(2 * cw, kw) * 8, &dbuf), "alloc");
  std::vector<uint64_t> host(std::max(2 * cw, kw));
  ckb(c, fhe_fill_uniform(c, (uint64_t *)dbuf, dnum * 2, 0, L + K, 0x524C4B), "fill key");
  ckb(c, fhe_memcpy_d2h(c, host.data(), dbuf, kw * 8), "d2h");
  {
    std::filesystem::create_directories(cfg.key_dir / "bench");
    std::ofstream kf(cfg.key_dir / "bench" / "0.key", std::ios::binary);
    herdsman_gpu::KeyFileHeader h;
    h.scheme = (uint8_t)p.scheme;
    h.log_n = p.log_n;
    h.L = L;
    h.K = K;
    h.dnum = dnum;
    h.n_keys = 1;
    h.moduli_digest = herdsman_gpu::moduli_digest(mods.data(), L + K);
    herdsman_gpu::KeyEntryHeader e;
    kf.write((const char *)&h, sizeof(h));
    kf.write((const char *)&e, sizeof(e));
    kf.write((const char *)host.data(), kw * 8);
  }
  herdsman_gpu::CtHeader ch;
  ch.scheme = (uint8_t)p.scheme;
  ch.domain = p.scheme == FHE_SCHEME_CKKS ? 1 : 0;
  ch.log_n = p.log_n;
  ch.n_limbs = L;
  ch.moduli_digest = herdsman_gpu::moduli_digest(mods.data(), L);
  for (int part = 0; part < parts; ++part) {
    std::vector<std::vector<uint8_t>> rs;
    for (int r = 0; r < rows; ++r) {
      ckb(c, fhe_fill_uniform(c, (uint64_t *)dbuf, 4, 0, L, 0x48455244ull + (uint64_t)part * rows + r), "fill");
      ckb(c, fhe_memcpy_d2h(c, host.data(), dbuf, 2 * cw * 8), "d2h");
      std::vector<uint8_t> row(2 * (sizeof(ch) + cw * 8));
      for (int k = 0; k < 2; ++k) {
        std::memcpy(row.data() + k * (sizeof(ch) + cw * 8), &ch, sizeof(ch));
        std::memcpy(row.data() + k * (sizeof(ch) + cw * 8) + sizeof(ch), host.data() + k * cw, cw * 8);
      }
      rs.push_back(std::move(row));
    }
    herdsman_gpu::write_partition(cfg.storage_dir / "bench" / "in" / std::to_string(part), rs);
  }
  fhe_dev_free(c, dbuf);
  fhe_ctx_destroy(c);
  // ---- the Executor's pattern: keep concurrent_workers() tasks in flight
  using herd::common::CtOp;
  herd::common::Circuit mul2, sq;
  mul2.program = {{CtOp::PUSH_INPUT, 0}, {CtOp::PUSH_INPUT, 1}, {CtOp::MUL_RELIN, 0}};
  sq.program = {{CtOp::PUSH_INPUT, 0}, {CtOp::PUSH_INPUT, 0}, {CtOp::MUL_RELIN, 0}};
  auto task = [&](const std::string &in, const std::string &out, int part, const herd::common::Circuit &c) {
    herd::common::MapTask t;
    t.session_uuid = {"bench"};
    t.input_data_frame_ptr.pointer = {{in}, (uint32_t)part};
    t.input_data_frame_ptr.row_count = (uint64_t)rows;
    t.output_data_frame_ptr = {{out}, (uint32_t)part};
    t.crypto_key_ptr.schema_type = herd::common::SchemaType::CKKS;
    t.circuit = c;
    return herd::common::task_t{t};
  };
  const bool chain = mode == "chainbench";
  std::vector<double> rates, rates2, rates2f;
  GpuWorkerGroup g(cfg);  // one long-lived group, as in a server
  herdsman_gpu::StageStats st1, st2;
  for (int rep = 0; rep <= reps; ++rep) {  // rep 0 warms contexts, keys, pinned and device buffers
    // each repetition writes fresh output frames, as every herdsman job does
    const std::string mid = "out" + std::to_string(rep), fin = "fin" + std::to_string(rep);
    if (rep > 0) {
      std::filesystem::remove_all(cfg.storage_dir / "bench" / ("out" + std::to_string(rep - 1)));
      std::filesystem::remove_all(cfg.storage_dir / "bench" / ("fin" + std::to_string(rep - 1)));
    }
    g.reset_stage_stats();
    // stage 1: "in0 in1 mul" over the input partitions (files)
    const double dt = run_all(g, parts, [&](int p) { return task("in", mid, p, mul2); });
    const double rate = (double)parts * rows / dt;
    std::printf("%s rep %d: %d MapTasks x %d rows in %.3f s = %.1f ct-mult+relin/s (%zu workers)\n",
                chain ? "stage-1" : "bench", rep, parts, rows, dt, rate, g.concurrent_workers());
    if (rep) rates.push_back(rate);
    if (!chain) {
      if (rep) st1 += g.stage_stats();
      continue;
    }
    if (!g.flush_frames()) throw std::runtime_error("write-behind failed");  // stage 1's files, off the clock
    if (rep) st1 += g.stage_stats();
    g.reset_stage_stats();
    // stage 2: "in0 in0 mul" over stage 1's output frame (intermediate-<job>-<node>
    // in herdsman), read from HBM when resident; then every file committed
    const double dt2 = run_all(g, parts, [&](int p) { return task(mid, fin, p, sq); });
    const auto t1 = std::chrono::steady_clock::now();
    if (!g.flush_frames()) throw std::runtime_error("write-behind failed");
    const double dtf = dt2 + std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    std::printf("stage-2 rep %d: %d MapTasks x %d rows in %.3f s = %.1f ct-mult+relin/s; with every file committed "
                "%.3f s = %.1f/s\n", rep, parts, rows, dt2, parts * rows / dt2, dtf, parts * rows / dtf);
    if (rep) {
      rates2.push_back(parts * rows / dt2);
      rates2f.push_back(parts * rows / dtf);
      st2 += g.stage_stats();
    }
  }
  auto summary = [&](const char *what, const std::vector<double> &v) {
    double mean = 0;
    for (double r : v) mean += r / v.size();
    const auto mm = std::minmax_element(v.begin(), v.end());
    std::printf("%s: %.1f ct-mult+relin/s mean of %zu warm reps (min %.1f, max %.1f); %d partitions x %d rows, "
                "max_batch %u, %zu lanes, %u io threads per lane, resident frames %s, write-behind %s\n",
                what, mean, v.size(), *mm.first, *mm.second, parts, rows, cfg.max_batch, g.concurrent_workers(),
                cfg.io_threads, cfg.resident_frame_bytes ? "on" : "off", cfg.write_behind ? "on" : "off");
  };
  summary(chain ? "stage-1" : "bench", rates);
  if (chain) {
    summary("stage-2 (tasks complete)", rates2);
    summary("stage-2 (files committed)", rates2f);
    std::printf("stage 1:\n");
    print_stages(st1);
    std::printf("stage 2:\n");
    print_stages(st2);
  } else {
    print_stages(st1);
  }
  return 0;
}

int main(int argc, char **argv) {
  try {
    if (argc < 2) throw std::runtime_error("usage: wg_run map|reduce|race ...");
    const std::string mode = argv[1];
    if (mode == "race") {
      const int n = argc > 2 ? std::atoi(argv[2]) : 100;
      GpuWorkerGroupConfig cfg;
      GpuWorkerGroup g(cfg);
      int delivered = 0;
      for (int i = 0; i < n; ++i) {
        // monostate = malformed task: completes (ERROR) immediately, long before the
        // callback is attached; the group must still deliver it exactly once
        if (run(g, herd::common::task_t{}, (i % 4) * 500) == Status::ERROR) ++delivered;
      }
      std::printf("race: %d/%d delivered, concurrent_workers=%zu\n", delivered, n, g.concurrent_workers());
      return delivered == n ? 0 : 1;
    }
    if (mode == "bench" || mode == "chainbench") return bench(argc, argv);
    if (argc < 8) throw std::runtime_error("missing arguments");
    GpuWorkerGroupConfig cfg;
    cfg.storage_dir = argv[2];
    cfg.key_dir = argv[3];
    const std::string session = argv[4];
    const int schema = std::atoi(argv[5]);
    cfg.schemas = {parse_params(schema, argv[6])};
    env_config(cfg);
    GpuWorkerGroup g(cfg);
    Status st;
    if (mode == "chain") {
      // herdsman's chained Map stages: stage 1 over every partition of IN_FRAME
      // into MID_FRAME, then (once all of stage 1 completed, as the
      // ExecutionService schedules the next stage) stage 2 over MID_FRAME into
      // OUT_FRAME, on the same group; then every file committed
      if (argc < 11) throw std::runtime_error("usage: wg_run chain ... IN_FRAME PARTS MID_FRAME OUT_FRAME PROG1 -- PROG2");
      const int parts = std::atoi(argv[8]);
      int sep = 11;
      while (sep < argc && std::string(argv[sep]) != "--") ++sep;
      if (sep >= argc) throw std::runtime_error("chain: PROG1 -- PROG2");
      // PROG2 "reduce [mul]": one ReduceTask over every partition of MID_FRAME into OUT_FRAME:0
      const bool reduce2 = sep + 1 < argc && std::string(argv[sep + 1]) == "reduce";
      const herd::common::Circuit c1 = parse_program(sep, argv, 11);
      const herd::common::Circuit c2 = reduce2 ? herd::common::Circuit{} : parse_program(argc, argv, sep + 1);
      auto make = [&](const char *in, const char *out, const herd::common::Circuit &c) {
        return [&, in, out](int p) {
          herd::common::MapTask t;
          t.session_uuid = {session};
          t.input_data_frame_ptr.pointer = {{in}, (uint32_t)p};
          t.output_data_frame_ptr = {{out}, (uint32_t)p};
          t.crypto_key_ptr.schema_type = static_cast<herd::common::SchemaType>(schema);
          t.circuit = c;
          return herd::common::task_t{t};
        };
      };
      run_all(g, parts, make(argv[7], argv[9], c1));
      if (const char *v = std::getenv("WG_FLUSH_BETWEEN"); v && v[0] == '1') {
        // every stage-1 file committed (or failed) before stage 2 is scheduled;
        // stage 2's statuses are then printed per partition instead of failing
        std::printf("stage1_flush: %s\n", g.flush_frames() ? "COMPLETED" : "ERROR");
        std::vector<Status> st2;
        run_all(g, parts, make(argv[9], argv[10], c2), &st2);
        std::printf("stage2:");
        for (Status x : st2) std::printf(" %s", name(x));
        std::printf("\n");
        const bool flushed = g.flush_frames();
        std::printf("status: %s\n", flushed ? "COMPLETED" : "ERROR");
        return 0;
      }
      if (reduce2) {
        herd::common::ReduceTask t;
        t.session_uuid = {session};
        t.output_data_frame_ptr = {{argv[10]}, 0};
        t.crypto_key_ptr.schema_type = static_cast<herd::common::SchemaType>(schema);
        if (sep + 2 < argc && std::string(argv[sep + 2]) == "mul")
          t.circuit.program.push_back({herd::common::CtOp::MUL_RELIN, 0});
        for (int p = 0; p < parts; ++p) {
          herd::common::InputDataFramePtr in;
          in.pointer = {{argv[9]}, (uint32_t)p};
          t.input_data_frame_ptrs.push_back(in);
        }
        if (run(g, t) != Status::COMPLETED) throw std::runtime_error("reduce stage failed");
      } else {
        run_all(g, parts, make(argv[9], argv[10], c2));
      }
      const bool flushed = g.flush_frames();
      const herdsman_gpu::StageStats ss = g.stage_stats();
      std::printf("chain: rows %llu resident_rows %llu flushed_rows %llu\n", (unsigned long long)ss.rows,
                  (unsigned long long)ss.resident_rows, (unsigned long long)ss.flushed_rows);
      std::printf("status: %s\n", flushed ? "COMPLETED" : "ERROR");
      return flushed ? 0 : 2;
    }
    if (mode == "map") {
      // PART may list several partitions ("1,0"): one MapTask each, in order, on
      // the same group (a failed task must leave its lane usable for the next)
      int rc = 0;
      std::string parts = argv[8];
      for (size_t b = 0; b <= parts.size();) {
        const size_t e = std::min(parts.find(',', b), parts.size());
        const uint32_t part = (uint32_t)std::stoul(parts.substr(b, e - b));
        herd::common::MapTask t;
        t.session_uuid = {session};
        t.input_data_frame_ptr.pointer = {{argv[7]}, part};
        t.output_data_frame_ptr = {{argv[9]}, part};
        t.crypto_key_ptr.schema_type = static_cast<herd::common::SchemaType>(schema);
        t.circuit = parse_program(argc, argv, 10);
        st = run(g, t);
        std::printf("status: %s\n", name(st));
        if (st != Status::COMPLETED) rc = 2;
        b = e + 1;
      }
      return rc;
    } else if (mode == "reduce") {
      herd::common::ReduceTask t;
      t.session_uuid = {session};
      t.output_data_frame_ptr = {{argv[7]}, (uint32_t)std::stoul(argv[8])};
      t.crypto_key_ptr.schema_type = static_cast<herd::common::SchemaType>(schema);
      for (int i = 9; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--") {
          if (i + 1 < argc && std::string(argv[i + 1]) == "mul")
            t.circuit.program.push_back({herd::common::CtOp::MUL_RELIN, 0});
          break;
        }
        const auto c = a.find(':');
        herd::common::InputDataFramePtr in;
        in.pointer = {{a.substr(0, c)}, (uint32_t)std::stoul(a.substr(c + 1))};
        t.input_data_frame_ptrs.push_back(in);
      }
      st = run(g, t);
    } else {
      throw std::runtime_error("unknown mode " + mode);
    }
    std::printf("status: %s\n", name(st));
    return st == Status::COMPLETED ? 0 : 2;
  } catch (const std::exception &e) {
    std::fprintf(stderr, "wg_run: %s\n", e.what());
    return 3;
  }
}
