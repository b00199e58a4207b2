// wg_run -- drive GpuWorkerGroup exactly the way herdsman's Executor does
// (/root/reference/src/execution/executor/executor.cpp:82-94: schedule_task,
// THEN set_completion_callback) and report the task status.  Used by the
// tests and usable by hand to run one Map/Reduce task over partition files.
//
//   wg_run map    STORAGE KEYS SESSION SCHEMA PARAMS IN_FRAME PART OUT_FRAME PROGRAM...
//   wg_run reduce STORAGE KEYS SESSION SCHEMA PARAMS OUT_FRAME OUT_PART IN_FRAME:PART... [-- mul]
//   wg_run race   N            (seam test: N malformed tasks, callback attached late)
// PARAMS = scheme,log_n,L,K,dnum,t[,moduli_file]   PROGRAM tokens: in<i> add sub mul rot:<k>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <future>
#include <iostream>
#include <sstream>
#include <string>
#include <thread>

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
  if (v.size() < 6) throw std::runtime_error("PARAMS = scheme,log_n,L,K,dnum,t[,moduli_file]");
  sp.params.scheme = std::stoul(v[0]);
  sp.params.log_n = std::stoul(v[1]);
  sp.params.num_q = std::stoul(v[2]);
  sp.params.num_p = std::stoul(v[3]);
  sp.params.dnum = std::stoul(v[4]);
  sp.params.plain_modulus = std::stoull(v[5]);
  sp.params.q_bits = 60;
  sp.params.p_bits = 61;
  if (v.size() > 6) {
    std::ifstream in(v[6]);
    uint64_t q;
    while (in >> q) sp.moduli.push_back(q);
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
    if (argc < 8) throw std::runtime_error("missing arguments");
    GpuWorkerGroupConfig cfg;
    cfg.storage_dir = argv[2];
    cfg.key_dir = argv[3];
    const std::string session = argv[4];
    const int schema = std::atoi(argv[5]);
    cfg.schemas.push_back(parse_params(schema, argv[6]));
    if (const char *d = std::getenv("WG_DEVICE")) cfg.devices = {std::atoi(d)};
    GpuWorkerGroup g(cfg);
    Status st;
    if (mode == "map") {
      herd::common::MapTask t;
      t.session_uuid = {session};
      t.input_data_frame_ptr.pointer = {{argv[7]}, (uint32_t)std::stoul(argv[8])};
      t.output_data_frame_ptr = {{argv[9]}, (uint32_t)std::stoul(argv[8])};
      t.crypto_key_ptr.schema_type = schema;
      t.circuit = parse_program(argc, argv, 10);
      st = run(g, t);
    } else if (mode == "reduce") {
      herd::common::ReduceTask t;
      t.session_uuid = {session};
      t.output_data_frame_ptr = {{argv[7]}, (uint32_t)std::stoul(argv[8])};
      t.crypto_key_ptr.schema_type = schema;
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
