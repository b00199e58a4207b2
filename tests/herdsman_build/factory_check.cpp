// Drives the herdsman-side factory of integration/herdsman-gpu-workers.patch
// (build_gpu_worker_group, called from main.cpp's build_worker_group) the way
// the Executor drives a worker group: schedule_task, then a late
// set_completion_callback (executor.cpp:86-93), through herdsman's REAL
// IWorkerGroup (include/execution/worker/i_worker_group.hpp + its .cpp).
#include <chrono>
#include <cstdio>
#include <future>
#include <thread>

#include "execution/worker/gpu/gpu_worker_group_factory.hpp"

int main() {
  Config::GpuWorkersConfig gpu;
  gpu.devices = {0};
  gpu.lanes_per_device = 3;
  Config::ServerConfig server;
  server.storage_directory = "/nonexistent/storage";
  server.key_directory = "/nonexistent/keys";
  std::unique_ptr<IWorkerGroup> g = build_gpu_worker_group(gpu, server);
  int ok = 0;
  for (int i = 0; i < 20; ++i) {
    // a malformed task and a MapTask whose partition file does not exist: both
    // must come back as ERROR exactly once, even though they finish before
    // the callback is attached
    herd::common::task_t task;
    if (i % 2) {
      herd::common::MapTask t;
      t.session_uuid = {"s"};
      t.input_data_frame_ptr.pointer = {{"in"}, 0};
      t.output_data_frame_ptr = {{"out"}, 0};
      t.crypto_key_ptr.schema_type = herd::common::SchemaType::CKKS;
      task = t;
    }
    auto h = g->schedule_task(task);
    std::this_thread::sleep_for(std::chrono::microseconds(300 * (i % 3)));
    std::promise<IWorkerGroup::TaskHandle::Status> p;
    auto f = p.get_future();
    h->set_completion_callback([&p](IWorkerGroup::TaskHandle::Status s) { p.set_value(s); });
    if (f.wait_for(std::chrono::seconds(120)) == std::future_status::ready &&
        f.get() == IWorkerGroup::TaskHandle::Status::ERROR && h->completed())
      ++ok;
  }
  std::printf("factory: %d/20 delivered as ERROR, concurrent_workers=%zu\n", ok, g->concurrent_workers());
  return ok == 20 && g->concurrent_workers() == 3 ? 0 : 1;
}
