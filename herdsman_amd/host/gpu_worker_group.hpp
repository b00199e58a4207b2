// gpu_worker_group.hpp -- in-process, MI355X-backed IWorkerGroup for herdsman.
//
// Replaces the remote-worker transports (GrpcWorkerGroup, LambdaWorkerGroup;
// /root/reference/src/execution/worker/grpc/grpc_worker_group.cpp:70-105) with
// a group that evaluates MapTask / ReduceTask circuits on local GPUs through
// the C ABI of include/plugins/fhe_backend.h.  The Executor
// (/root/reference/src/execution/executor/executor.cpp:82-113) and the
// service layer are unchanged: they see the same schedule_task /
// concurrent_workers / TaskHandle contract.
//
// Contract kept:
//   * schedule_task never blocks on GPU work: it enqueues and returns;
//   * every device runs `lanes_per_device` lanes; a lane is a host thread with
//     its own fhe_ctx per schema and its own HIP stream, so the kernels of
//     tasks on different lanes of one device overlap (DESIGN.md §4 "Concurrent
//     contexts"); evaluation keys are loaded once per (session, schema) per
//     device and shared by its lanes;
//   * concurrent_workers() = devices x lanes_per_device: exactly the number of
//     tasks that can be executing at once (the Executor keeps that many in
//     flight, executor.cpp:96-113);
//   * no exception crosses the seam: failures become Status::ERROR;
//   * the handle stays alive in the group until its completion is delivered;
//   * completion is delivered on the group's own completion thread, and is
//     re-tried until the executor's callback is attached: the executor sets
//     the callback only AFTER schedule_task returns (executor.cpp:86-93) and
//     TaskHandle::mark_completed silently drops a completion with no callback
//     (i_worker_group.cpp:9-12).  The handle detects delivery because the base
//     mark_completed evaluates the virtual status() exactly when it invokes
//     the callback.  Handles still undelivered when the group is destroyed are
//     dropped.
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <filesystem>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/plugins/fhe_backend.h"
#include "herd_seam.hpp"

namespace herdsman_gpu {

struct SchemaParams {
  int schema_type = 0;
  fhe_params params{};
  std::vector<uint64_t> moduli;  // optional explicit moduli (copied into params.moduli)
};

// BASELINE.json parameter sets keyed by herdsman schema_type (herd_common's
// SchemaType values are not in the snapshot; 0 = CKKS, 1 = BFV here).
inline std::vector<SchemaParams> default_schemas() {
  SchemaParams ckks, bfv;
  ckks.schema_type = 0;
  ckks.params = fhe_params{FHE_SCHEME_CKKS, 16, 12, 4, 3, 60, 61, 0, 0, nullptr};
  bfv.schema_type = 1;
  bfv.params = fhe_params{FHE_SCHEME_BFV, 15, 8, 4, 2, 60, 61, 0, 65537, nullptr};
  return {ckks, bfv};
}

// Where a lane's time goes over MapTasks (wg_run bench prints it): reading
// rows into pinned memory, enqueueing copies and kernels, waiting for a batch's
// GPU work (copies both ways + kernels, after the overlap with the host work),
// writing output rows.
struct StageStats {
  double read_s = 0, enqueue_s = 0, wait_s = 0, write_s = 0;
  double task_s = 0;  // whole tasks on the lanes, open to commit
  uint64_t batches = 0, rows = 0, tasks = 0;
  uint64_t resident_rows = 0;   // input rows read from a frame kept in HBM (no pread, no H2D)
  uint64_t flushed_rows = 0;    // rows the write-behind flusher wrote to partition files
  double flush_s = 0;           // the flusher's time (D2H + file writes), off the lanes
  StageStats &operator+=(const StageStats &o) {
    task_s += o.task_s;
    tasks += o.tasks;
    read_s += o.read_s;
    enqueue_s += o.enqueue_s;
    wait_s += o.wait_s;
    write_s += o.write_s;
    batches += o.batches;
    rows += o.rows;
    resident_rows += o.resident_rows;
    flushed_rows += o.flushed_rows;
    flush_s += o.flush_s;
    return *this;
  }
};

struct GpuWorkerGroupConfig {
  std::vector<int> devices{0};
  std::filesystem::path storage_dir;  // <storage>/<session>/<frame>/<partition>
  std::filesystem::path key_dir;      // <key_dir>/<session>/<schema>.key
  std::vector<SchemaParams> schemas = default_schemas();
  uint32_t lanes_per_device = 4;      // concurrent tasks per device (context + stream each)
  uint32_t max_batch = 64;            // rows per batched GPU call
  bool durable_outputs = false;       // fsync output partitions (PartitionWriter)
  uint32_t io_threads = 4;            // threads per lane reading / writing a batch's rows
  // Resident frames: every MapTask output partition (one ciphertext per row, one
  // level) also stays in HBM, per device, least recently used first out, at most
  // this many bytes per device (0: off).  A MapTask or ReduceTask on the same
  // device whose input partition is resident reads it from HBM: no pread, no H2D.
  // herdsman chains Map stages through intermediate-<job>-<node> frames that the
  // next stage reads back (execution_service.cpp:525-543), which is the case this
  // serves.  The partition file is still written (the storage contract holds).
  // Off by default: the budget is the deployer's share of HBM beside the
  // contexts, keys and workspaces (one budget per group per device).  A failed
  // device allocation evicts the frames first; a frame whose committed file
  // changed on disk (size or mtime) is dropped at lookup, not served.
  uint64_t resident_frame_bytes = 0;
  // write_behind: a MapTask whose output is resident completes once that output
  // is in HBM, and the group's flusher thread writes the partition file behind
  // it (D2H + file writes off the lanes).  flush_frames() returns once every
  // file is committed; a task that must read a file still being flushed waits
  // for it.  Off by default: then a task completes after its file is committed.
  bool write_behind = false;
  uint32_t flush_threads = 4;  // write-behind flusher threads (frames written in parallel)
};

class GpuWorkerGroup : public IWorkerGroup {
 public:
  explicit GpuWorkerGroup(GpuWorkerGroupConfig config);
  ~GpuWorkerGroup() override;

  std::shared_ptr<TaskHandle> schedule_task(const herd::common::task_t &task) override;
  std::size_t concurrent_workers() const noexcept override;
  // summed over the lanes since construction / the last reset (not part of the seam)
  StageStats stage_stats();
  void reset_stage_stats();
  // write_behind: block until every partition file queued so far is committed;
  // false if a flush failed (its message on stderr).  No-op otherwise.
  // A failed flush also fails every later task that reads that partition, and
  // the session's next scheduled task, with Status::ERROR (the executor then
  // fails the job, executor.cpp:168-178).
  bool flush_frames();
  // herdsman deleted a data frame (frame != nullptr) or a whole session: its
  // resident frames go now, not when another frame needs the budget
  void drop_frames(const herd::common::UUID &session, const herd::common::UUID *frame = nullptr);
  // false when herd_common's Circuit has no lowering to the backend's ops
  // (under HERDSMAN_REAL_SEAM): the group then fails every task at once
  static bool circuits_lowerable() noexcept;

  class Handle;

 private:
  struct Job;
  struct Device;
  struct Lane;
  struct Frames;

  void lane_loop(Device &dev, Lane &lane);
  void completion_loop();
  void flush_loop(uint32_t id);
  void complete(const std::shared_ptr<Handle> &h, TaskHandle::Status st);

  GpuWorkerGroupConfig config_;
  std::vector<std::unique_ptr<Device>> devices_;
  std::atomic<size_t> next_device_{0};

  std::mutex done_mutex_;
  std::condition_variable done_cv_;
  std::deque<std::shared_ptr<Handle>> done_;
  bool stopping_ = false;
  std::thread completion_thread_;
  std::mutex stats_m_;
  StageStats stats_;
  std::unique_ptr<Frames> frames_;  // resident frames and the write-behind flusher
  std::vector<std::thread> flush_threads_;
};

class GpuWorkerGroup::Handle : public IWorkerGroup::TaskHandle {
 public:
  Status status() const noexcept override {
    if (probing_.load()) probed_.store(true);
    return status_.load();
  }
  // completion thread only: true once the executor's callback has run
  bool try_deliver() {
    probed_.store(false);
    probing_.store(true);
    mark_completed();
    probing_.store(false);
    return probed_.load();
  }
  std::atomic<Status> status_{Status::PENDING};

 private:
  mutable std::atomic<bool> probing_{false};
  mutable std::atomic<bool> probed_{false};
};

}  // namespace herdsman_gpu
