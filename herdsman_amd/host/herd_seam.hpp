// herd_seam.hpp -- the herdsman worker-group seam, as this backend plugs into it.
//
// In a herdsman build this header is NOT used: the adaptor includes
// herdsman's own "execution/worker/i_worker_group.hpp"
// (/root/reference/include/execution/worker/i_worker_group.hpp:12-49) and
// herd_common's task types.  Those headers live in the `common` submodule,
// which is empty in the reference snapshot, so for building
// and testing outside herdsman this file restates the seam with the same
// names, members and semantics:
//   * TaskHandle::Status {COMPLETED, PENDING, TIME_OUT, ERROR}   (i_worker_group.hpp:18-24)
//   * completed(), virtual status(), set_completion_callback()  (:28-31)
//   * protected virtual mark_completed(): sets completed and calls the
//     callback under the handle's mutex iff one is set           (i_worker_group.cpp:4-13)
//   * schedule_task(const task_t&) -> shared_ptr<TaskHandle>, concurrent_workers()  (:46-48)
// and the task payload fields the executor fills in
// (/root/reference/src/service/execution_service.cpp:436-513).
// The ciphertext `Circuit` of herd_common is unknown (submodule absent); the
// stand-in below is this backend's own op list (documented in INTEGRATION.md).
#pragma once
#ifndef HERDSMAN_REAL_SEAM

#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <variant>
#include <vector>

namespace herd::common {

struct UUID {
  std::string value;
  const std::string &as_string() const { return value; }
};

struct DataFramePtr {
  UUID uuid;
  uint32_t partition = 0;
};

struct InputDataFramePtr {
  DataFramePtr pointer;
  uint64_t row_count = 0;
};

struct CryptoKeyPtr {
  int schema_type = 0;
};

// Stand-in circuit: a stack program over the ciphertexts of one row.
enum class CtOp : uint32_t { PUSH_INPUT = 0, ADD = 1, SUB = 2, MUL_RELIN = 3, ROTATE = 4 };
struct CircuitInstr {
  CtOp op;
  int32_t arg = 0;  // PUSH_INPUT: index of the ciphertext in the row; ROTATE: steps
};
struct Circuit {
  std::vector<CircuitInstr> program;
};

struct MapTask {
  UUID session_uuid;
  InputDataFramePtr input_data_frame_ptr;
  DataFramePtr output_data_frame_ptr;
  CryptoKeyPtr crypto_key_ptr;
  Circuit circuit;
};

struct ReduceTask {
  UUID session_uuid;
  std::vector<InputDataFramePtr> input_data_frame_ptrs;
  DataFramePtr output_data_frame_ptr;
  CryptoKeyPtr crypto_key_ptr;
  Circuit circuit;
};

using task_t = std::variant<std::monostate, MapTask, ReduceTask>;

}  // namespace herd::common

class IWorkerGroup {
 public:
  class TaskHandle {
   public:
    enum class Status { COMPLETED, PENDING, TIME_OUT, ERROR };

    virtual ~TaskHandle() noexcept = default;

    [[nodiscard]] bool completed() const noexcept { return completed_; }
    [[nodiscard]] virtual Status status() const noexcept = 0;

    void set_completion_callback(std::function<void(Status)> callback) noexcept {
      std::unique_lock lock(callback_mutex_);
      callback_ = std::move(callback);
    }

   protected:
    virtual void mark_completed() {
      std::unique_lock lock(callback_mutex_);
      completed_ = true;
      if (callback_) callback_(status());
    }

   private:
    std::function<void(Status)> callback_;
    std::mutex callback_mutex_;
    bool completed_ = false;
  };

  virtual ~IWorkerGroup() = default;
  virtual std::shared_ptr<TaskHandle> schedule_task(const herd::common::task_t &task) = 0;
  virtual std::size_t concurrent_workers() const noexcept = 0;
};

#endif  // HERDSMAN_REAL_SEAM
