// herd_seam.hpp -- the herdsman worker-group seam, as this backend plugs into it.
//
// With HERDSMAN_REAL_SEAM (a herdsman build) this header
// includes herdsman's own seam, "execution/worker/i_worker_group.hpp"
// (/root/reference/include/execution/worker/i_worker_group.hpp:12-49), which
// brings herd_common's task types with it; the adaptor is then compiled and
// linked against herdsman's IWorkerGroup and its i_worker_group.cpp
// (tests/test_herdsman_seam.py does exactly that against /root/reference).
//
// Without it (stand-alone builds and tests of this repo) the seam is restated
// here with the same names, members and semantics, over the herd_common
// stand-in types of herd_common_standin.hpp:
//   * TaskHandle::Status {COMPLETED, PENDING, TIME_OUT, ERROR}   (i_worker_group.hpp:18-24)
//   * completed(), virtual status(), set_completion_callback()  (:28-31)
//   * protected virtual mark_completed(): sets completed and calls the
//     callback under the handle's mutex iff one is set           (i_worker_group.cpp:4-13)
//   * schedule_task(const task_t&) -> shared_ptr<TaskHandle>, concurrent_workers()  (:46-48)
#pragma once
#ifdef HERDSMAN_REAL_SEAM

#include "execution/worker/i_worker_group.hpp"

#else

#include <functional>
#include <memory>
#include <mutex>

#include "herd_common_standin.hpp"

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
