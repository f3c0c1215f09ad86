// Native work queue (reference: src/work/source/{PDBWorkerQueue,PDBWorker,PDBBuzzer}.cc): a fixed pool
// of threads that the storage layer hands page I/O to, so reading evicted pages back from the page
// files and flushing dirty pages overlap the Python thread (which is feeding the GPU).
#include <chrono>
#include <stdexcept>

#include "runtime.h"

namespace nsdb_rt {

void Buzzer::buzz(const std::string& error) {
  {
    std::lock_guard<std::mutex> g(mu_);
    done_ = true;
    error_ = error;
  }
  cv_.notify_all();
}

bool Buzzer::wait(double timeout_s) {
  std::unique_lock<std::mutex> g(mu_);
  if (timeout_s < 0) {
    cv_.wait(g, [&] { return done_; });
    return true;
  }
  // system_clock deadline: libstdc++ maps it to pthread_cond_timedwait, which ThreadSanitizer intercepts
  // (steady_clock waits use pthread_cond_clockwait, invisible to TSan -> false "double lock" reports)
  const auto deadline = std::chrono::system_clock::now() +
                        std::chrono::duration_cast<std::chrono::system_clock::duration>(std::chrono::duration<double>(timeout_s));
  return cv_.wait_until(g, deadline, [&] { return done_; });
}

bool Buzzer::done() const {
  std::lock_guard<std::mutex> g(mu_);
  return done_;
}

std::string Buzzer::error() const {
  std::lock_guard<std::mutex> g(mu_);
  return error_;
}

WorkerQueue::WorkerQueue(int num_workers) {
  if (num_workers <= 0) throw std::runtime_error("WorkerQueue: num_workers must be > 0");
  for (int i = 0; i < num_workers; ++i) threads_.emplace_back([this] { loop(); });
}

WorkerQueue::~WorkerQueue() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

std::shared_ptr<Buzzer> WorkerQueue::submit(std::function<void()> work) {
  auto b = std::make_shared<Buzzer>();
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) throw std::runtime_error("WorkerQueue: stopped");
    q_.push_back(Item{std::move(work), b});
  }
  cv_.notify_one();
  return b;
}

void WorkerQueue::loop() {
  for (;;) {
    Item it;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;             // stop_ and nothing left
      it = std::move(q_.front());
      q_.pop_front();
      ++active_;
    }
    std::string err;
    try {
      it.fn();
    } catch (const std::exception& e) {
      err = e.what();
      if (err.empty()) err = "work item failed";
    } catch (...) {
      err = "work item failed";
    }
    it.buzzer->buzz(err);
    completed_.fetch_add(1);
    {
      std::lock_guard<std::mutex> g(mu_);
      --active_;
    }
    idle_cv_.notify_all();
  }
}

void WorkerQueue::drain() {
  std::unique_lock<std::mutex> g(mu_);
  idle_cv_.wait(g, [&] { return q_.empty() && active_ == 0; });
}

int64_t WorkerQueue::pending() const {
  std::lock_guard<std::mutex> g(mu_);
  return (int64_t)q_.size() + active_;
}

}  // namespace nsdb_rt
