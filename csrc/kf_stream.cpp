// kf_stream.cpp — HostRing: a ring of pinned (hipHostMalloc) slots filled by
// background reader threads (pread) and shipped with hipMemcpyAsync on a
// side stream, with one hipEvent per slot so the compute stream waits only
// for the slot it consumes.  Replaces the per-band GDAL reads of the
// reference (Sentinel2_Observations.py:148-185) with double-buffered,
// overlapped ingest.  Without a GPU (CI container) the slots fall back to
// pageable memory and h2d degenerates to memcpy.
#include "kf_stream.h"
#include "kf_tiff.h"

#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <pybind11/stl.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

class HostRing {
 public:
  HostRing(int n_slots, size_t slot_bytes, int n_threads) : slot_bytes_(slot_bytes) {
    if (n_slots <= 0 || slot_bytes == 0) throw std::runtime_error("HostRing: bad geometry");
    int ndev = 0;
    device_ = hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0;
    slots_.resize(n_slots, nullptr);
    events_.resize(n_slots, nullptr);
    pending_ = std::vector<std::atomic<int>>(n_slots);
    errors_.resize(n_slots);
    for (int i = 0; i < n_slots; ++i) {
      pending_[i] = 0;
      void* p = nullptr;
      if (device_ && hipHostMalloc(&p, slot_bytes, hipHostMallocDefault) == hipSuccess) {
        pinned_ = true;
      } else {
        p = aligned_alloc(4096, (slot_bytes + 4095) / 4096 * 4096);
        if (!p) throw std::runtime_error("HostRing: out of host memory");
      }
      slots_[i] = static_cast<char*>(p);
      if (device_) {
        if (hipEventCreateWithFlags(&events_[i], hipEventDisableTiming) != hipSuccess)
          throw std::runtime_error("HostRing: hipEventCreate failed");
      }
    }
    for (int t = 0; t < std::max(1, n_threads); ++t) workers_.emplace_back([this] { work(); });
    if (device_) {
      done_seq_.assign(n_slots, 0);
      want_seq_.assign(n_slots, 0);
      submitter_ = std::thread([this] { submit_loop(); });
    }
  }

  ~HostRing() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
    if (submitter_.joinable()) {
      {
        std::lock_guard<std::mutex> g(sub_mu_);
        sub_stop_ = true;
      }
      sub_cv_.notify_all();
      submitter_.join();
    }
    for (hipEvent_t e : dep_pool_) (void)hipEventDestroy(e);
    for (size_t i = 0; i < slots_.size(); ++i) {
      if (device_ && events_[i]) {
        (void)hipEventSynchronize(events_[i]);
        (void)hipEventDestroy(events_[i]);
      }
      if (pinned_) (void)hipHostFree(slots_[i]);
      else free(slots_[i]);
    }
  }

  uintptr_t slot(int i) const { return (uintptr_t)slots_.at(i); }
  size_t slot_bytes() const { return slot_bytes_; }
  int n_slots() const { return (int)slots_.size(); }
  bool pinned() const { return pinned_; }

  void read_file_async(int s, const std::string& path, size_t file_off, size_t nbytes, size_t slot_off) {
    check_range(s, slot_off, nbytes);
    pending_[s]++;
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back([=] {
        std::string err;
        int fd = open(path.c_str(), O_RDONLY);
        if (fd < 0) {
          err = "open failed: " + path;
        } else {
          size_t done = 0;
          while (done < nbytes) {
            ssize_t r = pread(fd, slots_[s] + slot_off + done, nbytes - done, (off_t)(file_off + done));
            if (r <= 0) { err = "short read: " + path; break; }
            done += (size_t)r;
          }
          close(fd);
        }
        if (!err.empty()) {
          std::lock_guard<std::mutex> g2(err_mu_);
          errors_[s] = err;
        }
        pending_[s]--;
      });
    }
    cv_.notify_one();
  }

  // Decode a window of one GeoTIFF band (kf_tiff.cpp, its own thread pool)
  // into slot s at slot_off, in the background.
  void read_tiff_async(int s, const std::string& path, int band, uint64_t r0, uint64_t r1, uint64_t c0, uint64_t c1,
                       size_t elem_bytes, size_t slot_off, int nthreads) {
    check_range(s, slot_off, (size_t)((r1 - r0) * (c1 - c0)) * elem_bytes);
    pending_[s]++;
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back([=] {
        try {
          kf::tiff::read_window(path, band, slots_[s] + slot_off, r0, r1, c0, c1, nthreads, (int)elem_bytes);
        } catch (const std::exception& e) {
          std::lock_guard<std::mutex> g2(err_mu_);
          errors_[s] = std::string(e.what()) + ": " + path;
        }
        pending_[s]--;
      });
    }
    cv_.notify_one();
  }

  void wait_reads(int s) {
    while (pending_.at(s).load() > 0) std::this_thread::yield();
    std::lock_guard<std::mutex> g(err_mu_);
    if (!errors_[s].empty()) {
      std::string e = errors_[s];
      errors_[s].clear();
      throw std::runtime_error("HostRing: " + e);
    }
  }

  void h2d(int s, uintptr_t dst, size_t nbytes, size_t slot_off, uintptr_t stream) {
    check_range(s, slot_off, nbytes);
    wait_reads(s);
    if (!device_) {
      memcpy(reinterpret_cast<void*>(dst), slots_[s] + slot_off, nbytes);
      return;
    }
    // an h2d_async of this slot still queued on the submitter would record the
    // slot event after this copy's, so stream_wait / host_wait would track the
    // older copy: let it be issued first (slot events in submission order)
    wait_submitted(s);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (hipMemcpyAsync(reinterpret_cast<void*>(dst), slots_[s] + slot_off, nbytes, hipMemcpyHostToDevice, st) !=
        hipSuccess)
      throw std::runtime_error("HostRing: hipMemcpyAsync failed");
    if (hipEventRecord(events_[s], st) != hipSuccess) throw std::runtime_error("HostRing: hipEventRecord failed");
  }

  // h2d from a dedicated submitter thread: the copy follows everything queued
  // on after_stream so far (an event recorded here, on the calling thread)
  // and is issued on copy_stream by the submitter.  hipMemcpyAsync can block
  // its calling thread for milliseconds (a one-off runtime stall of ~6 ms on
  // MI355X, scripts/probes/copy_stall_probe.py); issued here it blocks the
  // submitter, not the thread that launches the next kernel.  stream_wait /
  // host_wait of the slot first wait (on the host) until the copy is issued.
  void h2d_async(int s, uintptr_t dst, size_t nbytes, size_t slot_off, uintptr_t copy_stream,
                 uintptr_t after_stream) {
    if (!device_) {
      h2d(s, dst, nbytes, slot_off, copy_stream);
      return;
    }
    check_range(s, slot_off, nbytes);
    wait_reads(s);
    hipEvent_t dep = take_dep_event();
    if (hipEventRecord(dep, reinterpret_cast<hipStream_t>(after_stream)) != hipSuccess)
      throw std::runtime_error("HostRing: hipEventRecord failed");
    {
      std::lock_guard<std::mutex> g(sub_mu_);
      SubmitJob j{s, dst, nbytes, slot_off, copy_stream, dep, ++sub_seq_};
      want_seq_[s] = j.seq;
      sub_q_.push_back(j);
    }
    sub_cv_.notify_one();
  }

  void stream_wait(int s, uintptr_t stream) {
    if (!device_) return;
    wait_submitted(s);
    if (hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), events_.at(s), 0) != hipSuccess)
      throw std::runtime_error("HostRing: hipStreamWaitEvent failed");
  }

  void host_wait(int s) {
    if (!device_) return;
    wait_submitted(s);
    (void)hipEventSynchronize(events_.at(s));
  }

  void write_slot(int s, py::buffer b, size_t slot_off) {
    py::buffer_info info = b.request();
    size_t n = (size_t)info.size * (size_t)info.itemsize;
    check_range(s, slot_off, n);
    memcpy(slots_[s] + slot_off, info.ptr, n);
  }

 private:
  void check_range(int s, size_t off, size_t n) const {
    if (s < 0 || s >= (int)slots_.size()) throw std::runtime_error("HostRing: bad slot");
    if (off + n > slot_bytes_) throw std::runtime_error("HostRing: range exceeds slot");
  }
  struct SubmitJob {
    int s;
    uintptr_t dst;
    size_t nbytes, slot_off;
    uintptr_t stream;
    hipEvent_t dep;
    uint64_t seq;
  };

  hipEvent_t take_dep_event() {
    {
      std::lock_guard<std::mutex> g(sub_mu_);
      if (!dep_free_.empty()) {
        hipEvent_t e = dep_free_.back();
        dep_free_.pop_back();
        return e;
      }
    }
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
      throw std::runtime_error("HostRing: hipEventCreate failed");
    std::lock_guard<std::mutex> g(sub_mu_);
    dep_pool_.push_back(e);
    return e;
  }

  void wait_submitted(int s) {
    std::unique_lock<std::mutex> lk(sub_mu_);
    sub_done_cv_.wait(lk, [&] { return done_seq_.at(s) >= want_seq_.at(s); });
    if (!sub_error_.empty()) {
      std::string e = sub_error_;
      sub_error_.clear();
      throw std::runtime_error("HostRing: " + e);
    }
  }

  void submit_loop() {
    for (;;) {
      SubmitJob j;
      {
        std::unique_lock<std::mutex> lk(sub_mu_);
        sub_cv_.wait(lk, [this] { return sub_stop_ || !sub_q_.empty(); });
        if (sub_q_.empty()) return;
        j = sub_q_.front();
        sub_q_.pop_front();
      }
      hipStream_t st = reinterpret_cast<hipStream_t>(j.stream);
      std::string err;
      if (hipStreamWaitEvent(st, j.dep, 0) != hipSuccess) err = "hipStreamWaitEvent failed";
      else if (hipMemcpyAsync(reinterpret_cast<void*>(j.dst), slots_[j.s] + j.slot_off, j.nbytes,
                              hipMemcpyHostToDevice, st) != hipSuccess)
        err = "hipMemcpyAsync failed";
      else if (hipEventRecord(events_[j.s], st) != hipSuccess) err = "hipEventRecord failed";
      {
        std::lock_guard<std::mutex> g(sub_mu_);
        dep_free_.push_back(j.dep);   // the wait above has taken the record it needs
        done_seq_[j.s] = std::max(done_seq_[j.s], j.seq);
        if (!err.empty()) sub_error_ = err;
      }
      sub_done_cv_.notify_all();
    }
  }

  void work() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        job = std::move(q_.front());
        q_.pop_front();
      }
      job();
    }
  }

  size_t slot_bytes_;
  bool device_ = false, pinned_ = false, stop_ = false;
  std::vector<char*> slots_;
  std::vector<hipEvent_t> events_;
  std::vector<std::atomic<int>> pending_;
  std::vector<std::string> errors_;
  std::mutex mu_, err_mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  // h2d_async submitter
  std::thread submitter_;
  std::mutex sub_mu_;
  std::condition_variable sub_cv_, sub_done_cv_;
  std::deque<SubmitJob> sub_q_;
  std::vector<uint64_t> done_seq_, want_seq_;
  uint64_t sub_seq_ = 0;
  bool sub_stop_ = false;
  std::string sub_error_;
  std::vector<hipEvent_t> dep_pool_, dep_free_;
  std::vector<std::thread> workers_;
};

// Per-phase device timing for the engine's PhaseTimer: hipEvent pairs from a
// pool, recorded on the caller's stream, resolved in completion order.  One
// pybind call per phase edge instead of torch.cuda.Event's Python layers
// (identity7 resident: telemetry was ~40 us of a 165 us date).
class PhaseEvents {
 public:
  PhaseEvents() = default;
  PhaseEvents(const PhaseEvents&) = delete;
  PhaseEvents& operator=(const PhaseEvents&) = delete;
  ~PhaseEvents() {
    for (auto& sl : slots_) {
      if (sl.start) hipEventDestroy(sl.start);
      if (sl.stop) hipEventDestroy(sl.stop);
    }
  }

  // record the start of ``phase`` on ``stream``; returns the token for end().
  // The pool belongs to the device current at its first begin(): its events
  // are created there, and later begins switch to it (hipEventRecord needs the
  // event's device) and restore the caller's device.
  int begin(int phase, int64_t stream) {
    if (phase < 0) throw std::runtime_error("PhaseEvents: negative phase id");
    DeviceGuard g(device_);
    int t;
    if (!free_.empty()) {
      t = free_.back();
      free_.pop_back();
    } else {
      Slot sl;
      if (hipEventCreateWithFlags(&sl.start, hipEventDefault) != hipSuccess ||
          hipEventCreateWithFlags(&sl.stop, hipEventDefault) != hipSuccess)
        throw std::runtime_error("PhaseEvents: hipEventCreate failed");
      slots_.push_back(sl);
      t = static_cast<int>(slots_.size()) - 1;
    }
    slots_[t].phase = phase;
    if (hipEventRecord(slots_[t].start, reinterpret_cast<hipStream_t>(stream)) != hipSuccess)
      throw std::runtime_error("PhaseEvents: hipEventRecord failed");
    return t;
  }

  void end(int token, int64_t stream) {
    if (token < 0 || token >= static_cast<int>(slots_.size()))
      throw std::runtime_error("PhaseEvents: bad token");
    DeviceGuard g(device_);
    if (hipEventRecord(slots_[token].stop, reinterpret_cast<hipStream_t>(stream)) != hipSuccess)
      throw std::runtime_error("PhaseEvents: hipEventRecord failed");
    done_.push_back(token);
  }

  // (phase, ms) of the ended phases, oldest first: all of them when ``block``
  // (waits for the newest), else the finished prefix only
  std::vector<std::pair<int, float>> collect(bool block) {
    std::vector<std::pair<int, float>> out;
    if (block && !done_.empty()) {
      py::gil_scoped_release nogil;
      if (hipEventSynchronize(slots_[done_.back()].stop) != hipSuccess)
        throw std::runtime_error("PhaseEvents: hipEventSynchronize failed");
    }
    while (!done_.empty()) {
      Slot& sl = slots_[done_.front()];
      if (!block && hipEventQuery(sl.stop) != hipSuccess) break;
      float ms = 0.f;
      hipError_t e = hipEventElapsedTime(&ms, sl.start, sl.stop);
      if (e == hipErrorNotReady) {
        // a phase recorded on another stream than the newest one need not have
        // finished when that one has: wait for its own events, then read it
        py::gil_scoped_release nogil;
        if (hipEventSynchronize(sl.start) != hipSuccess || hipEventSynchronize(sl.stop) != hipSuccess)
          throw std::runtime_error("PhaseEvents: hipEventSynchronize failed");
        e = hipEventElapsedTime(&ms, sl.start, sl.stop);
      }
      if (e != hipSuccess) throw std::runtime_error("PhaseEvents: hipEventElapsedTime failed");
      out.emplace_back(sl.phase, ms);
      free_.push_back(done_.front());
      done_.pop_front();
    }
    return out;
  }

  size_t pending() const { return done_.size(); }

 private:
  struct Slot {
    hipEvent_t start = nullptr, stop = nullptr;
    int phase = 0;
  };
  // switches to the pool's device (fixed by the first use) for one call
  struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int& dev) {
      if (hipGetDevice(&prev) != hipSuccess) prev = -1;
      if (dev < 0) dev = prev;
      else if (prev != dev && hipSetDevice(dev) != hipSuccess)
        throw std::runtime_error("PhaseEvents: hipSetDevice failed");
    }
    ~DeviceGuard() {
      int cur = -1;
      if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
  };
  std::vector<Slot> slots_;
  std::vector<int> free_;
  std::deque<int> done_;
  int device_ = -1;
};

}  // namespace


void bind_stream(py::module_& m) {
  py::class_<HostRing>(m, "HostRing")
      .def(py::init<int, size_t, int>(), py::arg("n_slots"), py::arg("slot_bytes"), py::arg("n_threads") = 2)
      .def("slot", &HostRing::slot)
      .def_property_readonly("slot_bytes", &HostRing::slot_bytes)
      .def_property_readonly("n_slots", &HostRing::n_slots)
      .def_property_readonly("pinned", &HostRing::pinned)
      .def("read_file_async", &HostRing::read_file_async)
      .def("read_tiff_async", &HostRing::read_tiff_async)
      .def("wait_reads", &HostRing::wait_reads, py::call_guard<py::gil_scoped_release>())
      .def("h2d", &HostRing::h2d)
      .def("h2d_async", &HostRing::h2d_async)
      .def("stream_wait", &HostRing::stream_wait, py::call_guard<py::gil_scoped_release>())
      .def("host_wait", &HostRing::host_wait, py::call_guard<py::gil_scoped_release>())
      .def("write_slot", &HostRing::write_slot);
  py::class_<PhaseEvents>(m, "PhaseEvents")
      .def(py::init<>())
      .def("begin", &PhaseEvents::begin)
      .def("end", &PhaseEvents::end)
      .def("collect", &PhaseEvents::collect, py::arg("block"))
      .def_property_readonly("pending", &PhaseEvents::pending);
}
