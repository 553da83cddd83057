// Native bucketed data-parallel gradient reducer (the MI355X counterpart of torch DDP's C++ Reducer,
// torch/csrc/distributed/c10d/reducer.cpp, which the reference reaches through HF Trainer / Accelerate).
//
// Works on the flat gradient buffer of parallel/flat.py: bucket b is the contiguous slice
// [bounds[2b], bounds[2b+1]) of ONE buffer ("gradient as bucket view"), so a bucket's all-reduce runs in
// place with no flatten/unflatten copies.  Readiness is tracked per flat segment: mark_ready(seg) is called once per
// backward per segment — by FlatParams' post-accumulate hook for the few parameters autograd accumulates, and by the
// fused op that accumulated the gradient inside its GEMM / norm kernel for the rest (ops/linear.py _fire,
// ops/norms.py: AccumulateGrad never runs for them, so a C++ AccumulateGrad hook could not see them).
// A bucket is launched the moment its last segment is ready, strictly in bucket order on every rank (RCCL
// requires the same collective order everywhere), as an async all_reduce on the process group
// (ProcessGroupNCCL = RCCL over xGMI on ROCm: the collective runs on RCCL's own stream while backward
// keeps computing).  The first hook of a backward queues finalize() on the autograd engine; finalize
// launches leftovers (unused parameters) and makes the compute stream wait on the RCCL work — no host
// synchronisation on the GPU path.  Averaging uses ReduceOp::AVG (RCCL) or SUM + one scale (gloo).
// Compress-for-wire (set_wire_buffer, --grad-reduce-dtype bf16): a launch casts the fp32 bucket into its slice of a
// persistent bf16 shadow on the compute stream and all-reduces that; finalize widens it back after the wait.
// launch_upto(n) is the replay side of a segmented HIP-graph step (train/graph.py "overlap"): the buckets whose
// readiness the capture cut the backward graph at are launched between the graph segments, in bucket order.
#include <torch/extension.h>
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>

namespace dllm {

// roctx marker at every bucket launch (rocprofv3 --marker-trace), resolved at run time so the extension does not
// link libroctx64; DLLM_ROCTX=0 or a missing library makes it a no-op (utils/profiling.py is the Python side)
static void roctx_mark(const char* msg) {
  using MarkFn = void (*)(const char*);
  static MarkFn fn = [] {
    const char* e = std::getenv("DLLM_ROCTX");
    if (e && e[0] == '0') return (MarkFn) nullptr;
    void* h = dlopen("libroctx64.so", RTLD_LAZY | RTLD_NOLOAD);
    if (!h) h = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_LAZY);
    return h ? (MarkFn)dlsym(h, "roctxMarkA") : (MarkFn) nullptr;
  }();
  if (fn) fn(msg);
}

class NativeReducer {
 public:
  NativeReducer(at::Tensor grad_buf, std::vector<int64_t> bounds, std::vector<int64_t> seg_bucket,
                c10::intrusive_ptr<c10d::ProcessGroup> pg, bool average, bool use_avg_op)
      : grad_buf_(std::move(grad_buf)),
        bounds_(std::move(bounds)),
        seg_bucket_(std::move(seg_bucket)),
        pg_(std::move(pg)),
        average_(average),
        use_avg_op_(use_avg_op) {
    TORCH_CHECK(bounds_.size() % 2 == 0 && !bounds_.empty(), "bounds must be [start0, end0, start1, end1, ...]");
    TORCH_CHECK(grad_buf_.dim() == 1 && grad_buf_.is_contiguous(), "grad_buf must be a contiguous 1-D buffer");
    const int64_t nb = (int64_t)bounds_.size() / 2;
    counts_.assign(nb, 0);
    for (int64_t b : seg_bucket_) {
      TORCH_CHECK(b >= 0 && b < nb, "segment bucket index out of range");
      counts_[b] += 1;
    }
    reset_state();
  }

  void mark_ready(int64_t seg) {
    std::lock_guard<std::mutex> g(mu_);
    if (!enabled_) return;
    TORCH_CHECK(seg >= 0 && seg < (int64_t)seg_bucket_.size(), "segment index out of range");
    if (!callback_queued_) {
      callback_queued_ = true;
      torch::autograd::Engine::get_default_engine().queue_callback([this] { this->finalize(); });
    }
    const int64_t b = seg_bucket_[seg];
    if (--pending_[b] == 0) {
      ready_[b] = true;
      launch_ready_locked();
    }
  }

  // End of backward (queued on the engine): launch leftovers in order, order the compute stream after them.
  // With timing on (GPU buffers only) two events bracket that wait on the compute stream: the first fires when the
  // last backward kernel has run, the second when the last bucket's all-reduce has — their distance is the
  // communication NOT hidden under backward ("exposed" ms, bench.py reports it per step).
  void finalize() {
    std::lock_guard<std::mutex> g(mu_);
    const int64_t nb = num_buckets();
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = timing_ && grad_buf_.is_cuda();
    hipStream_t st = nullptr;
    if (timed) {
      st = c10::hip::getCurrentHIPStream(grad_buf_.device().index()).stream();
      if (hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess) {
        (void)hipEventRecord(e0, st);
      } else {
        e0 = e1 = nullptr;
      }
    }
    const auto h0 = std::chrono::steady_clock::now();
    while (next_ < nb) launch_locked(next_++);
    for (auto& bw : works_) {
      bw.second->wait();
      if (wire_.defined()) {
        const int64_t s = bounds_[2 * bw.first], e = bounds_[2 * bw.first + 1];
        grad_buf_.narrow(0, s, e - s).copy_(wire_.narrow(0, s, e - s));
      }
    }
    works_.clear();
    if (timed && e0) {
      (void)hipEventRecord(e1, st);
      events_.emplace_back(e0, e1);
    } else if (timing_ && !grad_buf_.is_cuda()) {  // CPU (gloo) rehearsal: wait() blocks the host
      host_ms_.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count());
    }
    if (average_ && !use_avg_op_) grad_buf_.div_(pg_->getSize());
    reset_state();
  }

  // train-task path: one coalesced all-reduce of the whole buffer, no hooks involved
  void sync_all() {
    if (wire_.defined()) wire_.copy_(grad_buf_);
    std::vector<at::Tensor> ts{wire_.defined() ? wire_ : grad_buf_};
    c10d::AllreduceOptions opts;
    opts.reduceOp = use_avg_op_ && average_ ? c10d::ReduceOp::AVG : c10d::ReduceOp::SUM;
    pg_->allreduce(ts, opts)->wait();
    if (wire_.defined()) grad_buf_.copy_(wire_);
    if (average_ && !use_avg_op_) grad_buf_.div_(pg_->getSize());
  }

  void set_wire_buffer(at::Tensor w) {
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(w.dim() == 1 && w.is_contiguous() && w.numel() == grad_buf_.numel() &&
                    w.device() == grad_buf_.device(),
                "wire buffer must be a contiguous 1-D tensor shaped like the gradient buffer");
    wire_ = std::move(w);
  }

  // launch buckets [launched, n) in order (no readiness check: the caller's schedule guarantees the gradients)
  void launch_upto(int64_t n) {
    std::lock_guard<std::mutex> g(mu_);
    n = std::min<int64_t>(n, num_buckets());
    while (next_ < n) launch_locked(next_++);
  }

  void set_enabled(bool e) {
    std::lock_guard<std::mutex> g(mu_);
    enabled_ = e;
  }
  void set_timing(bool on) {
    std::lock_guard<std::mutex> g(mu_);
    timing_ = on;
  }
  // exposed-communication ms of every timed backward since the last call (blocks until their events completed)
  std::vector<double> take_exposed_ms() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<double> out(host_ms_);
    host_ms_.clear();
    for (auto& pr : events_) {
      float ms = 0.f;
      if (hipEventSynchronize(pr.second) == hipSuccess && hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess)
        out.push_back((double)ms);
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
    events_.clear();
    return out;
  }
  bool enabled() const { return enabled_; }
  int64_t num_buckets() const { return (int64_t)bounds_.size() / 2; }
  int64_t launched() const { return next_; }
  void detach() {}

 private:
  void reset_state() {
    pending_ = counts_;
    ready_.assign(counts_.size(), false);
    next_ = 0;
    callback_queued_ = false;
  }

  void launch_locked(int64_t b) {
    const int64_t s = bounds_[2 * b], e = bounds_[2 * b + 1];
    char msg[64];
    std::snprintf(msg, sizeof msg, "allreduce bucket %ld (%.1f MiB)", (long)b,
                  (double)(e - s) * grad_buf_.element_size() / 1048576.0);
    roctx_mark(msg);
    at::Tensor view = grad_buf_.narrow(0, s, e - s);
    if (wire_.defined()) {
      at::Tensor w = wire_.narrow(0, s, e - s);
      w.copy_(view);  // compute stream: the all-reduce's stream waits on it
      view = w;
    }
    std::vector<at::Tensor> ts{view};
    c10d::AllreduceOptions opts;
    opts.reduceOp = use_avg_op_ && average_ ? c10d::ReduceOp::AVG : c10d::ReduceOp::SUM;
    works_.emplace_back(b, pg_->allreduce(ts, opts));
  }

  void launch_ready_locked() {
    const int64_t nb = num_buckets();
    while (next_ < nb && ready_[next_]) launch_locked(next_++);
  }

  at::Tensor grad_buf_;
  at::Tensor wire_;  // compress-for-wire shadow (undefined: all-reduce the buckets in place)
  std::vector<int64_t> bounds_, seg_bucket_, counts_, pending_;
  std::vector<bool> ready_;
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  bool average_, use_avg_op_;
  bool enabled_ = true;
  bool timing_ = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events_;
  std::vector<double> host_ms_;
  bool callback_queued_ = false;
  int64_t next_ = 0;
  std::vector<std::pair<int64_t, c10::intrusive_ptr<c10d::Work>>> works_;
  std::mutex mu_;
};

void bind_reducer(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<NativeReducer, std::shared_ptr<NativeReducer>>(m, "NativeReducer")
      .def(py::init<at::Tensor, std::vector<int64_t>, std::vector<int64_t>, c10::intrusive_ptr<c10d::ProcessGroup>,
                    bool, bool>(),
           py::arg("grad_buf"), py::arg("bounds"), py::arg("seg_bucket"), py::arg("process_group"),
           py::arg("average") = true, py::arg("use_avg_op") = true)
      .def("mark_ready", &NativeReducer::mark_ready)
      .def("finalize", &NativeReducer::finalize, py::call_guard<py::gil_scoped_release>())
      .def("sync_all", &NativeReducer::sync_all, py::call_guard<py::gil_scoped_release>())
      .def("set_wire_buffer", &NativeReducer::set_wire_buffer)
      .def("launch_upto", &NativeReducer::launch_upto, py::call_guard<py::gil_scoped_release>())
      .def("set_enabled", &NativeReducer::set_enabled)
      .def("set_timing", &NativeReducer::set_timing)
      .def("take_exposed_ms", &NativeReducer::take_exposed_ms, py::call_guard<py::gil_scoped_release>())
      .def("enabled", &NativeReducer::enabled)
      .def("num_buckets", &NativeReducer::num_buckets)
      .def("launched", &NativeReducer::launched)
      .def("detach", &NativeReducer::detach);
}

}  // namespace dllm
