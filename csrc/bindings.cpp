// pybind11 surface of the native HIP extension ``pytorch_ddp_mnist_amd._C``.
// Device buffers are owned by torch (HBM via its caching allocator) and passed as raw
// addresses; streams are passed as the integer handles of torch.cuda.Stream.cuda_stream.
#include <execinfo.h>
#include <pybind11/pybind11.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <pybind11/stl.h>

#include "kernels/launch.h"
#include "runtime/hip_check.h"
#include "runtime/rccl_comm.h"
#include "runtime/trainer.h"

namespace py = pybind11;

namespace {
// MNIST_AMD_SEGV_TRACE=1: print the native backtrace of a host SIGSEGV / SIGBUS / SIGILL / SIGFPE (faulthandler
// shows only Python frames), then hand the signal to the handler installed before ours -- Python's faulthandler
// (PYTHONFAULTHANDLER=1, set for bench.py's rank processes) prints every thread's Python stack and re-raises --
// or, without one, re-raise it with the default action (core / exit status 128 + sig).
constexpr int kTraced[] = {SIGSEGV, SIGBUS, SIGILL, SIGFPE};
struct sigaction g_prev[sizeof(kTraced) / sizeof(kTraced[0])];

void segv_trace(int sig, siginfo_t* info, void* uctx) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  char msg[128];
  const int len = snprintf(msg, sizeof(msg), "\n[mnist_amd] signal %d at address %p, native backtrace:\n", sig,
                           info ? info->si_addr : nullptr);
  (void)!write(2, msg, len > 0 ? (size_t)len : 0);
  backtrace_symbols_fd(frames, n, 2);
  for (size_t i = 0; i < sizeof(kTraced) / sizeof(kTraced[0]); ++i) {
    if (kTraced[i] != sig) continue;
    const struct sigaction& p = g_prev[i];
    sigaction(sig, &p, nullptr);  // the previous disposition, for the re-raise below as well
    if (p.sa_flags & SA_SIGINFO) {
      if (p.sa_sigaction) { p.sa_sigaction(sig, info, uctx); return; }
    } else if (p.sa_handler != SIG_DFL && p.sa_handler != SIG_IGN && p.sa_handler) {
      p.sa_handler(sig);
      return;
    }
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

void install_segv_trace() {
  for (size_t i = 0; i < sizeof(kTraced) / sizeof(kTraced[0]); ++i) {
    struct sigaction sa {};
    sa.sa_sigaction = segv_trace;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(kTraced[i], &sa, &g_prev[i]);
  }
}
}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X (gfx950) native kernels, step runtime and RCCL communicator";
  if (const char* e = std::getenv("MNIST_AMD_SEGV_TRACE"); e && *e == '1') install_segv_trace();

  m.def("model_nparam", [](int model) { return model_nparam(static_cast<ModelKind>(model)); });
  m.def("model_conv_params", [](int model) { return model_conv_params(static_cast<ModelKind>(model)); });
  m.def("model_phase_split", [](int model) { return model_phase_split(static_cast<ModelKind>(model)); });
  m.def("model_pack_size", [](int model) { return model_pack_size(static_cast<ModelKind>(model)); });
  m.def("conv_bwd_blocks", &lenet_conv_bwd_blocks, py::arg("B"), py::arg("target_blocks") = 0);
  m.def("fwd_head_applies", [](int dtype, int B) { return lenet_fwd_head_applies(static_cast<DType>(dtype), B); },
        py::arg("dtype"), py::arg("B"));
  m.def("conv_bwd_max_blocks", &lenet_conv_bwd_max_blocks, py::arg("B"), py::arg("target_blocks") = 0);
  m.attr("L1_KSPLIT") = L1_KSPLIT;
  m.def("metric_rows", [](int B) { return metric_rows(B); });
  m.attr("L1_SPLIT_MAX_B") = L1_SPLIT_MAX_B;
  m.attr("STAMP_ROWS") = STAMP_ROWS;
#ifdef MNIST_AMD_F32_SPLIT
  m.attr("F32_SPLIT") = 3;  // fp32 products as exact 3-part bf16 splits on 16x16x32 MFMAs (common.h Mma<float>, opt-in build)
#else
  m.attr("F32_SPLIT") = 0;
#endif
  m.attr("XB_MAX_B") = Trainer::XB_MAX_B;  // LeNet: batch-ordered pixel rows conv_fwd -> conv_bwd up to this batch
  m.def("device_count", [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("device_arch", [](int dev) {
    hipDeviceProp_t p;
    HIP_CHECK(hipGetDeviceProperties(&p, dev));
    return std::string(p.gcnArchName);
  });
  m.def("rccl_version", &RcclComm::version);
  // x[r] = normalize(images[idx[r]]) for r < B, fp32 (dtype 0) or bf16 (1), rows ld elements apart.
  // `zero` is a device int32 holding 0 (the kernel addresses idx through a device step counter).
  m.def("gather_normalize", [](int dtype, uintptr_t images, uintptr_t idx, uintptr_t zero, int B, uintptr_t out,
                               int ld, uintptr_t stream) {
    if (B <= 0) return;
    if (ld < 784) throw std::invalid_argument("gather_normalize: ld must be >= 784");
    BatchRef br{reinterpret_cast<const uint8_t*>(images), nullptr, reinterpret_cast<const int32_t*>(idx),
                reinterpret_cast<const int32_t*>(zero), 0, B};
    launch_gather_normalize(static_cast<DType>(dtype), br, reinterpret_cast<void*>(out), ld,
                            reinterpret_cast<hipStream_t>(stream));
    HIP_CHECK(hipGetLastError());
  });

  py::class_<TrainerPtrs>(m, "TrainerPtrs")
      .def(py::init<>())
#define RW(f) .def_readwrite(#f, &TrainerPtrs::f)
      RW(images) RW(labels) RW(idx) RW(step) RW(params) RW(grad) RW(mom) RW(pack) RW(slab_fc) RW(slab_conv)
      RW(metrics) RW(xT) RW(h1T) RW(h2T) RW(dy1T) RW(dy2T) RW(dy3T) RW(p1) RW(m1) RW(p2) RW(m2) RW(dp2) RW(z1p) RW(stamps) RW(xnext) RW(ynext) RW(xb);
#undef RW

  py::class_<Bucket>(m, "Bucket")
      .def(py::init([](int p0, int p1, int phase) { return Bucket{p0, p1, phase}; }))
      .def_readwrite("p0", &Bucket::p0)
      .def_readwrite("p1", &Bucket::p1)
      .def_readwrite("phase", &Bucket::phase)
      .def("__repr__", [](const Bucket& b) {
        return "Bucket(" + std::to_string(b.p0) + ", " + std::to_string(b.p1) + ", phase=" + std::to_string(b.phase) + ")";
      });

  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def_static("make_unique_id", [] { return py::bytes(RcclComm::make_unique_id()); })
      .def(py::init([](py::bytes uid, int rank, int world, int device, double init_timeout) {
             std::string id(uid);  // copy while holding the GIL; init waits on peers, so release it then
             py::gil_scoped_release nogil;
             return std::make_shared<RcclComm>(id, rank, world, device, init_timeout);
           }),
           py::arg("uid"), py::arg("rank"), py::arg("world"), py::arg("device"), py::arg("init_timeout") = 180.0)
      // The bounded-bring-up logic of the constructor against a FAKE communicator (no GPU, no RCCL state):
      // `ready_after` polls until it reports ready (< 0: never -- a peer that never arrives), `fail`: it reports
      // an error instead.  Returns (error message or "", seconds waited, whether abort was called).
      .def_static("_fake_init",
                  [](int rank, int world, double timeout, int ready_after, bool fail) {
                    int polls = 0;
                    bool aborted = false;
                    double waited = 0.0;
                    ncclResult_t st;
                    {
                      py::gil_scoped_release nogil;
                      st = RcclComm::poll_ready(
                          [&] {
                            ++polls;
                            if (fail && polls > 2) return ncclSystemError;
                            if (ready_after >= 0 && polls > ready_after) return ncclSuccess;
                            return ncclInProgress;
                          },
                          timeout, &waited);
                    }
                    const std::string err =
                        RcclComm::init_outcome(st, rank, world, timeout, waited, [&] { aborted = true; });
                    return py::make_tuple(err, waited, aborted);
                  },
                  py::arg("rank"), py::arg("world"), py::arg("timeout"), py::arg("ready_after") = -1,
                  py::arg("fail") = false)
      .def("destroy", &RcclComm::destroy, py::arg("timeout") = 600.0, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("destroyed", &RcclComm::destroyed)
      .def_property_readonly("nonblocking", &RcclComm::nonblocking)
      .def_property_readonly("init_seconds", &RcclComm::init_seconds)
      .def("all_reduce_sum_f32",
           [](RcclComm& c, uintptr_t buf, size_t n, uintptr_t s) {
             c.all_reduce_sum_f32(reinterpret_cast<float*>(buf), n, reinterpret_cast<hipStream_t>(s));
           })
      .def("broadcast_f32",
           [](RcclComm& c, uintptr_t buf, size_t n, int root, uintptr_t s) {
             c.broadcast_f32(reinterpret_cast<float*>(buf), n, root, reinterpret_cast<hipStream_t>(s));
           })
      .def("all_reduce_max_f64",
           [](RcclComm& c, uintptr_t buf, size_t n, uintptr_t s) {
             c.all_reduce_max_f64(reinterpret_cast<double*>(buf), n, reinterpret_cast<hipStream_t>(s));
           })
      .def("time_all_reduce",
           [](RcclComm& c, uintptr_t buf, size_t n, int warmup, int iters, uintptr_t s, double timeout, int per_graph) {
             return c.time_all_reduce(reinterpret_cast<float*>(buf), n, warmup, iters,
                                      reinterpret_cast<hipStream_t>(s), timeout, per_graph);
           },
           py::arg("buf"), py::arg("count"), py::arg("warmup"), py::arg("iters"), py::arg("stream"),
           py::arg("timeout") = 600.0, py::arg("per_graph") = 1, py::call_guard<py::gil_scoped_release>())
      .def("async_error", &RcclComm::async_error)
      .def("wait_stream",
           [](RcclComm& c, uintptr_t s, double timeout) { return c.wait_stream(reinterpret_cast<hipStream_t>(s), timeout); },
           py::call_guard<py::gil_scoped_release>())
      .def("probe_cross_stream_capture",
           [](RcclComm& c, uintptr_t buf, size_t n, uintptr_t s, int replays, double timeout) {
             return c.probe_cross_stream_capture(reinterpret_cast<float*>(buf), n, reinterpret_cast<hipStream_t>(s),
                                                 replays, timeout);
           },
           py::arg("buf"), py::arg("count"), py::arg("stream"), py::arg("replays") = 3, py::arg("timeout") = 60.0,
           py::call_guard<py::gil_scoped_release>())
      .def("abort", &RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("aborted", &RcclComm::aborted)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world);

  py::class_<OneShotAllReduce, std::shared_ptr<OneShotAllReduce>>(m, "OneShotAllReduce")
      .def(py::init<int, int, int, int, int, double>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("max_count"), py::arg("nblk") = 64, py::arg("timeout") = 5.0)
      .def("handle", [](const OneShotAllReduce& o) { return py::bytes(o.handle()); })
      .def("open_peers",
           [](OneShotAllReduce& o, const std::vector<py::bytes>& hs) {
             std::vector<std::string> v;
             for (const auto& h : hs) v.emplace_back(std::string(h));
             o.open_peers(v);
           })
      .def("all_reduce_sum_f32",
           [](OneShotAllReduce& o, uintptr_t buf, size_t n, uintptr_t s) {
             o.all_reduce_sum_f32(reinterpret_cast<float*>(buf), n, reinterpret_cast<hipStream_t>(s));
           })
      .def("check", &OneShotAllReduce::check)
      .def("clear_error", &OneShotAllReduce::clear_error)
      .def("enable_stamps", &OneShotAllReduce::enable_stamps)
      .def("stamps", &OneShotAllReduce::stamps)
      .def_property_readonly("calls", &OneShotAllReduce::calls)
      .def_property_readonly("rank", &OneShotAllReduce::rank)
      .def_property_readonly("world", &OneShotAllReduce::world)
      .def_property_readonly("max_count", &OneShotAllReduce::max_count)
      .def_property_readonly("ready", &OneShotAllReduce::ready);

  py::class_<Trainer>(m, "Trainer")
      .def(py::init<int, int, int, int, int, const TrainerPtrs&>(), py::arg("model"), py::arg("dtype"),
           py::arg("batch"), py::arg("ld_b"), py::arg("fc_splits"), py::arg("ptrs"))
      .def("set_comm", &Trainer::set_comm)
      .def("set_oneshot", &Trainer::set_oneshot)
      .def("set_overlap", &Trainer::set_overlap, py::arg("fc"), py::arg("conv"))
      .def_property_readonly("has_overlap", &Trainer::has_overlap)
      .def_property_readonly("has_oneshot", &Trainer::has_oneshot)
      .def("set_world", &Trainer::set_world)
      .def("set_optimizer", &Trainer::set_optimizer)
      .def("set_dropout", &Trainer::set_dropout)
      .def("set_buckets", &Trainer::set_buckets)
      .def_property("comm_enabled", &Trainer::comm_enabled, &Trainer::set_comm_enabled)
      .def_property_readonly("phase_split", &Trainer::phase_split)
      .def("buckets", &Trainer::buckets)
      .def("groups", [](const Trainer& t) {
        py::list out;
        for (const auto& g : t.groups()) out.append(py::make_tuple(g.p0, g.p1, g.mask));
        return out;
      })
      .def("time_units", &Trainer::time_units, py::arg("iters"), py::arg("warmup"), py::arg("stream"),
           py::call_guard<py::gil_scoped_release>())
      .def_static("job_begin", [](int model, int job) { return model_job_begin(static_cast<ModelKind>(model), job); })
      .def("set_plan", &Trainer::set_plan)
      .def_property_readonly("plan", &Trainer::plan)
      .def("set_concurrent", &Trainer::set_concurrent)
      .def("set_fwd_head", &Trainer::set_fwd_head)
      .def_property_readonly("fwd_head", &Trainer::fwd_head)
      .def_property_readonly("concurrent", &Trainer::concurrent)
      .def("set_bwd_blocks", &Trainer::set_bwd_blocks)
      .def_property_readonly("bwd_blocks", &Trainer::bwd_blocks)
      .def_property_readonly("bwd_grid", &Trainer::bwd_grid)
      .def("issued_collectives", &Trainer::issued_collectives)
      .def_property_readonly("has_comm", &Trainer::has_comm)
      .def_property_readonly("world", &Trainer::world)
      .def("spin", &Trainer::spin)
      .def("pack", &Trainer::pack)
      .def("train_step", &Trainer::train_step)
      .def("forward_backward", &Trainer::forward_backward)
      .def("reduce_grads", &Trainer::reduce_grads)
      .def("optimizer_step", &Trainer::optimizer_step)
      .def("eval_batch", &Trainer::eval_batch)
      .def("capture", &Trainer::capture)
      .def("replay", &Trainer::replay)
      .def("prime_next", &Trainer::prime_next)
      .def_property("fuse_wgrad_sgd", &Trainer::fuse_wgrad_sgd, &Trainer::set_fuse_wgrad_sgd)
      .def("capture_multi", &Trainer::capture_multi)
      .def("replay_multi", &Trainer::replay_multi)
      .def("capture_n", &Trainer::capture_n)
      .def("has_graph", &Trainer::has_graph)
      .def("replay_n", &Trainer::replay_n)
      .def_property_readonly("multi_steps", &Trainer::multi_steps)
      .def("invalidate", &Trainer::invalidate)
      .def("release", &Trainer::release, py::call_guard<py::gil_scoped_release>())
      .def("destroy", &Trainer::destroy, py::call_guard<py::gil_scoped_release>())
      .def("graph_nodes", &Trainer::graph_nodes)
      .def_property_readonly("captured", &Trainer::captured)
      .def_property_readonly("nparam", &Trainer::nparam)
      .def_property_readonly("pack_size", &Trainer::pack_size)
      .def_property_readonly("conv_slabs", &Trainer::conv_slabs)
      .def_property_readonly("conv_params", &Trainer::conv_params)
      .def_property_readonly("fc_splits", &Trainer::fc_splits)
      .def_property_readonly("fc_ld", &Trainer::fc_ld);
}
