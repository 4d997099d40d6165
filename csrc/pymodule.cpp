// Python bindings (`test_nccl_p2p_amd._p2pcore`), pybind11.
//
// Exposes the native engine to bench.py / the Python package: a Session owns
// a Bootstrap (TCP star, or local) and a Transport (RCCL on the MI355X, or
// host sockets).  Everything long-running releases the GIL.  Results cross
// the boundary as JSON text produced by report.cpp, so the Python side and
// the p2p_matrix executable share one result schema.
//
// The fill / verify kernels are also exposed on raw device pointers so they
// can be driven on torch tensors and checked against a PyTorch reference.
#include <hip/hip_runtime.h>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "app.hpp"
#include "bootstrap.hpp"
#include "common.hpp"
#include "kernels.hpp"
#include "provenance.hpp"
#include "report.hpp"
#include "runner.hpp"
#include "routing.hpp"
#include "schedule.hpp"
#include "transport.hpp"
#include "units.hpp"

namespace py = pybind11;
using namespace p2p;

namespace {

// Teardown of an engine object from Python's deallocation: the transports'
// waits (buffers freed, streams drained) run without the GIL, so bench.py's
// deadline watchdog keeps running meanwhile, and inside a NativeCall, so the
// watchdog does not abort these communicators from its thread (the drain
// honours its abort request instead).
template <class Fn>
void teardown_outside_gil(Fn&& fn) {
  NativeCall in_engine(std::nothrow);
  if (PyGILState_Check()) {
    py::gil_scoped_release nogil;
    fn();
  } else {
    fn();
  }
}

class Session {
 public:
  Session(int rank, int world, const std::string& host, int port, int device, const std::string& transport,
          double timeout_s, TcpListener* listener)
      : transport_kind_(transport) {
    if (world == 1)
      boot_ = make_local_bootstrap();
    else
      boot_ = make_tcp_bootstrap(rank, world, host, port, timeout_s, listener);
    TransportOptions opt;
    opt.device = device;
    opt.timeout_s = timeout_s;
    // "ipc" or "ipc:kernel" / "ipc:sdma" / "ipc:push"
    std::string kind = transport.substr(0, transport.find(':'));
    if (kind == "ipc" && transport.size() > 4) opt.ipc_engine = transport.substr(4);
    // "rccl:K": K communicators per rank (TransportOptions::rccl_comms)
    if (kind == "rccl" && transport.size() > 5) opt.rccl_comms = std::atoi(transport.substr(5).c_str());
    if (kind == "rccl")
      t_ = make_rccl_transport(*boot_, opt);
    else if (kind == "ipc")
      t_ = make_ipc_transport(*boot_, opt);
    else if (kind == "host")
      t_ = make_host_transport(*boot_, opt);
    else if (kind == "shm")
      t_ = make_shm_transport(*boot_, opt);
    else
      P2P_FATAL("transport must be 'rccl[:K]', 'ipc[:kernel|:sdma|:push|:relay]', 'host' or 'shm'");
  }

  ~Session() {
    teardown_outside_gil([this] {
      t_.reset();
      boot_.reset();
    });
  }

  int rank() const { return boot_->rank(); }
  int world() const { return boot_->size(); }
  std::string transport() const { return t_->name(); }
  std::string device_desc() const { return t_->device_desc(); }
  Bootstrap& boot() { return *boot_; }
  Transport& t() { return *t_; }

  void barrier() { boot_->barrier(); }
  double allreduce_max(double v) { return boot_->allreduce_max(v); }
  double allreduce_sum(double v) { return boot_->allreduce_sum(v); }

  // One (mode, dir, size) run; returns the run JSON (report.cpp schema).
  std::string run(const std::string& mode, const std::string& dir, size_t bytes, int iters, int warmup,
                  const std::string& timing, bool verify, bool warm, const std::vector<std::pair<int, int>>& cells) {
    Schedule s = make_schedule(parse_mode(mode), parse_direction(dir), world());
    restrict_cells(&s, cells, true);
    RunConfig cfg;
    cfg.bytes = bytes;
    cfg.iters = iters;
    cfg.warmup = warmup;
    cfg.timing = parse_timing(timing);
    cfg.verify = verify;
    cfg.salt = ++salt_;
    const int slots = std::max(1, s.max_recv_slots());
    // Verified runs: one receive generation per iteration, as far as memory
    // allows (runner.hpp RunConfig::gens).
    cfg.gens = verify ? verify_generations(*t_, *boot_, bytes, slots, std::max(iters, warmup)) : 1;
    if (const char* rc = std::getenv("P2P_RECHUNK")) cfg.rechunk = std::atoi(rc) != 0;
    Buffers bufs(*t_, bytes, slots * cfg.gens, slot_stride_bytes(bytes) * static_cast<size_t>(cfg.gens));
    if (warm) {
      warm_connections(*t_, *boot_, s, bufs);
      t_->refine_op_limits(*boot_);
    }
    RunRecord rec;
    rec.mode = s.mode;
    rec.dir = s.dir;
    rec.bytes = bytes;
    rec.cfg = cfg;
    rec.phases = run_schedule(*t_, *boot_, s, cfg, bufs);
    return run_to_json(rec, world());
  }

  std::string latency(size_t bytes, int iters, int warmup, int preposted) {
    Buffers bufs(*t_, std::max<size_t>(bytes, 16), 1);
    auto lat = run_latency(*t_, *boot_, bytes, iters, warmup, bufs, preposted);
    return latency_to_json(lat, world());
  }

  uint64_t fuzz(int rounds, uint64_t seed, size_t max_bytes) { return fuzz_transport(*t_, *boot_, rounds, seed, max_bytes); }

  // Test hook for the transports' watchdogs: a receive from this rank that
  // no send matches, then sync().  Returns the error the watchdog raised (""
  // if none did).  The buffer is kept: an aborted transfer may not have let go.
  std::string unmatched_recv(size_t bytes) {
    void* p = t_->alloc(bytes);
    try {
      t_->group_begin();
      t_->recv(p, bytes, rank());
      t_->group_end();
      t_->sync();
    } catch (const Error& e) {
      return e.what();
    }
    t_->release(p);
    return "";
  }

  // Test hook for teardown: a receive from `peer` that no send matches,
  // posted and left pending (no sync); the session's destructor must still
  // end, bounded by its timeout (RcclTransport::drain_quietly).  The buffer is
  // leaked on purpose: an aborted transfer may not have let go of it.
  void post_unmatched_recv(size_t bytes, int peer) {
    void* p = t_->alloc(bytes);
    t_->group_begin();
    t_->recv(p, bytes, peer);
    t_->group_end();
  }

  // Test hook for the stream gate: arm one, release it or not, wait for the
  // stream.  An unreleased gate must open by itself at its deadline.
  std::string gate_probe(double timeout_s, bool release) {
    const double t0 = now_seconds();
    if (!t_->gate_arm(timeout_s)) return "{\"supported\":false}";
    if (release) t_->gate_release();
    t_->sync();
    const double waited = now_seconds() - t0;
    const bool expired = t_->gate_timed_out();
    if (!release) t_->gate_release();  // keep the sequence consistent for later gates
    return strfmt("{\"supported\":true,\"timed_out\":%s,\"seconds\":%.4f}", expired ? "true" : "false", waited);
  }

  std::string device_latency(size_t bytes, int iters, int warmup) {
    return latency_to_json(run_device_latency(*t_, *boot_, bytes, iters, warmup), world());
  }

  // Dependent ring token chain (runner.hpp run_ring_latency); device=true
  // runs it as the one-wave kernel of the IPC transport.
  std::string ring_latency(size_t bytes, int laps, int warmup, bool device) {
    if (device) return ring_latency_to_json(run_device_ring_latency(*t_, *boot_, bytes, laps, warmup));
    Buffers bufs(*t_, std::max<size_t>(bytes, 16), 1);
    return ring_latency_to_json(run_ring_latency(*t_, *boot_, bytes, laps, warmup, bufs));
  }

  // Bounds every later wait of this session (transport and bootstrap).
  void set_timeout(double seconds) {
    t_->set_timeout(seconds);
    boot_->set_timeout(seconds);
  }

  // Largest op a message is posted as (RCCL: 16 MiB per p2p channel, see
  // transport_rccl.cpp), capped on every rank alike.
  bool set_chunk_cap(size_t bytes) { return t_->set_chunk_cap(bytes); }
  size_t max_chunk(int peer) const { return t_->max_chunk(peer); }
  // Collective: re-derive the op limits from what the transport connected.
  bool refine_op_limits() { return t_->refine_op_limits(*boot_); }

  // Collective: every rank's Transport::link_report() as a JSON list (rank
  // order; null where the transport has nothing to report).
  std::string link_reports() {
    const auto all = boot_->allgather_string(t_->link_report());
    std::string o = "[";
    for (size_t r = 0; r < all.size(); ++r) o += (r ? "," : "") + (all[r].empty() ? std::string("null") : all[r]);
    return o + "]";
  }

  // Collective: provenance_json() for this session's ranks.
  std::string provenance(int device) { return provenance_json(*boot_, device); }

 private:
  std::unique_ptr<Bootstrap> boot_;
  std::unique_ptr<Transport> t_;
  std::string transport_kind_;
  uint64_t salt_ = 1000;
};

class PyStepDriver {
 public:
  PyStepDriver(std::shared_ptr<Session> s, const std::string& mode, const std::string& dir, size_t bytes, int msgs,
               bool verify, bool batch, bool graph, int depth, size_t recv_budget, uint64_t salt)
      : session_(std::move(s)),
        d_(std::make_unique<StepDriver>(session_->t(), session_->boot(),
                                        make_schedule(parse_mode(mode), parse_direction(dir), session_->world()),
                                        bytes, msgs, verify, salt, StepOptions{batch, graph, depth, recv_budget})) {}
  ~PyStepDriver() {
    teardown_outside_gil([this] {
      // Drain first (bounded): the driver's buffers are freed next.
      if (!session_->t().drain_quietly()) {
        (void)d_.release();  // leaked: kernels may still use its buffers
        return;
      }
      d_.reset();
    });
  }
  StepDriver& d() { return *d_; }

 private:
  std::shared_ptr<Session> session_;  // keeps transport alive
  std::unique_ptr<StepDriver> d_;
};

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

// Kernel entry points on raw device pointers (torch tensors' data_ptr()).
struct KernelScratch {
  dev::VerifyAccum* d = nullptr;
  dev::VerifyAccum* h = nullptr;
  int device = -1;
};
KernelScratch& scratch() {
  static KernelScratch s;
  int dv = 0;
  if (hipGetDevice(&dv) != hipSuccess) P2P_FATAL("no HIP device");
  if (s.device != dv) {
    if (s.d) (void)hipFree(s.d);
    if (s.h) (void)hipHostFree(s.h);
    if (hipMalloc(&s.d, dev::verify_accum_bytes()) != hipSuccess) P2P_FATAL("hipMalloc failed");
    if (hipHostMalloc(&s.h, sizeof(dev::VerifyAccum), hipHostMallocDefault) != hipSuccess) P2P_FATAL("hipHostMalloc failed");
    s.device = dv;
  }
  return s;
}

dev::VerifyImpl verify_impl_arg(int impl) {
  if (impl < 0 || impl > static_cast<int>(dev::VerifyImpl::Stride))
    throw py::value_error(strfmt("verify: impl %d is not 0 (auto), 1 (lds8) or 2 (stride); round 5 removed the "
                                 "other variants (parse_verify_impl names them)", impl));
  return static_cast<dev::VerifyImpl>(impl);
}

py::tuple device_verify(uintptr_t ptr, size_t bytes, uint64_t seed, int impl, bool check, uintptr_t stream) {
  const dev::VerifyImpl vi = verify_impl_arg(impl);
  KernelScratch& ks = scratch();
  hipStream_t st = as_stream(stream);
  {
    py::gil_scoped_release nogil;
    dev::launch_verify_reset(ks.d, st);
    dev::launch_verify(reinterpret_cast<const void*>(ptr), bytes, seed, ks.d, vi, check, st);
    if (hipMemcpyAsync(ks.h, ks.d, sizeof(dev::VerifyAccum), hipMemcpyDeviceToHost, st) != hipSuccess)
      P2P_FATAL("hipMemcpyAsync failed");
    if (hipStreamSynchronize(st) != hipSuccess) P2P_FATAL("hipStreamSynchronize failed");
  }
  return py::make_tuple(ks.h->mismatches, ks.h->checksum, ks.h->first_bad);
}

// The batched verify on raw pointers: [(mismatches, checksum, first_bad)]
// per (ptr, bytes, seed) job, one readback (dev::BatchVerifier, per device).
// The verifiers are never destroyed (like KernelScratch): a static
// destructor would free device memory after the HIP runtime shut down.
py::list device_verify_many(const std::vector<std::tuple<uintptr_t, size_t, uint64_t>>& jobs, uintptr_t stream) {
  static auto* per_device = new std::vector<dev::BatchVerifier*>();
  int dv = 0;
  if (hipGetDevice(&dv) != hipSuccess) P2P_FATAL("no HIP device");
  if (static_cast<int>(per_device->size()) <= dv) per_device->resize(static_cast<size_t>(dv) + 1, nullptr);
  dev::BatchVerifier*& bv = (*per_device)[static_cast<size_t>(dv)];
  if (!bv) bv = new dev::BatchVerifier();
  std::vector<dev::VerifyJob> dj;
  for (const auto& j : jobs) dj.push_back({reinterpret_cast<const void*>(std::get<0>(j)), std::get<1>(j), std::get<2>(j)});
  hipStream_t st = as_stream(stream);
  {
    py::gil_scoped_release nogil;
    bv->reserve(static_cast<int>(dj.size()), [st] {
      if (hipStreamSynchronize(st) != hipSuccess) P2P_FATAL("hipStreamSynchronize failed");
    });
    bv->enqueue(dj.data(), static_cast<int>(dj.size()), st);
    if (hipStreamSynchronize(st) != hipSuccess) P2P_FATAL("hipStreamSynchronize failed");
  }
  py::list out;
  for (size_t i = 0; i < dj.size(); ++i)
    out.append(py::make_tuple(bv->results()[i].mismatches, bv->results()[i].checksum, bv->results()[i].first_bad));
  return out;
}

// Stream-ordered batched verify, no readback (timing with events): the
// scratch and results live per device and grow with the job count.
void device_verify_many_launch(const std::vector<std::tuple<uintptr_t, size_t, uint64_t>>& jobs, uintptr_t stream) {
  struct Buffers {
    dev::VerifyAccum* scratch = nullptr;
    dev::VerifyAccum* out = nullptr;
    int cap = 0;
  };
  static std::vector<Buffers> per_device;
  int dv = 0;
  if (hipGetDevice(&dv) != hipSuccess) P2P_FATAL("no HIP device");
  if (static_cast<int>(per_device.size()) <= dv) per_device.resize(static_cast<size_t>(dv) + 1);
  Buffers& b = per_device[static_cast<size_t>(dv)];
  const int n = static_cast<int>(jobs.size());
  if (!b.scratch && hipMalloc(&b.scratch, dev::multi_verify_scratch_bytes()) != hipSuccess) P2P_FATAL("hipMalloc failed");
  if (n > b.cap) {
    if (hipStreamSynchronize(as_stream(stream)) != hipSuccess) P2P_FATAL("hipStreamSynchronize failed");
    if (b.out) (void)hipFree(b.out);
    b.cap = std::max(n, 2 * b.cap);
    if (hipMalloc(&b.out, sizeof(dev::VerifyAccum) * static_cast<size_t>(b.cap)) != hipSuccess) P2P_FATAL("hipMalloc failed");
  }
  std::vector<dev::VerifyJob> dj;
  for (const auto& j : jobs) dj.push_back({reinterpret_cast<const void*>(std::get<0>(j)), std::get<1>(j), std::get<2>(j)});
  dev::launch_multi_verify(dj.data(), n, b.scratch, b.out, as_stream(stream));
}

py::list schedule_py(const std::string& mode, const std::string& dir, int n) {
  Schedule s = make_schedule(parse_mode(mode), parse_direction(dir), n);
  py::list phases;
  for (const auto& p : s.phases) {
    py::dict d;
    d["label"] = p.label;
    d["row"] = p.row;
    d["col"] = p.col;
    d["idle"] = p.idle;
    py::list flows;
    for (const auto& f : p.flows) flows.append(py::make_tuple(f.src, f.dst));
    d["flows"] = flows;
    py::list ranks;
    for (const auto& r : p.ranks) ranks.append(py::make_tuple(r.send_to, r.recv_from));
    d["ranks"] = ranks;
    phases.append(d);
  }
  return phases;
}

}  // namespace

PYBIND11_MODULE(_p2pcore, m) {
  m.doc() = "MI355X-native P2P benchmark engine (RCCL over xGMI, gfx950 kernels)";
  set_throw_on_fatal(true);

  py::class_<TcpListener>(m, "TcpListener")
      .def(py::init<int, const std::string&>(), py::arg("port") = 0, py::arg("bind_addr") = "0.0.0.0")
      .def_property_readonly("port", &TcpListener::port);

  py::class_<Session, std::shared_ptr<Session>>(m, "Session")
      .def(py::init<int, int, const std::string&, int, int, const std::string&, double, TcpListener*>(), py::arg("rank"),
           py::arg("world"), py::arg("host") = "127.0.0.1", py::arg("port") = 0, py::arg("device") = 0,
           py::arg("transport") = "rccl", py::arg("timeout_s") = 300.0, py::arg("listener") = nullptr,
           py::call_guard<NativeCall, py::gil_scoped_release>())
      .def_property_readonly("rank", &Session::rank)
      .def_property_readonly("world", &Session::world)
      .def_property_readonly("transport", &Session::transport)
      .def_property_readonly("device_desc", &Session::device_desc)
      .def("barrier", &Session::barrier, py::call_guard<NativeCall, py::gil_scoped_release>())
      .def("allreduce_max", &Session::allreduce_max, py::call_guard<NativeCall, py::gil_scoped_release>())
      .def("allreduce_sum", &Session::allreduce_sum, py::call_guard<NativeCall, py::gil_scoped_release>())
      .def("run", &Session::run, py::arg("mode") = "pair", py::arg("dir") = "uni", py::arg("bytes") = 32u << 20,
           py::arg("iters") = 128, py::arg("warmup") = 8, py::arg("timing") = "events", py::arg("verify") = false,
           py::arg("warm") = true, py::arg("cells") = std::vector<std::pair<int, int>>{}, py::call_guard<NativeCall, py::gil_scoped_release>())
      .def("gate_probe", &Session::gate_probe, py::arg("timeout_s") = 0.2, py::arg("release") = true,
           py::call_guard<NativeCall, py::gil_scoped_release>())
      .def("device_latency", &Session::device_latency, py::arg("bytes") = 8, py::arg("iters") = 1000,
           py::arg("warmup") = 100, py::call_guard<NativeCall, py::gil_scoped_release>())
      .def("latency", &Session::latency, py::arg("bytes") = 8, py::arg("iters") = 1000, py::arg("warmup") = 100,
           py::arg("preposted") = 0, py::call_guard<NativeCall, py::gil_scoped_release>(),
           "Ping-pong matrix (collective).  preposted=B: exchanges posted B at a time behind a stream gate and "
           "released together (GPU-timeline latency; host-posted where the transport has no gate).")
      .def("fuzz", &Session::fuzz, py::arg("rounds") = 20, py::arg("seed") = 1, py::arg("max_bytes") = size_t{4} << 20,
           py::call_guard<NativeCall, py::gil_scoped_release>(),
           "Random groups of verified messages through the transport (collective); returns mismatching words.")
      .def("ring_latency", &Session::ring_latency, py::arg("bytes") = 8, py::arg("laps") = 200, py::arg("warmup") = 20,
           py::arg("device") = false, py::call_guard<NativeCall, py::gil_scoped_release>(),
           "Dependent ring token chain 0 -> 1 -> ... -> 0 (collective); JSON with per-hop and per-lap times.")
      .def("set_timeout", &Session::set_timeout, py::arg("seconds"),
           "Bounds every later wait of the session (transport sync / rendezvous, bootstrap receives).")
      .def("set_chunk_cap", &Session::set_chunk_cap, py::arg("bytes"),
           "Caps the ops messages to every peer are posted as at `bytes` (0: lifts the cap, back to the limits the "
           "transport derived per peer); False where nothing is split. Call it on every rank with the same value.")
      .def("max_chunk", &Session::max_chunk, py::arg("peer"), "Largest op a message to `peer` is posted as (0: unsplit).")
      .def("refine_op_limits", &Session::refine_op_limits, py::call_guard<NativeCall, py::gil_scoped_release>(),
           "Collective: op limits from the connections made so far (RCCL: its connection lines).")
      .def("link_reports", &Session::link_reports, py::call_guard<NativeCall, py::gil_scoped_release>(),
           "Collective: what the data plane set up towards each peer, per rank (RCCL: p2p channels from its INFO log, "
           "each peer's transport, the op limit in use); JSON list.")
      .def("provenance", &Session::provenance, py::arg("device") = -1, py::call_guard<NativeCall, py::gil_scoped_release>(),
           "Collective: runtime, RCCL library, knobs, every rank's GPU and the links between them (JSON).")
      .def("_post_unmatched_recv", &Session::post_unmatched_recv, py::arg("bytes"), py::arg("peer"),
           py::call_guard<NativeCall, py::gil_scoped_release>(),
           "Test hook: a receive no send matches, left pending; the session's teardown must still end.")
      .def("_unmatched_recv", &Session::unmatched_recv, py::arg("bytes") = size_t{1} << 20,
           py::call_guard<NativeCall, py::gil_scoped_release>(), "Test hook: a receive no send matches; returns the watchdog's error.");

  py::class_<PyStepDriver>(m, "StepDriver")
      .def(py::init<std::shared_ptr<Session>, const std::string&, const std::string&, size_t, int, bool, bool, bool, int,
                    size_t, uint64_t>(),
           py::arg("session"), py::arg("mode") = "tournament", py::arg("dir") = "bi", py::arg("bytes") = 32u << 20,
           py::arg("msgs") = 8, py::arg("verify") = false, py::arg("batch") = false, py::arg("graph") = false,
           py::arg("depth") = 1, py::arg("recv_budget") = size_t{0}, py::arg("salt") = uint64_t{0},
           py::call_guard<NativeCall, py::gil_scoped_release>())
      .def("poison", [](PyStepDriver& s) { s.d().poison(); }, py::call_guard<NativeCall, py::gil_scoped_release>(),
           "Collective: zero every receive slot (after the warmup, before the timed steps) and arm the skip faults.")
      .def("clear", [](PyStepDriver& s) { s.d().clear(); }, py::call_guard<NativeCall, py::gil_scoped_release>(),
           "Collective: zero every receive slot once every rank has drained (no fault armed).")
      .def("recapture", [](PyStepDriver& s) { s.d().recapture(); }, py::call_guard<NativeCall, py::gil_scoped_release>(),
           "Collective: record the step graphs again after the op sizes changed (no-op without graphs).")
      .def_property_readonly("recaptures", [](PyStepDriver& s) { return s.d().recaptures(); })
      .def_property_readonly("limit_changes", [](PyStepDriver& s) { return s.d().limit_changes(); })
      .def_property_readonly("graphs", [](PyStepDriver& s) { return s.d().graphs(); })
      .def("verify_steps", [](PyStepDriver& s, long first, long count) {
            StepVerifyReport r;
            {
              NativeCall in_engine;
              py::gil_scoped_release nogil;
              r = s.d().verify_steps(first, count);
            }
            py::dict d;
            d["mismatches"] = r.mismatches;
            d["verified_msgs"] = r.verified_msgs;
            d["timed_msgs"] = r.timed_msgs;
            d["slots"] = r.slots;
            return d;
          }, py::arg("first"), py::arg("count"),
           "Collective: checks every receive slot steps [first, first+count) wrote (all ranks' totals).")
      .def("flows_per_step", [](PyStepDriver& s, long k) { return s.d().flows_per_step(k); })
      .def_property_readonly("depth", [](PyStepDriver& s) { return s.d().depth(); })
      .def_property_readonly("msgs", [](PyStepDriver& s) { return s.d().msgs(); })
      .def_property_readonly("recv_bytes", [](PyStepDriver& s) { return s.d().recv_bytes(); })
      .def("connect", [](PyStepDriver& s) { s.d().connect(); }, py::call_guard<NativeCall, py::gil_scoped_release>())
      .def("step", [](PyStepDriver& s, long k) { s.d().step(k); }, py::call_guard<NativeCall, py::gil_scoped_release>())
      .def("run_steps", [](PyStepDriver& s, long first, long count) { s.d().run_steps(first, count); },
           py::call_guard<NativeCall, py::gil_scoped_release>(),
           "Enqueue steps [first, first+count); consecutive steps share their boundary timestamp.")
      .def("sync", [](PyStepDriver& s) { s.d().sync(); }, py::call_guard<NativeCall, py::gil_scoped_release>())
      .def("step_ms", [](PyStepDriver& s) { return s.d().step_ms(); })
      .def("post_ms", [](PyStepDriver& s) { return s.d().post_ms(); },
           "Host time each recorded step took to post (ms).")
      .def("reset", [](PyStepDriver& s) { s.d().reset(); })
      .def("verify_last", [](PyStepDriver& s) { return s.d().verify_last(); }, py::call_guard<NativeCall, py::gil_scoped_release>())
      .def("bytes_sent_per_step", [](PyStepDriver& s, long k) { return s.d().bytes_sent_per_step(k); })
      .def("job_bytes_per_step", [](PyStepDriver& s, long k) { return s.d().job_bytes_per_step(k); })
      .def_property_readonly("phases", [](PyStepDriver& s) { return s.d().phases(); })
      .def("phase_flows", [](PyStepDriver& s, long k) {
        const auto& p = s.d().schedule().phases[static_cast<size_t>(k % s.d().phases())];
        std::vector<std::pair<int, int>> f;
        for (auto& x : p.flows) f.emplace_back(x.src, x.dst);
        return f;
      });

  // ---- kernels on raw pointers ----
  m.def("fill", [](uintptr_t ptr, size_t bytes, uint64_t seed, uintptr_t stream, int impl) {
        if (impl >= 2 && impl <= 6)
          throw py::value_error(strfmt("fill: impl %d (non-temporal / grid-stride / XCD-ordered / 2 or 4 stores per "
                                       "lane) was removed in round 5: it lost its A/B against the full grid "
                                       "(profiles/r3b_nt_ab/, r4_gpu_tier/); use 0 or 1", impl));
        if (impl < 0 || impl > static_cast<int>(dev::FillImpl::Grid)) throw py::value_error("fill: unknown impl");
        dev::launch_fill(reinterpret_cast<void*>(ptr), bytes, seed, as_stream(stream), static_cast<dev::FillImpl>(impl));
      }, py::arg("ptr"), py::arg("bytes"), py::arg("seed"), py::arg("stream") = 0, py::arg("impl") = 0,
      "impl: 0 auto = 1 full grid (one 16 B store per lane, one 4 KiB block per workgroup)");
  m.def("verify", &device_verify, py::arg("ptr"), py::arg("bytes"), py::arg("seed"), py::arg("impl") = 0,
        py::arg("check") = true, py::arg("stream") = 0,
        "impl: 0 auto (= 1), 1 LDS-DMA staged (lds8), 2 register staged (stride).  Returns (mismatching words, "
        "checksum, first bad byte offset or 2**64-1).");
  m.def("verify_many", &device_verify_many, py::arg("jobs"), py::arg("stream") = 0,
        "Batched verify of [(ptr, bytes, seed)]: one (mismatches, checksum, first_bad) per job, one readback.");
  m.def("verify_many_launch", &device_verify_many_launch, py::arg("jobs"), py::arg("stream") = 0,
        "Stream-ordered batched verify launches only (timing).");
  m.def("verify_launch", [](uintptr_t ptr, size_t bytes, uint64_t seed, int impl, bool check, uintptr_t stream,
                            unsigned max_grid) {
        // Stream-ordered launch only (reset + verify + finalize), no readback:
        // for timing the kernel with events.
        const dev::VerifyImpl vi = verify_impl_arg(impl);
        KernelScratch& ks = scratch();
        dev::launch_verify_reset(ks.d, as_stream(stream));
        dev::launch_verify(reinterpret_cast<const void*>(ptr), bytes, seed, ks.d, vi, check, as_stream(stream), max_grid);
      }, py::arg("ptr"), py::arg("bytes"), py::arg("seed"), py::arg("impl") = 0, py::arg("check") = true,
      py::arg("stream") = 0, py::arg("max_grid") = 0);
  m.def("copy", [](uintptr_t dst, uintptr_t src, size_t bytes, uintptr_t stream, int max_blocks, bool coherent) {
        dev::CopyOp op{reinterpret_cast<const void*>(src), reinterpret_cast<void*>(dst), bytes, coherent};
        dev::launch_multi_copy(&op, 1, as_stream(stream), max_blocks);
      }, py::arg("dst"), py::arg("src"), py::arg("bytes"), py::arg("stream") = 0, py::arg("max_blocks") = 0,
      py::arg("coherent") = false,
      "The IPC transport's gfx950 copy kernel on one (dst, src) pair (coherent: the cross-GPU form with "
      "system-scope sc0 sc1 buffer loads and stores).");
  m.def("copy_many", [](const std::vector<std::tuple<uintptr_t, uintptr_t, size_t>>& ops, uintptr_t stream,
                        bool coherent) {
        std::vector<dev::CopyOp> v;
        for (const auto& o : ops)
          v.push_back({reinterpret_cast<const void*>(std::get<1>(o)), reinterpret_cast<void*>(std::get<0>(o)),
                       std::get<2>(o), coherent});
        dev::launch_multi_copy(v.data(), static_cast<int>(v.size()), as_stream(stream));
      }, py::arg("ops"), py::arg("stream") = 0, py::arg("coherent") = false,
      "The copy kernel over several (dst, src, bytes) ops, as the IPC transport launches a group's receives.");
  m.def("fill_geometry", [](size_t bytes) {
    auto g = dev::fill_geometry(bytes);
    return py::make_tuple(g.grid, g.block, g.lds_bytes);
  });
  m.def("verify_geometry", [](size_t bytes, int impl) {
    auto g = dev::verify_geometry(bytes, verify_impl_arg(impl));
    return py::make_tuple(g.grid, g.block, g.lds_bytes);
  });
  m.def("rccl_available", &rccl_transport_available);
  m.def("runtime_json", &runtime_json, "HIP runtime / RCCL library versions and paths, visible devices and links.");
  m.def("env_knobs_json", &env_knobs_json, "Every NCCL_/RCCL_/HSA_/HIP_/GPU_... environment knob that is set.");
  m.def("request_abort", []() { request_abort(); },
        "Ask every transport wait of this process to abort its communicators on its own thread and fail.");
  m.def("abort_requested", []() { return abort_requested(); });
  m.def("abort_done", []() { return abort_done(); },
        "True once a transport wait has aborted its communicators after request_abort().");
  m.def("abort_if_idle", &abort_if_idle, py::call_guard<py::gil_scoped_release>(),
        "Watchdog: when no thread is inside the engine, abort every communicator from this thread, take no more "
        "engine calls and note the abort done; False (nothing done) while a call is in flight.  Releases the GIL "
        "(and holds no engine lock) while the aborts run, so a blocking abort stalls no other thread.");
  m.def("_push_blocking_abort_hook", [](double seconds) {
        push_abort_hook([seconds](int) { std::this_thread::sleep_for(std::chrono::duration<double>(seconds)); });
      }, py::arg("seconds"),
      "Test hook: an abort hook that blocks for `seconds` (an ncclCommAbort that does not return).");
  m.def("run_abort_hooks", []() { run_abort_hooks(1); }, py::call_guard<py::gil_scoped_release>(),
        "Aborts every live RCCL communicator / bootstrap (their kernels exit); for a watchdog about to end the "
        "process.");

  // ---- host reference (bit-compatible with the kernels) ----
  m.def("host_fill", [](size_t bytes, uint64_t seed) {
    std::string out(bytes, '\0');
    host_fill(&out[0], bytes, seed);
    return py::bytes(out);
  });
  m.def("host_verify", [](py::bytes data, uint64_t seed) {
    std::string s = data;
    VerifyResult r = host_verify(s.data(), s.size(), seed);
    return py::make_tuple(r.mismatches, r.checksum, r.first_bad);
  });
  m.def("prng_word", &prng_word);
  m.def("payload_seed", &payload_seed);

  // ---- pure host helpers ----
  m.def("schedule", &schedule_py, py::arg("mode"), py::arg("dir"), py::arg("n"));
  m.def("round_robin_rounds", &round_robin_rounds);
  m.def("plan_routes",
        [](int n, const std::vector<std::pair<int, int>>& flows, size_t bytes, size_t min_bytes, double relay_weight,
           int max_relays) {
          RouteOptions o;
          o.min_bytes = min_bytes;
          o.relay_weight = relay_weight;
          o.max_relays = max_relays;
          py::list out;
          for (const auto& stripes : plan_routes(n, flows, bytes, o)) {
            py::list l;
            for (const auto& st : stripes) l.append(py::make_tuple(st.via, st.offset, st.bytes));
            out.append(l);
          }
          return out;
        },
        py::arg("n"), py::arg("flows"), py::arg("bytes"), py::arg("min_bytes") = size_t{1} << 20,
        py::arg("relay_weight") = 1.0, py::arg("max_relays") = -1,
        "The relay engine's split of each flow of a group: [(via, offset, bytes), ...] per flow, direct stripe "
        "first (via = -1).");
  m.def("parse_size", &parse_size);
  m.def("parse_size_list", &parse_size_list);
  m.def("format_size", &format_size);
  m.def("host_hash", &host_hash);
  m.def("compute_placement", [](const std::vector<uint64_t>& h, int rank) {
    Placement p = compute_placement(h, rank);
    py::dict d;
    d["ok"] = p.ok;
    d["error"] = p.error;
    d["num_hosts"] = p.num_hosts;
    d["ranks_per_host"] = p.ranks_per_host;
    d["local_rank"] = p.local_rank;
    return d;
  });
  m.def("usage", &usage_text);
  m.def("parse_verify_impl", [](const std::string& name) {
        std::string note;
        const int v = parse_verify_impl(name, &note);
        if (v < 0) throw py::value_error("verify impl '" + name + "': " + note);
        return v;
      }, py::arg("name"), "Verify kernel name -> impl number (auto 0, lds8 1, stride 2), as p2p_matrix --verify-impl.");
  // The full p2p_matrix application in-process (TCP/env or local bootstrap),
  // e.g. `torchrun --nproc-per-node 8 -m test_nccl_p2p_amd --mode all`.
  m.def("run_cli", [](std::vector<std::string> args) {
    std::vector<char*> argv;
    for (auto& a : args) argv.push_back(&a[0]);
    AppConfig cfg;
    int code = 0;
    if (!parse_cli(static_cast<int>(argv.size()), argv.data(), &cfg, &code)) return code;
    // In the engine for the whole app: a watchdog's abort_if_idle
    // must not abort its communicators from another thread meanwhile.  Taken
    // with the GIL held, like every binding's NativeCall.
    NativeCall in_engine;
    py::gil_scoped_release nogil;
    std::string kind = cfg.bootstrap == "mpi" ? "env" : cfg.bootstrap;
    auto boot = make_bootstrap(kind, nullptr, nullptr);
    return run_app(cfg, *boot, stdout);
  }, py::arg("args"));
}
