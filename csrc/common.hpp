// Error policy, logging and small shared helpers for the p2p framework.
//
// Reference parity: the reference's MPICHECK / CUDACHECK / NCCLCHECK macros
// (/root/reference/p2p_matrix.cc:15-42) print to *stdout* and call exit()
// without telling the peers, so a failing rank leaves every other rank blocked
// in a barrier or a stream sync forever.  Here every check
// routes through p2p::fatal(), which prints to stderr and then runs the
// registered abort hook (MPI_Abort / ncclCommAbort / closing the TCP mesh) so
// the whole job goes down together.
#pragma once

#include <cstdint>
#include <cstdio>
#include <functional>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

namespace p2p {

// Called once by fatal() before the process exits.  Bootstraps and transports
// install hooks so that an error on one rank aborts the job instead of hanging.
using AbortHook = std::function<void(int code)>;
int push_abort_hook(AbortHook hook);  // returns a handle for remove_abort_hook
void remove_abort_hook(int handle);
void clear_abort_hooks();
// Runs (and removes) every registered hook, innermost first, without exiting:
// a watchdog that must end the process calls it so RCCL communicators are
// aborted (their kernels exit) before the process goes.
void run_abort_hooks(int code);
// Cooperative abort from another thread (bench.py's deadline watchdog): the
// transports' bounded waits poll abort_requested() and, on the thread that
// owns the communicators, abort them and fail.  Aborting a communicator from
// a second thread while its owner is inside RCCL crashed the owner (SIGSEGV,
// profiles/r4_rehearsal/); this keeps every RCCL call on one thread.
void request_abort();
bool abort_requested();
// Set by a transport once it has aborted its communicators on request.
void note_abort_done();
bool abort_done();
// The other half of the cooperative abort: a thread that is not
// inside the engine at all -- the main thread in a gloo barrier, a torch sync
// or plain Python -- never reaches a polling wait.  Every binding that can
// touch a communicator holds a NativeCall while it runs; abort_if_idle(),
// called by the watchdog, runs the abort hooks on its own thread only when
// no NativeCall is open (so no RCCL call can be running), refuses every
// later NativeCall and notes the abort done.  Returns false (nothing done)
// while a call is in flight.
class NativeCall {
 public:
  NativeCall();  // fatal (throws under the bindings) once the engine is closed
  // Never throws (destructors): entered() is false once the engine is closed.
  explicit NativeCall(std::nothrow_t);
  ~NativeCall();
  bool entered() const { return entered_; }
  NativeCall(const NativeCall&) = delete;
  NativeCall& operator=(const NativeCall&) = delete;

 private:
  bool entered_ = false;
};
bool abort_if_idle();
// A CPU transport's wait that saw abort_requested(): nothing to abort but the
// wait itself; notes the abort done and fails.
[[noreturn]] void abort_wait(const char* who);

[[noreturn]] void fatal(const char* file, int line, const std::string& what);

// When set (Python bindings), fatal() throws p2p::Error instead of exiting.
void set_throw_on_fatal(bool enable);

struct Error : public std::runtime_error {
  using std::runtime_error::runtime_error;
};

// printf-style std::string formatting.
std::string strfmt(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

// Verbosity: 0 quiet, 1 info, 2 debug.  Set from P2P_LOG / --verbose.
int log_level();
void set_log_level(int level);
void logf(int level, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

double now_seconds();  // monotonic (steady_clock), unlike the reference's system_clock

// Link-rate emulation for the CPU transports (P2P_EMULATE_LINK_GBS=<GB/s>, 0 or
// unset: off).  A group waits, before it moves any byte, as long as its
// busiest peer link would take at that rate (every peer its own full-duplex
// link, as on xGMI; self copies are free), so a CPU rehearsal with scaled-down
// sizes takes the time a node would (tests/test_torchrun_cpu.py).
// `send_bytes[p]` = bytes this rank sends to rank p in the group.
void emulate_link_delay(const std::vector<size_t>& send_bytes, int me);

// roctx ranges (visible in rocprofv3 --marker-trace / roctracer timelines).
// libroctx64 is dlopen'ed on first use and only when P2P_ROCTX=1, so nothing
// links against it and untraced runs pay nothing.
void trace_push(const char* name);
void trace_pop();
void trace_mark(const char* name);

// RAII helper.
struct TraceRange {
  explicit TraceRange(const char* name) { trace_push(name); }
  ~TraceRange() { trace_pop(); }
};

// While alive, file descriptor 1 points at stderr.  Libraries that print
// banners to stdout during init (RCCL prints its version block) would
// otherwise land in front of the reference-compatible matrices of a
// `mpirun ... > result.txt` run.  Inactive if `enable` is false.
class StdoutToStderr {
 public:
  explicit StdoutToStderr(bool enable = true);
  ~StdoutToStderr();
  StdoutToStderr(const StdoutToStderr&) = delete;
  StdoutToStderr& operator=(const StdoutToStderr&) = delete;

 private:
  int saved_ = -1;
};

}  // namespace p2p

#define P2P_FATAL(msg) ::p2p::fatal(__FILE__, __LINE__, (msg))

#define P2P_CHECK(cond, msg)                                             \
  do {                                                                   \
    if (!(cond)) ::p2p::fatal(__FILE__, __LINE__, std::string("check failed: " #cond ": ") + (msg)); \
  } while (0)

#define P2P_INFO(...) ::p2p::logf(1, __VA_ARGS__)
#define P2P_DEBUG(...) ::p2p::logf(2, __VA_ARGS__)
