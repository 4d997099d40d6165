#include "common.hpp"

#include <atomic>

#include <dlfcn.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

namespace p2p {

namespace {
std::mutex g_hook_mu;
std::vector<std::pair<int, AbortHook>>& hooks() {
  static std::vector<std::pair<int, AbortHook>> h;
  return h;
}
int g_next_hook = 1;
bool g_throw = false;
std::atomic<bool> g_abort_requested{false};
std::atomic<bool> g_abort_done{false};
std::atomic<int> g_log_level{-1};  // read by every thread that logs
}  // namespace

int push_abort_hook(AbortHook hook) {
  std::lock_guard<std::mutex> lk(g_hook_mu);
  int id = g_next_hook++;
  hooks().emplace_back(id, std::move(hook));
  return id;
}

void remove_abort_hook(int handle) {
  std::lock_guard<std::mutex> lk(g_hook_mu);
  auto& h = hooks();
  for (auto it = h.begin(); it != h.end(); ++it)
    if (it->first == handle) {
      h.erase(it);
      return;
    }
}

void clear_abort_hooks() {
  std::lock_guard<std::mutex> lk(g_hook_mu);
  hooks().clear();
}

void run_abort_hooks(int code) {
  std::vector<std::pair<int, AbortHook>> hs;
  {
    std::lock_guard<std::mutex> lk(g_hook_mu);
    hs.swap(hooks());
  }
  for (auto it = hs.rbegin(); it != hs.rend(); ++it) it->second(code);
}

void set_throw_on_fatal(bool enable) { g_throw = enable; }

namespace {
std::mutex g_call_mu;
int g_calls = 0;        // NativeCalls open
bool g_closed = false;  // abort_if_idle ran: the engine takes no more calls
}  // namespace

NativeCall::NativeCall() {
  std::lock_guard<std::mutex> lk(g_call_mu);
  if (g_closed) P2P_FATAL("the engine was aborted (the run's deadline passed)");
  ++g_calls;
  entered_ = true;
}

NativeCall::NativeCall(std::nothrow_t) {
  std::lock_guard<std::mutex> lk(g_call_mu);
  if (g_closed) return;
  ++g_calls;
  entered_ = true;
}

NativeCall::~NativeCall() {
  if (!entered_) return;
  std::lock_guard<std::mutex> lk(g_call_mu);
  --g_calls;
}

bool abort_if_idle() {
  {
    std::lock_guard<std::mutex> lk(g_call_mu);
    if (g_calls > 0) return false;
    g_closed = true;  // from here on every call is refused: none can enter while the hooks run
  }
  // The hooks run without g_call_mu: one that blocks
  // (ncclCommAbort on a kernel that never exits, a stuck proxy thread) must
  // not also stall every thread that tries to enter the engine; those are
  // refused at once.  The bindings release the GIL around this call, so the
  // bench watchdog's hard exit does not wait for it either.
  run_abort_hooks(1);
  note_abort_done();
  return true;
}

void abort_wait(const char* who) {
  note_abort_done();
  P2P_FATAL(strfmt("%s: wait aborted (the run's deadline passed)", who));
}

void request_abort() { g_abort_requested.store(true, std::memory_order_relaxed); }
bool abort_requested() { return g_abort_requested.load(std::memory_order_relaxed); }
void note_abort_done() { g_abort_done.store(true, std::memory_order_release); }
bool abort_done() { return g_abort_done.load(std::memory_order_acquire); }

void fatal(const char* file, int line, const std::string& what) {
  std::string msg = strfmt("p2p fatal error at %s:%d: %s", file, line, what.c_str());
  if (g_throw) throw Error(msg);
  std::fprintf(stderr, "%s\n", msg.c_str());
  std::fflush(stderr);
  std::vector<std::pair<int, AbortHook>> hs;
  {
    std::lock_guard<std::mutex> lk(g_hook_mu);
    hs.swap(hooks());
  }
  // Innermost (most recently installed) first: transport before bootstrap.
  for (auto it = hs.rbegin(); it != hs.rend(); ++it) it->second(EXIT_FAILURE);
  std::exit(EXIT_FAILURE);
}

std::string strfmt(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  va_list ap2;
  va_copy(ap2, ap);
  int n = std::vsnprintf(nullptr, 0, fmt, ap);
  va_end(ap);
  std::string out(n > 0 ? static_cast<size_t>(n) : 0, '\0');
  if (n > 0) std::vsnprintf(&out[0], static_cast<size_t>(n) + 1, fmt, ap2);
  va_end(ap2);
  return out;
}

int log_level() {
  int level = g_log_level.load(std::memory_order_relaxed);
  if (level < 0) {
    const char* e = std::getenv("P2P_LOG");
    int env_level = e ? std::atoi(e) : 0;
    // First caller wins; set_log_level may have run in between.
    if (g_log_level.compare_exchange_strong(level, env_level, std::memory_order_relaxed)) level = env_level;
  }
  return level;
}

void set_log_level(int level) { g_log_level.store(level, std::memory_order_relaxed); }

void logf(int level, const char* fmt, ...) {
  if (log_level() < level) return;
  va_list ap;
  va_start(ap, fmt);
  std::fprintf(stderr, "[p2p] ");
  std::vfprintf(stderr, fmt, ap);
  std::fprintf(stderr, "\n");
  va_end(ap);
}

namespace {

struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
  bool enabled = false;
};

Roctx& roctx() {
  static Roctx r = [] {
    Roctx x;
    const char* e = std::getenv("P2P_ROCTX");
    if (!e || std::atoi(e) == 0) return x;
    void* h = nullptr;
    // rocprofv3 (rocprofiler-sdk) records the markers of its own roctx
    // library; the legacy roctracer libroctx64 is only a fallback for the
    // older tools.
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", "libroctx64.so",
                            "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"}) {
      h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
      if (h) {
        std::fprintf(stderr, "[p2p] roctx ranges via %s\n", lib);
        break;
      }
    }
    if (!h) {
      std::fprintf(stderr, "[p2p] P2P_ROCTX=1 but no roctx library could be loaded; tracing disabled\n");
      return x;
    }
    x.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
    x.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    x.mark = reinterpret_cast<void (*)(const char*)>(dlsym(h, "roctxMarkA"));
    x.enabled = x.push && x.pop;
    return x;
  }();
  return r;
}

}  // namespace

void trace_push(const char* name) {
  if (roctx().enabled) roctx().push(name);
}

void trace_pop() {
  if (roctx().enabled) roctx().pop();
}

void trace_mark(const char* name) {
  if (roctx().enabled && roctx().mark) roctx().mark(name);
}

double now_seconds() {
  using clk = std::chrono::steady_clock;
  return std::chrono::duration<double>(clk::now().time_since_epoch()).count();
}

void emulate_link_delay(const std::vector<size_t>& send_bytes, int me) {
  static const double gbs = [] {
    const char* v = std::getenv("P2P_EMULATE_LINK_GBS");
    return v ? std::atof(v) : 0.0;
  }();
  if (gbs <= 0) return;
  size_t most = 0;
  for (size_t p = 0; p < send_bytes.size(); ++p)
    if (static_cast<int>(p) != me) most = std::max(most, send_bytes[p]);
  if (most == 0) return;
  const double until = now_seconds() + static_cast<double>(most) / (gbs * 1e9);
  while (now_seconds() < until) std::this_thread::sleep_for(std::chrono::microseconds(20));
}

StdoutToStderr::StdoutToStderr(bool enable) {
  if (!enable) return;
  std::fflush(stdout);
  saved_ = dup(1);
  if (saved_ >= 0 && dup2(2, 1) < 0) {
    close(saved_);
    saved_ = -1;
  }
}

StdoutToStderr::~StdoutToStderr() {
  if (saved_ < 0) return;
  std::fflush(stdout);
  dup2(saved_, 1);
  close(saved_);
}

}  // namespace p2p
