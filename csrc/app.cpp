#include "app.hpp"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>

#include "bootstrap.hpp"
#include "common.hpp"
#include "provenance.hpp"
#include "rccl_log.hpp"
#include "report.hpp"
#include "topology.hpp"
#include "transport.hpp"
#include "units.hpp"

namespace p2p {

int parse_verify_impl(const std::string& v, std::string* note) {
  if (v == "auto") return 0;
  if (v == "lds8" || v == "lds") return 1;
  if (v == "stride" || v == "reg" || v == "register") return 2;
  // Variants that lost their A/B against lds8 / stride and were removed in
  // round 5 (their measurements stay in profiles/).
  static const char* const kRemoved[][2] = {
      {"lds-cached", "profiles/r1_tuned/ (5.7-5.9 TB/s, default-cache LDS-DMA)"},
      {"lds-pipe", "profiles/r1_tuned/ (pipelined LDS loop, no gain)"},
      {"lds8-span", "profiles/r4_verify_span/ (per-workgroup spans, no gain)"},
      {"grid", "profiles/r1_tuned/ (full-grid register loop, 5.6-6.4 TB/s)"},
  };
  for (const auto& r : kRemoved)
    if (v == r[0]) {
      if (note) *note = strfmt("removed in round 5: it lost its A/B (%s); use lds8 or stride", r[1]);
      return -2;
    }
  if (note) *note = "unknown (auto | lds8 | stride; see --help)";
  return -1;
}

std::string usage_text() {
  return R"(p2p_matrix — MI355X inter-GPU point-to-point bandwidth / latency matrix (RCCL over xGMI)

usage: mpirun -n N ./p2p_matrix [options]          (reference-compatible launch)
       torchrun --nproc-per-node N ... ./p2p_matrix   (RANK/WORLD_SIZE/MASTER_ADDR bootstrap)
       ./p2p_matrix [options]                         (single rank: self path)

With no options: serial pair schedule, uni then bi, 32 MiB x 128 per cell, printed
exactly like the reference, followed by GB/s and per-message latency tables.

schedule
  -m, --mode LIST        pair | ring | allpairs | tournament | self | all   [pair]
                           pair       ordered pairs one at a time (reference schedule)
                           ring       r -> r+1 concurrently (PP hop pattern)
                           allpairs   every rank to every peer in one group (EP all-to-all)
                           tournament N-1 rounds of disjoint pairs (whole matrix, concurrent)
                           self       every rank to itself (1-GPU path)
  -d, --dir uni|bi|both  direction(s)                                         [both]
  -b, --size SIZE        message size, e.g. 4K 32M 1G                         [32M]
      --sizes LIST       sweep: 4K:4G (x2 steps), 4K:1G:4 (x4), 4K,1M,... ; overrides --size
      --cells LIST       pair mode: measure only these src-dst cells, e.g. 0-1,3-2 (others print 0.00)
timing
  -n, --iters N|auto     iterations per cell (auto: ~4 GiB per cell, 8..1000) [128]
  -w, --warmup N         untimed iterations per cell                          [8]
      --repeat R         run every (mode, dir, size) R times; the reference matrices print
                         the first run as it goes, then a repeat summary gives every run's
                         mean cell and their median / min / max (one wall-clock run of
                         the reference's method is a single noisy shot)       [1]
      --timing MODE      events    hipEvents, back-to-back messages, 1 sync  [events]
                         wallclock reference semantics: host clock, sync per message
      --reference        = --timing wallclock --warmup 0 --no-warm --two-streams, and RCCL's
                         own kernel unroll (P2P_RCCL_UNROLL is not applied): the reference's
                         methodology on a stock RCCL setup, p2p_matrix.cc:141-267; and its
                         buffers: one send and one receive region reused by every
                         iteration (:124-130), so --verify checks the last delivery
      --two-streams      RCCL: a receive posted in a group with a send goes on a second
                         stream, like the reference's bi loop (s_1); alone it stays on the first (its uni loop)
      --comms K          RCCL: K communicators per rank on K streams; the i-th message
                         of >= 1 MiB from a to b uses communicator (i + a + b) mod K on both
                         ends, smaller messages stay on the first (P2P_RCCL_SPLIT_MIN)  [1]
      --no-warm          do not pre-establish connections before timing
  -l, --latency          add a ping-pong latency matrix (with --mode ring also the dependent
                         ring token chain: per-hop latency of a pipeline 0 -> 1 -> ... -> 0)
      --device-latency   add a device-initiated ping-pong matrix (--transport ipc:
                         one wave per GPU writes into the peer's memory, no host
                         or runtime in the loop)
      --latency-preposted B  also the ping-pong posted B exchanges at a time behind a
                         stream gate (GPU transports), released together: the
                         operation's GPU-timeline latency without the host's posting
                         rate in it                                          [off]
      --latency-size S   [8]      --latency-iters N   [1000]
      --fuzz N           data-integrity stress: N groups of random messages (random
                         pairs incl. self, sizes 1 B .. the largest --size, at most
                         64 MiB), every one verified; failures exit 2
data
  -c, --verify           random-fill sends, verify every received buffer on the device,
                         outside the timed loop (the default)
      --no-verify        zero-filled sends, nothing read back (the reference's data)
      --verify-impl I    auto (= lds8) | lds8 (alias lds) | stride (alias reg)
                         (LDS-DMA- or register-staged verify kernel)
transport / launch
      --transport T      rccl  MI355X + RCCL ncclSend/ncclRecv over xGMI      [rccl]
                         ipc   one-sided pulls from hipIpc-mapped peer buffers (gfx950 copy
                               kernel or SDMA); ranks may share a GPU
                         host  CPU sockets, no GPU
                         shm   CPU shared-memory rings (one host), no GPU
      --ipc-engine E     kernel | sdma | push | relay (for --transport ipc)    [kernel]
                         kernel/sdma: one-sided pull of the peer's send buffer;
                         push: rendezvous + remote writes into the peer's slot;
                         relay: push, with stripes of each message routed
                         s -> k -> d through GPUs whose links are idle
                         (P2P_RELAY_MIN [1M], P2P_RELAY_WEIGHT [1], P2P_RELAY_MAX)
      --bootstrap B      auto | mpi | env | local                              [auto]
      --device N         GPU index (default: local rank from block placement)
      --timeout S        watchdog for init / waits, seconds                    [300]
      --min-gbs X        link check: exit 3 naming every off-diagonal flow below
                         X GB/s (use with the message size the check is for)
output
      --json FILE        JSON lines, one object per run, appended + flushed as each run ends
      --resume           skip the runs already in the --json file (restart a killed sweep;
                         with --repeat R, run only the repeats it is missing)
      --trace FILE       Chrome/Perfetto trace of every rank's timed phases
                         (P2P_ROCTX=1 also emits roctx ranges for rocprofv3 --marker-trace)
      --csv FILE         per-flow CSV
      --compat-only      only the reference matrices
      --no-compat        only the extended tables
      --dry-run          print the schedules and exit
      --topology         print the GPU link matrix (xGMI/PCIe, hops, peer access) and exit
  -v, --verbose          -h, --help      --version
environment (recorded in every --json provenance record; docs/OUTPUT.md)
  P2P_RCCL_MAX_CHUNK=B   RCCL: messages above B are posted as B-byte ops in one group, every peer
                         [16M x the p2p channels RCCL set up for the peer; 0 off]
  P2P_RCCL_UNROLL=U      RCCL kernels' unroll factor (RCCL_UNROLL_FACTOR unless the user set it;
                         0: RCCL's own choice, 1 on MI355X)                        [4]
  P2P_RCCL_LOG=0|keep    RCCL's INFO log (channels, transports per peer) is captured into a private
                         file unless NCCL_DEBUG asks for it on stderr; 0: off, keep: keep the file
  P2P_RECHUNK=0          --verify: a warmup that does not verify is reported, not retried with
                         smaller ops                                               [1]
  P2P_VERIFY_BUDGET=B    --verify: bytes of receive generations (one per timed iteration)
                         [free HBM / 4, <= 32G]
  P2P_RCCL_SPLIT_MIN=B   --comms: smaller messages stay on communicator 0       [1M]
  P2P_RCCL_REGISTER=1|2  ncclCommRegister every buffer (2: + ncclMemAlloc)
  P2P_RCCL_BLOCKING=1    blocking ncclCommInitRank instead of the polled non-blocking init
  P2P_RCCL_DISTINCT_HOSTS=1  one NCCL_HOSTID per rank: RCCL ranks may share a GPU (tests,
                         over RCCL's socket transport, e.g. NCCL_SOCKET_IFNAME=lo)
  P2P_IPC_POOL=B         exported IPC buffers kept for reuse                     [32G]
  P2P_SDMA_STREAMS=K     --ipc-engine sdma: side streams the receives share      [4]
  P2P_BOOTSTRAP_PORT, P2P_BOOTSTRAP_TIMEOUT   TCP bootstrap port / receive deadline
  P2P_HOSTNAME=name      hostname for the placement check (emulated hosts)
  P2P_DEVICE=N           default of --device
  P2P_INJECT_FAULT=kind@rank[:phase]   corrupt | exit | hang | skip | skip-some (tests)
  P2P_ROCTX=1, P2P_LOG=1 roctx ranges; engine log on stderr
)";
}

int auto_iters(size_t bytes, size_t target_bytes) {
  size_t it = target_bytes / std::max<size_t>(bytes, 1);
  return static_cast<int>(std::clamp<size_t>(it, 8, 1000));
}

namespace {

std::vector<Mode> parse_modes(const std::string& s) {
  if (s == "all") return {Mode::Pair, Mode::Tournament, Mode::Ring, Mode::AllPairs};
  std::vector<Mode> out;
  size_t pos = 0;
  while (pos <= s.size()) {
    size_t c = s.find(',', pos);
    std::string item = s.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
    if (!item.empty()) out.push_back(parse_mode(item));
    if (c == std::string::npos) break;
    pos = c + 1;
  }
  return out;
}

}  // namespace

bool parse_cli(int argc, char** argv, AppConfig* cfg, int* exit_code, FILE* out) {
  *exit_code = 0;
  bool size_given = false;
  // P2P_DEVICE: the default of --device (a multi-GPU rehearsal on one GPU
  // puts every rank on device 0 without editing the command lines).
  if (const char* d = std::getenv("P2P_DEVICE"); d && *d) cfg->device = std::atoi(d);
  for (int i = 0; i < argc; ++i) {
    std::string a = argv[i];
    std::string val;
    auto eq = a.find('=');
    bool has_eq = a.rfind("--", 0) == 0 && eq != std::string::npos;
    if (has_eq) {
      val = a.substr(eq + 1);
      a = a.substr(0, eq);
    }
    bool missing = false;
    auto next = [&]() -> std::string {
      if (has_eq) return val;
      if (i + 1 >= argc) {
        missing = true;
        return "";
      }
      return argv[++i];
    };
    auto value_ok = [&]() {
      if (!missing) return true;
      std::fprintf(stderr, "p2p_matrix: option %s needs a value\n", a.c_str());
      *exit_code = 1;
      return false;
    };
    // Numeric values are read whole and range-checked: a typo or a negative
    // count fails at the command line instead of running something else.
    bool bad = false;
    auto int_arg = [&](long lo) -> int {
      const std::string v = next();
      char* end = nullptr;
      long x = std::strtol(v.c_str(), &end, 10);
      if (v.empty() || *end || x < lo || x > INT_MAX) {
        if (!missing) std::fprintf(stderr, "p2p_matrix: %s needs a whole number >= %ld, got '%s'\n", a.c_str(), lo, v.c_str());
        bad = true;
        return 0;
      }
      return static_cast<int>(x);
    };
    auto num_arg = [&](double lo, bool strict) -> double {
      const std::string v = next();
      char* end = nullptr;
      double x = std::strtod(v.c_str(), &end);
      if (v.empty() || *end || !(strict ? x > lo : x >= lo)) {
        if (!missing)
          std::fprintf(stderr, "p2p_matrix: %s needs a number %s %g, got '%s'\n", a.c_str(), strict ? ">" : ">=", lo,
                       v.c_str());
        bad = true;
        return 0;
      }
      return x;
    };
    // Options taking a value check it before use.
    static const char* kValued[] = {"-m", "--mode", "-d", "--dir", "-b", "--size", "--sizes", "-n", "--iters", "-w",
                                    "--warmup", "--timing", "--latency-size", "--latency-iters", "--latency-preposted", "--verify-impl",
                                    "--transport", "--ipc-engine", "--bootstrap", "--device", "--timeout", "--min-gbs", "--json",
                                    "--csv", "--trace", "--cells", "--comms", "--fuzz", "--repeat"};
    for (const char* v : kValued)
      if (a == v && !has_eq && i + 1 >= argc) {
        missing = true;
        return value_ok();
      }
    if (a == "-h" || a == "--help") {
      std::fprintf(out, "%s", usage_text().c_str());
      return false;
    } else if (a == "--version") {
      std::fprintf(out, "p2p_matrix (MI355X / gfx950, RCCL) 1.0\n");
      return false;
    } else if (a == "-m" || a == "--mode") {
      cfg->modes = parse_modes(next());
    } else if (a == "-d" || a == "--dir") {
      std::string d = next();
      if (d == "both")
        cfg->dirs = {Direction::Uni, Direction::Bi};
      else
        cfg->dirs = {parse_direction(d)};
    } else if (a == "-b" || a == "--size") {
      if (!size_given) cfg->sizes = {parse_size(next())};
      else next();
    } else if (a == "--sizes") {
      cfg->sizes = parse_size_list(next());
      size_given = true;
    } else if (a == "-n" || a == "--iters") {
      std::string v = next();
      if (v == "auto") {
        cfg->iters_auto = true;
      } else {
        char* end = nullptr;
        long x = std::strtol(v.c_str(), &end, 10);
        if (v.empty() || *end || x < 1 || x > INT_MAX) {
          std::fprintf(stderr, "p2p_matrix: --iters must be >= 1 (or auto), got '%s'\n", v.c_str());
          *exit_code = 1;
          return false;
        }
        cfg->run.iters = static_cast<int>(x);
        cfg->iters_auto = false;
      }
    } else if (a == "-w" || a == "--warmup") {
      cfg->run.warmup = int_arg(0);
    } else if (a == "--timing") {
      cfg->run.timing = parse_timing(next());
    } else if (a == "--reference") {
      cfg->run.timing = Timing::Wallclock;
      cfg->run.warmup = 0;
      cfg->warm_connections = false;
      cfg->two_streams = true;
      cfg->reference_buffers = true;
      cfg->rccl_stock = true;
    } else if (a == "--two-streams") {
      cfg->two_streams = true;
    } else if (a == "--comms") {
      cfg->comms = int_arg(1);
    } else if (a == "--no-warm") {
      cfg->warm_connections = false;
    } else if (a == "-l" || a == "--latency") {
      cfg->latency = true;
    } else if (a == "--device-latency") {
      cfg->device_latency = true;
    } else if (a == "--latency-preposted") {
      cfg->latency_preposted = int_arg(0);
      cfg->latency = true;
    } else if (a == "--fuzz") {
      cfg->fuzz_rounds = int_arg(0);
    } else if (a == "--repeat") {
      cfg->repeat = int_arg(1);
    } else if (a == "--latency-size") {
      cfg->latency_bytes = parse_size(next());
      cfg->latency = true;
    } else if (a == "--latency-iters") {
      cfg->latency_iters = int_arg(1);
      cfg->latency = true;
    } else if (a == "-c" || a == "--verify") {
      cfg->run.verify = true;
    } else if (a == "--no-verify") {
      cfg->run.verify = false;
    } else if (a == "--verify-impl") {
      const std::string v = next();
      std::string note;
      cfg->verify_impl = parse_verify_impl(v, &note);
      if (cfg->verify_impl < 0) {
        std::fprintf(stderr, "p2p_matrix: --verify-impl '%s': %s\n", v.c_str(), note.c_str());
        *exit_code = 1;
        return false;
      }
    } else if (a == "--transport") {
      cfg->transport = next();
    } else if (a == "--ipc-engine") {
      cfg->ipc_engine = next();
    } else if (a == "--bootstrap") {
      cfg->bootstrap = next();
    } else if (a == "--device") {
      cfg->device = int_arg(-1);
    } else if (a == "--min-gbs") {
      cfg->min_gbs = num_arg(0, false);
    } else if (a == "--timeout") {
      cfg->timeout_s = num_arg(0, true);
    } else if (a == "--json") {
      cfg->json_path = next();
    } else if (a == "--csv") {
      cfg->csv_path = next();
    } else if (a == "--trace") {
      cfg->trace_path = next();
    } else if (a == "--cells") {
      // "0-1,2-3" (src-dst pairs, also "0:1")
      std::string v = next();
      size_t pos = 0;
      while (pos < v.size()) {
        size_t c = v.find(',', pos);
        std::string item = v.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
        size_t sep = item.find_first_of("-:");
        if (sep == std::string::npos) {
          std::fprintf(stderr, "p2p_matrix: bad --cells item '%s' (want src-dst)\n", item.c_str());
          *exit_code = 1;
          return false;
        }
        cfg->cells.emplace_back(std::atoi(item.substr(0, sep).c_str()), std::atoi(item.substr(sep + 1).c_str()));
        if (c == std::string::npos) break;
        pos = c + 1;
      }
    } else if (a == "--resume") {
      cfg->resume = true;
    } else if (a == "--compat-only") {
      cfg->extended = false;
      cfg->compat = true;
    } else if (a == "--no-compat") {
      cfg->compat = false;
    } else if (a == "--dry-run") {
      cfg->dry_run = true;
    } else if (a == "--topology") {
      cfg->topology_only = true;
    } else if (a == "-v" || a == "--verbose") {
      cfg->verbose++;
    } else {
      std::fprintf(stderr, "p2p_matrix: unknown option '%s' (see --help)\n", argv[i]);
      *exit_code = 1;
      return false;
    }
    if (bad) {
      *exit_code = 1;
      return false;
    }
  }
  if (cfg->run.iters < 1 && !cfg->iters_auto) {
    std::fprintf(stderr, "p2p_matrix: --iters must be >= 1\n");
    *exit_code = 1;
    return false;
  }
  if (cfg->run.warmup < 0) cfg->run.warmup = 0;
  if (cfg->transport != "rccl" && cfg->transport != "host" && cfg->transport != "ipc" && cfg->transport != "shm") {
    std::fprintf(stderr, "p2p_matrix: --transport must be rccl, ipc, host or shm\n");
    *exit_code = 1;
    return false;
  }
  // Known before any rank starts: fail at the command line, not mid-run.
  if (cfg->device_latency && cfg->transport != "ipc") {
    std::fprintf(stderr, "p2p_matrix: --device-latency needs a one-sided transport (--transport ipc); %s has none\n",
                 cfg->transport.c_str());
    *exit_code = 1;
    return false;
  }
  return true;
}

namespace {

void print_schedule(FILE* out, const Schedule& s) {
  std::fprintf(out, "schedule %s, %d ranks, %zu phases\n", s.name().c_str(), s.nranks, s.phases.size());
  for (const auto& p : s.phases) {
    std::fprintf(out, "  [%s]%s", p.label.c_str(), p.idle ? " idle" : "");
    for (const auto& f : p.flows) std::fprintf(out, " %d->%d", f.src, f.dst);
    std::fprintf(out, "\n");
  }
}

}  // namespace

namespace {

// Schedules: (mode, dir) pairs; Self and the concurrent all-pairs exchange
// have no meaningful uni/bi split, so they run once.  --cells: re-measure
// only some (src, dst) cells of the pair schedule; the others stay in the
// schedule as idle cells (barrier, reported 0.00), so the printed matrices
// keep their shape.
std::vector<Schedule> build_schedules(const AppConfig& cfg, int n) {
  std::vector<Schedule> scheds;
  for (Mode m : cfg.modes) {
    if (m == Mode::Self || m == Mode::AllPairs) {
      scheds.push_back(make_schedule(m, m == Mode::Self ? Direction::Uni : Direction::Bi, n));
      continue;
    }
    for (Direction d : cfg.dirs) scheds.push_back(make_schedule(m, d, n));
  }
  if (!cfg.cells.empty())
    for (auto& s : scheds) restrict_cells(&s, cfg.cells, false);
  for (const auto& s : scheds) {
    std::string bad = validate(s);
    P2P_CHECK(bad.empty(), "invalid schedule " + s.name() + ": " + bad);
  }
  return scheds;
}

std::unique_ptr<Transport> open_transport(const AppConfig& cfg, Bootstrap& boot, const Placement& pl,
                                          TransportOptions* topt) {
  topt->device = cfg.device >= 0 ? cfg.device : pl.local_rank;
  topt->timeout_s = cfg.timeout_s;
  topt->verify_impl = cfg.verify_impl;
  topt->ipc_engine = cfg.ipc_engine;
  topt->two_streams = cfg.two_streams;
  topt->rccl_comms = cfg.comms;
  topt->rccl_stock = cfg.rccl_stock;
  return cfg.transport == "host"  ? make_host_transport(boot, *topt)
         : cfg.transport == "shm" ? make_shm_transport(boot, *topt)
         : cfg.transport == "ipc" ? make_ipc_transport(boot, *topt)
                                  : make_rccl_transport(boot, *topt);
}

// Checkpoint / resume: every finished run is appended to the JSON-lines file
// and flushed at once, so a killed sweep keeps what it measured; --resume
// skips the (mode, dir, size) runs already present in that file (all R of
// them with --repeat R).  Returns how many each has (collective: rank 0 reads
// the file, every rank gets the counts).
std::vector<uint8_t> open_results(const AppConfig& cfg, Bootstrap& boot, const std::vector<Schedule>& scheds,
                                  const std::string& provenance, std::ofstream* js) {
  std::vector<uint8_t> skip(scheds.size() * cfg.sizes.size(), 0);
  if (boot.rank() == 0 && !cfg.json_path.empty()) {
    if (cfg.resume) {
      std::ifstream in(cfg.json_path);
      std::vector<std::string> done;
      for (std::string line; std::getline(in, line);) {
        std::string k = run_key_from_json(line);
        if (!k.empty()) done.push_back(k);
      }
      // How many runs of each (mode, dir, size) the file holds (with
      // --repeat R, a killed job resumes at the first missing repeat).
      for (size_t i = 0; i < scheds.size(); ++i)
        for (size_t j = 0; j < cfg.sizes.size(); ++j) {
          const auto c = std::count(done.begin(), done.end(), run_key(scheds[i].mode, scheds[i].dir, cfg.sizes[j]));
          skip[i * cfg.sizes.size() + j] = static_cast<uint8_t>(std::min<long>(c, 255));
        }
    }
    js->open(cfg.json_path, cfg.resume ? std::ios::app : std::ios::trunc);
    P2P_CHECK(js->good(), "cannot write " + cfg.json_path);
    *js << provenance << "\n";
    js->flush();
  }
  if (!skip.empty()) boot.bcast(skip.data(), skip.size(), 0);
  return skip;
}

// Every (schedule, size) run; rank 0 prints the reference-format matrices of
// pair runs as their cells finish (the reference prints and flushes per cell).
void run_all(const AppConfig& cfg, Transport& t, Bootstrap& boot, const std::vector<Schedule>& scheds,
             const std::vector<uint8_t>& skip, Buffers& bufs, std::ofstream& js, FILE* out, AppResult& res) {
  const int n = boot.size();
  const bool root = boot.rank() == 0;
  bool printed_compat = false;
  for (size_t sj = 0; sj < scheds.size(); ++sj) {
    const Schedule& s = scheds[sj];
    for (size_t si = 0; si < cfg.sizes.size(); ++si) {
      const int done = skip[sj * cfg.sizes.size() + si];
      if (done >= std::max(1, cfg.repeat)) {
        if (root) P2P_INFO("resume: skipping %s", run_key(s.mode, s.dir, cfg.sizes[si]).c_str());
        continue;
      }
      for (int rep = done; rep < std::max(1, cfg.repeat); ++rep) {
        RunRecord rec;
        rec.mode = s.mode;
        rec.dir = s.dir;
        rec.bytes = cfg.sizes[si];
        rec.cfg = cfg.run;
        rec.cfg.bytes = rec.bytes;
        rec.cfg.salt = static_cast<uint64_t>(res.runs.size());
        rec.repeat = rep;
        if (cfg.iters_auto) rec.cfg.iters = auto_iters(rec.bytes, cfg.target_bytes);
        // The reference matrices print the first run only, cell by cell.
        const bool compat = cfg.compat && s.mode == Mode::Pair && root && rep == 0;
        CompatPrinter cp(out, n);
        if (compat) {
          if (cfg.sizes.size() > 1)
            std::fprintf(out, "%s# message size %s\n", printed_compat ? "\n" : "", format_size(rec.bytes).c_str());
          cp.begin(s.dir, printed_compat && s.dir == Direction::Uni && cfg.sizes.size() == 1);
          printed_compat = true;
        }
        rec.phases = run_schedule(t, boot, s, rec.cfg, bufs, [&](const PhaseResult& r) {
          if (compat) cp.on_phase(r);
        });
        for (const auto& ph : rec.phases) res.mismatches += ph.total_mismatches;
        if (js.is_open()) {
          js << run_to_json(rec, n) << "\n";
          js.flush();
        }
        res.runs.push_back(std::move(rec));
      }
    }
  }
}

// Latency tables: host-posted and pre-posted ping-pong, the device ping-pong
// (one-sided transports), and in ring mode the dependent token chain.
void run_latencies(const AppConfig& cfg, Transport& t, Bootstrap& boot, Buffers& bufs, AppResult& res) {
  const int n = boot.size();
  const int warm = std::min(cfg.latency_iters, 100);
  if (cfg.latency) res.latency = run_latency(t, boot, cfg.latency_bytes, cfg.latency_iters, warm, bufs);
  if (cfg.latency && cfg.latency_preposted > 0)
    res.preposted_latency = run_latency(t, boot, cfg.latency_bytes, cfg.latency_iters, warm, bufs, cfg.latency_preposted);
  if (cfg.device_latency) res.device_latency = run_device_latency(t, boot, cfg.latency_bytes, cfg.latency_iters, warm);
  if (std::find(cfg.modes.begin(), cfg.modes.end(), Mode::Ring) != cfg.modes.end()) {
    const int laps = std::max(1, cfg.latency_iters / std::max(1, n));
    if (cfg.latency)
      res.ring_latency.push_back(run_ring_latency(t, boot, cfg.latency_bytes, laps, std::min(laps, 20), bufs));
    if (cfg.device_latency)
      res.ring_latency.push_back(run_device_ring_latency(t, boot, cfg.latency_bytes, laps, std::min(laps, 20)));
  }
}

// Rank 0: the extended tables after the reference matrices, and the JSON /
// trace / CSV files.
std::string links_to_json(const AppResult& res, int n);
void print_transport_matrix(FILE* out, const AppResult& res, int n);

void write_reports(const AppConfig& cfg, const Transport& t, const Bootstrap& boot, const Placement& pl,
                   const std::vector<char>& all_desc, size_t desc_len, const AppResult& res, uint64_t fuzz_bad,
                   size_t fuzz_max, std::ofstream& js, FILE* out) {
  const int n = boot.size();
  if (cfg.extended) {
    std::fprintf(out, "\n== p2p_matrix: %d rank(s), transport %s, bootstrap %s, %d host(s) ==\n", n, t.name().c_str(),
                 boot.name().c_str(), pl.num_hosts);
    for (int r = 0; r < n; ++r) std::fprintf(out, "  rank %d: %s\n", r, &all_desc[static_cast<size_t>(r) * desc_len]);
    if (t.name() != "host" && t.name() != "shm") std::fprintf(out, "%s", topology_report().c_str());
    print_transport_matrix(out, res, n);
    // The tables of the first run of each (mode, dir, size); with --repeat
    // the others are summarised below.
    std::vector<RunRecord> firsts;
    for (const auto& rec : res.runs)
      if (rec.repeat == 0) firsts.push_back(rec);
    for (const auto& rec : firsts) print_extended(out, rec, n);
    print_fabric_check(out, firsts, n);
    if (cfg.repeat > 1) print_repeat_summary(out, repeat_summaries(res.runs, n));
    print_latency(out, res.latency, n);
    print_latency(out, res.preposted_latency, n);
    print_latency(out, res.device_latency, n);
    for (const auto& rl : res.ring_latency) print_ring_latency(out, rl);
    if (cfg.fuzz_rounds > 0)
      std::fprintf(out, "\n== fuzz: %d groups of random messages (1 B .. %s, random pairs incl. self): %s ==\n",
                   cfg.fuzz_rounds, format_size(fuzz_max).c_str(),
                   fuzz_bad ? strfmt("%llu mismatching words", static_cast<unsigned long long>(fuzz_bad)).c_str()
                            : "all verified");
  }
  if (js.is_open()) {
    if (cfg.repeat > 1)
      for (const auto& rs : repeat_summaries(res.runs, n)) js << repeat_summary_json(rs) << "\n";
    js << links_to_json(res, n) << "\n";
    if (!res.latency.empty()) js << latency_to_json(res.latency, n) << "\n";
    if (!res.preposted_latency.empty()) js << latency_to_json(res.preposted_latency, n) << "\n";
    if (!res.device_latency.empty()) js << latency_to_json(res.device_latency, n) << "\n";
    for (const auto& rl : res.ring_latency) js << ring_latency_to_json(rl) << "\n";
    if (cfg.fuzz_rounds > 0)
      js << strfmt("{\"type\":\"fuzz\",\"rounds\":%d,\"max_bytes\":%zu,\"mismatches\":%llu}", cfg.fuzz_rounds, fuzz_max,
                   static_cast<unsigned long long>(fuzz_bad))
         << "\n";
  }
  if (!cfg.trace_path.empty()) {
    std::ofstream tr(cfg.trace_path);
    P2P_CHECK(tr.good(), "cannot write " + cfg.trace_path);
    tr << chrome_trace(res.runs, n) << "\n";
  }
  if (!cfg.csv_path.empty()) {
    std::ofstream cs(cfg.csv_path);
    P2P_CHECK(cs.good(), "cannot write " + cfg.csv_path);
    cs << csv_header();
    for (const auto& rec : res.runs) cs << run_to_csv(rec);
  }
  std::fflush(out);
}

// Collective: every rank's per-peer transport classes, the GPU link types
// between ranks and every rank's link report (AppResult).
void collect_links(Transport& t, Bootstrap& boot, int device, AppResult& res) {
  const int n = boot.size();
  std::vector<std::string> mine = t.peer_transports();
  mine.resize(static_cast<size_t>(n));
  std::string packed;
  for (const auto& tr : mine) packed += tr + "\n";
  const auto rows = boot.allgather_string(packed);
  res.transport_matrix.assign(static_cast<size_t>(n) * n, "");
  for (int r = 0; r < n; ++r) {
    size_t at = 0;
    for (int p = 0; p < n; ++p) {
      const size_t e = rows[static_cast<size_t>(r)].find('\n', at);
      if (e == std::string::npos) break;
      res.transport_matrix[static_cast<size_t>(r) * n + p] = rows[static_cast<size_t>(r)].substr(at, e - at);
      at = e + 1;
    }
  }
  res.link_matrix = rank_link_matrix(boot, device);
  res.link_reports = boot.allgather_string(t.link_report());
}

// {"type":"links"}: transport class and GPU link per pair, and every rank's
// link report (RCCL: p2p channels, per-peer transport and op limit).
std::string links_to_json(const AppResult& res, int n) {
  auto mat = [&](const std::vector<std::string>& m) {
    std::string o = "[";
    for (int a = 0; a < n; ++a) {
      o += a ? ",[" : "[";
      for (int b = 0; b < n; ++b) {
        const size_t i = static_cast<size_t>(a) * n + b;
        o += std::string(b ? "," : "") + "\"" + json_escape(i < m.size() ? m[i] : "") + "\"";
      }
      o += "]";
    }
    return o + "]";
  };
  std::string o = "{\"type\":\"links\",\"matrix_transport\":" + mat(res.transport_matrix) +
                  ",\"rank_links\":" + mat(res.link_matrix) + ",\"ranks\":[";
  for (size_t r = 0; r < res.link_reports.size(); ++r)
    o += (r ? "," : "") + (res.link_reports[r].empty() ? std::string("null") : res.link_reports[r]);
  return o + "]}";
}

// The transport class per pair, when the data plane reports one.
void print_transport_matrix(FILE* out, const AppResult& res, int n) {
  bool any = false;
  for (const auto& tr : res.transport_matrix) any = any || !tr.empty();
  if (!any) return;
  std::fprintf(out, "\n== data-plane transport per pair (row = rank, col = peer; RCCL INFO log) ==\n      ");
  for (int b = 0; b < n; ++b) std::fprintf(out, "%7d", b);
  std::fprintf(out, "\n");
  for (int a = 0; a < n; ++a) {
    std::fprintf(out, "%6d", a);
    for (int b = 0; b < n; ++b) {
      const std::string& tr = res.transport_matrix[static_cast<size_t>(a) * n + b];
      std::fprintf(out, "%7s", tr.empty() ? "-" : tr.c_str());
    }
    std::fprintf(out, "\n");
  }
}

// Link check (--min-gbs): every measured off-diagonal flow must reach the
// threshold, and a pair whose GPUs share a direct xGMI link must have been
// carried by RCCL's P2P transport (link_transport_mismatch: a silent SHM or
// NET fallback reads as a slow link); the failing ones are named so a bad
// link or GPU can be found.
int count_slow_flows(const AppConfig& cfg, const AppResult& res, bool root) {
  int slow = 0;
  if (cfg.min_gbs <= 0) return 0;
  const size_t n = static_cast<size_t>(std::sqrt(static_cast<double>(res.transport_matrix.size())) + 0.5);
  if (n > 0 && res.link_matrix.size() == n * n)
    for (size_t a = 0; a < n; ++a)
      for (size_t b = 0; b < n; ++b)
        if (a != b && link_transport_mismatch(res.link_matrix[a * n + b], res.transport_matrix[a * n + b])) {
          ++slow;
          if (root)
            std::fprintf(stderr, "p2p_matrix: WRONG TRANSPORT: %zu -> %zu went over %s although the GPUs share a %s link\n",
                         a, b, res.transport_matrix[a * n + b].c_str(), res.link_matrix[a * n + b].c_str());
        }
  for (const auto& rec : res.runs)
    for (const auto& ph : rec.phases)
      for (const auto& f : ph.flows)
        if (f.flow.src != f.flow.dst && f.gbs < cfg.min_gbs) {
          ++slow;
          if (root)
            std::fprintf(stderr, "p2p_matrix: SLOW LINK: %d -> %d %.2f GB/s < %.2f (%s-%s, %s)\n", f.flow.src,
                         f.flow.dst, f.gbs, cfg.min_gbs, mode_name(rec.mode), direction_name(rec.dir),
                         format_size(rec.bytes).c_str());
        }
  return slow;
}

}  // namespace

int run_app(const AppConfig& cfg, Bootstrap& boot, FILE* out, AppResult* result) {
  if (cfg.verbose) set_log_level(cfg.verbose);
  const int n = boot.size();
  const bool root = boot.rank() == 0;

  const std::vector<Schedule> scheds = build_schedules(cfg, n);
  if (cfg.dry_run) {
    if (root)
      for (const auto& s : scheds) print_schedule(out, s);
    return 0;
  }
  if (cfg.topology_only) {
    if (root) std::fprintf(out, "%s", topology_report().c_str());
    return 0;
  }

  Placement pl = check_placement(boot);
  if (!pl.ok) P2P_FATAL("process placement check failed: " + pl.error);
  TransportOptions topt;
  std::unique_ptr<Transport> t = open_transport(cfg, boot, pl, &topt);

  // Provenance (collective): the runtime, RCCL library and knobs, every
  // rank's GPU and the links between them -- the first line of --json.
  const bool gpu_transport = cfg.transport == "rccl" || cfg.transport == "ipc";
  const std::string provenance =
      cfg.json_path.empty() ? std::string() : provenance_json(boot, gpu_transport ? topt.device : -1);

  size_t max_bytes = *std::max_element(cfg.sizes.begin(), cfg.sizes.end());
  if (cfg.latency) max_bytes = std::max(max_bytes, cfg.latency_bytes);
  int slots = 1;
  for (const auto& s : scheds) slots = std::max(slots, s.max_recv_slots());
  // --verify: every timed iteration gets a receive generation of its own (its
  // own send region, seed and receive slots), as many as the memory budget
  // allows, so the check after timing covers each delivery, not only the last
  // one into a slot (runner.hpp RunConfig::gens; verify_coverage in the output).
  AppConfig run_cfg = cfg;
  // --reference keeps the reference's footprint (one 32 MiB send and receive
  // buffer for all 128 iterations, p2p_matrix.cc:124-130, which can stay in
  // the 256 MB Infinity Cache): one generation, the last delivery verified.
  if (cfg.run.verify && !cfg.reference_buffers) {
    int most_iters = std::max(cfg.run.iters, cfg.run.warmup);
    if (cfg.iters_auto)
      for (size_t b : cfg.sizes) most_iters = std::max(most_iters, auto_iters(b, cfg.target_bytes));
    run_cfg.run.gens = verify_generations(*t, boot, max_bytes, slots, most_iters);
  }
  if (const char* rc = std::getenv("P2P_RECHUNK")) run_cfg.run.rechunk = std::atoi(rc) != 0;
  Buffers bufs(*t, max_bytes, slots * run_cfg.run.gens, slot_stride_bytes(max_bytes) * static_cast<size_t>(run_cfg.run.gens));

  // Connection warm-up outside any timed cell (the reference pays lazy p2p
  // connection setup inside its first cells; --reference keeps that).
  if (cfg.warm_connections) {
    for (const auto& s : scheds) warm_connections(*t, boot, s, bufs);
    // Every peer of every schedule is connected: op limits from RCCL's
    // connection lines (transport.hpp refine_op_limits).
    t->refine_op_limits(boot);
  }

  AppResult local;
  AppResult& res = result ? *result : local;
  std::ofstream js;
  const std::vector<uint8_t> skip = open_results(cfg, boot, scheds, provenance, &js);
  run_all(run_cfg, *t, boot, scheds, skip, bufs, js, out, res);
  run_latencies(cfg, *t, boot, bufs, res);
  uint64_t fuzz_bad = 0;
  size_t fuzz_max = 0;
  if (cfg.fuzz_rounds > 0) {
    fuzz_max = std::max<size_t>(16, std::min<size_t>(max_bytes, size_t{64} << 20));
    fuzz_bad = boot.allreduce_sum_u64(fuzz_transport(*t, boot, cfg.fuzz_rounds, 0xF022, fuzz_max));
    res.mismatches += fuzz_bad;
  }

  // What the data plane set up per peer (RCCL: transports and channels from
  // its INFO log), now that every connection the runs used exists.
  collect_links(*t, boot, gpu_transport ? topt.device : -1, res);

  // Device descriptions of every rank, for the banner.
  char mine[256] = {0};
  std::snprintf(mine, sizeof(mine), "%s", t->device_desc().c_str());
  std::vector<char> all_desc(static_cast<size_t>(n) * sizeof(mine));
  boot.allgather(mine, all_desc.data(), sizeof(mine));
  if (root) write_reports(cfg, *t, boot, pl, all_desc, sizeof(mine), res, fuzz_bad, fuzz_max, js, out);

  res.slow_flows = count_slow_flows(cfg, res, root);
  boot.barrier();
  if (res.mismatches) {
    if (root) std::fprintf(stderr, "p2p_matrix: VERIFICATION FAILED: %llu mismatching words\n", static_cast<unsigned long long>(res.mismatches));
    return 2;
  }
  if (res.slow_flows) {
    if (root) std::fprintf(stderr, "p2p_matrix: LINK CHECK FAILED: %d flow(s) below %.2f GB/s\n", res.slow_flows, cfg.min_gbs);
    return 3;
  }
  return 0;
}

}  // namespace p2p
