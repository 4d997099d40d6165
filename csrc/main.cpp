// p2p_matrix: the executable.  `mpirun -n N ./p2p_matrix` as in the reference
// (README.md:5); see app.cpp for the flow and usage_text() for options.
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>

#include "app.hpp"
#include "bootstrap.hpp"
#include "common.hpp"

int main(int argc, char** argv) {
  p2p::AppConfig cfg;
  int code = 0;
  // Bootstrap flag must be known before MPI_Init (which may rewrite argv).
  std::string boot_kind = "auto";
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--bootstrap") && i + 1 < argc) boot_kind = argv[i + 1];
    if (!std::strncmp(argv[i], "--bootstrap=", 12)) boot_kind = argv[i] + 12;
  }
  bool dry = false;
  for (int i = 1; i < argc; ++i)
    if (!std::strcmp(argv[i], "--dry-run") || !std::strcmp(argv[i], "--help") || !std::strcmp(argv[i], "-h") ||
        !std::strcmp(argv[i], "--version") || !std::strcmp(argv[i], "--topology"))
      dry = true;
  if (dry && boot_kind == "auto" && !p2p::mpi_launch_detected()) boot_kind = "local";

  std::unique_ptr<p2p::Bootstrap> boot = p2p::make_bootstrap(boot_kind, &argc, &argv);
  p2p::Bootstrap* bp = boot.get();
  int hook = p2p::push_abort_hook([bp](int c) { bp->abort(c); });

  // Only rank 0 prints help / errors for the CLI.
  FILE* out = boot->rank() == 0 ? stdout : std::fopen("/dev/null", "w");
  if (!p2p::parse_cli(argc - 1, argv + 1, &cfg, &code, out)) {
    boot->barrier();
    p2p::remove_abort_hook(hook);
    return code;
  }
  code = p2p::run_app(cfg, *boot, stdout);
  p2p::remove_abort_hook(hook);
  boot.reset();  // MPI_Finalize (the reference leaves it commented out, p2p_matrix.cc:272)
  return code;
}
