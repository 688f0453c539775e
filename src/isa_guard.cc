// Linked into the executables only (not into hola_core or the Python module): the ISA check
// as the first static initialiser of the process, before any code compiled for the build's
// -march runs (main's own initialisers, libstdc++ streams aside, are all later: init
// priority 101 sorts ahead of every default-priority constructor at link time). Compiled for
// the x86-64 baseline like isa.cc. A CPU that cannot run the build gets one line on stderr and
// exit status 1 instead of a SIGILL crash loop.
#include <unistd.h>

#include <string>

#include "core/isa.h"

namespace {

__attribute__((constructor(101))) void hola_isa_guard() {
  const std::string missing = hola::isa::missing_features();
  if (missing.empty()) return;
  char exe[256];
  ssize_t n = readlink("/proc/self/exe", exe, sizeof exe - 1);
  exe[n > 0 ? n : 0] = 0;
  const char* base = exe;
  for (const char* p = exe; *p; ++p)
    if (*p == '/') base = p + 1;
  const std::string line = hola::isa::error_line(*base ? base : "hola");
  ssize_t w = ::write(2, line.data(), line.size());
  (void)w;
  _exit(1);
}

}  // namespace
