// Linked into the hola_amd._native module only: its ISA check as the module's first static
// initialiser (init priority 101 sorts ahead of the default-priority constructors of the
// module and of hola_core, which are built at the release -march), compiled for the x86-64
// baseline like src/isa_guard.cc. A Python process cannot be ended here the way an executable
// is, so on a CPU that lacks what the build assumes this prints the reason to stderr at once
// and records it; PYBIND11_MODULE then fails the import with it (src/pybind/module.cc). If a
// later initialiser of the module itself executes an instruction the CPU lacks, the process
// still dies with SIGILL, but the line naming the missing features has been written first
// (the module init alone ran after those initialisers).
#include <unistd.h>

#include <cstring>
#include <string>

#include "core/isa.h"

namespace hola::isa {

// Empty, or the error line (NUL-terminated): plain storage, constant-initialised, so it is
// valid before any dynamic initialiser of this module has run.
char g_module_isa_error[512];

namespace {

__attribute__((constructor(101))) void hola_module_isa_flag() {
  const std::string missing = missing_features();
  if (missing.empty()) return;
  const std::string line = error_line("hola_amd._native");
  ssize_t w = ::write(2, line.data(), line.size());
  (void)w;
  const size_t n = line.size() < sizeof g_module_isa_error - 1 ? line.size() : sizeof g_module_isa_error - 1;
  memcpy(g_module_isa_error, line.data(), n);
  g_module_isa_error[n] = 0;
}

}  // namespace
}  // namespace hola::isa
