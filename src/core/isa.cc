// Compiled with -march=x86-64 -mtune=generic (CMakeLists.txt): this file must run on a CPU
// that lacks what the rest of the build assumes.
#include "core/isa.h"

#include <cstdlib>
#include <cstring>

#ifndef HOLA_ISA_MARCH
#define HOLA_ISA_MARCH "x86-64-v3"
#endif

namespace hola::isa {

namespace {

struct Feature {
  const char* name;
  int level;  // first x86-64 psABI level that includes it
};

// x86-64 psABI micro-architecture levels (the features __builtin_cpu_supports can test).
constexpr Feature kFeatures[] = {
    {"sse3", 2}, {"ssse3", 2}, {"sse4.1", 2}, {"sse4.2", 2}, {"popcnt", 2},
    {"avx", 3},  {"avx2", 3},  {"bmi", 3},    {"bmi2", 3},   {"fma", 3},    {"f16c", 3}, {"lzcnt", 3}, {"movbe", 3},
    {"avx512f", 4}, {"avx512bw", 4}, {"avx512cd", 4}, {"avx512dq", 4}, {"avx512vl", 4},
};

int level_of(const char* march) {
  if (!strcmp(march, "x86-64-v4")) return 4;
  if (!strcmp(march, "x86-64-v3")) return 3;
  if (!strcmp(march, "x86-64-v2")) return 2;
  if (!strcmp(march, "x86-64")) return 1;
  return 3;  // a named CPU (znver3, native, ...): at least the AVX2 the request path uses
}

bool supports(const char* f) {
  __builtin_cpu_init();
  if (!strcmp(f, "sse3")) return __builtin_cpu_supports("sse3");
  if (!strcmp(f, "ssse3")) return __builtin_cpu_supports("ssse3");
  if (!strcmp(f, "sse4.1")) return __builtin_cpu_supports("sse4.1");
  if (!strcmp(f, "sse4.2")) return __builtin_cpu_supports("sse4.2");
  if (!strcmp(f, "popcnt")) return __builtin_cpu_supports("popcnt");
  if (!strcmp(f, "avx")) return __builtin_cpu_supports("avx");
  if (!strcmp(f, "avx2")) return __builtin_cpu_supports("avx2");
  if (!strcmp(f, "bmi")) return __builtin_cpu_supports("bmi");
  if (!strcmp(f, "bmi2")) return __builtin_cpu_supports("bmi2");
  if (!strcmp(f, "fma")) return __builtin_cpu_supports("fma");
  if (!strcmp(f, "f16c")) return __builtin_cpu_supports("f16c");
  if (!strcmp(f, "lzcnt")) return __builtin_cpu_supports("lzcnt");
  if (!strcmp(f, "movbe")) return __builtin_cpu_supports("movbe");
  if (!strcmp(f, "avx512f")) return __builtin_cpu_supports("avx512f");
  if (!strcmp(f, "avx512bw")) return __builtin_cpu_supports("avx512bw");
  if (!strcmp(f, "avx512cd")) return __builtin_cpu_supports("avx512cd");
  if (!strcmp(f, "avx512dq")) return __builtin_cpu_supports("avx512dq");
  if (!strcmp(f, "avx512vl")) return __builtin_cpu_supports("avx512vl");
  return true;
}

bool pretend_missing(const char* f) {
  const char* p = getenv("HOLA_ISA_PRETEND_MISSING");
  if (!p) return false;
  const size_t n = strlen(f);
  for (const char* s = p; *s;) {
    const char* e = strchr(s, ',');
    const size_t len = e ? size_t(e - s) : strlen(s);
    if (len == n && !strncmp(s, f, n)) return true;
    if (!e) break;
    s = e + 1;
  }
  return false;
}

}  // namespace

const char* build_level() { return HOLA_ISA_MARCH; }

std::string missing_features() {
  const int need = level_of(HOLA_ISA_MARCH);
  std::string out;
  for (const Feature& f : kFeatures) {
    if (f.level > need) continue;
    if (supports(f.name) && !pretend_missing(f.name)) continue;
    if (!out.empty()) out += ',';
    out += f.name;
  }
  return out;
}

std::string error_line(const char* program) {
  return std::string(program) + ": this build needs an " + HOLA_ISA_MARCH + " CPU and this one lacks " +
         missing_features() + "; run the portable build on this node (cmake --preset portable, or docker build "
         "--build-arg HOLA_MARCH=x86-64-v2)\n";
}

}  // namespace hola::isa
