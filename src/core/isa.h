// The x86-64 ISA level a build was compiled for, checked against the CPU it runs on.
//
// Release builds use -march=x86-64-v3 (AVX2 and friends: every EPYC host of an MI355X node has
// them) and the request path uses AVX2 intrinsics, so such a binary on an older node would die
// with SIGILL somewhere in start-up, with no message. The check runs first and says what is
// missing; a pre-AVX2 node runs the `portable` preset (HOLA_MARCH=x86-64-v2), whose parser
// and line scan take their byte loops. isa.cc is compiled for the x86-64 baseline, so the
// check itself runs on any x86-64 CPU.
#pragma once
#include <string>

namespace hola::isa {

// The -march level this build was compiled for ("x86-64-v3", ...).
const char* build_level();
// Comma-separated CPU features the build needs that this CPU lacks; empty when it can run.
// HOLA_ISA_PRETEND_MISSING=feat[,feat] (tests) adds features to the answer as if absent.
std::string missing_features();
// One line for stderr when missing_features() is not empty.
std::string error_line(const char* program);

}  // namespace hola::isa
