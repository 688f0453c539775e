// What this binary is: the release it implements (the reference's Maven version, which the
// image is tagged with), the source revision it was built from, and how it was built. Shown by
// `hola --version` and `/metrics` (`hola_build_info`); written at build time by
// cmake/build_info.cmake.
#pragma once

namespace hola::build_info {

const char* version();     // "0.0.1-SNAPSHOT" (pom.xml:24 of the reference)
const char* revision();    // short git revision, "-dirty" with uncommitted changes, or "unknown"
const char* compiler();    // e.g. "GNU 11.4.0"
const char* build_type();  // CMAKE_BUILD_TYPE, plus the sanitizers of the build

}  // namespace hola::build_info
