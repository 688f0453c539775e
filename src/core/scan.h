// Short-line scanning for the HTTP heads on the request path.
//
// A header line is almost always shorter than 32 bytes, and libc's memchr costs a call plus
// its size dispatch (~27 instructions on the box, bench/micro.cc) for every line. When 32
// bytes of the buffer are at hand, one AVX2 compare finds the newline inline; otherwise, or
// past the first 32 bytes, memchr does. Never reads past `avail`. A build below x86-64-v3
// (HOLA_MARCH=x86-64-v2, preset `portable`) has no __AVX2__ and uses memchr throughout.
#pragma once
#if defined(__AVX2__)
#include <immintrin.h>
#endif

#include <cstddef>
#include <cstring>

namespace hola {

inline const char* find_newline(const char* p, size_t avail) {
#if defined(__AVX2__)
  if (avail >= 32) {
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p));
    const unsigned m = unsigned(_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, _mm256_set1_epi8('\n'))));
    if (m) return p + __builtin_ctz(m);
    return static_cast<const char*>(memchr(p + 32, '\n', avail - 32));
  }
#endif
  return static_cast<const char*>(memchr(p, '\n', avail));
}

}  // namespace hola
