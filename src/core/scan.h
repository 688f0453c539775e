// Short-line scanning for the HTTP heads on the request path.
//
// A header line is almost always shorter than 32 bytes, and libc's memchr costs a call plus
// its size dispatch (~27 instructions on the box, bench/micro.cc) for every line. When 32
// bytes of the buffer are at hand, one AVX2 compare finds the newline inline; otherwise, or
// past the first 32 bytes, memchr does. Never reads past `avail`. A build below x86-64-v3
// (HOLA_MARCH=x86-64-v2, preset `portable`) has no __AVX2__ and uses memchr throughout.
#pragma once
#if defined(__AVX2__) || defined(__SSE2__)
#include <immintrin.h>
#endif

#include <cstddef>
#include <cstdint>
#include <cstring>

namespace hola {

template <char C>
inline const char* find_byte(const char* p, size_t avail) {
#if defined(__AVX2__)
  if (avail >= 32) {
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p));
    const unsigned m = unsigned(_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, _mm256_set1_epi8(C))));
    if (m) return p + __builtin_ctz(m);
    return static_cast<const char*>(memchr(p + 32, C, avail - 32));
  }
#endif
  return static_cast<const char*>(memchr(p, C, avail));
}

inline const char* find_newline(const char* p, size_t avail) { return find_byte<'\n'>(p, avail); }

}  // namespace hola

namespace hola {

// Length of the prefix of p[0..n) that a JSON string holds verbatim: no control character
// (< 0x20), no '"' and no '\\'. Sixteen bytes per SSE2 compare (every x86-64 has SSE2),
// eight per word below that (the tail word is padded with spaces, which are plain, so
// nothing past n is read). The per-byte loop it replaces was most of the JSON encoder's and
// decoder's instructions on the chaining path (profiles/round6/03_chain_instr).
inline size_t json_plain_prefix(const char* p, size_t n) {
  size_t i = 0;
#if defined(__SSE2__)
  const __m128i quote = _mm_set1_epi8('"'), bslash = _mm_set1_epi8('\\'), ctl = _mm_set1_epi8(0x1f);
  for (; i + 16 <= n; i += 16) {
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p + i));
    // bytes <= 0x1f: unsigned min(v, 0x1f) == v
    const __m128i bad = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, quote), _mm_cmpeq_epi8(v, bslash)),
                                     _mm_cmpeq_epi8(_mm_min_epu8(v, ctl), v));
    const unsigned m = unsigned(_mm_movemask_epi8(bad));
    if (m) return i + size_t(__builtin_ctz(m));
  }
#endif
  constexpr uint64_t kOnes = 0x0101010101010101ull, kHigh = 0x8080808080808080ull;
  auto zero_bytes = [](uint64_t x) { return (x - kOnes) & ~x & kHigh; };  // high bit of each 0x00 byte
  while (i < n) {
    const size_t k = n - i < 8 ? n - i : 8;
    uint64_t w = 0x2020202020202020ull;
    memcpy(&w, p + i, k);
    // high bit of each byte < 0x20 (bytes >= 0x80 are excluded by ~w), '"' or '\\'
    const uint64_t m = ((w - 0x2020202020202020ull) & ~w & kHigh) | zero_bytes(w ^ ('"' * kOnes)) |
                       zero_bytes(w ^ ('\\' * kOnes));
    if (m) return i + size_t(__builtin_ctzll(m) / 8);
    i += k;
  }
  return n;
}

}  // namespace hola
