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
// (< 0x20), no '"' and no '\\'. Sixteen bytes per SSE2 compare (every x86-64 has SSE2); the
// last partial block is the buffer's last 16 bytes, overlapping what was already passed (the
// bytes before i shifted out of the mask), so nothing outside p[0..n) is read and no
// variable-length copy is made. Shorter buffers take overlapping 8- or 4-byte words, the
// bytes already passed replaced by spaces (plain). The per-byte loop this replaces was most
// of the JSON encoder's and decoder's instructions on the chaining path
// (profiles/round6/03_chain_instr).
namespace scan_detail {
constexpr uint64_t kOnes = 0x0101010101010101ull, kHigh = 0x8080808080808080ull, kSpaces = 0x2020202020202020ull;
// high bit of each byte of w that is < 0x20, '"' or '\\' (bytes >= 0x80 are plain); exact for
// the first such byte (the zero-byte test's borrow can only mark bytes above a true one)
inline uint64_t json_bad_bytes(uint64_t w) {
  auto zero_bytes = [](uint64_t x) { return (x - kOnes) & ~x & kHigh; };
  return ((w - kSpaces) & ~w & kHigh) | zero_bytes(w ^ ('"' * kOnes)) | zero_bytes(w ^ ('\\' * kOnes));
}
}  // namespace scan_detail

inline size_t json_plain_prefix(const char* p, size_t n) {
  using namespace scan_detail;
  size_t i = 0;
#if defined(__SSE2__)
  const __m128i quote = _mm_set1_epi8('"'), bslash = _mm_set1_epi8('\\'), ctl = _mm_set1_epi8(0x1f);
  auto bad16 = [&](const char* q) {
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(q));
    // bytes <= 0x1f: unsigned min(v, 0x1f) == v
    const __m128i bad = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, quote), _mm_cmpeq_epi8(v, bslash)),
                                     _mm_cmpeq_epi8(_mm_min_epu8(v, ctl), v));
    return unsigned(_mm_movemask_epi8(bad));
  };
  for (; i + 16 <= n; i += 16)
    if (const unsigned m = bad16(p + i)) return i + size_t(__builtin_ctz(m));
  if (i == n) return n;
  if (n >= 16) {  // the last n - i < 16 bytes, as the top of the buffer's last 16
    const unsigned m = bad16(p + n - 16) >> (16 - (n - i));
    return m ? i + size_t(__builtin_ctz(m)) : n;
  }
#endif
  // fewer than 16 bytes from i (i == 0 with SSE2): 8-byte words, the last one overlapping
  while (n - i >= 8) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    if (const uint64_t m = json_bad_bytes(w)) return i + size_t(__builtin_ctzll(m) / 8);
    i += 8;
  }
  if (i == n) return n;
  if (n >= 8) {
    uint64_t w;
    memcpy(&w, p + n - 8, 8);
    const unsigned seen = unsigned(8 - (n - i));  // leading bytes of w before i
    const uint64_t low = (uint64_t(1) << (8 * seen)) - 1;
    w = (w & ~low) | (kSpaces & low);
    const uint64_t m = json_bad_bytes(w);
    return m ? n - 8 + size_t(__builtin_ctzll(m) / 8) : n;
  }
  if (n >= 4) {  // 4..7 bytes in all (i == 0): two overlapping 4-byte words
    uint32_t a, b;
    memcpy(&a, p, 4);
    memcpy(&b, p + n - 4, 4);
    const unsigned seen = unsigned(8 - n);  // bytes of b already in a
    const uint64_t w = uint64_t(a) | (uint64_t(b) << 32);
    const uint64_t low = ((uint64_t(1) << (8 * seen)) - 1) << 32;
    const uint64_t m = json_bad_bytes((w & ~low) | (kSpaces & low));
    if (!m) return n;
    const size_t j = size_t(__builtin_ctzll(m) / 8);
    return j < 4 ? j : n - 4 + (j - 4);
  }
  for (; i < n; ++i) {
    const unsigned char c = (unsigned char)p[i];
    if (c < 0x20 || c == '"' || c == '\\') return i;
  }
  return n;
}

}  // namespace hola
