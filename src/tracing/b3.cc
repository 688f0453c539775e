#include "tracing/b3.h"

#include <cstring>
#if defined(__SSSE3__)
#include <immintrin.h>
#endif

namespace hola::tracing {

namespace {
int hexdigit(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
bool is_true(std::string_view s) { return s == "1" || s == "true" || s == "TRUE" || s == "True"; }
bool is_false(std::string_view s) { return s == "0" || s == "false" || s == "FALSE" || s == "False"; }
}  // namespace

bool parse_hex64(std::string_view s, uint64_t* out) {
  if (s.empty() || s.size() > 16) return false;
  uint64_t v = 0;
  for (char c : s) {
    int d = hexdigit(c);
    if (d < 0) return false;
    v = (v << 4) | uint64_t(d);
  }
  *out = v;
  return true;
}

bool parse_trace_id(std::string_view s, uint64_t* hi, uint64_t* lo) {
  if (s.size() > 16) {
    if (s.size() != 32) return false;
    return parse_hex64(s.substr(0, 16), hi) && parse_hex64(s.substr(16), lo);
  }
  *hi = 0;
  return parse_hex64(s, lo);
}

void hex64(uint64_t v, char out[16]) {
#if defined(__SSSE3__)
  // all 16 digits at once: the id's bytes in print order, split into nibbles, interleaved
  // high/low, looked up in a 16-entry table with one shuffle (three ids per traced
  // downstream call; the nibble loop was ~64 instructions each)
  const __m128i x = _mm_cvtsi64_si128(int64_t(__builtin_bswap64(v)));
  const __m128i mask = _mm_set1_epi8(0x0f);
  const __m128i nib = _mm_unpacklo_epi8(_mm_and_si128(_mm_srli_epi16(x, 4), mask), _mm_and_si128(x, mask));
  const __m128i lut = _mm_setr_epi8('0', '1', '2', '3', '4', '5', '6', '7', '8', '9', 'a', 'b', 'c', 'd', 'e', 'f');
  _mm_storeu_si128(reinterpret_cast<__m128i*>(out), _mm_shuffle_epi8(lut, nib));
#else
  static const char* d = "0123456789abcdef";
  for (int i = 15; i >= 0; --i) {
    out[i] = d[v & 15];
    v >>= 4;
  }
#endif
}

std::string hex64(uint64_t v) {
  char b[16];
  hex64(v, b);
  return std::string(b, 16);
}

std::string trace_id_hex(uint64_t hi, uint64_t lo) { return hi ? hex64(hi) + hex64(lo) : hex64(lo); }

Extract extract(std::string_view trace_id, std::string_view span_id, std::string_view parent_id,
                std::string_view sampled, std::string_view flags, std::string_view single,
                SpanContext* out) {
  *out = SpanContext();
  if (!single.empty()) {
    // b3: {TraceId}-{SpanId}[-{SamplingState}[-{ParentSpanId}]]  or just {SamplingState}
    if (single == "0") return Extract::kNotSampled;
    // Split on '-' by hand (gcc 11 mis-warns on chained string_view::find here).
    std::string_view part[4];
    int n = 0;
    size_t from = 0;
    for (size_t i = 0; i <= single.size() && n < 3; ++i) {
      if (i == single.size() || single[i] == '-') {
        part[n++] = single.substr(from, i - from);
        from = i + 1;
      }
    }
    if (n == 3 && from <= single.size()) part[n++] = single.substr(from);  // parent: the rest
    if (n < 2) return Extract::kNone;  // "1"/"d": no ids
    std::string_view t = part[0], sp = part[1], state = n > 2 ? part[2] : std::string_view(),
                     parent = n > 3 ? part[3] : std::string_view();
    if (state == "0") return Extract::kNotSampled;
    if (!parse_trace_id(t, &out->trace_hi, &out->trace_id) || !parse_hex64(sp, &out->span_id))
      return Extract::kNone;
    if (!parent.empty() && parse_hex64(parent, &out->parent_id)) out->has_parent = true;
    out->sampled = true;
    out->debug = state == "d";
    return Extract::kContext;
  }
  bool debug = flags == "1";
  if (sampled.empty() && !debug) return Extract::kNone;
  if (!debug && is_false(sampled)) return Extract::kNotSampled;
  if (!debug && !is_true(sampled)) return Extract::kNone;
  if (trace_id.empty() || span_id.empty()) return Extract::kNone;
  if (!parse_trace_id(trace_id, &out->trace_hi, &out->trace_id) || !parse_hex64(span_id, &out->span_id))
    return Extract::kNone;
  if (!parent_id.empty() && parse_hex64(parent_id, &out->parent_id)) out->has_parent = true;
  out->sampled = true;
  out->debug = debug;
  return Extract::kContext;
}

void inject(const SpanContext& ctx, std::string* h) {
  // Formatted into a local buffer with fixed-size copies (inlined moves), then one append:
  // this runs on every traced downstream call, and an append per piece was a memcpy call each.
  char buf[192];
  char* p = buf;
  auto lit = [&](const auto& s) {
    memcpy(p, s, sizeof s - 1);
    p += sizeof s - 1;
  };
  auto put = [&](uint64_t v) {
    hex64(v, p);
    p += 16;
  };
  lit("X-B3-TraceId: ");
  if (ctx.trace_hi) put(ctx.trace_hi);
  put(ctx.trace_id);
  lit("\r\nX-B3-SpanId: ");
  put(ctx.span_id);
  if (ctx.has_parent) {
    lit("\r\nX-B3-ParentSpanId: ");
    put(ctx.parent_id);
  }
  if (ctx.sampled) lit("\r\nX-B3-Sampled: 1\r\n");
  else lit("\r\nX-B3-Sampled: 0\r\n");
  if (ctx.debug) lit("X-B3-Flags: 1\r\n");
  h->append(buf, size_t(p - buf));  // at most 14+32+16+16+21+16+19+15 = 149 bytes
}

}  // namespace hola::tracing
