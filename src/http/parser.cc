#include "http/parser.h"

#include "core/scan.h"

#if defined(__AVX2__)
#include <immintrin.h>
#endif

#include <cstring>
#include <type_traits>

namespace hola::http {

namespace {

// A fresh Request, copied from a constant in 32-byte vector moves. `*req = Request()` built the
// temporary on the stack with `rep stos` and copied it out with 16-byte loads of 8-byte
// stores, which miss store forwarding; a plain copy or memset of the constant compiles to
// `rep stos`/`rep movs` too, whose start-up alone costs tens of cycles at this size. Together
// about half of parse_request's time for a wrk-style request (bench/micro.cc).
static_assert(std::is_trivially_copyable_v<Request>);
const Request kFreshRequest{};
inline void reset_request(Request* req) {
#if !defined(__AVX2__)
  memcpy(static_cast<void*>(req), &kFreshRequest, sizeof(Request));  // portable build (x86-64-v2)
#else
  constexpr size_t kVec = sizeof(Request) / 32, kTail = sizeof(Request) % 32;
  const auto* src = reinterpret_cast<const unsigned char*>(&kFreshRequest);
  auto* dst = reinterpret_cast<unsigned char*>(req);
  for (size_t i = 0; i < kVec; ++i)
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + 32 * i),
                        _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + 32 * i)));
  if constexpr (kTail > 0) memcpy(dst + 32 * kVec, src + 32 * kVec, kTail);
#endif
}

inline char lower(char c) { return (c >= 'A' && c <= 'Z') ? char(c + 32) : c; }

// RFC 9110 token characters, as a constant table (no initialisation guard on the hot path).
struct TcharTable {
  bool t[256] = {};
  constexpr TcharTable() {
    for (int c = '0'; c <= '9'; ++c) t[c] = true;
    for (int c = 'a'; c <= 'z'; ++c) t[c] = true;
    for (int c = 'A'; c <= 'Z'; ++c) t[c] = true;
    for (char c : std::string_view("!#$%&'*+-.^_`|~")) t[(unsigned char)c] = true;
  }
};
constexpr TcharTable kTchar;

inline bool is_tchar(unsigned char c) { return kTchar.t[c]; }

// Header-name comparison with a lowercase literal, eight bytes at a time. OR 0x20 folds the
// letters, and on token characters (a validated field name) it maps nothing else onto a
// literal's letters, digits or '-': the only other preimages, 0x0d/0x10-0x19, are controls. Not
// for field values, which may hold control characters. (The per-character iequals loop was
// ~35 instructions per known header.)
template <size_t N>
inline bool name_is(std::string_view name, const char (&lit)[N]) {
  constexpr size_t n = N - 1;
  static_assert(n >= 2 && n <= 24);
  if (name.size() != n) return false;
  auto word = [](const char* p, size_t k) {
    uint64_t w = 0;
    memcpy(&w, p, k);
    return w;
  };
  constexpr uint64_t kFold = 0x2020202020202020ull;
  if constexpr (n <= 8) {
    const uint64_t mask = n == 8 ? kFold : kFold & ((uint64_t(1) << (8 * n)) - 1);
    return (word(name.data(), n) | mask) == word(lit, n);
  } else {
    // words at 0, 8, ... and one ending at the last byte (overlapping)
    for (size_t off = 0; off + 8 < n; off += 8)
      if ((word(name.data() + off, 8) | kFold) != word(lit + off, 8)) return false;
    return (word(name.data() + n - 8, 8) | kFold) == word(lit + n - 8, 8);
  }
}

inline std::string_view trim_ows(std::string_view s) {
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t')) s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t')) s.remove_suffix(1);
  return s;
}

// Iterates comma-separated tokens of a Connection header.
template <class F>
void for_each_token(std::string_view v, F f) {
  while (!v.empty()) {
    size_t c = v.find(',');
    std::string_view t = trim_ows(v.substr(0, c));
    if (!t.empty()) f(t);
    if (c == std::string_view::npos) break;
    v.remove_prefix(c + 1);
  }
}

bool parse_uint(std::string_view s, int64_t* out) {
  if (s.empty() || s.size() > 18) return false;
  int64_t v = 0;
  for (char c : s) {
    if (c < '0' || c > '9') return false;
    v = v * 10 + (c - '0');
  }
  *out = v;
  return true;
}

}  // namespace

bool percent_decode(std::string_view in, char* out, size_t* out_len, bool keep_encoded_slash) {
  auto hex = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    c = lower(c);
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    return -1;
  };
  size_t o = 0;
  for (size_t i = 0; i < in.size(); ++i) {
    if (in[i] == '%') {
      if (i + 2 >= in.size()) return false;
      int h = hex(in[i + 1]), l = hex(in[i + 2]);
      if (h < 0 || l < 0) return false;
      const char d = char(h * 16 + l);
      if (keep_encoded_slash && d == '/') {
        memcpy(out + o, in.data() + i, 3);
        o += 3;
      } else {
        out[o++] = d;
      }
      i += 2;
    } else {
      out[o++] = in[i];
    }
  }
  *out_len = o;
  return true;
}

void strip_path_parameters(std::string_view in, char* out, size_t* out_len) {
  size_t o = 0;
  bool skipping = false;
  for (char ch : in) {
    if (ch == '/') skipping = false;
    else if (ch == ';') skipping = true;
    if (!skipping) out[o++] = ch;
  }
  *out_len = o;
}

bool remove_dot_segments(std::string_view in, char* out, size_t* out_len) {
  // RFC 3986 §5.2.4 on an absolute path, segment by segment: "." segments vanish, ".."
  // drops the last output segment (never above the root). A trailing "." or ".." leaves
  // the path ending in "/", as the RFC's "/." and "/.." rules do.
  if (in.empty() || in[0] != '/') return false;
  size_t o = 0;
  size_t i = 0;
  while (i < in.size()) {
    size_t j = i + 1;  // in[i] == '/'
    while (j < in.size() && in[j] != '/') ++j;
    std::string_view seg = in.substr(i + 1, j - i - 1);
    const bool last = j == in.size();
    if (seg == ".") {
      if (last) out[o++] = '/';
    } else if (seg == "..") {
      while (o > 0 && out[o - 1] != '/') --o;  // strip the last segment's text ...
      if (o > 0) --o;                          // ... and its leading '/'
      if (last) out[o++] = '/';
    } else {
      out[o++] = '/';
      memcpy(out + o, seg.data(), seg.size());
      o += seg.size();
    }
    i = j;
  }
  if (o == 0) out[o++] = '/';
  *out_len = o;
  return true;
}

Parse parse_request(const char* buf, size_t len, Request* req, int* status) {
  reset_request(req);
  size_t pos = 0;
  // RFC 9112 §2.2: ignore at least one empty line before the request-line.
  while (pos < len && (buf[pos] == '\r' || buf[pos] == '\n')) ++pos;
  if (pos > kMaxHeadBytes) {  // a stream of bare line breaks must not grow the buffer forever
    *status = 400;
    return Parse::kError;
  }
  if (pos == len) return Parse::kIncomplete;

  // ---- request line ----
  const char* line = buf + pos;
  const char* nl = find_newline(line, len - pos);
  if (!nl) {
    if (len - pos > kMaxRequestLine) {
      *status = 414;
      return Parse::kError;
    }
    return Parse::kIncomplete;
  }
  size_t line_len = size_t(nl - line);
  if (line_len > kMaxRequestLine) {
    *status = 414;
    return Parse::kError;
  }
  if (line_len && line[line_len - 1] == '\r') --line_len;
  // One pass over the request line: method (token chars up to the first SP), target (up to
  // the next SP, noting control characters and the '?'), then the 8-byte version.
  size_t i = 0;
  while (i < line_len && is_tchar((unsigned char)line[i])) ++i;
  if (i == 0 || i == line_len || line[i] != ' ') {
    *status = 400;
    return Parse::kError;
  }
  req->method = std::string_view(line, i);
  const size_t t0 = ++i;
  size_t q = std::string_view::npos;
  bool bad_target = false;
  // Target: up to the next SP. With 32 bytes of the buffer at hand (within `len`: no read past
  // the data), one AVX2 compare finds the SP, the first '?' and any control byte at once; a
  // target of 32 bytes or more, or one with a control byte, takes the byte loop below, which
  // decides the same (about 10 instructions per byte of "/api/hola" before). A portable
  // (x86-64-v2) build always takes the byte loop.
#if defined(__AVX2__)
  if (len - pos - t0 >= 32) {
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(line + t0));
    const uint32_t sp = uint32_t(_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, _mm256_set1_epi8(' '))));
    if (sp != 0) {
      const uint32_t p = uint32_t(__builtin_ctz(sp));
      const uint32_t before = (uint32_t(1) << p) - 1;  // p <= 31
      const uint32_t ctl =
          uint32_t(_mm256_movemask_epi8(_mm256_or_si256(
              _mm256_cmpeq_epi8(_mm256_min_epu8(v, _mm256_set1_epi8(0x1f)), v),
              _mm256_cmpeq_epi8(v, _mm256_set1_epi8(0x7f)))));
      if (t0 + p < line_len && (ctl & before) == 0) {
        const uint32_t qm = uint32_t(_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, _mm256_set1_epi8('?')))) & before;
        if (qm) q = __builtin_ctz(qm);
        i = t0 + p;
      }
    }
  }
#endif
  if (i == t0) {
    for (; i < line_len && line[i] != ' '; ++i) {
      const unsigned char c = (unsigned char)line[i];
      if (c <= 0x20 || c == 0x7f) bad_target = true;
      else if (c == '?' && q == std::string_view::npos) q = i - t0;
    }
  }
  if (i == line_len || i == t0) {
    *status = 400;
    return Parse::kError;
  }
  req->target = std::string_view(line + t0, i - t0);
  std::string_view ver(line + i + 1, line_len - i - 1);
  if (ver.size() != 8 || ver.substr(0, 5) != "HTTP/" || ver[6] != '.' || ver[5] < '0' ||
      ver[5] > '9' || ver[7] < '0' || ver[7] > '9') {
    *status = 400;
    return Parse::kError;
  }
  if (ver[5] != '1') {
    *status = 505;
    return Parse::kError;
  }
  req->version_minor = ver[7] - '0';
  if (bad_target) {
    *status = 400;
    return Parse::kError;
  }
  req->path = req->target.substr(0, q);
  if (q != std::string_view::npos) req->query = req->target.substr(q + 1);
  // Absolute-form targets (proxies): strip scheme://authority.
  if (req->path.size() > 7 && req->path[0] != '/' &&
      (req->path.substr(0, 7) == "http://" || req->path.substr(0, 8) == "https://")) {
    size_t s = req->path.find('/', req->path.find("//") + 2);
    req->path = s == std::string_view::npos ? std::string_view("/") : req->path.substr(s);
  }

  // ---- header fields ----
  bool conn_close = false, conn_keep = false, have_cl = false, have_te = false;
  size_t p = size_t(nl - buf) + 1;
  for (;;) {
    if (p >= len) {
      if (len > kMaxHeadBytes) {
        *status = 431;
        return Parse::kError;
      }
      return Parse::kIncomplete;
    }
    const char* hl = buf + p;
    const char* he = find_newline(hl, len - p);
    if (!he) {
      if (len > kMaxHeadBytes) {
        *status = 431;
        return Parse::kError;
      }
      return Parse::kIncomplete;
    }
    size_t hlen = size_t(he - hl);
    p = size_t(he - buf) + 1;
    if (p > kMaxHeadBytes) {
      *status = 431;
      return Parse::kError;
    }
    if (hlen && hl[hlen - 1] == '\r') --hlen;
    if (hlen == 0) break;  // end of head
    // Field name: token characters up to the colon. Anything else before it (obs-fold
    // leading whitespace, spaces before the colon, a missing colon) is a 400 (RFC 9112 §5).
    size_t colon = 0;
    while (colon < hlen && is_tchar((unsigned char)hl[colon])) ++colon;
    if (colon == 0 || colon == hlen || hl[colon] != ':') {
      *status = 400;
      return Parse::kError;
    }
    std::string_view h(hl, hlen);
    std::string_view name = h.substr(0, colon);
    std::string_view value = trim_ows(h.substr(colon + 1));
    switch (name.size()) {
      case 2:
        if (name_is(name, "b3")) req->b3_single = value;
        break;
      case 4:
        if (name_is(name, "host")) req->host = value;
        break;
      case 6:
        if (name_is(name, "expect")) {
          req->expect_continue = iequals(value, "100-continue");
        } else if (name_is(name, "accept")) {
          // Multiple Accept fields are equivalent to one comma-joined field; keep the first
          // and let the negotiation treat a second one conservatively (rare in practice).
          if (!req->has_accept) req->accept = value;
          req->has_accept = true;
        }
        break;
      case 10:
        if (name_is(name, "connection")) {
          for_each_token(value, [&](std::string_view t) {
            if (iequals(t, "close")) conn_close = true;
            else if (iequals(t, "keep-alive")) conn_keep = true;
          });
        } else if (name_is(name, "x-b3-flags")) {
          req->b3_flags = value;
        }
        break;
      case 12:
        if (name_is(name, "x-b3-traceid")) req->b3_trace_id = value;
        else if (name_is(name, "x-b3-sampled")) req->b3_sampled = value;
        break;
      case 11:
        if (name_is(name, "x-b3-spanid")) req->b3_span_id = value;
        break;
      case 14:
        if (name_is(name, "content-length")) {
          int64_t v;
          if (!parse_uint(value, &v) || (have_cl && v != req->content_length)) {
            *status = 400;
            return Parse::kError;
          }
          have_cl = true;
          req->content_length = v;
        }
        break;
      case 17:
        if (name_is(name, "transfer-encoding")) {
          have_te = true;
          std::string_view last;
          for_each_token(value, [&](std::string_view t) { last = t; });
          if (iequals(last, "chunked")) {
            req->chunked = true;
          } else {
            *status = 501;
            return Parse::kError;
          }
        } else if (name_is(name, "x-b3-parentspanid")) {
          req->b3_parent_id = value;
        }
        break;
      default:
        break;
    }
  }
  if (have_te && have_cl) {  // request smuggling guard (RFC 9112 §6.3)
    *status = 400;
    return Parse::kError;
  }
  if (req->version_minor == 0) req->keep_alive = conn_keep && !conn_close;
  else req->keep_alive = !conn_close;
  req->head_bytes = p;
  return Parse::kOk;
}

Parse skip_chunked_body(const char* buf, size_t len, size_t* consumed) {
  return decode_chunked_body(buf, len, consumed, nullptr);
}

Parse decode_chunked_body(const char* buf, size_t len, size_t* consumed, std::string* body) {
  size_t p = 0;
  for (;;) {
    const char* nl = static_cast<const char*>(memchr(buf + p, '\n', len - p));
    if (!nl) return len - p > 1024 ? Parse::kError : Parse::kIncomplete;
    std::string_view line(buf + p, size_t(nl - (buf + p)));
    if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
    size_t semi = line.find(';');
    std::string_view hexs = line.substr(0, semi);
    while (!hexs.empty() && (hexs.back() == ' ' || hexs.back() == '\t')) hexs.remove_suffix(1);
    if (hexs.empty() || hexs.size() > 15) return Parse::kError;
    uint64_t sz = 0;
    for (char c : hexs) {
      int d;
      if (c >= '0' && c <= '9') d = c - '0';
      else if ((c | 32) >= 'a' && (c | 32) <= 'f') d = (c | 32) - 'a' + 10;
      else return Parse::kError;
      sz = sz * 16 + uint64_t(d);
    }
    p = size_t(nl - buf) + 1;
    if (sz == 0) {
      // trailer section, terminated by an empty line
      for (;;) {
        const char* tl = static_cast<const char*>(memchr(buf + p, '\n', len - p));
        if (!tl) return Parse::kIncomplete;
        size_t l = size_t(tl - (buf + p));
        bool empty = l == 0 || (l == 1 && buf[p] == '\r');
        p = size_t(tl - buf) + 1;
        if (empty) {
          *consumed = p;
          return Parse::kOk;
        }
      }
    }
    if (len - p < sz + 2) return Parse::kIncomplete;
    if (body) body->append(buf + p, size_t(sz));
    p += sz;
    if (buf[p] == '\r') ++p;
    if (p >= len) return Parse::kIncomplete;
    if (buf[p] != '\n') return Parse::kError;
    ++p;
  }
}

}  // namespace hola::http
