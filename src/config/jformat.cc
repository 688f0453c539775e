#include "config/jformat.h"

#include <algorithm>
#include <cstdint>
#include <cstdio>

#include "config/properties.h"

namespace hola::config {

namespace {

// Decodes UTF-8 into code points; invalid bytes map to U+FFFD (as a Java decoder would).
std::vector<uint32_t> decode_utf8(std::string_view s) {
  std::vector<uint32_t> cps;
  for (size_t i = 0; i < s.size();) {
    unsigned char c = (unsigned char)s[i];
    uint32_t cp;
    int n;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 6) { cp = c & 0x1F; n = 2; }
    else if ((c >> 4) == 14) { cp = c & 0x0F; n = 3; }
    else if ((c >> 3) == 30) { cp = c & 0x07; n = 4; }
    else { cps.push_back(0xFFFD); ++i; continue; }
    if (i + size_t(n) > s.size()) { cps.push_back(0xFFFD); ++i; continue; }
    bool bad = false;
    for (int k = 1; k < n; ++k) {
      unsigned char d = (unsigned char)s[i + size_t(k)];
      if ((d >> 6) != 2) { bad = true; break; }
      cp = (cp << 6) | (d & 0x3F);
    }
    if (bad) { cps.push_back(0xFFFD); ++i; continue; }
    cps.push_back(cp);
    i += size_t(n);
  }
  return cps;
}

// Java measures width/precision in UTF-16 code units.
size_t utf16_len(const std::vector<uint32_t>& cps) {
  size_t n = 0;
  for (uint32_t c : cps) n += c >= 0x10000 ? 2 : 1;
  return n;
}

std::string encode(const std::vector<uint32_t>& cps) {
  std::string s;
  for (uint32_t c : cps) append_utf8(&s, c);
  return s;
}

// String.toUpperCase(Locale.ROOT-ish) for the characters a greeting plausibly contains.
std::vector<uint32_t> to_upper(const std::vector<uint32_t>& in) {
  std::vector<uint32_t> out;
  for (uint32_t c : in) {
    if (c >= 'a' && c <= 'z') out.push_back(c - 32);
    else if (c == 0xDF) { out.push_back('S'); out.push_back('S'); }
    else if (c >= 0xE0 && c <= 0xFE && c != 0xF7) out.push_back(c - 32);
    else if (c == 0xFF) out.push_back(0x178);
    else if (c >= 0x100 && c <= 0x17F && (c & 1) && c != 0x131 && c != 0x138 && c != 0x149 && c != 0x17F &&
             !(c >= 0x139 && c <= 0x148) && !(c >= 0x179 && c <= 0x17E)) out.push_back(c - 1);
    else if (((c >= 0x139 && c <= 0x148) || (c >= 0x179 && c <= 0x17E)) && !(c & 1)) out.push_back(c - 1);
    else if (c >= 0x3B1 && c <= 0x3C9 && c != 0x3C2) out.push_back(c - 32);
    else if (c >= 0x430 && c <= 0x44F) out.push_back(c - 32);
    else if (c >= 0x450 && c <= 0x45F) out.push_back(c - 80);
    else out.push_back(c);
  }
  return out;
}

struct Spec {
  int index = 0;       // >0 explicit, 0 ordinary, -1 relative ('<')
  std::string flags;
  int width = -1;
  int precision = -1;
  bool dt = false;     // 't' / 'T' prefix
  char conv = 0;
};

bool has(const std::string& f, char c) { return f.find(c) != std::string::npos; }

FormatResult fail(const char* name, std::string detail) {
  FormatResult r;
  r.ok = false;
  r.error = name;
  r.detail = std::move(detail);
  return r;
}

bool parse_int(std::string_view s, size_t* i, int* out) {
  size_t st = *i;
  long v = 0;
  while (*i < s.size() && s[*i] >= '0' && s[*i] <= '9') {
    v = v * 10 + (s[*i] - '0');
    if (v > 1000000000) v = 1000000000;
    ++*i;
  }
  if (*i == st) return false;
  *out = int(v);
  return true;
}

// Digits as Formatter's width()/precision() read them: a value past Integer.MAX_VALUE fails
// Integer.parseInt, which Formatter reports as an illegal width/precision of MIN_VALUE.
bool parse_long(std::string_view s, size_t* i, long long* out) {
  size_t st = *i;
  long long v = 0;
  while (*i < s.size() && s[*i] >= '0' && s[*i] <= '9') {
    v = v * 10 + (s[*i] - '0');
    if (v > 1000000000000LL) v = 1000000000000LL;
    ++*i;
  }
  if (*i == st) return false;
  *out = v;
  return true;
}
constexpr long long kIntMax = 2147483647LL;

// The reference's JVM runs with -Xmx512m (the manifests' JAVA_OPTIONS), so a translation
// whose widths pad the greeting to hundreds of millions of characters ends in an
// OutOfMemoryError, a 500. The output here is bounded well below that (32 Mi code units), so
// such a configuration costs a 500 per request instead of the process's memory.
constexpr size_t kMaxOutput = size_t(32) << 20;

void justify(std::string* out, const std::vector<uint32_t>& cps, int width, bool left) {
  size_t len = utf16_len(cps);
  std::string body = encode(cps);
  if (width > 0 && size_t(width) > len) {
    std::string pad(size_t(width) - len, ' ');
    if (left) body += pad;
    else body = pad + body;
  }
  *out += body;
}

}  // namespace

int32_t java_string_hash(std::string_view utf8) {
  uint32_t h = 0;
  for (uint32_t c : decode_utf8(utf8)) {
    if (c >= 0x10000) {
      uint32_t v = c - 0x10000;
      h = 31 * h + (0xD800 + (v >> 10));
      h = 31 * h + (0xDC00 + (v & 0x3FF));
    } else {
      h = 31 * h + c;
    }
  }
  return int32_t(h);
}

FormatResult java_format(std::string_view fmt, const std::vector<std::string>& args) {
  std::string out;
  int ordinary = 0;    // next ordinary index (0-based)
  int last = -1;       // last used index for '<'
  size_t i = 0;
  while (i < fmt.size()) {
    size_t pct = fmt.find('%', i);
    if (pct == std::string_view::npos) {
      out.append(fmt.substr(i));
      break;
    }
    out.append(fmt.substr(i, pct - i));
    i = pct + 1;
    // Formatter's pattern: %(\d+\$)?([-#+ 0,(\<]*)?(\d+)?(\.\d+)?([tT])?([a-zA-Z%])
    Spec sp;
    size_t save = i;
    int n;
    if (parse_int(fmt, &i, &n) && i < fmt.size() && fmt[i] == '$') {
      sp.index = n;
      ++i;
    } else {
      i = save;
    }
    while (i < fmt.size() && std::string_view("-#+ 0,(<").find(fmt[i]) != std::string_view::npos) {
      if (has(sp.flags, fmt[i]))
        return fail("DuplicateFormatFlagsException", std::string("Flags = '") + fmt[i] + "'");
      sp.flags.push_back(fmt[i]);
      ++i;
    }
    long long wide = 0;
    if (parse_long(fmt, &i, &wide)) {
      if (wide > kIntMax) return fail("IllegalFormatWidthException", "-2147483648");
      sp.width = int(wide);
    }
    if (i < fmt.size() && fmt[i] == '.') {
      size_t j = i + 1;
      if (parse_long(fmt, &j, &wide)) {
        if (wide > kIntMax) return fail("IllegalFormatPrecisionException", "-2147483648");
        sp.precision = int(wide);
        i = j;
      } else {
        return fail("UnknownFormatConversionException", "Conversion = '.'");
      }
    }
    if (i < fmt.size() && (fmt[i] == 't' || fmt[i] == 'T')) {
      sp.dt = true;
      ++i;
    }
    if (i >= fmt.size()) {
      return fail("UnknownFormatConversionException", "Conversion = '%'");
    }
    char c = fmt[i++];
    if (!((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '%'))
      return fail("UnknownFormatConversionException", std::string("Conversion = '") + c + "'");
    sp.conv = c;
    if (sp.dt) {
      // %tX with a String argument
      int idx = sp.index > 0 ? sp.index - 1 : (has(sp.flags, '<') ? last : ordinary++);
      if (idx < 0 || size_t(idx) >= args.size())
        return fail("MissingFormatArgumentException", "Format specifier '%t" + std::string(1, c) + "'");
      return fail("IllegalFormatConversionException", std::string(1, c) + " != java.lang.String");
    }
    bool left = has(sp.flags, '-');
    if (c == '%' || c == 'n') {
      if (c == 'n') {
        if (sp.width >= 0) return fail("IllegalFormatWidthException", std::to_string(sp.width));
        if (!sp.flags.empty()) return fail("IllegalFormatFlagsException", "Flags = '" + sp.flags + "'");
        if (sp.precision >= 0) return fail("IllegalFormatPrecisionException", std::to_string(sp.precision));
        out.push_back('\n');
        continue;
      }
      if (sp.precision >= 0) return fail("IllegalFormatPrecisionException", std::to_string(sp.precision));
      for (char f : sp.flags)
        if (f != '-') return fail("IllegalFormatFlagsException", "Flags = '" + sp.flags + "'");
      if (left && sp.width < 0) return fail("MissingFormatWidthException", "%-%");
      if (size_t(std::max(sp.width, 0)) + out.size() > kMaxOutput) return fail("OutOfMemoryError", "Java heap space");
      justify(&out, {uint32_t('%')}, sp.width, left);
      continue;
    }
    bool known = std::string_view("bBhHsScCdoxXeEfgGaA").find(c) != std::string_view::npos;
    if (!known) return fail("UnknownFormatConversionException", std::string("Conversion = '") + c + "'");
    if (left && sp.width < 0) return fail("MissingFormatWidthException", std::string("%-") + c);
    // resolve the argument
    int idx;
    if (sp.index > 0) idx = sp.index - 1;
    else if (has(sp.flags, '<')) idx = last;
    else idx = ordinary++;
    if (idx < 0 || size_t(idx) >= args.size())
      return fail("MissingFormatArgumentException", std::string("Format specifier '%") + c + "'");
    last = idx;
    if (size_t(std::max(sp.width, 0)) + out.size() > kMaxOutput) return fail("OutOfMemoryError", "Java heap space");
    const std::string& arg = args[size_t(idx)];
    switch (c) {
      case 's':
      case 'S': {
        if (has(sp.flags, '#'))
          return fail("FormatFlagsConversionMismatchException", std::string("Conversion = s, Flags = #"));
        for (char f : sp.flags)
          if (f != '-' && f != '<')
            return fail("FormatFlagsConversionMismatchException",
                        std::string("Conversion = ") + c + ", Flags = " + f);
        std::vector<uint32_t> cps = decode_utf8(arg);
        if (sp.precision >= 0) {
          std::vector<uint32_t> cut;
          size_t units = 0;
          for (uint32_t cp : cps) {
            size_t u = cp >= 0x10000 ? 2 : 1;
            if (units + u > size_t(sp.precision)) break;
            units += u;
            cut.push_back(cp);
          }
          cps.swap(cut);
        }
        if (c == 'S') cps = to_upper(cps);
        justify(&out, cps, sp.width, left);
        break;
      }
      case 'b':
      case 'B':
      case 'h':
      case 'H': {
        for (char f : sp.flags)
          if (f != '-' && f != '<')
            return fail("FormatFlagsConversionMismatchException",
                        std::string("Conversion = ") + c + ", Flags = " + f);
        std::string v;
        if (c == 'b' || c == 'B') {
          v = "true";  // non-null, non-Boolean argument
        } else {
          char hex[16];
          snprintf(hex, sizeof hex, "%x", uint32_t(java_string_hash(arg)));
          v = hex;
        }
        std::vector<uint32_t> cps = decode_utf8(v);
        if (sp.precision >= 0 && size_t(sp.precision) < cps.size()) cps.resize(size_t(sp.precision));
        if (c == 'B' || c == 'H') cps = to_upper(cps);
        justify(&out, cps, sp.width, left);
        break;
      }
      default:
        // c, d, o, x, X, e, E, f, g, G, a, A applied to a java.lang.String
        return fail("IllegalFormatConversionException", std::string(1, c) + " != java.lang.String");
    }
  }
  if (out.size() > kMaxOutput) return fail("OutOfMemoryError", "Java heap space");
  FormatResult r;
  r.value = std::move(out);
  return r;
}

}  // namespace hola::config
