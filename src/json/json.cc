#include "json/json.h"

#include <cstdio>

#include "config/properties.h"
#include "core/scan.h"

namespace hola::json {

namespace {
// 1 = must be escaped: control characters, '"' and '\\'.
constexpr bool needs_escape(unsigned char c) { return c < 0x20 || c == '"' || c == '\\'; }
}  // namespace

void append_string(std::string* out, std::string_view s) {
  const size_t plain = json_plain_prefix(s.data(), s.size());
  if (plain == s.size()) {  // nothing to escape (aloha's greetings): three appends
    out->push_back('"');
    out->append(s.data(), s.size());
    out->push_back('"');
    return;
  }
  out->reserve(out->size() + s.size() + 8);
  out->push_back('"');
  size_t run = 0;  // start of the pending run of characters copied verbatim
  for (size_t i = plain; i < s.size(); ++i) {
    unsigned char c = (unsigned char)s[i];
    if (!needs_escape(c)) continue;
    out->append(s.data() + run, i - run);
    run = i + 1;
    switch (c) {
      case '"': out->append("\\\""); break;
      case '\\': out->append("\\\\"); break;
      case '\b': out->append("\\b"); break;
      case '\f': out->append("\\f"); break;
      case '\n': out->append("\\n"); break;
      case '\r': out->append("\\r"); break;
      case '\t': out->append("\\t"); break;
      default: {
        char buf[8];
        snprintf(buf, sizeof buf, "\\u%04X", c);
        out->append(buf);
      }
    }
  }
  out->append(s.data() + run, s.size() - run);
  out->push_back('"');
}

size_t quoted_size(std::string_view s) {
  size_t n = s.size() + 2;
  const size_t plain = json_plain_prefix(s.data(), s.size());
  for (unsigned char c : s.substr(plain))
    if (needs_escape(c)) n += (c == '"' || c == '\\' || c == '\b' || c == '\f' || c == '\n' || c == '\r' || c == '\t') ? 1 : 5;
  return n;
}

std::string quote(std::string_view s) {
  std::string r;
  append_string(&r, s);
  return r;
}

std::string string_array(const std::vector<std::optional<std::string>>& items) {
  std::string r = "[";
  for (size_t i = 0; i < items.size(); ++i) {
    if (i) r.push_back(',');
    if (items[i]) append_string(&r, *items[i]);
    else r.append("null");
  }
  r.push_back(']');
  return r;
}

const Value* Value::get(std::string_view key) const {
  for (const auto& kv : obj)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

namespace {

struct Parser {
  std::string_view s;
  size_t i = 0;
  std::string err;
  int depth = 0;

  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  bool fail(const char* m) {
    if (err.empty()) err = std::string(m) + " at offset " + std::to_string(i);
    return false;
  }
  bool lit(std::string_view w) {
    if (s.substr(i, w.size()) != w) return fail("bad literal");
    i += w.size();
    return true;
  }
  bool hex4(uint32_t* v) {
    if (i + 4 > s.size()) return fail("short \\u escape");
    *v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s[i++];
      int h = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
      if (h < 0) return fail("bad \\u escape");
      *v = *v * 16 + uint32_t(h);
    }
    return true;
  }
  bool str(std::string* out) {
    if (i >= s.size() || s[i] != '"') return fail("expected string");
    ++i;
    out->clear();
    while (i < s.size()) {
      // the run of plain characters up to the next quote, escape or control character goes
      // in with one append (aloha's greetings have no escapes)
      const size_t run = i + json_plain_prefix(s.data() + i, s.size() - i);
      if (run != i) {
        out->append(s.data() + i, run - i);
        i = run;
        if (i >= s.size()) break;
      }
      char c = s[i++];
      if (c == '"') return true;
      if ((unsigned char)c < 0x20) return fail("control character in string");
      if (c != '\\') {
        out->push_back(c);
        continue;
      }
      if (i >= s.size()) break;
      c = s[i++];
      switch (c) {
        case '"': out->push_back('"'); break;
        case '\\': out->push_back('\\'); break;
        case '/': out->push_back('/'); break;
        case 'b': out->push_back('\b'); break;
        case 'f': out->push_back('\f'); break;
        case 'n': out->push_back('\n'); break;
        case 'r': out->push_back('\r'); break;
        case 't': out->push_back('\t'); break;
        case 'u': {
          uint32_t v = 0;
          if (!hex4(&v)) return false;
          if (v >= 0xD800 && v <= 0xDBFF && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
            size_t save = i;
            i += 2;
            uint32_t lo = 0;
            if (hex4(&lo) && lo >= 0xDC00 && lo <= 0xDFFF) {
              config::append_utf8(out, 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00));
              break;
            }
            i = save;
            err.clear();
          }
          if (v >= 0xD800 && v <= 0xDFFF) out->push_back('?');
          else config::append_utf8(out, v);
          break;
        }
        default: return fail("bad escape");
      }
    }
    return fail("unterminated string");
  }
  bool num(Value* v) {
    size_t st = i;
    if (i < s.size() && s[i] == '-') ++i;
    if (i >= s.size()) return fail("bad number");
    if (s[i] == '0') ++i;
    else if (s[i] >= '1' && s[i] <= '9') while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
    else return fail("bad number");
    if (i < s.size() && s[i] == '.') {
      ++i;
      if (i >= s.size() || s[i] < '0' || s[i] > '9') return fail("bad fraction");
      while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
    }
    if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
      ++i;
      if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
      if (i >= s.size() || s[i] < '0' || s[i] > '9') return fail("bad exponent");
      while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
    }
    v->type = Value::Type::kNumber;
    v->text = std::string(s.substr(st, i - st));
    return true;
  }
  bool value(Value* v) {
    if (++depth > 64) return fail("nesting too deep");
    ws();
    if (i >= s.size()) return fail("unexpected end");
    char c = s[i];
    bool ok;
    if (c == '"') {
      v->type = Value::Type::kString;
      ok = str(&v->text);
    } else if (c == '[') {
      ++i;
      v->type = Value::Type::kArray;
      ws();
      ok = true;
      if (i < s.size() && s[i] == ']') {
        ++i;
      } else {
        for (;;) {
          v->arr.emplace_back();
          if (!value(&v->arr.back())) { ok = false; break; }
          ws();
          if (i < s.size() && s[i] == ',') { ++i; continue; }
          if (i < s.size() && s[i] == ']') { ++i; break; }
          ok = fail("expected , or ]");
          break;
        }
      }
    } else if (c == '{') {
      ++i;
      v->type = Value::Type::kObject;
      ws();
      ok = true;
      if (i < s.size() && s[i] == '}') {
        ++i;
      } else {
        for (;;) {
          ws();
          std::string k;
          if (!str(&k)) { ok = false; break; }
          ws();
          if (i >= s.size() || s[i] != ':') { ok = fail("expected :"); break; }
          ++i;
          v->obj.emplace_back(std::move(k), Value());
          if (!value(&v->obj.back().second)) { ok = false; break; }
          ws();
          if (i < s.size() && s[i] == ',') { ++i; continue; }
          if (i < s.size() && s[i] == '}') { ++i; break; }
          ok = fail("expected , or }");
          break;
        }
      }
    } else if (c == 't') {
      v->type = Value::Type::kBool;
      v->b = true;
      ok = lit("true");
    } else if (c == 'f') {
      v->type = Value::Type::kBool;
      ok = lit("false");
    } else if (c == 'n') {
      v->type = Value::Type::kNull;
      ok = lit("null");
    } else {
      ok = num(v);
    }
    --depth;
    return ok;
  }
};

}  // namespace

bool parse(std::string_view in, Value* out, std::string* err) {
  Parser p;
  p.s = in;
  *out = Value();
  if (!p.value(out)) {
    if (err) *err = p.err;
    return false;
  }
  p.ws();
  if (p.i != in.size()) {
    if (err) *err = "trailing characters at offset " + std::to_string(p.i);
    return false;
  }
  return true;
}

bool plain_string_list(std::string_view in, size_t* count) {
  const size_t n = in.size();
  if (n < 2 || in[0] != '[' || in[n - 1] != ']') return false;
  size_t k = 0;
  if (n > 2) {
    const size_t end = n - 1;  // the closing bracket: no string may run into it
    size_t i = 1;
    for (;;) {
      if (in[i] != '"') return false;
      ++i;
      i += json_plain_prefix(in.data() + i, end - i);  // stops at the closing quote, an escape or a control
      if (i >= end || in[i] != '"') return false;
      ++i;
      ++k;
      if (i == end) break;
      if (in[i] != ',' || i + 1 >= end) return false;
      ++i;
    }
  }
  *count = k;
  return true;
}

bool decode_string_list(std::string_view in, std::vector<std::optional<std::string>>* out,
                        std::string* err) {
  // Streams straight into *out (no DOM): this runs once per aloha response. The elements
  // already in *out are reused (a string keeps its capacity), so a caller that decodes into
  // the same vector every time allocates nothing in the steady state.
  Parser p;
  p.s = in;
  size_t n = 0;
  auto next_str = [&]() -> std::string* {
    if (n < out->size()) {
      auto& o = (*out)[n++];
      if (!o) o.emplace();
      o->clear();
      return &*o;
    }
    out->emplace_back(std::string());
    ++n;
    return &*out->back();
  };
  auto next_null = [&] {
    if (n < out->size()) (*out)[n++].reset();
    else {
      out->emplace_back(std::nullopt);
      ++n;
    }
  };
  auto fail = [&](const std::string& m) {
    if (err) *err = p.err.empty() ? m : p.err;
    return false;
  };
  p.ws();
  if (p.i >= in.size() || in[p.i] != '[') {
    if (p.i < in.size() && in[p.i] == '{') return fail("expected a JSON array");
    Value v;  // not an array: report what a full parse would (syntax error or wrong type)
    std::string e;
    if (!parse(in, &v, &e)) return fail(e);
    return fail("expected a JSON array");
  }
  ++p.i;
  p.ws();
  if (p.i < in.size() && in[p.i] == ']') {
    ++p.i;
  } else {
    for (;;) {
      p.ws();
      if (p.i >= in.size()) return fail("unexpected end at offset " + std::to_string(p.i));
      char c = in[p.i];
      if (c == '"') {
        if (!p.str(next_str())) return fail("bad string");
      } else if (c == 'n') {
        if (!p.lit("null")) return fail("bad literal");
        next_null();
      } else if (c == 't' || c == 'f') {
        if (!p.lit(c == 't' ? "true" : "false")) return fail("bad literal");
        next_str()->assign(c == 't' ? "true" : "false");
      } else if (c == '[' || c == '{') {
        return fail("cannot deserialize java.lang.String out of a nested array/object");
      } else {
        Value v;
        if (!p.num(&v)) return fail("bad number");
        *next_str() = std::move(v.text);
      }
      p.ws();
      if (p.i < in.size() && in[p.i] == ',') {
        ++p.i;
        continue;
      }
      if (p.i < in.size() && in[p.i] == ']') {
        ++p.i;
        break;
      }
      return fail("expected , or ] at offset " + std::to_string(p.i));
    }
  }
  p.ws();
  if (p.i != in.size()) return fail("trailing characters at offset " + std::to_string(p.i));
  out->resize(n);
  return true;
}

}  // namespace hola::json
