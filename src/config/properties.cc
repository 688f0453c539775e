#include "config/properties.h"

#include <cstdint>

namespace hola::config {

void append_utf8(std::string* out, uint32_t cp) {
  if (cp < 0x80) {
    out->push_back(char(cp));
  } else if (cp < 0x800) {
    out->push_back(char(0xC0 | (cp >> 6)));
    out->push_back(char(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    out->push_back(char(0xE0 | (cp >> 12)));
    out->push_back(char(0x80 | ((cp >> 6) & 0x3F)));
    out->push_back(char(0x80 | (cp & 0x3F)));
  } else {
    out->push_back(char(0xF0 | (cp >> 18)));
    out->push_back(char(0x80 | ((cp >> 12) & 0x3F)));
    out->push_back(char(0x80 | ((cp >> 6) & 0x3F)));
    out->push_back(char(0x80 | (cp & 0x3F)));
  }
}

namespace {

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\f'; }

// Splits text into logical lines the way java.util.Properties.LineReader does.
std::vector<std::string> logical_lines(std::string_view in) {
  std::vector<std::string> lines;
  std::string buf;
  bool skip_ws = true, comment = false, new_line = true, appended_begin = false;
  bool preceding_backslash = false, skip_lf = false;
  for (size_t i = 0; i < in.size(); ++i) {
    char c = in[i];
    if (skip_lf) {
      skip_lf = false;
      if (c == '\n') continue;
    }
    if (skip_ws) {
      if (is_ws(c)) continue;
      if (!appended_begin && (c == '\r' || c == '\n')) continue;
      skip_ws = false;
      appended_begin = false;
    }
    if (new_line) {
      new_line = false;
      if (c == '#' || c == '!') {
        comment = true;
        continue;
      }
    }
    if (c != '\n' && c != '\r') {
      buf.push_back(c);
      preceding_backslash = (c == '\\') ? !preceding_backslash : false;
      continue;
    }
    // end of a natural line
    if (comment || buf.empty()) {
      comment = false;
      new_line = true;
      skip_ws = true;
      buf.clear();
      preceding_backslash = false;
      continue;
    }
    if (preceding_backslash) {
      buf.pop_back();  // the continuation backslash
      skip_ws = true;
      appended_begin = true;
      preceding_backslash = false;
      if (c == '\r') skip_lf = true;
    } else {
      lines.push_back(std::move(buf));
      buf.clear();
      skip_ws = true;
      new_line = true;
      preceding_backslash = false;
    }
  }
  if (!buf.empty() && !comment) {
    if (preceding_backslash) buf.pop_back();
    lines.push_back(std::move(buf));
  }
  return lines;
}

int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// Properties.loadConvert: resolves escapes. UTF-16 surrogate pairs written as two \u
// escapes are combined; a lone surrogate becomes '?' (what a Java String encoder emits).
bool load_convert(std::string_view s, std::string* out, std::string* err) {
  out->clear();
  uint32_t pending_high = 0;
  auto flush_high = [&] {
    if (pending_high) {
      out->push_back('?');
      pending_high = 0;
    }
  };
  for (size_t i = 0; i < s.size();) {
    char c = s[i++];
    if (c != '\\') {
      flush_high();
      out->push_back(c);
      continue;
    }
    if (i >= s.size()) {  // lone trailing backslash (only reachable at EOF): dropped
      flush_high();
      break;
    }
    c = s[i++];
    if (c == 'u') {
      uint32_t v = 0;
      for (int k = 0; k < 4; ++k) {
        int h = i < s.size() ? hexval(s[i]) : -1;
        if (h < 0) {
          *err = "Malformed \\uxxxx encoding.";
          return false;
        }
        v = v * 16 + uint32_t(h);
        ++i;
      }
      if (v >= 0xD800 && v <= 0xDBFF) {
        flush_high();
        pending_high = v;
      } else if (v >= 0xDC00 && v <= 0xDFFF) {
        if (pending_high) {
          uint32_t cp = 0x10000 + ((pending_high - 0xD800) << 10) + (v - 0xDC00);
          pending_high = 0;
          append_utf8(out, cp);
        } else {
          out->push_back('?');
        }
      } else {
        flush_high();
        append_utf8(out, v);
      }
      continue;
    }
    flush_high();
    switch (c) {
      case 't': out->push_back('\t'); break;
      case 'r': out->push_back('\r'); break;
      case 'n': out->push_back('\n'); break;
      case 'f': out->push_back('\f'); break;
      default: out->push_back(c); break;
    }
  }
  flush_high();
  return true;
}

}  // namespace

PropertiesResult parse_properties(std::string_view text) {
  PropertiesResult r;
  for (const std::string& line : logical_lines(text)) {
    size_t limit = line.size(), key_len = 0, value_start = limit;
    bool has_sep = false, preceding_backslash = false;
    while (key_len < limit) {
      char c = line[key_len];
      if ((c == '=' || c == ':') && !preceding_backslash) {
        value_start = key_len + 1;
        has_sep = true;
        break;
      }
      if (is_ws(c) && !preceding_backslash) {
        value_start = key_len + 1;
        break;
      }
      preceding_backslash = (c == '\\') ? !preceding_backslash : false;
      ++key_len;
    }
    while (value_start < limit) {
      char c = line[value_start];
      if (!is_ws(c)) {
        if (!has_sep && (c == '=' || c == ':')) has_sep = true;
        else break;
      }
      ++value_start;
    }
    std::string key, value;
    if (!load_convert(std::string_view(line).substr(0, key_len), &key, &r.error) ||
        !load_convert(std::string_view(line).substr(value_start), &value, &r.error)) {
      // Properties.load throws; Configuration.java:34-36 swallows it -> empty map.
      r.ok = false;
      r.entries.clear();
      r.map.clear();
      return r;
    }
    r.map[key] = value;
    r.entries.emplace_back(std::move(key), std::move(value));
  }
  return r;
}

}  // namespace hola::config
