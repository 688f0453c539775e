#include "http/negotiate.h"

#include "http/parser.h"

namespace hola::http {

namespace {
std::string_view trim(std::string_view s) {
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t')) s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t')) s.remove_suffix(1);
  return s;
}

// Parses a qvalue ("0", "0.5", "1.000"); returns thousandths, -1 on error.
int parse_q(std::string_view v) {
  v = trim(v);
  if (v.size() >= 2 && v.front() == '"' && v.back() == '"') v = v.substr(1, v.size() - 2);
  if (v.empty()) return -1;
  int whole;
  size_t i = 0;
  if (v[0] == '.') whole = 0;  // ".2" (seen from Java's HttpURLConnection default)
  else if (v[0] == '0' || v[0] == '1') whole = v[i++] - '0';
  else return -1;
  int frac = 0, digits = 0;
  if (i < v.size()) {
    if (v[i] != '.') return -1;
    ++i;
    for (; i < v.size(); ++i) {
      if (v[i] < '0' || v[i] > '9' || digits == 3) return -1;
      frac = frac * 10 + (v[i] - '0');
      ++digits;
    }
  }
  while (digits < 3) {
    frac *= 10;
    ++digits;
  }
  int q = whole * 1000 + frac;
  return q > 1000 ? -1 : q;
}
}  // namespace

bool accepts(std::string_view accept, std::string_view type, std::string_view subtype) {
  int best_spec = -1, best_q = 0;
  bool any_valid = false;
  while (true) {
    size_t comma = accept.find(',');
    std::string_view range = trim(accept.substr(0, comma));
    if (!range.empty()) {
      size_t semi = range.find(';');
      std::string_view mt = trim(range.substr(0, semi));
      std::string_view params = semi == std::string_view::npos ? std::string_view() : range.substr(semi + 1);
      std::string_view t, st;
      size_t slash = mt.find('/');
      bool ok = true;
      if (mt == "*") {
        t = "*";
        st = "*";
      } else if (slash != std::string_view::npos && slash > 0 && slash + 1 < mt.size()) {
        t = mt.substr(0, slash);
        st = mt.substr(slash + 1);
        if (t == "*" && st != "*") ok = false;
      } else {
        ok = false;
      }
      int q = 1000, nparams = 0;
      while (ok && !params.empty()) {
        size_t sc = params.find(';');
        std::string_view p = trim(params.substr(0, sc));
        size_t eq = p.find('=');
        if (eq != std::string_view::npos) {
          std::string_view k = trim(p.substr(0, eq));
          if (k == "q" || k == "Q") {
            q = parse_q(p.substr(eq + 1));
            if (q < 0) ok = false;
          } else {
            ++nparams;
          }
        }
        if (sc == std::string_view::npos) break;
        params.remove_prefix(sc + 1);
      }
      if (ok) {
        any_valid = true;
        bool tmatch = t == "*" || iequals(t, type);
        bool smatch = st == "*" || iequals(st, subtype);
        if (tmatch && smatch) {
          int spec = (t == "*" ? 0 : 2) + (st == "*" ? 0 : 1) + (nparams ? 4 : 0);
          if (spec > best_spec || (spec == best_spec && q > best_q)) {
            best_spec = spec;
            best_q = q;
          }
        }
      }
    }
    if (comma == std::string_view::npos) break;
    accept.remove_prefix(comma + 1);
  }
  if (!any_valid) return true;
  return best_spec >= 0 && best_q > 0;
}

}  // namespace hola::http
