// java.util.Properties.load(Reader) semantics, byte-exact for UTF-8 input.
//
// The reference reads `-Dconf=<file>` with `Properties.load(new FileReader(file))`
// (Configuration.java:27-29) on every request. This parser reproduces that grammar:
// natural/logical lines with odd-backslash continuation, `#`/`!` comments, the `=`, `:` and
// whitespace separators, and the \t \n \r \f \uXXXX escapes — so translation.properties:15
// (`...configuraciones\n`, a literal backslash-n) decodes to a trailing newline character.
#pragma once
#include <map>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace hola::config {

struct PropertiesResult {
  bool ok = true;
  std::string error;  // e.g. "Malformed \\uxxxx encoding." (IllegalArgumentException)
  // Insertion order kept for diagnostics; later duplicates win in `map`.
  std::vector<std::pair<std::string, std::string>> entries;
  std::map<std::string, std::string> map;
};

PropertiesResult parse_properties(std::string_view text);

// Appends the UTF-8 encoding of a code point.
void append_utf8(std::string* out, uint32_t cp);

}  // namespace hola::config
