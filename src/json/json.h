// Minimal JSON codec: the reference serialises List<String> responses with the
// JAX-RS JSON provider and decodes aloha's reply with Feign's JacksonDecoder
// (HolaResource.java:110). Only what those paths need: a string escaper, a compact writer
// for string arrays, and a small DOM parser for decoding `List<String>`.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <string_view>
#include <vector>

namespace hola::json {

// Appends `s` as a JSON string literal (Jackson-style escaping: \" \\ \b \f \n \r \t, other
// control characters as \u00XX, everything else — including non-ASCII UTF-8 — raw).
void append_string(std::string* out, std::string_view s);
// The length append_string() writes for `s` (quotes and escapes included): a response's
// Content-Length before its body is written.
size_t quoted_size(std::string_view s);
std::string quote(std::string_view s);

// Serialises a list of optional strings (nullopt -> null), compact: ["a","b"].
std::string string_array(const std::vector<std::optional<std::string>>& items);

struct Value {
  enum class Type { kNull, kBool, kNumber, kString, kArray, kObject } type = Type::kNull;
  bool b = false;
  std::string text;  // number literal or string contents
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;
  const Value* get(std::string_view key) const;
};

// Parses a complete JSON document; false with *err on syntax error or trailing garbage.
bool parse(std::string_view in, Value* out, std::string* err);

// Jackson's List<String> binding: array of scalars; numbers/booleans coerce to their text,
// null stays null; objects/arrays inside are a mismatch. false with *err on failure (then
// *out holds a partial result). Elements already in *out are reused, so decoding into the
// same vector again allocates nothing once its strings are large enough.
bool decode_string_list(std::string_view in, std::vector<std::optional<std::string>>* out,
                        std::string* err);

// True when `in` is a list of strings exactly as a serializer writes one: `[` then
// `"..."` separated by `,` then `]`, no whitespace, nothing escaped in any string. Such a
// list decodes to strings that re-encode to the same bytes, so a caller that only passes the
// list on can copy its text instead of decoding and re-encoding every element. *count is the
// number of strings. Anything else (whitespace, escapes, null, numbers, malformed) is false:
// decode_string_list() then says what it decodes to or why it fails.
bool plain_string_list(std::string_view in, size_t* count);

}  // namespace hola::json
