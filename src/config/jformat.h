// The subset of java.util.Formatter needed for `String.format(translation, hostname)`
// (HolaResource.java:65): one String argument, so every conversion either formats a String
// or throws. Errors carry the Java exception class name so the 500 path is testable.
//
// Supported: %s %S %b %B %h %H %n %% with flags '-' and '#', width, precision, explicit
// (`2$`) and relative (`<`) argument indices. Numeric/char/date conversions applied to a
// String raise IllegalFormatConversionException exactly as Java does.
#pragma once
#include <string>
#include <string_view>
#include <vector>

namespace hola::config {

struct FormatResult {
  bool ok = true;
  std::string value;
  std::string error;  // Java exception simple name, e.g. "MissingFormatArgumentException"
  std::string detail;
};

FormatResult java_format(std::string_view fmt, const std::vector<std::string>& args);

// java.lang.String.hashCode() of a UTF-8 string (computed over its UTF-16 code units).
int32_t java_string_hash(std::string_view utf8);

}  // namespace hola::config
