// Response serialisation. Hot responses are prepared once per (config generation, worker)
// and only their Date bytes are patched once per second — so answering GET /api/hola is a
// memcpy into the connection's output buffer, not a String.format + JAX-RS writer pass
// (HolaResource.java:65, SURVEY.md §2c "hot ops").
#pragma once
#include <cstring>
#include <string>
#include <string_view>

namespace hola::http {

const char* reason_phrase_for(int status);

struct ResponseSpec {
  int status = 200;
  std::string_view content_type;  // empty: no Content-Type header
  bool cors = false;              // Access-Control-Allow-Origin: * (CorsFilter.java:31)
  std::string extra_headers;      // pre-formatted "Name: value\r\n" lines
  std::string_view body;
  bool head = false;              // HEAD: headers only (Content-Length kept)
  bool keep_alive = true;
};

struct Prepared {
  std::string bytes;
  size_t date_off = std::string::npos;
  void set_date(const char* date29) {
    if (date_off != std::string::npos) memcpy(&bytes[date_off], date29, 29);
  }
  std::string_view view() const { return bytes; }
};

Prepared build_response(const ResponseSpec& spec, const char* date29);

}  // namespace hola::http
