#include "http/response.h"

namespace hola::http {

const char* reason_phrase_for(int status) {
  switch (status) {
    case 200: return "OK";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 406: return "Not Acceptable";
    case 413: return "Request Entity Too Large";
    case 414: return "Request-URI Too Long";
    case 431: return "Request Header Fields Too Large";
    case 500: return "Internal Server Error";
    case 501: return "Not Implemented";
    case 503: return "Service Unavailable";
    case 505: return "HTTP Version Not Supported";
    default: return "Unknown";
  }
}

Prepared build_response(const ResponseSpec& s, const char* date29) {
  Prepared p;
  std::string& b = p.bytes;
  b.reserve(192 + s.body.size() + s.extra_headers.size());
  b += "HTTP/1.1 ";
  b += std::to_string(s.status);
  b += ' ';
  b += reason_phrase_for(s.status);
  b += s.keep_alive ? "\r\nConnection: keep-alive\r\n" : "\r\nConnection: close\r\n";
  if (s.cors) b += "Access-Control-Allow-Origin: *\r\n";
  if (!s.content_type.empty()) {
    b += "Content-Type: ";
    b += s.content_type;
    b += "\r\n";
  }
  b += "Content-Length: ";
  b += std::to_string(s.body.size());
  b += "\r\n";
  b += s.extra_headers;
  b += "Date: ";
  p.date_off = b.size();
  b.append(date29, 29);
  b += "\r\n\r\n";
  if (!s.head) b += s.body;
  return p;
}

}  // namespace hola::http
