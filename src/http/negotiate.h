// Accept-header negotiation for a single produced media type — the JAX-RS @Produces check
// (HolaResource.java:54,71,82) that RESTEasy turns into 406 Not Acceptable.
#pragma once
#include <string_view>

namespace hola::http {

// True if `accept` (an Accept header value) admits type/subtype with q > 0. The most
// specific matching media range decides (RFC 9110 §12.5.1), so "*/*, text/plain;q=0"
// rejects text/plain. Unparseable ranges are ignored; an Accept with no usable range
// accepts everything (lenient, like RESTEasy's fallback to */*).
bool accepts(std::string_view accept, std::string_view type, std::string_view subtype);

}  // namespace hola::http
