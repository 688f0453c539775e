// B3 propagation codec: X-B3-TraceId/SpanId/ParentSpanId/Sampled/Flags
// multi-header form and the single `b3` header; 64- and 128-bit trace ids.
#pragma once
#include <cstdint>
#include <string>
#include <string_view>

namespace hola::tracing {

struct SpanContext {
  uint64_t trace_hi = 0;  // upper 64 bits of a 128-bit trace id (0 for 64-bit ids)
  uint64_t trace_id = 0;
  uint64_t span_id = 0;
  uint64_t parent_id = 0;
  bool has_parent = false;
  bool sampled = true;
  bool debug = false;
};

// Parses 1..16 hex digits (Brave 3 IdConversion accepts short ids); false on bad input.
bool parse_hex64(std::string_view s, uint64_t* out);
// Parses a 16- or 32-hex-digit trace id.
bool parse_trace_id(std::string_view s, uint64_t* hi, uint64_t* lo);
// 16 lower-case hex digits.
void hex64(uint64_t v, char out[16]);
std::string hex64(uint64_t v);
std::string trace_id_hex(uint64_t hi, uint64_t lo);

enum class Extract { kNone, kNotSampled, kContext };

// Brave 3.9 server-side semantics (HttpServerRequestAdapter.getTraceData): incoming ids are
// honoured only together with an X-B3-Sampled header; Sampled 0/false means "do not trace";
// X-B3-Flags: 1 forces debug (and sampling). The single `b3` header is also accepted.
Extract extract(std::string_view trace_id, std::string_view span_id, std::string_view parent_id,
                std::string_view sampled, std::string_view flags, std::string_view single,
                SpanContext* out);

// Appends the B3 headers for an outbound request whose span is `ctx` ("Name: v\r\n" lines).
void inject(const SpanContext& ctx, std::string* headers);

}  // namespace hola::tracing
