// Downstream call abstraction for GET /api/hola-chaining (HolaResource.java:69-78): the
// handler asks a Chainer for aloha's greetings and gets either the decoded list or the
// Hystrix fallback `["Aloha response (fallback)"]` (HolaResource.java:111-112).
#pragma once
#include <optional>
#include <string>
#include <string_view>
#include <vector>

#include "core/inline_function.h"

namespace hola::http {
class Worker;
}
namespace hola::tracing {
struct SpanContext;
}

namespace hola::app {

constexpr std::string_view kFallbackGreeting = "Aloha response (fallback)";

struct ChainResult {
  std::vector<std::optional<std::string>> items;
  // aloha's body when it is a list of plain strings as a serializer writes it
  // (json::plain_string_list): the list is then passed on as this text and `items` is not
  // filled. The view is valid only while the callback runs; `raw_count` strings.
  bool raw = false;
  std::string_view raw_list;
  size_t raw_count = 0;
  bool fallback = false;
  // aloha answered 2xx without a list (empty body, or JSON null): Feign's JacksonDecoder
  // returns null, the command succeeds, and greetings.addAll(null) then throws in
  // HolaResource.holaChaining() (HolaResource.java:76), so the request fails with a 500.
  bool null_list = false;
  // The command failed with hystrix.command.*.fallback.enabled=false: HystrixRuntimeException
  // escapes aloha() and holaChaining() answers a 500, like null_list.
  bool error = false;
  std::string reason;  // why the fallback was used (timeout, short-circuited, ...)
};

// The continuation of a parked /api/hola-chaining request: its captures (connection,
// content, server span, start time) live inline, so a call allocates nothing for it.
using ChainDone = InlineFunction<void(const ChainResult&), 256>;

class Chainer {
 public:
  virtual ~Chainer() = default;
  // Runs on the worker thread; `done` is invoked exactly once, on the same thread. It may run
  // before call() returns: Hystrix runs the fallback of a short-circuited or rejected command
  // on the caller's thread, and so does this (no timer round trip).
  virtual void call(http::Worker& w, const tracing::SpanContext* parent,
                    ChainDone done) = 0;
};

}  // namespace hola::app
