// Static files compiled into the binary (cmake/embed_assets.cmake): the landing page
// (src/main/webapp/index.html role), the Swagger 2.0 document (SwaggerListener.java:29-42
// role) and an offline stand-in for the swagger-ui 2.1.4 webjar (pom.xml:207-211).
#pragma once
#include <cstddef>
#include <string_view>

namespace hola::assets {

struct Asset {
  const char* name;
  const char* data;
  size_t size;
  std::string_view view() const { return {data, size}; }
};

const Asset* find(std::string_view name);

}  // namespace hola::assets
