#include "core/clock.h"

#include <cstdio>

namespace hola {

void format_http_date(int64_t sec, char out[29]) {
  static const char* kDays[] = {"Sun", "Mon", "Tue", "Wed", "Thu", "Fri", "Sat"};
  static const char* kMonths[] = {"Jan", "Feb", "Mar", "Apr", "May", "Jun",
                                  "Jul", "Aug", "Sep", "Oct", "Nov", "Dec"};
  time_t t = static_cast<time_t>(sec);
  tm g;
  gmtime_r(&t, &g);
  char buf[40];
  snprintf(buf, sizeof buf, "%s, %02d %s %04d %02d:%02d:%02d GMT", kDays[g.tm_wday], g.tm_mday,
           kMonths[g.tm_mon], g.tm_year + 1900, g.tm_hour, g.tm_min, g.tm_sec);
  for (int i = 0; i < 29; ++i) out[i] = buf[i];
}

}  // namespace hola
