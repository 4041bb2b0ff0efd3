// Logging stand-in for the reference headers' `#include <spdlog/spdlog.h>` (spdlog is a
// FetchContent dependency of the reference, absent from this image). Used ONLY by
// tests/cpp/reference_binding.cpp, which compiles the reference's own data_structures.h /
// metrics_tracker.h against freeimpala_amd::BasicLearner to check the INTEGRATION.md section 2
// alias. Supports the calls those two headers make: spdlog::{trace,debug,info,warn,error,
// critical}(fmt, args...) with "{}" placeholders, printed to stderr.
#pragma once
#include <cstdio>
#include <sstream>
#include <string>

namespace spdlog {
namespace detail {
inline void fmt_into(std::ostringstream& o, const char* f) { o << f; }
template <class T, class... R>
void fmt_into(std::ostringstream& o, const char* f, const T& v, const R&... rest) {
    for (; *f; ++f) {
        if (f[0] == '{' && f[1] == '}') {
            o << v;
            fmt_into(o, f + 2, rest...);
            return;
        }
        o << *f;
    }
}
template <class... A>
void log(const char* level, const char* f, const A&... a) {
    std::ostringstream o;
    fmt_into(o, f, a...);
    std::fprintf(stderr, "[ref] [%s] %s\n", level, o.str().c_str());
}
}  // namespace detail
template <class... A> void trace(const char* f, const A&... a) { detail::log("trace", f, a...); }
template <class... A> void debug(const char* f, const A&... a) { detail::log("debug", f, a...); }
template <class... A> void info(const char* f, const A&... a) { detail::log("info", f, a...); }
template <class... A> void warn(const char* f, const A&... a) { detail::log("warn", f, a...); }
template <class... A> void error(const char* f, const A&... a) { detail::log("error", f, a...); }
template <class... A> void critical(const char* f, const A&... a) { detail::log("critical", f, a...); }
}  // namespace spdlog
