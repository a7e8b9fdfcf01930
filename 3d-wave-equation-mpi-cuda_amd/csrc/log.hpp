// Log levels (the reference has no levels and no machine-readable output).
//   WAVE_LOG=error|warn|info|debug   (default warn), messages go to stderr:
//   wave3d[info] <message>
#pragma once

#include <cstdlib>
#include <cstring>
#include <iostream>
#include <sstream>

namespace wave3d {

enum class LogLevel { Error = 0, Warn = 1, Info = 2, Debug = 3 };

inline LogLevel log_level() {
    static const LogLevel lvl = [] {
        const char* e = std::getenv("WAVE_LOG");
        if (!e) return LogLevel::Warn;
        if (!std::strcmp(e, "error")) return LogLevel::Error;
        if (!std::strcmp(e, "info")) return LogLevel::Info;
        if (!std::strcmp(e, "debug")) return LogLevel::Debug;
        return LogLevel::Warn;
    }();
    return lvl;
}

inline bool log_on(LogLevel l) { return int(l) <= int(log_level()); }

template <class... A>
void log_msg(LogLevel l, const A&... a) {
    if (!log_on(l)) return;
    static const char* names[] = {"error", "warn", "info", "debug"};
    std::ostringstream s;
    s << "wave3d[" << names[int(l)] << "] ";
    (s << ... << a);
    s << '\n';
    std::cerr << s.str();
}

}  // namespace wave3d
