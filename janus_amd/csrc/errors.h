// Thread-local last-error message shared by every translation unit of libprio3gpu.so
// (engine.hip, codec.cpp, hpke.cpp); read through prio3gpu_last_error().
#pragma once

namespace p3g {
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
}
