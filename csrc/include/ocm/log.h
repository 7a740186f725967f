// Logging and error helpers.
//
// Parity with reference inc/debug.h:22-65: `printd` output is enabled by the
// *presence* of OCM_VERBOSE. Unlike the reference, prefix and body go to the
// same stream (stderr) in one write, and failures return errors instead of
// assert(0) so a daemon survives a bad request.
#pragma once
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

namespace ocm {

bool verbose();
void log_line(const char *level, const char *file, const char *func, int line,
              const char *fmt, ...) __attribute__((format(printf, 5, 6)));

// Thread-local last error string for the C API (ocm_last_error).
void set_last_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
const char *last_error();

}  // namespace ocm

#define OCM_LOG(...)                                                                  \
    do {                                                                              \
        if (::ocm::verbose()) ::ocm::log_line("D", __FILE__, __func__, __LINE__, __VA_ARGS__); \
    } while (0)
#define OCM_INFO(...) ::ocm::log_line("I", __FILE__, __func__, __LINE__, __VA_ARGS__)
#define OCM_WARN(...) ::ocm::log_line("W", __FILE__, __func__, __LINE__, __VA_ARGS__)
#define OCM_ERR(...) ::ocm::log_line("E", __FILE__, __func__, __LINE__, __VA_ARGS__)

// Fail the current function with `rv` after recording an error.
#define OCM_FAIL(rv, ...)                    \
    do {                                     \
        ::ocm::set_last_error(__VA_ARGS__);  \
        OCM_LOG(__VA_ARGS__);                \
        return rv;                           \
    } while (0)
