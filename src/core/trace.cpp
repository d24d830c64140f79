#include "trace.hpp"

#include <dlfcn.h>

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "core.hpp"

namespace qa {
namespace trace {

namespace {
struct State {
    FILE* out = nullptr;
    bool enabled = false;
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    std::mutex mu;
    State() {
        const char* e = getenv("QUEST_TRACE");
        if (e && *e && strcmp(e, "0") != 0) {
            enabled = true;
            if (!strcmp(e, "1") || !strcmp(e, "stderr"))
                out = stderr;
            else
                out = fopen(e, "a");
            if (!out) out = stderr;
            // the process clock's origin on CLOCK_MONOTONIC (Python's
            // time.monotonic()), so host marks of a driver line up with "t"
            const double mono = std::chrono::duration<double>(t0.time_since_epoch()).count();
            fprintf(out, "{\"t\": 0, \"rank\": -1, \"ev\": \"trace_start\", \"monotonic\": %.6f}\n", mono);
            fflush(out);
        }
        const char* r = getenv("QUEST_ROCTX");
        if (r && atoi(r) == 1) {
            void* h = dlopen("libroctx64.so", RTLD_NOW | RTLD_LOCAL);
            if (!h) h = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_NOW | RTLD_LOCAL);
            if (h) {
                push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
                pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
            }
        }
    }
};
State& S() {
    static State s;
    return s;
}
}  // namespace

bool on() { return S().enabled; }

double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - S().t0).count();
}

void event(const char* ev, const char* fmt, ...) {
    State& s = S();
    if (!s.enabled) return;
    char body[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(body, sizeof body, fmt, ap);
    va_end(ap);
    std::lock_guard<std::mutex> g(s.mu);
    fprintf(s.out, "{\"t\": %.6f, \"rank\": %d, \"ev\": \"%s\"%s%s}\n", now(), rt().rank, ev, body[0] ? ", " : "",
            body);
    fflush(s.out);
}

void rangePush(const char* name) {
    if (S().push) S().push(name);
}
void rangePop() {
    if (S().pop) S().pop();
}

}  // namespace trace
}  // namespace qa
