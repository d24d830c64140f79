// Lightweight tracing (the reference has none).
//
//  QUEST_TRACE=<file>|stderr  one JSON line per event: register create /
//                             destroy, every flush (ops in, ops after block
//                             fusion, passes), every distributed swap (qubits,
//                             bytes, host time), checkpoints.
//  QUEST_ROCTX=1              roctx ranges around flushes and swaps, so that
//                             `rocprofv3 --marker-trace` shows them next to
//                             the kernels (libroctx64 is dlopen'ed).
#pragma once

namespace qa {
namespace trace {

bool on();
// printf-style payload: the JSON members after "t", "rank", "ev"
void event(const char* ev, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
double now();  // seconds since the first call

void rangePush(const char* name);
void rangePop();

struct Range {
    explicit Range(const char* name) { rangePush(name); }
    ~Range() { rangePop(); }
};

}  // namespace trace
}  // namespace qa
