// marf_prof.h -- per-kernel HIP-event timing hooks (see marf_prof.hip).
#pragma once
#include <hip/hip_runtime.h>

bool marf_prof_on();
void* marf_prof_begin(const char* name, hipStream_t s);
void marf_prof_end(void* handle, hipStream_t s);

// RAII scope: times everything launched on `s` inside it.
struct MarfProfScope {
    void* h;
    hipStream_t s;
    MarfProfScope(const char* name, hipStream_t st) : h(marf_prof_begin(name, st)), s(st) {}
    ~MarfProfScope() { marf_prof_end(h, s); }
};
