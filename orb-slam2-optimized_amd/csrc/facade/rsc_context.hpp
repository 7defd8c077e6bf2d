// rsc_context.hpp — per-thread engine context for the C++ facade.
// The reference runs relocalization on the Tracking thread and loop closure on the LoopClosing
// thread (System.cpp:58-69); each host thread gets its own rsc_context (HIP stream + buffers), so
// the facade is re-entrant without locks.  Device = $RSC_DEVICE (default 0).
#pragma once
#include <cstdlib>
#include <stdexcept>
#include <string>
#include "rsc.h"

namespace rsc_orb {

inline void check(int status, const char* what) {
    if (status != RSC_OK)
        throw std::runtime_error(std::string("rsc: ") + what + ": " + rsc_status_string(status));
}

struct ThreadContext {
    rsc_context* ctx = nullptr;
    ThreadContext() {
        const char* d = std::getenv("RSC_DEVICE");
        check(rsc_context_create(d ? std::atoi(d) : 0, &ctx), "rsc_context_create");
    }
    ~ThreadContext() { rsc_context_destroy(ctx); }
};

inline rsc_context* thread_context() {
    thread_local ThreadContext tc;
    return tc.ctx;
}

}  // namespace rsc_orb
