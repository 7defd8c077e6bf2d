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

// rand() (Q3): the reference draws every RANSAC sample from glibc's process-global, never seeded
// rand() (Random.cpp:47-50).  By default each facade solver owns a stream seeded with its
// constructor's `seed` (H4).  With reference_rand(true) — or RSC_REFERENCE_RAND=1 in the environment —
// every solver constructed afterwards on this thread is bound to the thread's ONE stream (srand(1) on
// first use), so the calls of a single-threaded Relocalization() / ComputeSim3() draw exactly the
// samples the reference binary draws (other rand() users in between: rsc_stream_skip).
struct ThreadContext {
    rsc_context* ctx = nullptr;
    rsc_stream* stream = nullptr;
    bool reference_rand = false;
    ThreadContext() {
        const char* d = std::getenv("RSC_DEVICE");
        check(rsc_context_create(d ? std::atoi(d) : 0, &ctx), "rsc_context_create");
        const char* r = std::getenv("RSC_REFERENCE_RAND");
        reference_rand = r && std::atoi(r) != 0;
    }
    ~ThreadContext() {
        if (stream) rsc_stream_destroy(stream);
        rsc_context_destroy(ctx);
    }
};

inline ThreadContext& thread_state() {
    thread_local ThreadContext tc;
    return tc;
}

inline rsc_context* thread_context() { return thread_state().ctx; }

inline void reference_rand(bool on) { thread_state().reference_rand = on; }

// The thread's shared stream (created as srand(1) on first use).
inline rsc_stream* thread_stream() {
    ThreadContext& t = thread_state();
    if (!t.stream) check(rsc_stream_create(t.ctx, 1, &t.stream), "rsc_stream_create");
    return t.stream;
}

// Stream a newly constructed solver binds to: the thread's stream in reference_rand mode, else none.
inline rsc_stream* construction_stream() { return thread_state().reference_rand ? thread_stream() : nullptr; }

}  // namespace rsc_orb
