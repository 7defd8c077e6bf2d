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
// rand() (Random.cpp:47-50).  By default (round 6) every solver constructed on a thread is bound to
// the thread's ONE stream (srand(1) on first use), so the calls of a single-threaded Relocalization()
// / ComputeSim3() draw exactly the samples the reference binary draws (other rand() users in between:
// rsc_stream_skip); the constructor's `seed` is then unused.  The stream is per host thread, not
// process-global: the reference's Tracking and LoopClosing threads race on one rand(), which no
// replay can reproduce.  reference_rand(false) — or RSC_REFERENCE_RAND=0 in the environment — is the
// opt-in to per-solver streams srand(seed) (H4) for solvers constructed afterwards on this thread.
// Lifetime: facade solvers use their thread's context (and stream); they must not outlive the thread
// that constructed them.
struct ThreadContext {
    rsc_context* ctx = nullptr;
    rsc_stream* stream = nullptr;
    bool reference_rand = true;
    ThreadContext() {
        const char* d = std::getenv("RSC_DEVICE");
        check(rsc_context_create(d ? std::atoi(d) : 0, &ctx), "rsc_context_create");
        const char* r = std::getenv("RSC_REFERENCE_RAND");
        if (r) reference_rand = std::atoi(r) != 0;
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
