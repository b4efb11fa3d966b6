// Reverse-communication as C++20 coroutines.
//
// The reference keeps each solve's control state in Fortran SAVE variables and
// re-enters its routines through `go to` ladders keyed by logical flags
// (SRC/dsaitr.f:347-351, SRC/dsaup2.f:349-362).  Here the algorithm is written
// as straight-line coroutines: an RCI request (ido = -1/1/2/3) is a
// `co_await rci(...)` that suspends the whole call chain and hands control back
// to the caller of dsaupd_c; the next dsaupd_c call resumes the innermost
// suspended coroutine.  The coroutine frames ARE the per-solve state (heap
// allocated, one chain per solve), so several solves can be in flight.
#pragma once
#include <coroutine>
#include <cstdint>
#include <exception>
#include <utility>

namespace ahip {

struct RciReq {
    int ido = 0;
    int64_t x = -1, y = -1, bx = -1;  // 0-based offsets into workd (ipntr(1..3) - 1)
};

struct RciCtx {
    RciReq req;
    std::coroutine_handle<> leaf;  // coroutine to resume on the next call
    bool done = false;
};

// A lazily-started coroutine that returns to its awaiter when it finishes.
struct [[nodiscard]] Task {
    struct promise_type {
        std::coroutine_handle<> cont;
        RciCtx* ctx = nullptr;
        Task get_return_object() {
            return Task{std::coroutine_handle<promise_type>::from_promise(*this)};
        }
        std::suspend_always initial_suspend() noexcept { return {}; }
        struct Final {
            bool await_ready() noexcept { return false; }
            std::coroutine_handle<> await_suspend(std::coroutine_handle<promise_type> h) noexcept {
                auto& p = h.promise();
                if (p.cont) return p.cont;
                if (p.ctx) p.ctx->done = true;
                return std::noop_coroutine();
            }
            void await_resume() noexcept {}
        };
        Final final_suspend() noexcept { return {}; }
        void return_void() {}
        void unhandled_exception() { std::terminate(); }
    };
    std::coroutine_handle<promise_type> h;

    explicit Task(std::coroutine_handle<promise_type> hh) : h(hh) {}
    Task(Task&& o) noexcept : h(std::exchange(o.h, {})) {}
    Task& operator=(Task&& o) noexcept {
        if (this != &o) {
            if (h) h.destroy();
            h = std::exchange(o.h, {});
        }
        return *this;
    }
    Task(const Task&) = delete;
    ~Task() {
        if (h) h.destroy();
    }

    // Awaiting a child task: run it, come back when it completes.
    bool await_ready() const noexcept { return false; }
    template <class P>
    std::coroutine_handle<> await_suspend(std::coroutine_handle<P> parent) noexcept {
        h.promise().cont = parent;
        h.promise().ctx = parent.promise().ctx;
        return h;
    }
    void await_resume() const noexcept {}
};

// `co_await RciAwait{ctx, req}` parks the chain and returns to the caller.
struct RciAwait {
    RciCtx* ctx;
    RciReq req;
    bool await_ready() const noexcept { return false; }
    void await_suspend(std::coroutine_handle<> h) noexcept {
        ctx->req = req;
        ctx->leaf = h;
    }
    void await_resume() const noexcept {}
};

// Start a root task bound to `ctx`.
inline void start_root(Task& t, RciCtx& ctx) {
    t.h.promise().ctx = &ctx;
    t.h.promise().cont = {};
    ctx.done = false;
    ctx.leaf = t.h;
}

}  // namespace ahip
