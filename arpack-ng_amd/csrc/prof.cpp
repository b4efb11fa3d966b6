// Per-kernel-class hipEvent profiler (see device.hpp).  Events are recorded on
// the stream the kernel is launched on, so the measured duration is the
// kernel's own device time inside the timed region, not host wall time.
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

#include "device.hpp"

namespace ahip {

namespace {
// countdown of the fault-injection hook; AHIP_FAULT_AT=k arms it (read on the
// first checked call, like ARPACK_HIP_DETERMINISTIC below)
constexpr long kUnread = -1;
std::atomic<long> g_fault_at{kUnread};
}  // namespace

hipError_t fault_filter(hipError_t e) {
    long v = g_fault_at.load(std::memory_order_relaxed);
    if (v == kUnread) {
        const char* s = getenv("AHIP_FAULT_AT");
        long unread = kUnread;
        g_fault_at.compare_exchange_strong(unread, s && atol(s) > 0 ? atol(s) : 0L);
        v = g_fault_at.load(std::memory_order_relaxed);
    }
    if (v <= 0) return e;
    return g_fault_at.fetch_sub(1) == 1 ? hipErrorInvalidValue : e;
}

void fault_inject(long k) { g_fault_at.store(k > 0 ? k : 0); }

namespace {
// -1: not read yet -- ARPACK_HIP_DETERMINISTIC is read on first use (a value
// computed in a static initializer read 0 in the built library)
std::atomic<int> g_det{-1};
}  // namespace

bool deterministic() {
    int v = g_det.load(std::memory_order_relaxed);
    if (v < 0) {
        const char* e = getenv("ARPACK_HIP_DETERMINISTIC");
        int unset = -1;
        g_det.compare_exchange_strong(unset, e && e[0] == '1' ? 1 : 0);
        v = g_det.load(std::memory_order_relaxed);
    }
    return v != 0;
}
void set_deterministic(bool on) { g_det.store(on ? 1 : 0); }

}  // namespace ahip

namespace ahip::dev {

namespace {
struct Pending {
    ProfClass c;
    hipEvent_t a, b;
    double bytes;
};
std::mutex g_mu;
bool g_on = false;
std::vector<hipEvent_t> g_pool;
std::vector<Pending> g_pending;
hipEvent_t g_open[kProfClasses] = {};
ProfStat g_acc[kProfClasses];
// kernel mode: the open span (one at a time; nested spans count in the outer),
// bound to the stream and thread that armed it: launches on other streams or
// threads get no events and do not count in it
int g_arm = -1, g_depth = 0;
hipStream_t g_arm_stream = nullptr;
std::thread::id g_arm_thread;
hipEvent_t g_kstart = nullptr, g_kstop = nullptr;
std::vector<hipEvent_t> g_retire;  // stop events superseded by a later launch

// superseded stop events go back to the pool once their launch has completed
void recycle_retired_locked() {
    size_t k = 0;
    for (hipEvent_t e : g_retire) {
        if (hipEventQuery(e) == hipSuccess) g_pool.push_back(e);
        else g_retire[k++] = e;
    }
    g_retire.resize(k);
}

hipEvent_t take() {
    if (!g_pool.empty()) {
        hipEvent_t e = g_pool.back();
        g_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

void drain_locked() {
    for (auto& p : g_pending) {
        (void)hipEventSynchronize(p.b);
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            g_acc[p.c].ms += ms;
            g_acc[p.c].bytes += p.bytes;
            g_acc[p.c].count += 1;
        }
        g_pool.push_back(p.a);
        g_pool.push_back(p.b);
    }
    g_pending.clear();
    for (hipEvent_t e : g_retire) {
        (void)hipEventSynchronize(e);
        g_pool.push_back(e);
    }
    g_retire.clear();
}
}  // namespace

void prof_enable(bool on) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_on = on;
}

bool prof_on() { return g_on; }

void prof_begin(ProfClass c, hipStream_t s) {
    if (!g_on) return;
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_pending.size() > 4096) drain_locked();  // bound the number of live events
    hipEvent_t e = take();
    (void)hipEventRecord(e, s);
    g_open[c] = e;
}

void prof_end(ProfClass c, hipStream_t s, double bytes) {
    if (!g_on) return;
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_open[c]) return;
    hipEvent_t e = take();
    (void)hipEventRecord(e, s);
    g_pending.push_back(Pending{c, g_open[c], e, bytes});
    g_open[c] = nullptr;
}

void prof_arm(ProfClass c, hipStream_t s) {
    if (!g_on) return;
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_arm >= 0) {
        ++g_depth;
        return;
    }
    if (g_pending.size() > 4096) drain_locked();
    g_arm = c;
    g_arm_stream = s;
    g_arm_thread = std::this_thread::get_id();
    g_kstart = g_kstop = nullptr;
}

void prof_disarm(ProfClass c, double bytes) {
    if (!g_on) return;
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_depth > 0) {
        --g_depth;
        return;
    }
    if (g_arm != c) return;
    if (g_kstart && g_kstop) g_pending.push_back(Pending{c, g_kstart, g_kstop, bytes});
    g_arm = -1;
    g_kstart = g_kstop = nullptr;
}

bool prof_kernel_events(hipStream_t s, hipEvent_t* start, hipEvent_t* stop) {
    *start = *stop = nullptr;
    if (!g_on) return false;
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_arm < 0 || s != g_arm_stream || std::this_thread::get_id() != g_arm_thread) return false;
    if (!g_kstart) *start = g_kstart = take();
    if (g_kstop) {
        g_retire.push_back(g_kstop);
        if (g_retire.size() > 64) recycle_retired_locked();
    }
    *stop = g_kstop = take();
    return true;
}

void prof_collect(ProfStat out[kProfClasses]) {
    std::lock_guard<std::mutex> lk(g_mu);
    drain_locked();
    for (int c = 0; c < kProfClasses; ++c) {
        out[c] = g_acc[c];
        g_acc[c] = ProfStat{};
    }
}

}  // namespace ahip::dev
