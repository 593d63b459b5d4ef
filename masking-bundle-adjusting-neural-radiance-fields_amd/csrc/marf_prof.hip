// marf_prof.hip -- optional per-kernel timing with HIP events recorded on the launch stream
// (the stream the kernel runs on), so bench.py can report each kernel's average duration live.
// Off by default; when off the hooks are two predictable branches per launch.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "marf_args.h"
#include "marf_prof.h"

namespace {
struct Pending {
    const char* name;
    hipEvent_t a, b;
};
std::mutex g_mu;
bool g_on = false;
std::string g_filter;  // ",name1,name2," or empty (every kernel)
std::vector<Pending> g_pending;
std::vector<hipEvent_t> g_pool;
std::map<std::string, std::pair<double, long long>> g_acc;

hipEvent_t take() {
    if (!g_pool.empty()) {
        hipEvent_t e = g_pool.back();
        g_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}
}  // namespace

bool marf_prof_on() { return g_on; }

void* marf_prof_begin(const char* name, hipStream_t s) {
    if (!g_on) return nullptr;
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_filter.empty() && g_filter.find("," + std::string(name) + ",") == std::string::npos) return nullptr;
    Pending* p = new Pending{name, take(), take()};
    if (!p->a || !p->b) {
        delete p;
        return nullptr;
    }
    (void)hipEventRecord(p->a, s);
    return p;
}

void marf_prof_end(void* h, hipStream_t s) {
    if (!h) return;
    Pending* p = static_cast<Pending*>(h);
    (void)hipEventRecord(p->b, s);
    std::lock_guard<std::mutex> lk(g_mu);
    g_pending.push_back(*p);
    delete p;
}

static void drain() {
    for (auto& p : g_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            auto& e = g_acc[p.name];
            e.first += ms;
            e.second += 1;
        }
        g_pool.push_back(p.a);
        g_pool.push_back(p.b);
    }
    g_pending.clear();
}

namespace marf {

hipError_t ensure_dynamic_lds(const void* kernel, size_t lds) {
    static std::mutex mu;
    static std::map<std::pair<int, const void*>, size_t> set_so_far;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(mu);
    size_t& cur = set_so_far[{dev, kernel}];
    if (cur >= lds) return hipSuccess;
    e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e == hipSuccess) cur = lds;
    return e;
}

}  // namespace marf

extern "C" {

int marf_profile_enable(int on) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_on = on != 0;
    return 0;
}

int marf_profile_filter(const char* names) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_filter.clear();
    if (names && names[0]) g_filter = "," + std::string(names) + ",";
    return 0;
}

int marf_profile_reset(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    drain();
    g_acc.clear();
    return 0;
}

int marf_profile_read(char* names, int name_len, double* total_ms, long long* count, int cap) {
    std::lock_guard<std::mutex> lk(g_mu);
    drain();
    int i = 0;
    for (auto& kv : g_acc) {
        if (i >= cap) break;
        if (names && name_len > 0) {
            std::string n = kv.first.substr(0, (size_t)name_len - 1);
            for (size_t c = 0; c < (size_t)name_len; ++c) names[(size_t)i * name_len + c] = c < n.size() ? n[c] : 0;
        }
        if (total_ms) total_ms[i] = kv.second.first;
        if (count) count[i] = kv.second.second;
        ++i;
    }
    return i;
}

}  // extern "C"
