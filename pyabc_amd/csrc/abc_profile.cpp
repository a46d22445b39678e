// HIP-event timing of the dominant kernel (the transition-density GEMM +
// exp2 + sum launch), for bench.py's roofline: events are recorded on the
// stream the kernel is launched on, directly around that one launch.
#include <mutex>
#include <vector>
#include "abc_common.h"

namespace {
struct Pair { hipEvent_t a, b; };
std::mutex g_mu;
bool g_on = false;
std::vector<Pair> g_pool;   // created once, reused
size_t g_used = 0;
}  // namespace

namespace abc {
void profile_start(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_on) return;
  if (g_used == g_pool.size()) {
    Pair p;
    if (hipEventCreate(&p.a) != hipSuccess || hipEventCreate(&p.b) != hipSuccess) return;
    g_pool.push_back(p);
  }
  hipEventRecord(g_pool[g_used].a, s);
}
void profile_stop(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_on || g_used == g_pool.size()) return;
  hipEventRecord(g_pool[g_used].b, s);
  ++g_used;
}
}  // namespace abc

extern "C" int abc_profile_begin(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_on = true;
  g_used = 0;
  return ABC_OK;
}

extern "C" int abc_profile_end(double* total_ms, int64_t* launches) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_on = false;
  double tot = 0.0;
  for (size_t i = 0; i < g_used; ++i) {
    ABC_HIP(hipEventSynchronize(g_pool[i].b));
    float ms = 0.f;
    ABC_HIP(hipEventElapsedTime(&ms, g_pool[i].a, g_pool[i].b));
    tot += ms;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = (int64_t)g_used;
  return ABC_OK;
}
