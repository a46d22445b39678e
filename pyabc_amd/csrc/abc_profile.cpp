// HIP-event timing of the engine's kernels for bench.py (roofline and
// per-stage split of the timed region): events are recorded on the stream a
// kernel is launched on, directly around that one launch, per channel
// (ABC_PROF_DENSITY: the transition-density GEMM + exp2 + sum launch;
// ABC_PROF_CANDIDATES: the fused candidate round; ABC_PROF_REGEN: the
// regeneration of kept rows; ABC_PROF_RESCUE: the unhinted density re-run of
// rescued candidates).
#include <mutex>
#include <vector>
#include "abc_common.h"

namespace {
struct Pair { hipEvent_t a, b; };
constexpr int NCH = 4;
std::mutex g_mu;
bool g_on = false;
std::vector<Pair> g_pool[NCH];   // created once, reused
size_t g_used[NCH] = {0, 0, 0, 0};
double g_ms[NCH] = {0, 0, 0, 0};
int64_t g_n[NCH] = {0, 0, 0, 0};
}  // namespace

namespace abc {
void profile_start(hipStream_t s, int ch) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_on || ch < 0 || ch >= NCH) return;
  if (g_used[ch] == g_pool[ch].size()) {
    Pair p;
    if (hipEventCreate(&p.a) != hipSuccess || hipEventCreate(&p.b) != hipSuccess) return;
    g_pool[ch].push_back(p);
  }
  hipEventRecord(g_pool[ch][g_used[ch]].a, s);
}
void profile_stop(hipStream_t s, int ch) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_on || ch < 0 || ch >= NCH || g_used[ch] == g_pool[ch].size()) return;
  hipEventRecord(g_pool[ch][g_used[ch]].b, s);
  ++g_used[ch];
}
}  // namespace abc

extern "C" int abc_profile_begin(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_on = true;
  for (int c = 0; c < NCH; ++c) g_used[c] = 0;
  return ABC_OK;
}

extern "C" int abc_profile_end(double* total_ms, int64_t* launches) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_on = false;
  for (int c = 0; c < NCH; ++c) {
    double tot = 0.0;
    for (size_t i = 0; i < g_used[c]; ++i) {
      ABC_HIP(hipEventSynchronize(g_pool[c][i].b));
      float ms = 0.f;
      ABC_HIP(hipEventElapsedTime(&ms, g_pool[c][i].a, g_pool[c][i].b));
      tot += ms;
    }
    g_ms[c] = tot;
    g_n[c] = (int64_t)g_used[c];
  }
  if (total_ms) *total_ms = g_ms[ABC_PROF_DENSITY];
  if (launches) *launches = g_n[ABC_PROF_DENSITY];
  return ABC_OK;
}

extern "C" int abc_profile_channel(int channel, double* total_ms, int64_t* launches) {
  std::lock_guard<std::mutex> lk(g_mu);
  ABC_CHECK_ARG(channel >= 0 && channel < NCH, "profile_channel: bad channel");
  if (total_ms) *total_ms = g_ms[channel];
  if (launches) *launches = g_n[channel];
  return ABC_OK;
}
