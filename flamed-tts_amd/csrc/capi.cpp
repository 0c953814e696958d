// Error plumbing, device pinning and tuning knobs shared by every C-ABI entry point.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>

#include "common.hpp"
#include "flamed_hip.h"

namespace fl {
static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const char* last_error() { return g_err; }

int device_of(const void* p, int* dev) {
  if (!p || !dev) return kBadArg;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // clear the sticky error of an unknown (host) pointer
    return kBadArg;
  }
  if (a.type != hipMemoryTypeDevice && a.type != hipMemoryTypeManaged) return kBadArg;
  *dev = a.device;
  return kOk;
}

static std::mutex g_tune_mu;
static Tune g_tune_defaults;
static int g_tune_epoch = 0;
thread_local const Tune* tl_tune = nullptr;
struct SplitCtx;                               // gemm.hpp
thread_local SplitCtx* g_split = nullptr;      // the calling thread's split-K context (SplitScope)

const Tune& tune_defaults_unlocked() { return g_tune_defaults; }

Tune tune_snapshot(int* epoch) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  if (epoch) *epoch = g_tune_epoch;
  return g_tune_defaults;
}

int tune_epoch() {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  return g_tune_epoch;
}

int tune_apply(Tune& t, const char* key, int value) {
  FL_REQUIRE(key, "flamed_tune: null key");
  struct Knob { const char* name; int Tune::*field; int lo, hi; const int* allowed; };
  static const int k_dwcg[] = {16, 32, 0};
  static const int k_dmans[] = {3, 4, 6, 8, 0};
  static const int k_dwtc[] = {64, 128, 0};
  static const int k_bigns[] = {2, 3, 0};
  static const int k_stages[] = {3, 5, 7, 0};
  static const int k_smax[] = {1, 2, 4, 0};
  static const Knob knobs[] = {
      {"splitk_target", &Tune::split_target, 1, 1 << 20, nullptr},
      {"splitk_max", &Tune::split_max, 1, 4, k_smax},
      {"small_stages", &Tune::small_stages, 3, 7, k_stages},
      {"xcd_strips", &Tune::xcd_strips, 0, 64, nullptr},
      {"bn32", &Tune::bn32, 0, 1, nullptr},
      {"dma", &Tune::use_dma, 0, 2, nullptr},
      {"dma_ns", &Tune::dma_ns, 3, 8, k_dmans},
      {"noctr", &Tune::noctr, 0, 1, nullptr},
      {"dup_class", &Tune::dup_class, -1, FLAMED_DEN_KERNEL_CLASSES - 1, nullptr},
      {"stamp_class", &Tune::stamp_class, -1, FLAMED_DEN_KERNEL_CLASSES - 1, nullptr},
      {"dw_cg32", &Tune::dw_cg32_rows, 0, 1 << 30, nullptr},
      {"dw_cg", &Tune::dw_cg_small, 16, 32, k_dwcg},
      {"dw_tc", &Tune::dw_tc_big, 64, 128, k_dwtc},
      {"big", &Tune::big, 0, 1, nullptr},
      {"big_rows", &Tune::big_min_rows, 1024, 1 << 30, nullptr},
      {"big_ns", &Tune::big_ns, 2, 3, k_bigns},
      {"lnfold", &Tune::lnfold, 0, 1, nullptr},
      {"fold_rows", &Tune::fold_big_rows, 0, 1 << 30, nullptr},
      {"graph_steps", &Tune::graph_steps, 1, 1024, nullptr},
      {"x16", &Tune::x16, 0, 1, nullptr},
      {"g8p_rows", &Tune::g8p_rows, 0, 1 << 30, nullptr},
      {"dwgn", &Tune::dwgn, 0, 1, nullptr},
      {"dwgn_small", &Tune::dwgn_small, 0, 1, nullptr},
      {"fuse_euler", &Tune::fuse_euler, 0, 1, nullptr},
      {"pva_split", &Tune::pva_split, 0, 1, nullptr},
      {"persist", &Tune::persist, 0, 1, nullptr},
      {"split_batch", &Tune::split_batch, 1, 4, nullptr},
      {"split_graph", &Tune::split_graph, 0, 1, nullptr},
      {"split_prio", &Tune::split_prio, 0, 2, nullptr},
      {"prio_all", &Tune::prio_all, 0, 1, nullptr},
      {"split_min_rows", &Tune::split_min_rows, 1024, 1 << 30, nullptr},
      {"persist_opt", &Tune::persist_opt, 0, 1 << 20, nullptr},
      {"persist_seal_skip", &Tune::persist_seal_skip, -1, 1 << 20, nullptr},
      {"persist_inject", &Tune::persist_inject, -1, 1 << 20, nullptr},
      {"persist_multi", &Tune::persist_multi, 0, 1, nullptr},
      {"persist_pad", &Tune::persist_pad, 0, 1, nullptr},
      {"persist_pad_ntw", &Tune::persist_pad_ntw, 1, 8, nullptr},
      {"persist_multi_ntw", &Tune::persist_multi_ntw, 1, 8, nullptr},
      {"persist_ntw", &Tune::persist_ntw, 1, 8, nullptr},
      {"persist_capmode", &Tune::persist_capmode, 0, 1, nullptr},
      {"pva_persist", &Tune::pva_persist, 0, 1, nullptr},
      {"attn_mfma", &Tune::attn_mfma, 0, 1, nullptr},
      {"prior_split", &Tune::prior_split, 0, 1, nullptr},
      {"stop_after", &Tune::stop_after, -1, 1 << 20, nullptr},
      {"coop", &Tune::coop, 0, 1, nullptr},
      {"dwgn_var", &Tune::dwgn_var, 0, 2, nullptr},
      {"pva_stage", &Tune::pva_stage, 0, 3, nullptr},
      {"pva_inject", &Tune::pva_inject, -1, 1 << 20, nullptr},
  };
  for (const Knob& k : knobs) {
    if (std::strcmp(k.name, key) != 0) continue;
    int v = value;
    if (k.lo == 0 && k.hi == 1) v = value != 0;  // boolean knobs
    FL_REQUIRE(v >= k.lo && v <= k.hi, "flamed_tune: %s must be in [%d, %d] (got %d)", key, k.lo, k.hi, value);
    if (k.allowed) {
      bool ok = false;
      for (const int* a = k.allowed; *a; ++a) ok = ok || *a == v;
      FL_REQUIRE(ok, "flamed_tune: %s = %d is not a supported value", key, value);
    }
    t.*(k.field) = v;
    return kOk;
  }
  set_error("flamed_tune: unknown key '%s'", key);
  return kBadArg;
}
}  // namespace fl

extern "C" {
FLAMED_API const char* flamed_last_error(void) { return fl::last_error(); }
FLAMED_API int flamed_version(void) { return 2; }

FLAMED_API int flamed_tune(const char* key, int value) {
  std::lock_guard<std::mutex> lk(fl::g_tune_mu);
  fl::Tune t = fl::g_tune_defaults;
  const int rc = fl::tune_apply(t, key, value);
  if (rc) return rc;
  fl::g_tune_defaults = t;
  ++fl::g_tune_epoch;
  return fl::kOk;
}
}
