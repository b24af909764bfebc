// sph_util.h -- host-side helpers shared by the pair-style layer and the engine.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/sph_hip.h"

namespace sph {

void set_error(const char *fmt, ...);

struct Failure {
  int code;
};

#define SPH_HIP_TRY(expr)                                                             \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) {                                                           \
      ::sph::set_error("%s:%d: %s -> %s", __FILE__, __LINE__, #expr,                  \
                       hipGetErrorString(_e));                                        \
      throw ::sph::Failure{_e == hipErrorOutOfMemory ? SPH_HIP_ENOMEM                 \
                                                     : SPH_HIP_ERUNTIME};             \
    }                                                                                 \
  } while (0)

#define SPH_REQUIRE(cond, code, ...)                                                  \
  do {                                                                                \
    if (!(cond)) {                                                                    \
      ::sph::set_error(__VA_ARGS__);                                                  \
      throw ::sph::Failure{code};                                                     \
    }                                                                                 \
  } while (0)

#define SPH_API_BEGIN try {
#define SPH_API_END                                                                   \
  }                                                                                   \
  catch (const ::sph::Failure &f) {                                                   \
    return f.code;                                                                    \
  }                                                                                   \
  catch (const std::exception &ex) {                                                  \
    ::sph::set_error("exception: %s", ex.what());                                     \
    return SPH_HIP_ERUNTIME;                                                          \
  }                                                                                   \
  return SPH_HIP_OK;

// allocation log (SPH_ALLOC_LOG=1 at engine creation): every device buffer growth to stderr
extern int g_alloc_log;

// Growable device buffer (never shrinks; contents not preserved on growth unless asked).
template <class T>
struct DBuf {
  T *p = nullptr;
  size_t cap = 0;
  void reserve(size_t n, bool keep = false, hipStream_t s = 0) {
    if (n <= cap) return;
    size_t nc = n + n / 8 + 64;
    if (g_alloc_log)
      fprintf(stderr, "[sph] DBuf<%zu B> %p grows %zu -> %zu%s\n", sizeof(T), (void *)this, cap,
              nc, keep ? " (kept)" : "");
    T *q = nullptr;
    SPH_HIP_TRY(hipMalloc(&q, nc * sizeof(T)));
    if (keep && p && cap) SPH_HIP_TRY(hipMemcpyAsync(q, p, cap * sizeof(T), hipMemcpyDeviceToDevice, s));
    if (p) {
      if (keep) SPH_HIP_TRY(hipStreamSynchronize(s));
      (void)hipFree(p);
    }
    p = q;
    cap = nc;
  }
  // grow to exactly n (no headroom): scratch twins that are swapped with a buffer of
  // capacity n keep equal capacities, so the swap never triggers a reallocation
  void reserve_exact(size_t n) {
    if (n <= cap) return;
    T *q = nullptr;
    SPH_HIP_TRY(hipMalloc(&q, n * sizeof(T)));
    if (p) (void)hipFree(p);
    p = q;
    cap = n;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

void require_device(int device);

}  // namespace sph
