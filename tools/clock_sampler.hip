// tools/clock_sampler.hip -- measurement helper (not part of the product): a one-wave kernel on
// a stream of its own that samples the shader clock counter against the constant 100 MHz
// real-time counter while the engine's kernels run beside it, so the clock during a pass is
// read without serialising the dispatches (rocprofv3 --pmc does).  Built by
// `hipcc --offload-arch=gfx950 -shared -fPIC tools/clock_sampler.hip -o tools/libclock_sampler.so`
// (tools/clock_probe.sh); used by tools/inner_probe.py --sampler.
#include <hip/hip_runtime.h>

__global__ void k_clock_sampler(unsigned long long *out, int n, unsigned long long span) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const unsigned long long step = span / (unsigned long long)n;
  for (int k = 0; k < n; k++) {
    const unsigned long long target = t0 + (unsigned long long)(k + 1) * step;
    unsigned long long t, c;
    do {
      t = __builtin_amdgcn_s_memrealtime();
      c = __builtin_amdgcn_s_memtime();
    } while (t < target);
    out[2 * k] = t - t0;
    out[2 * k + 1] = c - c0;
  }
}

static hipStream_t g_s = nullptr;
static unsigned long long *g_d = nullptr;
static int g_n = 0;

extern "C" {
// n samples over span_us microseconds, launched now on the sampler's own stream
int clk_start(int n, double span_us) {
  if (!g_s && hipStreamCreateWithFlags(&g_s, hipStreamNonBlocking) != hipSuccess) return 1;
  if (n > g_n) {
    if (g_d) (void)hipFree(g_d);
    if (hipMalloc(&g_d, sizeof(unsigned long long) * 2 * n) != hipSuccess) return 2;
    g_n = n;
  }
  const unsigned long long span = (unsigned long long)(span_us * 100.0);  // 100 MHz ticks
  hipLaunchKernelGGL(k_clock_sampler, dim3(1), dim3(64), 0, g_s, g_d, n, span);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
// wait for the sampler; out[2k] = real-time ticks (10 ns), out[2k+1] = shader clock cycles
int clk_read(unsigned long long *out, int n) {
  if (hipStreamSynchronize(g_s) != hipSuccess) return 1;
  return hipMemcpy(out, g_d, sizeof(unsigned long long) * 2 * n, hipMemcpyDeviceToHost) ==
                 hipSuccess ? 0 : 2;
}
}
