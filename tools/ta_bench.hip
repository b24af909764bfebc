// ta_bench.hip -- gather micro-benchmark: cost of one 64-lane vector load instruction on
// gfx950 as a function of how many distinct cache lines its lanes touch and of the bytes
// per lane.  Every lane issues NL loads (independent, accumulated) from a table of N
// records; the lane's record index comes from a per-lane LCG so the set of lines a wave
// instruction touches is controlled by the `share` parameter (lanes per record).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ta_bench tools/ta_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));

// W = bytes per lane (4, 8, 16); SHARE lanes read consecutive W-byte pieces of one record
// of REC bytes (REC = SHARE*W, aligned); window = records the random index ranges over
template <int W, int SHARE>
__global__ void __launch_bounds__(256) k_gather(const unsigned char *__restrict__ tab,
                                                unsigned nrec, unsigned window, int iters,
                                                unsigned *__restrict__ out) {
  constexpr int REC = W * SHARE;
  const unsigned lane = threadIdx.x & 63;
  const unsigned grp = lane / SHARE, sub = lane % SHARE;
  unsigned seed = (blockIdx.x * 4 + threadIdx.x / 64) * 2654435761u + grp * 40503u + 7u;
  const unsigned base = (blockIdx.x % 8) * (nrec / 8);  // per-XCD window
  unsigned acc = 0;
  for (int it = 0; it < iters; it++) {
    unsigned idx[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      seed = seed * 1664525u + 1013904223u;
      idx[k] = base + (seed >> 8) % window;
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const unsigned char *p = tab + (size_t)idx[k] * REC + sub * W;
      if (W == 16) {
        const v4u v = *reinterpret_cast<const v4u *>(p);
        acc += v.x ^ v.y ^ v.z ^ v.w;
      } else if (W == 8) {
        const v2u v = *reinterpret_cast<const v2u *>(p);
        acc += v.x ^ v.y;
      } else {
        acc += *reinterpret_cast<const unsigned *>(p);
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// fully coalesced 16 B/lane stream over the same table (reference rate)
__global__ void __launch_bounds__(256) k_stream(const v4u *__restrict__ tab, unsigned n16,
                                                int iters, unsigned *__restrict__ out) {
  unsigned acc = 0;
  const unsigned stride = gridDim.x * blockDim.x;
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  for (int it = 0; it < iters * 8; it++) {
    const v4u v = tab[i % n16];
    acc += v.x ^ v.y ^ v.z ^ v.w;
    i += stride;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int W, int SHARE>
void run(const unsigned char *tab, unsigned bytes, unsigned window_rec, unsigned *out,
         const char *name) {
  const unsigned nrec = bytes / (W * SHARE);
  const int blocks = 256 * 16, iters = 64;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_gather<W, SHARE>), dim3(blocks), dim3(256), 0, 0, tab, nrec,
                     window_rec, iters, out);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL((k_gather<W, SHARE>), dim3(blocks), dim3(256), 0, 0, tab, nrec,
                     window_rec, iters, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double instr = (double)blocks * 4 * iters * 8;  // wave-instructions
  const double per_cu = instr / 256.0;
  printf("%-28s W=%2d share=%2d window=%8u rec: %.3f ms, %.1f ns/instr/CU, %.1f cyc@2.4GHz\n",
         name, W, SHARE, window_rec, ms, ms * 1e6 / per_cu, ms * 1e6 / per_cu * 2.4);
}

int main() {
  const unsigned bytes = 64u << 20;  // 64 MB table (Infinity-cache resident)
  unsigned char *tab;
  unsigned *out;
  CK(hipMalloc(&tab, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(tab, 1, bytes));
  for (unsigned wkb : {512u, 8192u}) {  // per-XCD window in KB (L2-resident / beyond L2)
    printf("-- per-XCD window %u KB\n", wkb);
    const unsigned wb = wkb * 1024u;
    run<16, 1>(tab, bytes, wb / 16, out, "16B random, own line");
    run<16, 2>(tab, bytes, wb / 32, out, "16B, 2 lanes/32B rec");
    run<16, 4>(tab, bytes, wb / 64, out, "16B, 4 lanes/64B rec");
    run<16, 8>(tab, bytes, wb / 128, out, "16B, 8 lanes/128B line");
    run<8, 1>(tab, bytes, wb / 8, out, "8B random");
    run<8, 4>(tab, bytes, wb / 32, out, "8B, 4 lanes/32B rec");
    run<4, 1>(tab, bytes, wb / 4, out, "4B random");
  }
  {
    const int blocks = 256 * 16, iters = 64;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(256), 0, 0, (const v4u *)tab, bytes / 16,
                       iters, out);
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(256), 0, 0, (const v4u *)tab, bytes / 16,
                       iters, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double per_cu = (double)blocks * 4 * iters * 8 / 256.0;
    printf("%-28s W=16 coalesced: %.3f ms, %.1f cyc/instr/CU\n", "stream", ms,
           ms * 1e6 / per_cu * 2.4);
  }
  return 0;
}
