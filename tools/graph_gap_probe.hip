// Dispatch gap between dependent kernels on one stream, plain launches against a captured
// hipGraph of the same chain.  A chain is K kernels that each read and write n doubles (the
// step's short kernels: integrate, forward, ...); the gap is (chain time - K x one kernel's
// time) / K.  Build: hipcc -O3 --offload-arch=gfx950 tools/graph_gap_probe.hip -o
// tools/graph_gap_probe.  usage: graph_gap_probe [n_doubles=1048576] [K=5] [reps=200]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void k_touch(double *a, size_t n, double s) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = a[i] * s + 1.0;
}

static void chain(hipStream_t st, double *a, size_t n, int K) {
  const int bl = 256;
  const unsigned g = (unsigned)((n + bl - 1) / bl);
  for (int k = 0; k < K; k++) hipLaunchKernelGGL(k_touch, dim3(g), dim3(bl), 0, st, a, n, 0.5);
}

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1u << 20);
  const int K = argc > 2 ? atoi(argv[2]) : 5;
  const int reps = argc > 3 ? atoi(argv[3]) : 200;
  double *a;
  CK(hipMalloc(&a, n * sizeof(double)));
  CK(hipMemset(a, 0, n * sizeof(double)));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms;
  // one kernel's time: many independent... (dependent anyway on one stream) -- time one
  // launch bracketed by events, averaged
  double one = 0.0;
  for (int r = 0; r < 50; r++) {
    CK(hipEventRecord(e0, st));
    chain(st, a, n, 1);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 10) one += ms / 40.0;
  }
  // plain launches
  for (int r = 0; r < 20; r++) chain(st, a, n, K);
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; r++) chain(st, a, n, K);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double plain = ms / reps;
  // captured graph of one chain
  hipGraph_t gr;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  chain(st, a, n, K);
  CK(hipStreamEndCapture(st, &gr));
  CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
  for (int r = 0; r < 20; r++) CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; r++) CK(hipGraphLaunch(ge, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double graph = ms / reps;
  printf("{\"n_doubles\": %zu, \"K\": %d, \"one_kernel_us\": %.2f, \"chain_plain_us\": %.2f, "
         "\"chain_graph_us\": %.2f, \"gap_plain_us\": %.2f, \"gap_graph_us\": %.2f}\n",
         n, K, one * 1e3, plain * 1e3, graph * 1e3, (plain - K * one) * 1e3 / K,
         (graph - K * one) * 1e3 / K);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(gr));
  CK(hipFree(a));
  return 0;
}
