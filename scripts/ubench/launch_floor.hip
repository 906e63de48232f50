// Launch-floor probe: per-launch wall time of back-to-back small kernels on
// one stream, plain launches vs the same sequence replayed from a hipGraph.
// Build: hipcc --offload-arch=gfx950 -O3 launch_floor.hip -o launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void touch(double* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.0;
}

int main() {
  const int n = 640 * 256;
  double* p;
  CK(hipMalloc(&p, n * sizeof(double)));
  CK(hipMemset(p, 0, n * sizeof(double)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 2000;
  struct Cfg { int blocks, threads; } cfgs[] = {{1, 64}, {640, 256}, {157, 1024}};
  for (auto c : cfgs) {
    for (int w = 0; w < 50; ++w) hipLaunchKernelGGL(touch, dim3(c.blocks), dim3(c.threads), 0, s, p, n);
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(touch, dim3(c.blocks), dim3(c.threads), 0, s, p, n);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    // same sequence as a graph of 100 launches, replayed
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int r = 0; r < 100; ++r) hipLaunchKernelGGL(touch, dim3(c.blocks), dim3(c.threads), 0, s, p, n);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps / 100; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float msg;
    CK(hipEventElapsedTime(&msg, a, b));
    std::printf("blocks %4d x %4d: stream %.2f us/launch, graph %.2f us/launch\n", c.blocks,
                c.threads, 1e3 * ms / reps, 1e3 * msg / reps);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipFree(p));
  return 0;
}
