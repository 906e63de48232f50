// Host cost of submitting the headline's launch pair (event record, a kernel with a
// ~200-byte argument struct, a second kernel, event record) directly, as a replayed
// hipGraph, and as a hipGraph whose two kernel nodes get new arguments before each
// replay; wall time from submission to completion, first shot after an idle pause
// and repeated shots.
//   hipcc --offload-arch=gfx950 -O3 graph_launch.hip -o graph_launch
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

struct Args {
  double d[24];
  long long step0;
  double* out;
};

__global__ void k1(Args a) {
  if (threadIdx.x == 0 && blockIdx.x == 0) a.out[0] = a.d[0] + (double)a.step0;
}
__global__ void k2(const double* in, double* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[1] = in[0] * 2.0;
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double, std::micro>(b - a).count();
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  double* out;
  (void)hipMalloc(&out, 64);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  Args a{};
  a.out = out;
  auto direct = [&](long long step) {
    a.step0 = step;
    (void)hipEventRecord(e0, s);
    hipLaunchKernelGGL(k1, dim3(506), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k2, dim3(20), dim3(1024), 0, s, (const double*)out, out);
    (void)hipEventRecord(e1, s);
  };
  // graph of the same four operations
  hipGraph_t g;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  direct(0);
  (void)hipStreamEndCapture(s, &g);
  hipGraphExec_t ge;
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  size_t nn = 0;
  (void)hipGraphGetNodes(g, nullptr, &nn);
  hipGraphNode_t nodes[8];
  (void)hipGraphGetNodes(g, nodes, &nn);
  hipGraphNode_t kn = nullptr;
  for (size_t i = 0; i < nn; ++i) {
    hipGraphNodeType ty;
    (void)hipGraphNodeGetType(nodes[i], &ty);
    if (ty == hipGraphNodeTypeKernel && !kn) kn = nodes[i];
  }
  hipKernelNodeParams kp{};
  (void)hipGraphKernelNodeGetParams(kn, &kp);
  auto graph = [&](long long step, bool update) {
    if (update) {
      a.step0 = step;
      void* args[] = {&a};
      hipKernelNodeParams p = kp;
      p.kernelParams = args;
      (void)hipGraphExecKernelNodeSetParams(ge, kn, &p);
    }
    (void)hipGraphLaunch(ge, s);
  };
  for (int w = 0; w < 20; ++w) { direct(w); graph(w, true); }
  (void)hipStreamSynchronize(s);
  const char* names[3] = {"direct (record, launch, launch, record)", "graph replay", "graph + node update"};
  for (int mode = 0; mode < 3; ++mode) {
    double first = 0, rep = 0, sub_first = 0, sub_rep = 0;
    const int R = 20;
    for (int r = 0; r < R; ++r) {
      std::this_thread::sleep_for(std::chrono::milliseconds(20));   // the host comes back cold
      for (int k = 0; k < 2; ++k) {   // first shot after the pause, then a hot one
        const auto t0 = clk::now();
        if (mode == 0) direct(r);
        else graph(r, mode == 2);
        const auto t1 = clk::now();
        (void)hipStreamSynchronize(s);
        const auto t2 = clk::now();
        if (k == 0) { first += us(t0, t2); sub_first += us(t0, t1); }
        else { rep += us(t0, t2); sub_rep += us(t0, t1); }
      }
    }
    printf("%-42s first shot: submit %6.2f us, total %6.2f us | hot: submit %6.2f us, total %6.2f us\n",
           names[mode], sub_first / R, first / R, sub_rep / R, rep / R);
  }
  return 0;
}
