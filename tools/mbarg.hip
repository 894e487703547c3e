// Latency of the first dependent loads of a kernel: kernarg s_load, device s_load,
// vector load (GPU box).  Build: hipcc --offload-arch=gfx950 -O3 tools/mbarg.hip -o sac-td3-td7_amd/lib/mbarg
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

__device__ unsigned long long* g_out;

struct Args {
  const int* const* pp;  // device pointer to a device pointer
  int pad[64];
};

__global__ void probe(Args a) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0);
  const int* const* pp = a.pp;               // kernarg s_load
  const int* p = *(const int* const __attribute__((address_space(4)))*)pp;  // device s_load (constant)
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  const int v = __builtin_nontemporal_load(p + threadIdx.x);  // vector load
  const int w = v + 1;
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    unsigned long long* o = g_out;
    o[0] = t0;
    o[1] = t1;
    o[2] = t2;
    o[3] = (unsigned long long)w;
  }
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int* data;
  CK(hipMalloc(&data, 4096));
  CK(hipMemset(data, 0, 4096));
  int** pp;
  CK(hipMalloc(&pp, 64));
  CK(hipMemcpy(pp, &data, 8, hipMemcpyHostToDevice));
  unsigned long long* o;
  CK(hipMalloc(&o, 64));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_out), &o, 8));
  Args a{};
  a.pp = pp;
  for (int graph = 0; graph < 2; ++graph) {
    for (int rep = 0; rep < 4; ++rep) {
      if (!graph) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, st, a);
      } else {
        hipGraph_t g;
        hipGraphExec_t x;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, st, a);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(x, st));
        CK(hipStreamSynchronize(st));
        CK(hipGraphLaunch(x, st));
      }
      CK(hipStreamSynchronize(st));
      unsigned long long r[4];
      CK(hipMemcpy(r, o, 32, hipMemcpyDeviceToHost));
      printf("%s rep %d: kernarg->device s_load chain %6.2f us, vector load %6.2f us\n", graph ? "graph " : "stream",
             rep, (r[1] - r[0]) * 0.01, (r[2] - r[1]) * 0.01);
    }
  }
  return 0;
}
