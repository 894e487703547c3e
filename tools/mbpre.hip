// Kernel-argument preload vs kernarg-segment loads for the level op table (GPU box).
// Chains of 40 dependent launches (1024 workgroups each) in a hipGraph; per-launch time.
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-kernarg-preload-count=16 tools/mbpre.hip -o sac-td3-td7_amd/lib/mbpre
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

struct LA {
  const unsigned* ops;
  unsigned e[12];
};
__device__ __forceinline__ void body(const unsigned* ops, const unsigned* ee, unsigned long long* out) {
  int k = 0;
  unsigned e = ee[0];
#pragma unroll
  for (int q = 1; q < 12; ++q) {
    const unsigned x = ee[q];
    const bool in = (int)(x & 0xffffu) <= (int)blockIdx.x;
    e = in ? x : e;
    k = in ? q : k;
  }
  // one dependent descriptor load (scalar), then one vector load, as a GEMM prologue
  const unsigned d = __builtin_amdgcn_readfirstlane(ops[k * 16]);
  const unsigned v = ops[(d + threadIdx.x) & 1023];
  if (v == 0xdeadbeef) out[blockIdx.x] = e;
}
__global__ __launch_bounds__(256) void kstruct(const LA la, unsigned long long* out) { body(la.ops, la.e, out); }
__global__ __launch_bounds__(256) void kflat(const unsigned* ops, unsigned e0, unsigned e1, unsigned e2, unsigned e3,
                                             unsigned e4, unsigned e5, unsigned e6, unsigned e7, unsigned e8,
                                             unsigned e9, unsigned e10, unsigned e11) {
  const unsigned ee[12] = {e0, e1, e2, e3, e4, e5, e6, e7, e8, e9, e10, e11};
  body(ops, ee, nullptr);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned* ops;
  CK(hipMalloc(&ops, 1 << 20));
  CK(hipMemset(ops, 0, 1 << 20));
  unsigned long long* out;
  CK(hipMalloc(&out, 1 << 20));
  const int L = 40, reps = 50;
  for (int nwg : {256, 1024}) {
    for (int kind = 0; kind < 2; ++kind) {
      hipGraph_t g;
      hipGraphExec_t x;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      for (int l = 0; l < L; ++l) {
        LA la{};
        la.ops = ops + l * 256;
        for (int q = 0; q < 12; ++q) la.e[q] = q < 6 ? (unsigned)(q * nwg / 6) | (1u << 16) : 0xffffu;
        if (kind == 0) hipLaunchKernelGGL(kstruct, dim3(nwg), dim3(256), 0, st, la, out);
        else
          hipLaunchKernelGGL(kflat, dim3(nwg), dim3(256), 0, st, la.ops, la.e[0], la.e[1], la.e[2], la.e[3],
                             la.e[4], la.e[5], la.e[6], la.e[7], la.e[8], la.e[9], la.e[10], la.e[11]);
      }
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
      for (int w = 0; w < 5; ++w) CK(hipGraphLaunch(x, st));
      CK(hipStreamSynchronize(st));
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a, st));
      for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(x, st));
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("%-7s nwg %5d: %6.3f us per launch\n", kind ? "preload" : "kernarg", nwg, ms * 1e3 / (reps * L));
    }
  }
  return 0;
}
