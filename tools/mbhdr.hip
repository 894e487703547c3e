// Dependent-load chain at kernel entry (GPU box): where each level's prologue time goes.
// Chains of 40 launches of 1024 workgroups in a hipGraph, per-launch time for:
//   A: kernarg op table -> vector load (descriptor fields in the kernel arguments)
//   B: kernarg op table -> device s_load of a 80-byte descriptor -> vector load (current)
//   C: kernarg -> vector load, but 4 KB of kernel arguments
// Build: hipcc --offload-arch=gfx950 -O3 tools/mbhdr.hip -o sac-td3-td7_amd/lib/mbhdr
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

struct Hot {
  unsigned w[20];
};
struct LAk {  // descriptors in kernel arguments
  unsigned entry[16];
  Hot hot[16];
};
struct LAd {  // descriptors in device memory
  const Hot* ops;
  unsigned entry[16];
};
__device__ __forceinline__ int pick(const unsigned* ent) {
  int k = 0;
#pragma unroll
  for (int q = 1; q < 16; ++q) k = (int)(ent[q] & 0xffffu) <= (int)blockIdx.x ? q : k;
  return k;
}
__device__ __forceinline__ void body(const Hot& h, unsigned long long* out) {
  const float* p = (const float*)(((unsigned long long)h.w[15] << 32) | h.w[14]);
  const float v = p[(h.w[3] + threadIdx.x) & 4095];
  if (v == 1234.5f) out[blockIdx.x] = h.w[0];
}
__global__ __launch_bounds__(256) void kA(const LAk la, unsigned long long* out) {
  const int k = pick(la.entry);
  body(la.hot[k], out);
}
__global__ __launch_bounds__(256) void kB(const LAd la, unsigned long long* out) {
  const int k = pick(la.entry);
  const Hot h = la.ops[k];
  body(h, out);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  float* data;
  CK(hipMalloc(&data, 1 << 20));
  CK(hipMemset(data, 0, 1 << 20));
  Hot* dops;
  CK(hipMalloc(&dops, 40 * 16 * sizeof(Hot)));
  Hot hh[40 * 16];
  for (int i = 0; i < 40 * 16; ++i) {
    for (int j = 0; j < 20; ++j) hh[i].w[j] = j;
    hh[i].w[14] = (unsigned)(unsigned long long)data;
    hh[i].w[15] = (unsigned)((unsigned long long)data >> 32);
  }
  CK(hipMemcpy(dops, hh, sizeof(hh), hipMemcpyHostToDevice));
  unsigned long long* out;
  CK(hipMalloc(&out, 1 << 20));
  const int L = 40, reps = 50, nwg = 1024;
  for (int kind = 0; kind < 2; ++kind) {
    hipGraph_t g;
    hipGraphExec_t x;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int l = 0; l < L; ++l) {
      unsigned ent[16];
      for (int q = 0; q < 16; ++q) ent[q] = q < 6 ? (unsigned)(q * nwg / 6) : 0xffffu;
      if (kind == 0) {
        LAk la{};
        for (int q = 0; q < 16; ++q) la.entry[q] = ent[q], la.hot[q] = hh[l * 16 + q];
        hipLaunchKernelGGL(kA, dim3(nwg), dim3(256), 0, st, la, out);
      } else {
        LAd la{};
        la.ops = dops + l * 16;
        for (int q = 0; q < 16; ++q) la.entry[q] = ent[q];
        hipLaunchKernelGGL(kB, dim3(nwg), dim3(256), 0, st, la, out);
      }
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
    printf("%s: %6.3f us per launch (kernarg bytes %zu)\n", kind ? "B descriptor in device memory" : "A descriptor in kernargs",
           ms * 1e3 / (reps * L), kind ? sizeof(LAd) : sizeof(LAk));
  }
  return 0;
}
