// Instruction-fetch cost probe: straight-line code of N bytes per wave (GPU box).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mbic.hip -o build/mbic
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

#define NOP16 "s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n"
#define NOP64 NOP16 NOP16 NOP16 NOP16
#define NOP256 NOP64 NOP64 NOP64 NOP64

template <int N256>
__global__ void body(int* out) {
#pragma unroll
  for (int i = 0; i < N256; ++i) asm volatile(NOP256 ::);  // 1 KB of code each
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

template <int N256>
static double t(int nwg, int* o, hipStream_t st) {
  const int reps = 100;
  hipGraph_t g;
  hipGraphExec_t x;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(body<N256>, dim3(nwg), dim3(256), 0, st, o);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(x, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, st));
  CK(hipGraphLaunch(x, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.0 / reps;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int* o;
  CK(hipMalloc(&o, 64));
  for (int nwg : {1, 256, 1024}) {
    printf("nwg %4d: 0 KB %6.2f | 1 KB %6.2f | 4 KB %6.2f | 8 KB %6.2f | 16 KB %6.2f us\n", nwg, t<0>(nwg, o, st),
           t<1>(nwg, o, st), t<4>(nwg, o, st), t<8>(nwg, o, st), t<16>(nwg, o, st));
  }
  return 0;
}
