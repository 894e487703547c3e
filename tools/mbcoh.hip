// Cross-launch visibility of control values on MI355X (gfx950) under hipGraph replay: what the
// engine's `sload` (kernels.hip: a scalar load of a value an earlier launch wrote) and its
// Ctrl-block false sharing rely on.  Each test is a chain of captured kernel nodes
//   prime (every workgroup loads the line: K$ / every XCD's L2 hold the OLD value)
//   -> write (workgroup w writes the line: plain store, device-scope atomic, or two
//            workgroups on different XCDs storing different bytes of the same 128-B line)
//   -> read  (every workgroup loads it: scalar load, or vector load)
// repeated `iters` times per graph with a new value each time, the graph replayed `reps` times.
// A cache that a kernel-node boundary does not refresh returns the previous iteration's value.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mbcoh.hip -o build/mbcoh
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); }  \
  } while (0)

#define CAS __attribute__((address_space(4)))

constexpr int kNwg = 2048, kThr = 256;

__device__ __forceinline__ int sld(const int* p) { return *(const CAS int*)p; }
// plain vector load (a buffer load: the compiler cannot turn it into a scalar one)
__device__ __forceinline__ int vld(const int* p, int off) {
  return (int)__builtin_amdgcn_raw_buffer_load_b32(__builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 0x7fff0000, 0x00020000),
                                                   off * 4, 0, 0);
}

// every workgroup pulls the line into its CU's scalar cache and its XCD's L2
__global__ __launch_bounds__(kThr) void k_prime(const int* ctl, int* sink) {
  const int a = sld(ctl), b = sld(ctl + 16), c = sld(ctl + 8);
  if (threadIdx.x == 0) sink[blockIdx.x] = a + b + c + ((const volatile int*)ctl)[4];
}

// MODE 0: workgroup w stores ctl[0] = val (plain vector store)
// MODE 1: workgroup w atomicMax(ctl[0], val) (device scope)
// MODE 2: workgroups w and w + 1 (adjacent: different XCDs) store ctl[0] and ctl[16] = val
//         (two XCDs dirty different bytes of one 128-B line in the same launch)
// MODE 3: as 1, while every other workgroup scalar-loads ctl[8] (same line) and atomically adds 1
//         to ctl[24] (the engine's Ctrl: head atomics beside Adam scalars read by GEMMs)
template <int MODE>
__global__ __launch_bounds__(kThr) void k_write(int* ctl, int val, int w, int* sink) {
  const int b = blockIdx.x;
  if (threadIdx.x != 0) return;
  if (MODE == 0 && b == w) ctl[0] = val;
  if ((MODE == 1 || MODE == 3) && b == w) atomicMax(ctl, val);
  if (MODE == 2) {
    if (b == w) ctl[0] = val;
    if (b == w + 1) ctl[16] = val;
  }
  if (MODE == 3 && b != w) {
    sink[b] = sld(ctl + 8);
    atomicAdd(ctl + 24, 1);
  }
}

// every workgroup reads ctl[0] (and ctl[16] for MODE 2): scalar (VEC 0) or vector (VEC 1) loads
template <int VEC, int MODE>
__global__ __launch_bounds__(kThr) void k_read(const int* ctl, int want, int* bad) {
  int a, c = want;
  if (VEC) {
    a = vld(ctl, 0);
    if (MODE == 2) c = vld(ctl, 16);
  } else {
    a = sld(ctl);
    if (MODE == 2) c = sld(ctl + 16);
  }
  if (threadIdx.x == 0 && (a != want || c != want)) atomicAdd(bad, 1);
}

template <int VEC, int MODE>
static void run(const char* name, int iters, int reps) {
  int *ctl, *sink, *bad;
  CK(hipMalloc(&ctl, 4096));
  CK(hipMalloc(&sink, kNwg * 4));
  CK(hipMalloc(&bad, 4));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t x;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < iters; ++i) {
    const int w = (i * 37) % (kNwg - 1);
    k_prime<<<kNwg, kThr, 0, st>>>(ctl, sink);
    k_write<MODE><<<kNwg, kThr, 0, st>>>(ctl, i + 1, w, sink);
    k_read<VEC, MODE><<<kNwg, kThr, 0, st>>>(ctl, i + 1, bad);
  }
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipMemsetAsync(bad, 0, 4, st));
  for (int r = 0; r < reps; ++r) {
    CK(hipMemsetAsync(ctl, 0, 4096, st));
    CK(hipGraphLaunch(x, st));
  }
  int nb = 0;
  CK(hipMemcpyAsync(&nb, bad, 4, hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  printf("%-44s %8lld workgroup reads, %lld stale\n", name, (long long)iters * reps * kNwg, (long long)nb);
  CK(hipGraphExecDestroy(x));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(st));
  CK(hipFree(ctl));
  CK(hipFree(sink));
  CK(hipFree(bad));
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200, reps = argc > 2 ? atoi(argv[2]) : 20;
  CK(hipSetDevice(0));
  run<0, 0>("plain store -> scalar load", iters, reps);
  run<1, 0>("plain store -> vector load", iters, reps);
  run<0, 1>("atomicMax -> scalar load", iters, reps);
  run<1, 1>("atomicMax -> vector load", iters, reps);
  run<0, 2>("2 XCDs, 2 halves of a line -> scalar load", iters, reps);
  run<1, 2>("2 XCDs, 2 halves of a line -> vector load", iters, reps);
  run<0, 3>("atomicMax + line sharers -> scalar load", iters, reps);
  run<1, 3>("atomicMax + line sharers -> vector load", iters, reps);
  printf("done\n");
  return 0;
}
