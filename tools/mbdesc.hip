// Where should a level's op descriptor live?  A graph of 200 dependent launches (1024
// workgroups each, the engine's level geometry); every workgroup reads a descriptor
// (pointer + offset), then one 16-B vector load through it and a store.  Variants:
//   kernarg: descriptor in the kernel-argument segment (s_load from the kernarg pointer)
//   table:   descriptor in a device table written once at setup (s_load, constant space)
//   table2:  as table, with a second dependent descriptor record (a GEMM's epilogue fields)
// Reports us per launch (graph replay, HIP events).  GPU box only.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mbdesc.hip -o sac-td3-td7_amd/lib/mbdesc
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)
#define CAS __attribute__((address_space(4)))

struct Desc {
  const float* src;
  float* dst;
  int off, pad;
  const float* src2;
  long long pad2[12];
};
struct KArgs {
  Desc d[16];
  int which;
};
struct TArgs {
  const Desc* table;
  int which;
};

__global__ __launch_bounds__(256) void k_kernarg(const KArgs a) {
  const Desc& d = a.d[blockIdx.x & 15];
  const float v = d.src[(blockIdx.x * 256 + threadIdx.x) & 4095];
  d.dst[blockIdx.x * 256 + threadIdx.x] = v + 1.f;
}
__global__ __launch_bounds__(256) void k_table(const TArgs a) {
  const CAS Desc* t = (const CAS Desc*)a.table;
  const CAS Desc& d = t[blockIdx.x & 15];
  const float v = d.src[(blockIdx.x * 256 + threadIdx.x) & 4095];
  d.dst[blockIdx.x * 256 + threadIdx.x] = v + 1.f;
}
__global__ __launch_bounds__(256) void k_table2(const TArgs a) {
  const CAS Desc* t = (const CAS Desc*)a.table;
  const CAS Desc& d = t[blockIdx.x & 15];
  const float v = d.src[(blockIdx.x * 256 + threadIdx.x) & 4095];
  const CAS Desc& d2 = t[16 + (blockIdx.x & 15)];
  const float w = d2.src2[(blockIdx.x * 256 + threadIdx.x) & 4095];
  d.dst[blockIdx.x * 256 + threadIdx.x] = v + w;
}

template <class F>
static double run(F launch, hipStream_t st) {
  const int reps = 200;
  hipGraph_t g;
  hipGraphExec_t x;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < reps; ++i) launch(i);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(x, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  double best = 1e30;
  for (int t = 0; t < 5; ++t) {
    CK(hipEventRecord(a, st));
    CK(hipGraphLaunch(x, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms * 1000.0 / reps < best ? ms * 1000.0 / reps : best;
  }
  return best;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int nwg = 1024;
  float *buf, *src;
  CK(hipMalloc(&buf, (size_t)nwg * 256 * 4 * 2));
  CK(hipMalloc(&src, 4096 * 4));
  CK(hipMemset(src, 0, 4096 * 4));
  // per launch i: its own descriptor table (as the engine's per-level op tables)
  const int reps = 200;
  Desc* tables;
  CK(hipMalloc(&tables, sizeof(Desc) * 32 * reps));
  Desc h[32 * 200];
  KArgs ka[200];
  for (int i = 0; i < reps; ++i)
    for (int q = 0; q < 32; ++q) {
      Desc d{};
      d.src = (i & 1) ? buf : src;  // dependent chain: odd launches read what even ones wrote
      d.dst = (i & 1) ? buf + (size_t)nwg * 256 : buf;
      d.src2 = src;
      h[i * 32 + q] = d;
      if (q < 16) ka[i].d[q] = d;
    }
  CK(hipMemcpy(tables, h, sizeof(h), hipMemcpyHostToDevice));
  printf("sizeof(KArgs) = %zu\n", sizeof(KArgs));
  for (int rep = 0; rep < 3; ++rep) {
    const double tk = run([&](int i) { hipLaunchKernelGGL(k_kernarg, dim3(nwg), dim3(256), 0, st, ka[i]); }, st);
    const double tt = run([&](int i) {
      TArgs t{tables + (size_t)i * 32, 0};
      hipLaunchKernelGGL(k_table, dim3(nwg), dim3(256), 0, st, t);
    }, st);
    const double t2 = run([&](int i) {
      TArgs t{tables + (size_t)i * 32, 0};
      hipLaunchKernelGGL(k_table2, dim3(nwg), dim3(256), 0, st, t);
    }, st);
    printf("us per dependent launch: kernarg %6.3f | table %6.3f | table + 2nd record %6.3f\n", tk, tt, t2);
  }
  return 0;
}
