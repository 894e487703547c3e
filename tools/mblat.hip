// Pointer-chase latency per hop on one lane, for several strides (GPU box).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mblat.hip -o sac-td3-td7_amd/lib/mblat
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

__global__ void chase(const unsigned* p, int hops, unsigned start, unsigned long long* out) {
  if (threadIdx.x != 0) return;
  unsigned idx = start;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int h = 0; h < hops; ++h) idx = __builtin_nontemporal_load(p + idx) + 0 * h, idx = p[idx];
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  out[0] = t1 - t0;
  out[1] = idx;
}

__global__ void chase1(const unsigned* p, int hops, unsigned start, unsigned long long* out) {
  if (threadIdx.x != 0) return;
  unsigned idx = start;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int h = 0; h < hops; ++h) idx = p[idx];
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  out[0] = t1 - t0;
  out[1] = idx;
}

__global__ void touch(unsigned* p, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = p[i];
}

int main() {
  const size_t N = (size_t)256 << 20;  // 1 GB of u32
  unsigned* d;
  CK(hipMalloc(&d, N * 4));
  unsigned long long* o;
  CK(hipMalloc(&o, 64));
  std::vector<unsigned> h(N);
  const int hops = 64;
  for (size_t stride : {(size_t)16, (size_t)1024, (size_t)16384, (size_t)(512 << 10), (size_t)(4 << 20)}) {
    // ring with the given stride in u32 elements
    for (size_t i = 0; i < N; ++i) h[i] = (unsigned)((i + stride) % N);
    CK(hipMemcpy(d, h.data(), N * 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(chase1, dim3(1), dim3(64), 0, 0, d, hops, (unsigned)(rep * 7), o);
      CK(hipDeviceSynchronize());
      unsigned long long r[2];
      CK(hipMemcpy(r, o, 16, hipMemcpyDeviceToHost));
      printf("stride %9zu B rep %d: %7.1f ns/hop\n", stride * 4, rep, r[0] * 10.0 / hops);
    }
    // after another kernel rewrote the data (dirty lines elsewhere)
    hipLaunchKernelGGL(touch, dim3(1024), dim3(256), 0, 0, d, N);
    hipLaunchKernelGGL(chase1, dim3(1), dim3(64), 0, 0, d, hops, 0u, o);
    CK(hipDeviceSynchronize());
    unsigned long long r[2];
    CK(hipMemcpy(r, o, 16, hipMemcpyDeviceToHost));
    printf("stride %9zu B after rewrite: %7.1f ns/hop\n", stride * 4, r[0] * 10.0 / hops);
  }
  return 0;
}
