// RESULT (MI355X, ROCm 7.2): launch per level 4.0 us; in-launch seam 6.8 us per level with sc1
// stores, 6.5 us with plain stores (co-located teams) -> kernel boundaries stay.
// Cost of an in-launch level seam for the row-partitioned chain (GPU box).
// 1024 workgroups (4 per CU) of 256 threads; team = blockIdx % 8 (same-XCD hint), rank =
// blockIdx / 8.  Each level every workgroup reads a 16-row x 256-col fp32 slab of the
// previous level (rows owned by its team; sc1 buffer loads), does a little math, writes
// a 16 x 64 tile (sc1 stores), then a sharded team barrier (agent atomics, sc1 poll).
// Output is checked against the host.  Compared with the same per-level body as one
// kernel launch per level.  Build: hipcc --offload-arch=gfx950 -O3 tools/mbchain.hip -o build/mbchain
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

constexpr int R = 256, C = 256;  // rows (batch) x cols per level buffer
constexpr int NT = 1024;         // workgroups
// tile t of a level: rows 16*(t/4)... 16 row tiles x 4 col tiles (64 cols) = 64 tiles; 1024 WGs
// -> each tile computed by... we use 16 x 16 tiles: 16 row tiles x 16 col tiles = 256 tiles;
// team x (blockIdx%8) owns row tiles 2x, 2x+1 (32 tiles); rank<32 computes one tile, others idle.

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 0x7fff0000, 0x00020000);
}
template <int AUX>
__device__ __forceinline__ float4 ld(__amdgpu_buffer_rsrc_t r, int off) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
template <int AUX>
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, int off, float4 v) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  u4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, AUX);
}

// one tile of level l: out[r][c] = sum_k in[r][k] * w(k, c) for r in the 16-row tile, c in
// the 16-col tile; here w(k,c) = ((k + c) % 7 - 3) / 64 (cheap, exact in fp32 for small sums)
template <int AUX, int SAUX = AUX>
__device__ void tile(const float* in, float* out, int t, float* lds) {
  const int it = t >> 4, jt = t & 15;
  const int tid = threadIdx.x;
  __amdgpu_buffer_rsrc_t ri = rsrc(in), ro = rsrc(out);
  // load the 16 x 256 slab: 4096 floats = 1024 float4, 4 per thread
  for (int q = 0; q < 4; ++q) {
    const int f4 = tid + q * 256;
    const int r = f4 >> 6, c4 = f4 & 63;
    float4 v = ld<AUX>(ri, ((it * 16 + r) * C + c4 * 4) * 4);
    *(float4*)(lds + r * C + c4 * 4) = v;
  }
  __syncthreads();
  const int r = tid >> 4, c = jt * 16 + (tid & 15);
  float acc = 0.f;
  const float wc = (float)((c & 7) - 3) * (1.f / 64.f);
#pragma unroll 8
  for (int k = 0; k < C; k += 4) {
    const float4 v = *(const float4*)(lds + r * C + k);
    acc += (v.x + v.y) * wc + (v.z - v.w) * (1.f / 128.f);
  }
  acc = tanhf(acc);
  __syncthreads();
  // store 16 x 16 via lanes (tid < 64 store float4)
  lds[r * 16 + (tid & 15)] = acc;
  __syncthreads();
  if (tid < 64) {
    const int rr = tid >> 2, cc = (tid & 3) * 4;
    st<SAUX>(ro, ((it * 16 + rr) * C + jt * 16 + cc) * 4, *(float4*)(lds + rr * 16 + cc));
  }
}

template <int SAUX>
__global__ __launch_bounds__(256) void chain(float* bufs, int L, unsigned* bar, unsigned base, unsigned* err) {
  __shared__ float lds[16 * C];
  const int team = blockIdx.x & 7, rank = blockIdx.x >> 3;  // 128 per team
  const int shard = rank & 3;
  for (int l = 0; l < L; ++l) {
    const float* in = bufs + (size_t)l * R * C;
    float* out = bufs + (size_t)(l + 1) * R * C;
    if (rank < 32) tile<16, SAUX>(in, out, (team * 2 + (rank >> 4)) * 16 + (rank & 15), lds);
    if (l + 1 == L) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned target = base + 32u * (l + 1);
    unsigned* cnt = bar + team * 1024;  // one counter per team, 4 KB apart
    if (threadIdx.x == 0) {
      if (rank < 32) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      long long spins = 0;
      while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > 20000000) { atomicOr(err, 2u); break; }
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void one(const float* in, float* out) {
  __shared__ float lds[16 * C];
  if (blockIdx.x < 256) tile<0>(in, out, blockIdx.x, lds);
}

int main() {
  const int L = 32;
  float* bufs;
  CK(hipMalloc(&bufs, (size_t)(L + 1) * R * C * 4));
  std::vector<float> h0((size_t)R * C);
  for (size_t i = 0; i < h0.size(); ++i) h0[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(bufs, h0.data(), h0.size() * 4, hipMemcpyHostToDevice));
  unsigned *bar, *err;
  CK(hipMalloc(&bar, 8 * 4096));
  CK(hipMemset(bar, 0, 8 * 4096));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // reference: per-level launches
  hipGraph_t g;
  hipGraphExec_t x;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int l = 0; l < L; ++l) hipLaunchKernelGGL(one, dim3(256), dim3(256), 0, st, bufs + (size_t)l * R * C, bufs + (size_t)(l + 1) * R * C);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(x, st));
  CK(hipStreamSynchronize(st));
  std::vector<float> ref((size_t)R * C), got((size_t)R * C);
  CK(hipMemcpy(ref.data(), bufs + (size_t)L * R * C, ref.size() * 4, hipMemcpyDeviceToHost));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 40;
  CK(hipEventRecord(a, st));
  for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(x, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("launch per level : %6.3f us per level\n", ms * 1e3 / (reps * L));
  // chain: base advances by 32 per level boundary per shard
  unsigned base = 0;
  {
    unsigned e0;
    CK(hipMemcpy(&e0, err, 4, hipMemcpyDeviceToHost));
    printf("err before %u  err %p bar %p bufs %p\n", e0, (void*)err, (void*)bar, (void*)bufs);
  }
  for (int var = 0; var < 2; ++var)
  for (int Lc : {1, L}) {
    auto K = var ? chain<0> : chain<16>;
    CK(hipMemset(bufs + (size_t)R * C, 0, (size_t)L * R * C * 4));
    // warm + check
    hipLaunchKernelGGL(K, dim3(NT), dim3(256), 0, st, bufs, Lc, bar, base, err);
    base += 32u * (Lc - 1);
    CK(hipStreamSynchronize(st));
    if (Lc == L) {
      CK(hipMemcpy(got.data(), bufs + (size_t)L * R * C, got.size() * 4, hipMemcpyDeviceToHost));
      double md = 0;
      for (size_t i = 0; i < got.size(); ++i) md = fmax(md, fabs(got[i] - ref[i]));
      unsigned e;
      CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
      printf("chain check: max |diff| vs launches %.3g, err %u\n", md, e);
    }
    CK(hipEventRecord(a, st));
    for (int r = 0; r < reps; ++r) {
      hipLaunchKernelGGL(K, dim3(NT), dim3(256), 0, st, bufs, Lc, bar, base, err);
      base += 32u * (Lc - 1);
    }
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%s chain L=%2d: %7.3f us per launch\n", var ? "plain-store" : "sc1-store", Lc, ms * 1e3 / reps);
  }
  unsigned e;
  CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
  printf("err %u\n", e);
  return 0;
}
