// Level handoff cost on MI355X (gfx950): kernel boundary vs in-launch dataflow (diagnostics, GPU box).
// A chain of S stages of W workgroups; every workgroup of stage s reads a 4 KB block that a workgroup of
// stage s - 1 on another XCD wrote (block (7 w + 3) mod W), adds to it and writes its own block.
//   boundary: one launch per stage (stream order = the engine's level boundaries)
//   dataflow: all S x W workgroups in ONE launch; stage s waits for stage s - 1's counter to reach W
//             (agent-scope acquire), its producers store, release (agent scope) and count.  Workgroups are
//             dispatched in index order, so every producer of a stage is resident or done before any of
//             its consumers is dispatched: a wait always ends.  Each wait is bounded anyway (err counts
//             the waits that gave up; the result is then wrong, never a hang).
//   nowait:   the same single launch without the waits (the stages' work alone, overlapped)
// Prints microseconds per stage.  Build: hipcc --offload-arch=gfx950 -O3 tools/mbflow.hip -o build/mbflow
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); }  \
  } while (0)

constexpr int kThr = 256;

__device__ __forceinline__ void stage_work(const float4* in, float4* out, int W, int w) {
  const int src = (7 * w + 3) % W;
  float4 v = in[(size_t)src * kThr + threadIdx.x];
  v.x += 1.f;
  out[(size_t)w * kThr + threadIdx.x] = v;
}

__global__ __launch_bounds__(kThr) void k_stage(const float4* in, float4* out, int W) {
  stage_work(in, out, W, blockIdx.x);
}

template <bool WAIT>
__global__ __launch_bounds__(kThr) void k_flow(float4* buf, int* cnt, int* err, int W) {
  const int s = blockIdx.x / W, w = blockIdx.x - s * W;
  if (WAIT && s > 0) {
    if (threadIdx.x == 0) {
      int it = 0;
      while (__hip_atomic_load(cnt + s - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < W) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > (1 << 22)) {
          atomicAdd(err, 1);
          break;
        }
      }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (the producers' stores are visible)
  }
  stage_work(buf + (size_t)s * W * kThr, buf + (size_t)(s + 1) * W * kThr, W, w);
  if (WAIT) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt + s, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int main(int argc, char** argv) {
  const int S = argc > 1 ? atoi(argv[1]) : 32, W = argc > 2 ? atoi(argv[2]) : 512, reps = argc > 3 ? atoi(argv[3]) : 20;
  float4* buf;
  int *cnt, *err;
  CK(hipMalloc(&buf, (size_t)(S + 1) * W * kThr * sizeof(float4)));
  CK(hipMemset(buf, 0, (size_t)(S + 1) * W * kThr * sizeof(float4)));
  CK(hipMalloc(&cnt, S * sizeof(int)));
  CK(hipMalloc(&err, sizeof(int)));
  CK(hipMemset(err, 0, sizeof(int)));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // boundary chain as a captured graph (the engine's hipGraph path)
  hipGraph_t g;
  hipGraphExec_t gx;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int s = 0; s < S; ++s)
    k_stage<<<W, kThr, 0, st>>>(buf + (size_t)s * W * kThr, buf + (size_t)(s + 1) * W * kThr, W);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&gx, g, nullptr, nullptr, 0));
  auto timeit = [&](auto&& launch) {
    launch();
    CK(hipStreamSynchronize(st));
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0, st));
      launch();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    return best * 1e3f / S;
  };
  const float t_graph = timeit([&] { CK(hipGraphLaunch(gx, st)); });
  const float t_stream = timeit([&] {
    for (int s = 0; s < S; ++s)
      k_stage<<<W, kThr, 0, st>>>(buf + (size_t)s * W * kThr, buf + (size_t)(s + 1) * W * kThr, W);
  });
  const float t_flow = timeit([&] {
    CK(hipMemsetAsync(cnt, 0, S * sizeof(int), st));
    k_flow<true><<<S * W, kThr, 0, st>>>(buf, cnt, err, W);
  });
  const float t_nowait = timeit([&] { k_flow<false><<<S * W, kThr, 0, st>>>(buf, cnt, err, W); });
  int h_err = 0;
  CK(hipMemcpy(&h_err, err, sizeof(int), hipMemcpyDeviceToHost));
  // check: stage S's blocks hold S (each stage adds 1 along its source chain) -- dataflow ordering held
  std::vector<float4> last((size_t)W * kThr);
  CK(hipMemsetAsync(cnt, 0, S * sizeof(int), st));
  CK(hipMemsetAsync(buf, 0, (size_t)(S + 1) * W * kThr * sizeof(float4), st));
  k_flow<true><<<S * W, kThr, 0, st>>>(buf, cnt, err, W);
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(last.data(), buf + (size_t)S * W * kThr, last.size() * sizeof(float4), hipMemcpyDeviceToHost));
  int bad = 0;
  for (auto& v : last) bad += v.x != (float)S;
  printf("S %d W %d: us per stage  graph %.2f  stream %.2f  dataflow %.2f  nowait %.2f  (waits given up %d, "
         "wrong blocks %d)\n", S, W, t_graph, t_stream, t_flow, t_nowait, h_err, bad);
  return 0;
}
