// Microbenchmark of the LAP sampler level (OP_SAMPLE_GATHER over a 1M-row replay) with
// fine phase stamps (GPU box only).  Build (kernels with -DRLE_TRACE_FINE):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DRLE_TRACE_FINE -I include -I sac-td3-td7_amd/csrc \
//         -c sac-td3-td7_amd/csrc/kernels.hip -o sac-td3-td7_amd/lib/mb_kernels_fine.o
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I sac-td3-td7_amd/csrc -c tools/mbs.cpp -o /tmp/mbs.o
//   hipcc --offload-arch=gfx950 /tmp/mbs.o sac-td3-td7_amd/lib/mb_kernels_fine.o -o sac-td3-td7_amd/lib/mb_sampler
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "ops.h"

namespace rle {
hipError_t launch_level(const Op* d_ops, const Op* h_ops, int nops, int nwg, hipStream_t st,
                        unsigned long long* trace = nullptr);
}
using namespace rle;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)

template <class T>
static T* dmake(size_t n) {
  T* p;
  CK(hipMalloc(&p, n * sizeof(T)));
  CK(hipMemset(p, 0, n * sizeof(T)));
  return p;
}

int main() {
  const long long N = 1000000;
  const int S = 376, Sp = 384, A = 17, Ap = 32, B = 256, nblk = (int)((N + 4095) / 4096);
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  SampleArgs s{};
  s.state = dmake<float>((size_t)N * Sp);
  s.next_state = dmake<float>((size_t)N * Sp);
  s.action = dmake<float>((size_t)N * Ap);
  s.reward = dmake<float>(N);
  s.notdone = dmake<float>(N);
  float* prio = dmake<float>(N);
  {
    std::vector<float> p(N);
    for (long long i = 0; i < N; ++i) p[i] = 1.f + (float)((i * 2654435761u) % 97) / 32.f;
    CK(hipMemcpy(prio, p.data(), N * 4, hipMemcpyHostToDevice));
  }
  s.priority = prio;
  long long* size = dmake<long long>(1);
  CK(hipMemcpy(size, &N, 8, hipMemcpyHostToDevice));
  s.size = size;
  s.cap = N;
  s.S = S; s.Sp = Sp; s.A = A; s.Ap = Ap; s.B = B; s.lap = 1;
  s.bsum = dmake<double>(nblk);
  s.nblk = nblk;
  s.ss.t = dmake<float>((size_t)2 * B * Sp); s.ss.rbs = 2 * B / 16; s.ss.cbn = Sp / 16;
  s.ss.n = dmake<float>((size_t)2 * B * Sp);
  s.a.t = dmake<float>((size_t)B * Ap); s.a.n = dmake<float>((size_t)B * Ap); s.a.rbs = B / 16; s.a.cbn = Ap / 16;
  s.r = dmake<float>(B); s.nd = dmake<float>(B);
  s.ind = dmake<long long>(B);
  s.u_out = dmake<float>(B);
  s.eps.t = dmake<float>((size_t)B * Ap); s.eps.rbs = B / 16; s.eps.cbn = Ap / 16;
  long long* cnt = dmake<long long>(2);
  int* mode = dmake<int>(1);
  s.ctrl_rng = cnt; s.tape_mode = mode; s.tape_pos = cnt + 1;
  s.seed = 1234;
  // block sums
  Op red{}; red.kind = OP_SAMPLE_REDUCE; red.sample = s; red.wg_count = nblk;
  Op* dred = dmake<Op>(1);
  CK(hipMemcpy(dred, &red, sizeof(Op), hipMemcpyHostToDevice));
  CK(launch_level(dred, &red, 1, nblk, st));
  Op g{}; g.kind = OP_SAMPLE_GATHER; g.sample = s; g.wg_count = B;
  Op* dg = dmake<Op>(1);
  CK(hipMemcpy(dg, &g, sizeof(Op), hipMemcpyHostToDevice));
  // plain timing (graph of 200 launches)
  const int reps = 200;
  hipGraph_t gr; hipGraphExec_t gx;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < reps; ++i) CK(launch_level(dg, &g, 1, B, st));
  CK(hipStreamEndCapture(st, &gr));
  CK(hipGraphInstantiate(&gx, gr, nullptr, nullptr, 0));
  CK(hipGraphLaunch(gx, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  CK(hipGraphLaunch(gx, st));
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("sampler level (256 WG, LAP over 1M): %.2f us per launch\n", ms * 1000 / reps);
  // traced
  unsigned long long* tr = dmake<unsigned long long>((size_t)B * 16);  // kTraceStride (fine build)
  for (int rep = 0; rep < 3; ++rep) {
    CK(launch_level(dg, &g, 1, B, st, tr));
    CK(hipStreamSynchronize(st));
  }
  std::vector<unsigned long long> a((size_t)B * 16);
  CK(hipMemcpy(a.data(), tr, a.size() * 8, hipMemcpyDeviceToHost));
  // stamps in order: entry t0, ctrl f0, noise f1, bsum f2, scan f3, found t1, prio loads f4,
  // scan2 f5, hit t2, gather f6, exit t3
  const char* names[] = {"ctrl loads", "noise", "bsum loads", "scan1", "found1", "prio loads",
                         "scan2", "hit", "gather", "exit"};
  std::vector<std::vector<double>> d(10);
  for (int w = 0; w < B; ++w) {
    const unsigned long long* t = &a[(size_t)w * 16];
    const unsigned long long* f = t + 4;
    unsigned long long seq[11] = {t[0], f[0], f[1], f[2], f[3], t[1], f[4], f[5], t[2], f[6], t[3]};
    for (int i = 0; i < 10; ++i) d[i].push_back(((double)seq[i + 1] - (double)seq[i]) * 0.01);
  }
  for (int i = 0; i < 10; ++i) {
    std::sort(d[i].begin(), d[i].end());
    printf("  %-12s median %6.2f us  p90 %6.2f\n", names[i], d[i][B / 2], d[i][B * 9 / 10]);
  }
  return 0;
}
