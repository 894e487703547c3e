// Microbenchmark of the level-dispatch kernel on synthetic ops (GPU box only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I sac-td3-td7_amd/csrc \
//        tools/mb.cpp sac-td3-td7_amd/lib/kernels.o -o /tmp/mb
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
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

static float* dalloc(size_t n) {
  float* p;
  CK(hipMalloc(&p, n * 4));
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice));
  return p;
}

// Y = relu(X W^T + b); X: N image [M][K], W: N image [N][K], Y: T image [M][N].
static Op fwd_op(float* X, float* W, float* b, float* Y, int M, int N, int K) {
  Op op{};
  op.kind = OP_GEMM;
  GemmArgs& g = op.gemm;
  g.mode = GEMM_FWD;
  g.M = M; g.N = N; g.R = K;
  g.A.nseg = 1;
  g.A.seg[0].p = X; g.A.seg[0].xs = K / 16; g.A.seg[0].x0 = 0; g.A.seg[0].x1 = M; g.A.seg[0].r0 = 0; g.A.seg[0].r1 = K;
  g.B.nseg = 1;
  g.B.seg[0].p = W; g.B.seg[0].xs = K / 16; g.B.seg[0].x0 = 0; g.B.seg[0].x1 = N; g.B.seg[0].r0 = 0; g.B.seg[0].r1 = K;
  g.tn = 16;
  g.tiles_m = (M + kTileM - 1) / kTileM; g.tiles_n = (N + g.tn - 1) / g.tn;
  g.vid = gemm_vid(GEMM_FWD, EPI_STORE, ACT_RELU, 0);
  g.ks_log = 2;
  g.inv_tiles_n = 1.f / (float)g.tiles_n;
  g.epi = EPI_STORE; g.act = ACT_RELU; g.bias = b;
  g.out.t = Y; g.out.rbs = M / 16; g.out.cbn = N / 16;
  op.wg_count = g.tiles_m * g.tiles_n;
  return op;
}

static size_t nidx(int cbn, int r, int c) {
  return ((size_t)(r >> 4) * cbn + (c >> 4)) * 256 + ((c >> 2) & 3) * 64 + (r & 15) * 4 + (c & 3);
}
static size_t tidx(int rbs, int r, int c) {
  return ((size_t)(c >> 4) * rbs + (r >> 4)) * 256 + ((r >> 2) & 3) * 64 + (c & 15) * 4 + (r & 3);
}

static unsigned long long* g_trace = nullptr;  // [wg][4] phase stamps of the last rep

static double time_level(std::vector<Op> ops, int reps, hipStream_t st) {
  int wg = 0;
  for (auto& o : ops) { o.wg_begin = wg; wg += o.wg_count; }
  Op* d;
  CK(hipMalloc(&d, ops.size() * sizeof(Op)));
  CK(hipMemcpy(d, ops.data(), ops.size() * sizeof(Op), hipMemcpyHostToDevice));
  // capture reps launches in a graph, like the engine
  hipGraph_t g; hipGraphExec_t x;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < reps; ++i) CK(launch_level(d, ops.data(), (int)ops.size(), wg, st, g_trace));
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(x, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a, st));
  CK(hipGraphLaunch(x, st));
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGraphExecDestroy(x)); CK(hipGraphDestroy(g)); CK(hipFree(d));
  return ms * 1000.0 / reps;
}

// entry-relative phase medians of the last traced level: prologue, loop, epilogue, total
static void phases(const char* name, int nwg) {
  std::vector<unsigned long long> t((size_t)nwg * 4);
  CK(hipMemcpy(t.data(), g_trace, t.size() * 8, hipMemcpyDeviceToHost));
  unsigned long long t0 = ~0ull, t3 = 0;
  std::vector<double> pro, loop, epi;
  for (int w = 0; w < nwg; ++w) {
    t0 = std::min(t0, t[w * 4]);
    t3 = std::max(t3, t[w * 4 + 3]);
    pro.push_back((t[w * 4 + 1] - t[w * 4]) * 0.01);
    loop.push_back((t[w * 4 + 2] - t[w * 4 + 1]) * 0.01);
    epi.push_back((t[w * 4 + 3] - t[w * 4 + 2]) * 0.01);
  }
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  printf("   %-28s span %6.2f us | pro %5.2f loop %5.2f epi %5.2f\n", name, (t3 - t0) * 0.01, med(pro), med(loop),
         med(epi));
}


int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int K = 256, N = 256;
  float* X = dalloc(2048 * 1100);
  float* W = dalloc(16 * 256 * 1100);
  float* bb = dalloc(4096);
  float* Y = dalloc(16 * 2048 * 256);
  long long* cnt; CK(hipMalloc(&cnt, 128)); CK(hipMemset(cnt, 0, 128));
  const int reps = 200;
  {
    Op e{}; e.kind = 0; e.wg_count = 1;
    printf("empty 1 WG          : %8.2f us\n", time_level({e}, reps, st));
    e.wg_count = 256;
    printf("empty 256 WG        : %8.2f us\n", time_level({e}, reps, st));
    e.wg_count = 2048;
    printf("empty 2048 WG       : %8.2f us\n", time_level({e}, reps, st));
  }
  {
    Op e{}; e.kind = OP_STEP_END; e.wg_count = 1; e.end.counters = cnt; e.end.cmask = 1;
    printf("step_end counters   : %8.2f us\n", time_level({e}, reps, st));
  }
  {  // correctness of one fwd tile set vs CPU
    const int M = 256, Kc = 384;
    Op o = fwd_op(X, W, bb, Y, M, N, Kc);
    time_level({o}, 1, st);
    std::vector<float> hx((size_t)M * Kc), hw((size_t)N * Kc), hb(N), hy((size_t)M * N);
    CK(hipMemcpy(hx.data(), X, hx.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hw.data(), W, hw.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), bb, hb.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hy.data(), Y, hy.size() * 4, hipMemcpyDeviceToHost));
    double md = 0;
    for (int i = 0; i < M; ++i)
      for (int n = 0; n < N; ++n) {
        double s = hb[n];
        for (int k = 0; k < Kc; ++k) s += (double)hx[nidx(Kc / 16, i, k)] * hw[nidx(Kc / 16, n, k)];
        s = s > 0 ? s : 0;
        md = std::max(md, std::abs(s - hy[tidx(M / 16, i, n)]));
      }
    printf("fwd correctness max|d| = %.3g\n", md);
  }
  for (int Kk : {16, 64, 128, 256, 512, 1024}) {
    Op o = fwd_op(X, W, bb, Y, 256, N, Kk);
    printf("fwd 256x256xK=%4d (64 WG): %8.2f us\n", Kk, time_level({o}, reps, st));
  }
  for (int Kk : {16, 256, 1024}) {
    Op o = fwd_op(X, W, bb, Y, 16, 64, Kk);
    printf("fwd 16x64xK=%4d (1 WG)   : %8.2f us\n", Kk, time_level({o}, reps, st));
  }
  CK(hipMalloc(&g_trace, 8 * 4 * 4096));
  for (int Kk : {16, 256, 1024}) {
    Op o = fwd_op(X, W, bb, Y, 256, N, Kk);
    time_level({o}, 20, st);
    char nm[64];
    snprintf(nm, sizeof nm, "traced fwd 256x256xK=%d", Kk);
    phases(nm, o.wg_count);
  }
  {
    Op e{}; e.kind = 0; e.wg_count = 256;
    time_level({e}, 20, st);
    std::vector<unsigned long long> t(256 * 4);
    CK(hipMemcpy(t.data(), g_trace, t.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long a = ~0ull, b = 0;
    for (int w = 0; w < 256; ++w) { a = std::min(a, t[w * 4]); b = std::max(b, t[w * 4 + 3]); }
    printf("   traced empty 256 WG span %6.2f us\n", (b - a) * 0.01);
  }
  CK(hipFree(g_trace));
  g_trace = nullptr;
  {  // contention: copies of the same-shaped GEMM in one level (tn 16 -> 256 WG each)
    CK(hipMalloc(&g_trace, 8 * 4 * 8192));
    for (int Kk : {256, 768}) {
      for (int copies : {1, 2, 4, 8}) {
        std::vector<Op> v;
        for (int i = 0; i < copies; ++i) {
          Op o = fwd_op(X, W + (size_t)i * 256 * 800, bb, Y + (size_t)i * 2048 * 256, 256, N, Kk);
          o.gemm.tn = 16;
          o.gemm.tiles_n = 16;
          o.gemm.ks_log = 2;
          o.gemm.inv_tiles_n = 1.f / 16.f;
          o.wg_count = 256;
          v.push_back(o);
        }
        const double us = time_level(v, 50, st);
        char nm[64];
        snprintf(nm, sizeof nm, "%dx fwd 256x256x%d (%d WG)", copies, Kk, 256 * copies);
        printf("%-34s %8.2f us\n", nm, us);
        time_level(v, 5, st);
        phases(nm, 256 * copies);
      }
    }
    CK(hipFree(g_trace));
    g_trace = nullptr;
  }
  for (int M : {256, 512}) {
    Op o = fwd_op(X, W, bb, Y, M, N, K);
    printf("fwd %dx%dx%d (%d WG): %8.2f us\n", M, N, K, o.wg_count, time_level({o}, reps, st));
  }
  {
    Op o = fwd_op(X, W, bb, Y, 256, N, 384);
    printf("fwd 256x256x384     : %8.2f us\n", time_level({o}, reps, st));
    std::vector<Op> v;
    for (int i = 0; i < 8; ++i) v.push_back(fwd_op(X, W + (size_t)i * 256 * 400, bb, Y + (size_t)i * 2048 * 256, 256, N, 384));
    printf("8x fwd 256x256x384 (2048 WG): %8.2f us\n", time_level(v, reps, st));
  }
  return 0;
}
