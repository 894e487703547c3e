// Gate for splitting a level into specialised launches (VERDICT r5 "do this" #1): per dependency level
// of N GEMM ops (M x 256 x 256 each, 16 x 64 tiles: M / 4 workgroups per op), the time per level of
//   A  one `mega` launch (rle_level's structure: op from a preloaded table, descriptor load, variant switch);
//   B  N `spec` launches as AQL packets, the barrier bit on the level's first only (agent acquire on it,
//      none on the others -- they launch after it), agent release on every one (they retire in any order);
//   B2 as B, agent acquire on every packet;
//   C  N `spec` packets without release fences, then one barrier-AND packet per level that waits for them
//      all and releases at agent scope;
//   D  as B with `specd` (the descriptor loaded from memory instead of preloaded kernel arguments);
//   E  N `spec` packets, each with the barrier bit (the ops of a level serialised).
// Every mode's final buffers are compared with A's (bitwise: the same tiles, the same sums).
// Build (CPU container): hipcc --offload-arch=gfx950 --offload-device-only --no-gpu-bundle-output -O3
//   -mllvm -amdgpu-kernarg-preload-count=14 -c tools/mbsplit_k.hip -o build/mbsplit_k.co &&
//   hipcc -O2 tools/mbsplit.cpp -o build/mbsplit -lhsa-runtime64
// Run (GPU box): build/mbsplit build/mbsplit_k.co
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <algorithm>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)
#define HK(x)                                                                    \
  do {                                                                           \
    hsa_status_t s = (x);                                                        \
    if (s != HSA_STATUS_SUCCESS) { printf("%s: %d\n", #x, (int)s); exit(1); }    \
  } while (0)

static hsa_agent_t g_gpu;
static hsa_status_t find_gpu(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) { g_gpu = a; return HSA_STATUS_INFO_BREAK; }
  return HSA_STATUS_SUCCESS;
}
struct Kern { uint64_t obj; uint32_t gseg, pseg; };
struct Desc { const float *a, *w; float* out; const float* bias; unsigned long long pad[4]; };
constexpr int kMaxOps = 12, L = 48;

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "build/mbsplit_k.co";
  std::ifstream f(path, std::ios::binary);
  std::vector<char> co((std::istreambuf_iterator<char>(f)), {});
  if (co.empty()) { printf("no code object %s\n", path); return 1; }
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  HK(hsa_init());
  hsa_iterate_agents(find_gpu, nullptr);
  hsa_code_object_reader_t rdr;
  HK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rdr));
  hsa_executable_t exe;
  HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
  HK(hsa_executable_load_agent_code_object(exe, g_gpu, rdr, nullptr, nullptr));
  HK(hsa_executable_freeze(exe, nullptr));
  auto kern = [&](const std::string& name) {
    Kern k;
    hsa_executable_symbol_t sym;
    HK(hsa_executable_get_symbol_by_name(exe, (name + ".kd").c_str(), &g_gpu, &sym));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.obj));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.gseg));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.pseg));
    return k;
  };
  Kern kmega = kern("mega"), kspec[6], kspecd[6];
  for (int v = 0; v < 6; ++v) {
    kspec[v] = kern("spec" + std::to_string(v));
    kspecd[v] = kern("specd" + std::to_string(v));
  }
  hsa_queue_t* q;
  HK(hsa_queue_create(g_gpu, 16384, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
  hsa_signal_t sig;
  HK(hsa_signal_create(1, 0, nullptr, &sig));

  const int Mmax = 1024;
  const size_t act = (size_t)Mmax * 256;  // floats per op buffer
  float *buf, *wts, *bias;
  CK(hipMalloc(&buf, 2 * kMaxOps * act * 4));
  CK(hipMalloc(&wts, kMaxOps * 65536 * 4));
  CK(hipMalloc(&bias, kMaxOps * 256 * 4));
  {
    std::vector<float> h(kMaxOps * 65536);
    for (size_t i = 0; i < h.size(); ++i) h[i] = ((float)((i * 2654435761u) % 2001) / 1000.f - 1.f) / 16.f;
    CK(hipMemcpy(wts, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    std::vector<float> hb(kMaxOps * 256);
    for (size_t i = 0; i < hb.size(); ++i) hb[i] = (float)((i * 40503u) % 101) / 1000.f - 0.05f;
    CK(hipMemcpy(bias, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  }
  std::vector<float> h0(kMaxOps * act);
  for (size_t i = 0; i < h0.size(); ++i) h0[i] = (float)((i * 2246822519u) % 1000) / 1000.f - 0.5f;
  auto reset = [&] {
    CK(hipMemcpy(buf, h0.data(), h0.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(buf + kMaxOps * act, 0, kMaxOps * act * 4));
    CK(hipDeviceSynchronize());
  };
  auto in_of = [&](int parity, int j) { return buf + ((size_t)parity * kMaxOps + j) * act; };

  // kernel arguments in device memory: [parity][slot] 128 B apart
  // slot 0: mega's 12 entries + ops pointer; slots 1..12: spec (a, w, out, bias); slots 13..24: specd (desc ptr)
  // descriptors: [parity][op] 64 B
  constexpr int kSlots = 1 + 2 * kMaxOps;
  char* kargs;
  Desc* descs;
  CK(hipMalloc(&kargs, 2 * kSlots * 128));
  CK(hipMalloc(&descs, 2 * kMaxOps * sizeof(Desc)));
  auto ka = [&](int parity, int slot) { return kargs + ((size_t)parity * kSlots + slot) * 128; };

  auto setup = [&](int N, int M) {
    const int W = M / 4;  // workgroups per op
    std::vector<char> hk(2 * kSlots * 128, 0);
    std::vector<Desc> hd(2 * kMaxOps);
    for (int p = 0; p < 2; ++p) {
      unsigned* e = (unsigned*)(hk.data() + ((size_t)p * kSlots) * 128);
      for (int qq = 0; qq < 12; ++qq) e[qq] = qq < N ? (unsigned)(qq * W) | ((unsigned)(qq % 6) << 20) : 0xffffu;
      *(Desc**)(hk.data() + ((size_t)p * kSlots) * 128 + 48) = descs + p * kMaxOps;
      for (int j = 0; j < N; ++j) {
        Desc d{in_of(p, j), wts + (size_t)j * 65536, in_of(1 - p, j), bias + j * 256, {}};
        hd[p * kMaxOps + j] = d;
        const void** s = (const void**)(hk.data() + ((size_t)p * kSlots + 1 + j) * 128);
        s[0] = d.a; s[1] = d.w; s[2] = d.out; s[3] = d.bias;
        *(Desc**)(hk.data() + ((size_t)p * kSlots + 1 + kMaxOps + j) * 128) = descs + p * kMaxOps + j;
      }
    }
    CK(hipMemcpy(kargs, hk.data(), hk.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(descs, hd.data(), hd.size() * sizeof(Desc), hipMemcpyHostToDevice));
  };

  uint64_t wi = 0;  // packets written (== the queue's write index: one writer)
  auto slot = [&]() {
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
    while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {}
    wi = idx + 1;
    return (hsa_kernel_dispatch_packet_t*)q->base_address + (idx & (q->size - 1));
  };
  auto hdr = [](int type, bool barrier, int acq, int rel) {
    return (uint16_t)((type << HSA_PACKET_HEADER_TYPE) | ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
                      (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) | (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  };
  auto dispatch = [&](const Kern& k, unsigned wgs, const void* args, bool barrier, int acq, int rel, bool last) {
    auto* pk = slot();
    pk->workgroup_size_x = 256; pk->workgroup_size_y = 1; pk->workgroup_size_z = 1; pk->reserved0 = 0;
    pk->grid_size_x = wgs * 256; pk->grid_size_y = 1; pk->grid_size_z = 1;
    pk->private_segment_size = k.pseg; pk->group_segment_size = k.gseg;
    pk->kernel_object = k.obj; pk->kernarg_address = const_cast<void*>(args); pk->reserved2 = 0;
    pk->completion_signal = last ? sig : hsa_signal_t{0};
    __atomic_store_n((uint32_t*)pk, (uint32_t)hdr(HSA_PACKET_TYPE_KERNEL_DISPATCH, barrier, acq, rel) | (1u << 16),
                     __ATOMIC_RELEASE);
  };
  auto barrier_and = [&](int rel, bool last) {
    auto* pk = (hsa_barrier_and_packet_t*)slot();
    pk->reserved0 = 0; pk->reserved1 = 0;
    for (int i = 0; i < 5; ++i) pk->dep_signal[i] = hsa_signal_t{0};
    pk->reserved2 = 0;
    pk->completion_signal = last ? sig : hsa_signal_t{0};
    __atomic_store_n((uint32_t*)pk, (uint32_t)hdr(HSA_PACKET_TYPE_BARRIER_AND, true, 0, rel), __ATOMIC_RELEASE);
  };
  const int AG = HSA_FENCE_SCOPE_AGENT, SY = HSA_FENCE_SCOPE_SYSTEM, NO = HSA_FENCE_SCOPE_NONE;
  // one burst of `levels` levels in mode m; returns host wall us from the doorbell to completion
  auto burst = [&](char m, int N, int M, int levels) {
    const int W = M / 4;
    hsa_signal_store_relaxed(sig, 1);
    for (int l = 0; l < levels; ++l) {
      const int p = l & 1;
      const bool first = l == 0, lastl = l == levels - 1;
      if (m == 'A') {
        dispatch(kmega, N * W, ka(p, 0), true, first ? SY : AG, lastl ? SY : AG, lastl);
        continue;
      }
      for (int j = 0; j < N; ++j) {
        const bool fj = j == 0, lj = j == N - 1;
        const Kern& k = m == 'D' ? kspecd[j % 6] : kspec[j % 6];
        const void* a = m == 'D' ? ka(p, 1 + kMaxOps + j) : ka(p, 1 + j);
        const int acq = (first && fj) ? SY : (fj || m == 'E' || m == '2') ? AG : NO;
        if (m == 'C') {
          dispatch(k, W, a, fj, acq, NO, false);
        } else {
          dispatch(k, W, a, fj || m == 'E', acq, (lastl && lj) ? SY : AG, lastl && lj);
        }
      }
      if (m == 'C') barrier_and(lastl ? SY : AG, lastl);
    }
    auto t0 = std::chrono::steady_clock::now();
    hsa_signal_store_screlease(q->doorbell_signal, wi - 1);
    while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 1000000000ull, HSA_WAIT_STATE_ACTIVE) >= 1) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 20) { printf("timeout\n"); exit(3); }
    }
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  };
  std::vector<float> ref(kMaxOps * act), got(kMaxOps * act);
  const char modes[] = {'A', 'B', '2', 'C', 'D', 'E'};
  printf("us per level (median of 5 bursts of %d levels); N ops x (M/4) workgroups per level\n", L * 4);
  printf("%5s %3s %8s %8s %8s %8s %8s %8s\n", "M", "N", "A mega", "B split", "B2 acq", "C bar", "D desc", "E serial");
  for (int M : {256, 1024}) {
    for (int N : {1, 2, 4, 6, 8, 12}) {
      setup(N, M);
      printf("%5d %3d", M, N);
      for (char m : modes) {
        reset();
        burst(m, N, M, L);  // (L even: the result is back in parity 0)
        CK(hipMemcpy(got.data(), buf, (size_t)N * act * 4, hipMemcpyDeviceToHost));
        if (m == 'A') ref = got;
        bool same = std::memcmp(got.data(), ref.data(), (size_t)N * act * 4) == 0;
        std::vector<double> t;
        for (int r = 0; r < 5; ++r) t.push_back(burst(m, N, M, L * 4) / (L * 4));
        std::sort(t.begin(), t.end());
        printf(" %7.3f%s", t[2], same ? " " : "!");
      }
      printf("\n");
      fflush(stdout);
    }
  }
  printf("('!' = final buffers differ from A's)\n");

  // ---- F: row-block fused chains (P chains x L layers in ONE launch, 16 workgroups per chain, the activations in
  // LDS) against the same work as L dependent `mega` levels of P ops (M = 256: 64 workgroups of 16 x 64 tiles each)
  Kern kchain = kern("chain");
  float *cx, *cw, *cout;
  CK(hipMalloc(&cx, 12 * 65536 * 4));
  CK(hipMalloc(&cw, 12 * 8 * 65536 * 4));
  CK(hipMalloc(&cout, 12 * 65536 * 4));
  CK(hipMemset(cx, 0, 12 * 65536 * 4));
  CK(hipMemset(cw, 0, 12 * 8 * 65536 * 4));
  char* cka;
  CK(hipMalloc(&cka, 128));
  printf("\nfused chains: us per chain pass (median of 5 bursts of 48) vs L x the level time of mode A (N = P, M = 256)\n");
  printf("%3s %3s %9s %9s %9s\n", "P", "L", "F fused", "L x A", "F / LxA");
  for (int P : {1, 2, 4, 6, 12}) {
    setup(P, 256);
    std::vector<double> ta;
    for (int r = 0; r < 5; ++r) ta.push_back(burst('A', P, 256, L * 4) / (L * 4));
    std::sort(ta.begin(), ta.end());
    for (int Lc : {2, 3, 4, 8}) {
      struct { const float *x, *w; float* o; const float* b; int L; } a{cx, cw, cout, bias, Lc};
      CK(hipMemcpy(cka, &a, sizeof(a), hipMemcpyHostToDevice));
      std::vector<double> tf;
      for (int r = 0; r < 5; ++r) {
        hsa_signal_store_relaxed(sig, 1);
        const int nb = 48;
        for (int i = 0; i < nb; ++i) dispatch(kchain, P * 16, cka, true, i == 0 ? SY : AG, i == nb - 1 ? SY : AG, i == nb - 1);
        auto t0 = std::chrono::steady_clock::now();
        hsa_signal_store_screlease(q->doorbell_signal, wi - 1);
        while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 1000000000ull, HSA_WAIT_STATE_ACTIVE) >= 1) {}
        tf.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / nb);
      }
      std::sort(tf.begin(), tf.end());
      printf("%3d %3d %9.3f %9.3f %9.3f\n", P, Lc, tf[2], Lc * ta[2], tf[2] / (Lc * ta[2]));
      fflush(stdout);
    }
  }
  printf("done\n");
  return 0;
}
