// RESULT (MI355X, ROCm 7.2, 256 workgroups, 16 KB slab per workgroup): hipGraph 4.08 us per
// level, AQL agent/agent 3.83, acquire none + release agent 3.68, none/none with sc1 loads and
// stores 3.52 (exact); plain loads/stores without a release are stale.  Empty kernel: 1.53 / 1.26.
// Kernel arguments must live in device memory (host kernarg pool: 23-29 us per level).
// => at most ~0.5 us per level (~6% of a TD7 step) from owning the queue: not pursued.
// Launch cost of a dependent level chain: hipGraph vs AQL packets written straight into an HSA
// queue with chosen acquire / release fence scopes (GPU box).  Ring of two 256 x 256 fp32
// buffers (level l reads buf[l & 1], writes buf[(l + 1) & 1]): a cache that is not refreshed
// across levels returns stale values, and the final buffer differs from the hipGraph run.
// Build: hipcc --offload-arch=gfx950 --offload-device-only --no-gpu-bundle-output -O3 -c
//   tools/mbaql_k.hip -o build/mbaql_k.co &&
//   hipcc -O2 tools/mbaql.cpp -o build/mbaql -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
  } while (0)
#define HK(x)                                                        \
  do {                                                               \
    hsa_status_t s = (x);                                            \
    if (s != HSA_STATUS_SUCCESS) { printf("%s: %d\n", #x, (int)s); exit(1); } \
  } while (0)

constexpr int R = 256, C = 256, L = 32;
static hsa_agent_t g_gpu;
static hsa_region_t g_karg;

static hsa_status_t find_gpu(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) { g_gpu = a; return HSA_STATUS_INFO_BREAK; }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_karg(hsa_region_t r, void*) {
  uint32_t f;
  hsa_region_get_info(r, HSA_REGION_INFO_GLOBAL_FLAGS, &f);
  if (f & HSA_REGION_GLOBAL_FLAG_KERNARG) { g_karg = r; return HSA_STATUS_INFO_BREAK; }
  return HSA_STATUS_SUCCESS;
}

struct Kern { uint64_t obj; uint32_t gseg, pseg; hipFunction_t hf; };
static hsa_executable_t g_mine;
static std::string g_want;
static uint64_t g_found;
static hsa_status_t find_exe(hsa_executable_t e, void*) {
  if (e.handle == g_mine.handle) return HSA_STATUS_SUCCESS;
  hsa_executable_symbol_t sym;
  if (hsa_executable_get_symbol_by_name(e, g_want.c_str(), &g_gpu, &sym) == HSA_STATUS_SUCCESS) {
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &g_found);
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "build/mbaql_k.co";
  std::ifstream f(path, std::ios::binary);
  std::vector<char> co((std::istreambuf_iterator<char>(f)), {});
  if (co.empty()) { printf("no code object %s\n", path); return 1; }
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  HK(hsa_init());
  hsa_iterate_agents(find_gpu, nullptr);
  hsa_agent_iterate_regions(g_gpu, find_karg, nullptr);
  hsa_code_object_reader_t rdr;
  HK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rdr));
  hsa_executable_t exe;
  HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
  HK(hsa_executable_load_agent_code_object(exe, g_gpu, rdr, nullptr, nullptr));
  HK(hsa_executable_freeze(exe, nullptr));
  hipModule_t mod;
  CK(hipModuleLoadData(&mod, co.data()));
  auto kern = [&](const char* name) {
    Kern k;
    hsa_executable_symbol_t sym;
    HK(hsa_executable_get_symbol_by_name(exe, (std::string(name) + ".kd").c_str(), &g_gpu, &sym));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.obj));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.gseg));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.pseg));
    CK(hipModuleGetFunction(&k.hf, mod, name));
    if (getenv("HIPOBJ")) {  // the kernel object of HIP's own loaded copy of the module
      g_mine = exe; g_want = std::string(name) + ".kd"; g_found = 0;
      hsa_ven_amd_loader_1_03_pfn_t tbl;
      HK(hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(tbl), &tbl));
      tbl.hsa_ven_amd_loader_iterate_executables(find_exe, nullptr);
      if (!g_found) { printf("HIP copy of %s not found\n", name); exit(1); }
      k.obj = g_found;
    }
    return k;
  };
  hsa_queue_t* q;
  HK(hsa_queue_create(g_gpu, 8192, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
  hsa_signal_t sig;
  HK(hsa_signal_create(1, 0, nullptr, &sig));
  const int reps = 40;
  // kernel arguments in DEVICE memory (each workgroup's kernarg loads would otherwise cross
  // PCIe to the host kernarg pool), written once: level l's arguments are the same every rep
  void* kargs;
  CK(hipMalloc(&kargs, (size_t)L * 64));

  float* buf;
  CK(hipMalloc(&buf, 2ull * R * C * 4));
  std::vector<float> h0((size_t)R * C), ref((size_t)R * C), got((size_t)R * C);
  for (size_t i = 0; i < h0.size(); ++i) h0[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  auto reset = [&] { CK(hipMemcpy(buf, h0.data(), h0.size() * 4, hipMemcpyHostToDevice)); CK(hipMemset(buf + R * C, 0, R * C * 4)); CK(hipDeviceSynchronize()); };

  // ---- hipGraph reference
  Kern k00 = kern("one_0_0");
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  auto graph_of = [&](Kern& k) {
    hipGraph_t g;
    hipGraphExec_t x;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int l = 0; l < L; ++l) {
      struct { float* in; float* out; } a = {buf + (l & 1) * R * C, buf + ((l + 1) & 1) * R * C};
      size_t sz = sizeof(a);
      void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
      CK(hipModuleLaunchKernel(k.hf, 256, 1, 1, 256, 1, 1, 0, st, nullptr, cfg));
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    return x;
  };
  hipGraphExec_t gx = graph_of(k00);
  reset();
  CK(hipGraphLaunch(gx, st));
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(ref.data(), buf, ref.size() * 4, hipMemcpyDeviceToHost));
  auto time_graph = [&](hipGraphExec_t x, const char* what) {
    CK(hipGraphLaunch(x, st));
    CK(hipStreamSynchronize(st));
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(x, st));
    CK(hipStreamSynchronize(st));
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    printf("%-34s %7.3f us per level\n", what, us / (reps * L));
  };
  time_graph(gx, "hipGraph one_0_0");
  printf("one_0_0: group %u private %u\n", k00.gseg, k00.pseg);
  {
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r)
      for (int l = 0; l < L; ++l) {
        struct { float* in; float* out; } a = {buf + (l & 1) * R * C, buf + ((l + 1) & 1) * R * C};
        size_t sz = sizeof(a);
        void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
        CK(hipModuleLaunchKernel(k00.hf, 256, 1, 1, 256, 1, 1, 0, st, nullptr, cfg));
      }
    CK(hipStreamSynchronize(st));
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    printf("%-34s %7.3f us per level\n", "stream launches one_0_0", us / (reps * L));
  }
  Kern ke = kern("empty");
  hipGraphExec_t gxe = graph_of(ke);
  time_graph(gxe, "hipGraph empty");

  // ---- AQL
  {
    std::vector<char> hk((size_t)L * 64, 0);
    for (int l = 0; l < L; ++l) {
      float** ka = (float**)(hk.data() + (size_t)l * 64);
      ka[0] = buf + (l & 1) * R * C;
      ka[1] = buf + ((l + 1) & 1) * R * C;
    }
    CK(hipMemcpy(kargs, hk.data(), hk.size(), hipMemcpyHostToDevice));
  }
  auto run_aql = [&](Kern& k, int acq, int rel, int nrep) {
    hsa_signal_store_relaxed(sig, 1);
    const int n = nrep * L;
    uint64_t idx0 = hsa_queue_add_write_index_relaxed(q, n);
    for (int i = 0; i < n; ++i) {
      const int l = i % L;
      void* ka = (char*)kargs + (size_t)l * 64;
      auto* pk = (hsa_kernel_dispatch_packet_t*)q->base_address + ((idx0 + i) & (q->size - 1));
      pk->workgroup_size_x = 256; pk->workgroup_size_y = 1; pk->workgroup_size_z = 1; pk->reserved0 = 0;
      pk->grid_size_x = 256 * 256; pk->grid_size_y = 1; pk->grid_size_z = 1;
      pk->private_segment_size = k.pseg; pk->group_segment_size = k.gseg;
      pk->kernel_object = k.obj; pk->kernarg_address = ka; pk->reserved2 = 0;
      const bool first = i == 0, last = i == n - 1;
      pk->completion_signal = last ? sig : hsa_signal_t{0};
      const int a = first ? HSA_FENCE_SCOPE_SYSTEM : acq, r = last ? HSA_FENCE_SCOPE_SYSTEM : rel;
      const uint16_t hdr = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                           (a << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) | (r << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
      __atomic_store_n((uint32_t*)pk, (uint32_t)hdr | (1u << 16), __ATOMIC_RELEASE);
    }
    auto t0 = std::chrono::steady_clock::now();
    hsa_signal_store_screlease(q->doorbell_signal, idx0 + n - 1);
    while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 1000000000ull, HSA_WAIT_STATE_ACTIVE) >= 1) {
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 20) { printf("AQL timeout\n"); exit(3); }
    }
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  };
  const char* sc[] = {"none", "agent", "system"};
  struct Case { const char* k; int acq, rel; };
  Case cases[] = {{"one_0_0", 1, 1}, {"one_0_0", 2, 2}, {"one_0_0", 0, 1}, {"one_16_0", 0, 1}, {"one_0_0", 1, 0},
                  {"one_0_16", 1, 0}, {"one_16_16", 0, 0}, {"one_17_17", 0, 0}, {"one_0_0", 0, 0},
                  {"empty", 1, 1}, {"empty", 0, 0}};
  for (auto& c : cases) {
    Kern k = kern(c.k);
    int bad = 0;
    double md = 0;
    for (int rep = 0; rep < 5; ++rep) {
      reset();
      run_aql(k, c.acq, c.rel, 1);
      CK(hipMemcpy(got.data(), buf, got.size() * 4, hipMemcpyDeviceToHost));
      double d = 0;
      for (size_t i = 0; i < got.size(); ++i) d = fmax(d, fabs(got[i] - ref[i]));
      md = fmax(md, d);
      bad += d != 0;
    }
    run_aql(k, c.acq, c.rel, 2);
    const double us = run_aql(k, c.acq, c.rel, reps);
    printf("AQL %-10s acq %-6s rel %-6s %7.3f us per level | %s (max diff %.3g, %d/5 runs differ)\n", c.k, sc[c.acq], sc[c.rel],
           us / (reps * L), strcmp(c.k, "empty") ? (bad ? "STALE" : "exact") : "-", md, bad);
  }
  printf("done\n");
  return 0;
}
