// Host side of the MI355X off-policy update engine: device memory, the
// per-agent step programs (built as op DAGs), the level scheduler, hipGraph
// capture and the C ABI declared in include/rle.h.
//
// A step program is written in the reference's order (td7.py:287-332,
// td3.py:206-242, sac.py:251-295) as a list of ops with read/write resource
// sets.  `Prog::schedule` assigns every op the lowest dependency level that
// respects RAW, WAR and WAW hazards; each level becomes one launch of the
// device dispatch kernel, and the whole step is captured into a hipGraph.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "ops.h"
#include "rle.h"

namespace rle {
// next_ops / next_nops: descriptors of the level launched after this one (prefetched into
// every XCD's L2 during this level; 0: none)
// ext: the extended kernel instance (register-blocked / 32-row tiles, fused priority sampler)
hipError_t launch_level(const Op* d_ops, const Op* h_ops, int nops, int nwg, hipStream_t st,
                        unsigned long long* trace = nullptr, const Op* next_ops = nullptr, int next_nops = 0,
                        int ks = KS_EXT);
int level_capacity();
int trace_stride();
extern std::vector<LevelLaunch>* g_level_rec;
const char* level_kernel_symbol(int ks);
hipError_t launch_append(float* state, float* next_state, float* action, float* reward, float* notdone,
                         float* priority, const float* st_s, const float* st_ns, const float* st_a,
                         const float* st_r, const float* st_d, long long ptr, long long cap, int count,
                         int Sp, int Ap, const float* max_priority, int lap, double* bsum, double* ssum,
                         long long size_before, hipStream_t st);
hipError_t launch_act_chain(const ActChainArgs& a, hipStream_t st);
hipError_t launch_fill(float* state, float* next_state, float* action, float* reward, float* notdone,
                       float* priority, long long n, int S, int Sp, int A, int Ap, unsigned long long seed,
                       hipStream_t st);

static thread_local std::string g_err;

struct Error {
  int code;
  std::string msg;
};

#define HIPCHK(x)                                                                               \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) throw Error{RLE_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)}; \
  } while (0)
#define REQUIRE(c, m)                              \
  do {                                                \
    if (!(c)) throw Error{RLE_EINVAL, std::string(m)}; \
  } while (0)

static inline int r4(int x) { return (x + 3) & ~3; }
static inline int r16(int x) { return (x + 15) & ~15; }
static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

static int host_fkey(float f) {
  int i;
  std::memcpy(&i, &f, 4);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
static float host_unkey(int k) {
  int i = k >= 0 ? k : k ^ 0x7FFFFFFF;
  float f;
  std::memcpy(&f, &i, 4);
  return f;
}

// Live device allocations (address -> bytes) for the RLE_AUDIT=1 operand-range check and the
// RLE_HAZARD=1 level check.  Engines and replays on other host threads allocate concurrently
// (ctypes drops the GIL), so every access holds live_mu().
static std::map<uintptr_t, size_t>& live_allocs() {
  static std::map<uintptr_t, size_t> m;
  return m;
}
static std::mutex& live_mu() {
  static std::mutex mu;
  return mu;
}

// Zero-filled device buffers.  Small ones (< 1 MB: step scratch, vectors, op tables, ...) are
// carved out of 32 MB slabs that are zeroed once, each rounded up to a whole page plus a guard
// page (as a hipMalloc of its own would be padded), so an engine's thousands of buffers cost a
// few hipMalloc / hipMemset calls instead of one synchronised pair each.
struct DevMem {
  static constexpr size_t kSlab = 32u << 20, kSmall = 1u << 20, kPage = 4096;
  std::vector<std::pair<void*, size_t>> ptrs;  // hipMalloc'd blocks (slabs and large buffers)
  char* slab = nullptr;
  size_t slab_used = 0;
  void* fresh(size_t bytes) {
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, bytes));
    HIPCHK(hipMemset(p, 0, bytes));
    // hipMemset runs on the null stream, which does not order against our
    // non-blocking streams: finish it before any stream touches the buffer.
    HIPCHK(hipDeviceSynchronize());
    ptrs.emplace_back(p, bytes);
    return p;
  }
  void* alloc(size_t bytes) {
    if (bytes == 0) bytes = 16;
    void* p;
    if (bytes >= kSmall) {
      p = fresh(bytes);
    } else {
      const size_t need = (bytes + kPage - 1) / kPage * kPage + kPage;
      if (!slab || slab_used + need > kSlab) {
        slab = static_cast<char*>(fresh(kSlab));
        slab_used = 0;
      }
      p = slab + slab_used;
      slab_used += need;
    }
    {
      std::lock_guard<std::mutex> lk(live_mu());
      live_allocs()[(uintptr_t)p] = bytes;
    }
    return p;
  }
  template <class T>
  T* make(size_t n) {
    return reinterpret_cast<T*>(alloc(n * sizeof(T)));
  }
  ~DevMem() {
    std::lock_guard<std::mutex> lk(live_mu());
    for (auto& [p, bytes] : ptrs) {
      auto& m = live_allocs();  // the block's buffers (a large buffer, or a slab's carved ones)
      const uintptr_t lo = (uintptr_t)p, hi = lo + bytes;
      for (auto it = m.lower_bound(lo); it != m.end() && it->first < hi;) it = m.erase(it);
      (void)hipFree(p);
    }
  }
};

// Pinned host allocations (coherent, mapped into the device's address space): act-call
// staging and the zero-copy action output.
struct PinMem {
  std::vector<void*> ptrs;
  void* alloc(size_t bytes) {
    void* p = nullptr;
    HIPCHK(hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(p, 0, bytes);
    ptrs.push_back(p);
    std::lock_guard<std::mutex> lk(live_mu());
    live_allocs()[(uintptr_t)p] = bytes;
    return p;
  }
  ~PinMem() {
    std::lock_guard<std::mutex> lk(live_mu());
    for (void* p : ptrs) {
      live_allocs().erase((uintptr_t)p);
      (void)hipHostFree(p);
    }
  }
};

// Named device buffers reused across calls (grown on demand, never shrunk): the replay's eager
// entry points (sample_indices, update_priority, ...) allocate once instead of per call.
struct Scratch {
  DevMem mem;
  std::map<std::string, std::pair<void*, size_t>> bufs;
  template <class T>
  T* get(const std::string& name, size_t n) {
    const size_t bytes = std::max<size_t>(n * sizeof(T), 16);
    auto& b = bufs[name];
    if (b.second < bytes) {
      b.first = mem.alloc(bytes);
      b.second = bytes;
    }
    return static_cast<T*>(b.first);
  }
};

// ------------------------------------------------------------------ replay

struct Engine;

struct Replay {
  int device;
  long long cap;
  int S, Sp, A, Ap, lap;
  long long ptr = 0, size = 0;
  float *state, *next_state, *action, *reward, *notdone, *priority;
  long long* size_d;
  float* maxp_d;
  double* bsum;
  double* ssum;  // LAP sub-block sums (64 priorities each), nblk * 64
  int nblk;
  float* maxred_part;
  int maxred_nwg = 256;
  hipStream_t stream = nullptr;
  DevMem mem;
  Scratch scratch;  // eager entry points' temporaries
  // append staging
  float* stage = nullptr;
  long long stage_rows = 0;
  // bumped by every change of what sampling draws from (appends, priority writes):
  // an engine's batch prefetched under another version is stale
  unsigned long long version = 0;
  // engines bound to this replay, each with an event recorded on its stream after every
  // enqueued step: replay operations on `stream` wait for them first (an append after
  // rle_step_async must not race the step's priority scatter and block sums)
  std::vector<std::pair<Engine*, hipEvent_t>> users;
  void wait_users();   // (after Engine: also drains the users' direct-dispatch bursts)
  void drain_users();  // the users' rle_step_async bursts on their own queues retired (host wait)
};

// ------------------------------------------------------------------ programs

// A tensor of the step program: fragment images (ops.h "tensor images") for
// anything a GEMM touches, or a plain vector for 1-column tensors outside GEMMs.
struct View {
  Mat m{};                      // images (m.n / m.t may be null)
  float* p = nullptr;           // plain vector data (1-column tensors), else null
  int rows = 0, cols = 0;       // rows (16-multiple for images), padded columns
  int id = -1;
  const float* norm = nullptr;  // AvgL1Norm partials (producer |x| column-tile sums)
  int norm_ld = 0, norm_row0 = 0, nparts = 0, width = 0, norm_id = -1;
  // EPI_NBDOT output (the gradient g of an AvgL1Norm output whose backward is deferred
  // into the consuming DW, kDwNb): row partials of sum_j g x
  const float* nbdot = nullptr;
  int nbdot_ld = 0, nbdot_n = 0, nbdot_id = -1;
  // EPI_QDOT output: row partials [qd_n][qd_ld] of sum_j y_j w_j (a critic's q before its bias)
  const float* qd = nullptr;
  int qd_ld = 0, qd_n = 0, qd_id = -1;
  View sub(int r0, int n) const {
    View v = *this;
    if (m.n || m.t) {
      if (r0 % 16) throw Error{RLE_EINVAL, "sub-view of an image must start at a 16-row boundary"};
      if (m.n) v.m.n = m.n + (size_t)(r0 / 16) * m.cbn * 256;
      if (m.t) v.m.t = m.t + (size_t)(r0 / 16) * 256;
    }
    if (p) v.p = p + r0;
    v.rows = n;
    v.norm_row0 += r0;
    return v;
  }
  NormRef nref() const {
    NormRef r{};
    if (norm) {
      r.part = norm;
      r.ld = norm_ld;
      r.row0 = norm_row0;
      r.nparts = nparts;
      r.width = width;
    }
    return r;
  }
};

// GEMM tile width: the narrowest tile (more workgroups, reduction split across the
// 4 waves) while the output has at most 640 16x16 blocks per width step.
static int pick_tn(int M, int N) {
  const int blocks = cdiv(M, 16) * cdiv(N, 16);
  if (blocks <= 640) return 16;
  if (blocks <= 1280) return 32;
  return 64;
}

// Layout invariants the GEMM main loop relies on (kernels.hip, "GEMM"): reduction
// segments 16-aligned, sorted and disjoint; every segment of a FWD/DX operand
// and of a DW A operand spans the whole operand row range (x0 == 0); DW B
// segments split the columns at 16-aligned bounds and share one reduction range.
static void check_gemm(const GemmArgs& g) {
  auto chk = [&](const Operand& o, bool xsplit, int xn) {
    REQUIRE(o.nseg >= 1 && o.nseg <= kMaxSeg, "gemm: bad segment count");
    for (int q = 0; q < o.nseg; ++q) {
      const Seg& s = o.seg[q];
      REQUIRE(s.p != nullptr && s.r0 % 16 == 0 && s.r1 > s.r0, "gemm: bad reduction segment");
      if (!xsplit) {
        REQUIRE(s.x0 == 0 && s.x1 >= xn, "gemm: segment must span the operand rows");
        if (q) REQUIRE(s.r0 == r16(o.seg[q - 1].r1), "gemm: reduction segments must be back to back");
      } else {
        REQUIRE(s.x0 % 16 == 0 && s.x1 % 16 == 0 && s.r0 == o.seg[0].r0 && s.r1 == o.seg[0].r1,
                "gemm: bad column split");
      }
    }
  };
  chk(g.A, false, g.M);
  chk(g.B, g.mode == GEMM_DW, g.N);
  if (g.mode == GEMM_DX || (g.mode == GEMM_FWD && g.B.nseg > 1)) {  // W segment q pairs with A segment q
    REQUIRE(g.B.nseg == g.A.nseg, "gemm: one W segment per A segment");
    for (int q = 0; q < g.A.nseg; ++q)
      REQUIRE(g.B.seg[q].r0 == g.A.seg[q].r0 && g.B.seg[q].r1 == g.A.seg[q].r1, "gemm: W / A segment mismatch");
  }
  REQUIRE(g.R <= 16 * 1024, "gemm: reduction too long");
}

static void xcd_plan(GemmArgs& g, bool xcd);

// (ks < 0: in any kernel set)
static bool gemm_variant_compiled(int vid, int ks = -1) {
#define RLE_VID(mode, epi, act, norm, pre, pk, sets) \
  (vid == gemm_vid(mode, epi, act, norm, pre) && (ks < 0 || ks == KS_EXT || (((sets) >> ks_family(ks)) & 1))) ||
  return RLE_GEMM_VARIANTS(RLE_VID) false;
#undef RLE_VID
}

// Device-side dispatch fields of a GEMM op: compiled variant, split count, tile-row
// reciprocal (kernels.hip gemm_v).
static void gemm_finalize(GemmArgs& g, bool xcd = true) {
  int norm = 0;
  for (int q = 0; q < g.A.nseg; ++q) norm |= g.A.seg[q].norm.part != nullptr;
  for (int q = 0; q < g.B.nseg; ++q) norm |= g.B.seg[q].norm.part != nullptr;
  const int act = g.mode == GEMM_FWD ? g.act : (g.mode == GEMM_DX ? g.dact : g.act);
  REQUIRE(g.mode != GEMM_DX || !norm, "gemm: no DX variant with normed operands");
  REQUIRE(g.mode != GEMM_DW || g.epi == EPI_ADAM, "gemm: DW is always fused with Adam");
  REQUIRE(g.mode != GEMM_DW || act == ACT_NONE || (act == kDwNb && !norm && g.nbx.t && g.nbm.part && g.nbdot &&
                                                   g.R <= 1024),
          "gemm: deferred AvgL1Norm backward operands");
  REQUIRE(g.epi != EPI_NBDOT || (g.mode == GEMM_DX && act == ACT_NONE && g.nbx.t && g.norm_out),
          "gemm: EPI_NBDOT is a plain DX with x and partials");
  REQUIRE(g.epi != EPI_MSE || act == ACT_NONE, "gemm: MSE epilogue takes no activation");
  REQUIRE((g.dact == ACT_NONE) == (g.dsrc.t == nullptr) || g.mode != GEMM_DX, "gemm: DX derivative source");
  REQUIRE(g.has_pre != 1 || ((g.mode == GEMM_FWD || g.mode == GEMM_DX) && g.prea.N <= 32 && g.prea.seg < g.A.nseg &&
                               g.A.seg[g.prea.seg].r1 - g.A.seg[g.prea.seg].r0 <= 32 && g.prea.mode == g.mode &&
                               g.prea.R % 16 == 0),
          "gemm: pre-GEMM layout");
  {  // the fused head (kernels.hip headdx_reduce): q of every twin from EPI_QDOT partials
    const HeadArgs& h = g.hd;
    const bool pol = h.mode == HEAD_MLP_POLICY;
    const bool modes = (h.mode == HEAD_TD7_LOSS && h.tgt_mode == HEAD_TD7_TARGET && h.vt && h.vmax_key && h.vmin_key) ||
                       (h.mode == HEAD_MLP_LOSS && h.tgt_mode == HEAD_MLP_TARGET && !h.vt) ||
                       (pol && h.tgt_mode < 0 && !h.lap && h.tp_n[0] == 0 && h.tp_n[1] == 0);
    const bool parts = h.qp[0] && h.qp[1] && h.qp_n[0] <= 64 && h.qp_n[1] <= 64 &&
                       (pol || (h.tp[0] && h.tp[1] && h.tp_n[0] <= 64 && h.tp_n[1] <= 64));
    REQUIRE(g.has_pre != 2 || (g.mode == GEMM_DX && g.epi == EPI_STORE && (act == ACT_ELU || act == ACT_RELU) &&
                               !norm && g.A.nseg == 1 && modes && parts && h.dact == act && (!h.sac || h.logpi) &&
                               (!h.lap || h.prio) && h.H <= 256 && h.H % 4 == 0 && g.R == r16(h.H) &&
                               g.M % 16 == 0 && h.rows == h.nvalid && h.rows <= g.M && g.M - h.rows < 16 &&
                               (g.head_n == 0 || g.head_n == 1)),
            "gemm: fused loss head layout");
  }
  REQUIRE(g.epi != EPI_SACFWD || (g.mode == GEMM_FWD && act == ACT_NONE && !norm && g.has_pre == 0 && g.tn == 64 &&
                                   g.tiles_n == 1 && g.sf.A <= 32 && g.sf.ls_off + g.sf.A <= g.N && g.sf.eps.t &&
                                   g.sf.eps2.t && (g.sf.act.n || g.sf.act.t) && g.sf.logpi),
          "gemm: SAC actor forward epilogue operands");
  REQUIRE(g.epi != EPI_SACBWD || (g.mode == GEMM_DX && act == ACT_NONE && !norm && g.has_pre == 0 && g.sb.raw.t &&
                                   g.sb.eps2.t && (g.sb.dout.n || g.sb.dout.t) && g.sb.log_alpha &&
                                   g.sb.ls_off >= g.sb.mean_off + g.N),
          "gemm: SAC actor backward epilogue operands");
  REQUIRE((g.has_pre != 3 && g.has_pre != 4) || (((g.mode == GEMM_FWD && (g.epi == EPI_STORE || g.epi == EPI_QDOT) && g.prea.bias) ||
                                (g.mode == GEMM_DX && g.epi == EPI_STORE && g.prea.dsrc.t)) &&
                               act == ACT_RELU && !norm && g.A.nseg == 1 && g.prea.seg == 0 && g.prea.mode == g.mode &&
                               g.prea.act == ACT_RELU && g.prea.N == g.A.seg[0].r1 - g.A.seg[0].r0 && g.prea.N <= 256 &&
                               g.prea.N % 16 == 0 && g.prea.R % 16 == 0 && g.prea.R <= 48 && g.prea.B.nseg == 1 &&
                               g.R == g.prea.N &&  // (<= 16 chunks per wave: kernels.hip PK 3 holds them all)
                               !g.pre.t && g.B.nseg == 1),
          "gemm: pre-layer layout");
  {  // has_pre 4: the pre-layer's input segment prea2.seg from the pre-GEMM prea2 (kernels.hip PK 4: its
     // output, at most 2 column blocks, in LDS; FWD with target smoothing, as pre_actor_fwd builds it)
    const PreArgs& q = g.prea2;
    REQUIRE(g.has_pre != 4 || (g.mode == GEMM_FWD && g.epi == EPI_QDOT && q.mode == GEMM_FWD && q.N <= 32 &&
                               q.R % 16 == 0 && q.R <= 16 * 1024 && q.A.nseg == 1 && q.B.nseg == 1 &&
                               q.seg == 1 && g.prea.A.nseg == 2 && g.prea.A.seg[0].r0 == 0 &&
                               g.prea.A.seg[q.seg].r1 - g.prea.A.seg[q.seg].r0 <= 16 &&
                               g.prea.A.seg[q.seg].r0 % 16 == 0),
            "gemm: two-stage pre-layer layout");
  }
  {  // has_pre 5: SAC's raw head + rsample (kernels.hip sacraw_*, PK 5) as segment prea.seg of a ReLU forward
    const PreArgs& q = g.prea;
    REQUIRE(g.has_pre != 5 || (g.mode == GEMM_FWD && g.epi == EPI_STORE && act == ACT_RELU && !norm &&
                               q.mode == GEMM_FWD && q.A.nseg == 1 && q.B.nseg == 1 && q.sac_a >= 1 &&
                               q.N == 2 * q.sac_a && q.N <= 48 && q.R % 16 == 0 && q.R <= 256 && q.bias &&
                               q.noise.t && q.seg < g.A.nseg && g.A.seg[q.seg].r1 - g.A.seg[q.seg].r0 <= 32 &&
                               g.A.seg[q.seg].r1 - g.A.seg[q.seg].r0 >= q.sac_a),
            "gemm: SAC pre-GEMM layout");
  }
  REQUIRE(g.epi != EPI_SACFWD || (g.R <= 256 && g.N <= 48 && g.A.nseg == 1 && g.B.nseg == 1),
          "gemm: SAC raw head (kernels.hip sacraw_*: three column blocks, R <= 256)");
  REQUIRE(g.has_pre >= 0 && g.has_pre <= 5, "gemm: pre kind");
  // (has_pre 4 takes the pre-layer's id with the norm bit, which no pre-layer variant uses; has_pre 5 a
  // pre-GEMM id with the norm bit on a ReLU forward, which no pre-GEMM consumer has)
  g.vid = g.has_pre == 4   ? gemm_vid(g.mode, g.epi, act, 1, 3)
          : g.has_pre == 5 ? gemm_vid(g.mode, g.epi, act, 1, 1)
                           : gemm_vid(g.mode, g.epi, act, norm, g.has_pre);
  REQUIRE(gemm_variant_compiled(g.vid), "gemm: no compiled variant for this mode / epilogue / activation / norm / pre "
                                        "(ops.h RLE_GEMM_VARIANTS)");
  REQUIRE(g.tn == 16 || g.tn == 32 || g.tn == 64, "gemm: tile width");
  g.ks_log = g.tn == 16 ? 2 : (g.tn == 32 ? 1 : 0);
  REQUIRE(g.R % 16 == 0, "gemm: reduction length must be a multiple of 16");
  REQUIRE((long long)g.tiles_m * g.tiles_n < 65536, "gemm: too many tiles");
  // 64-row LDS-staged tiles (kernels.hip gemm_wide): one of its variants, 64-wide tiles over whole 64-row blocks,
  // no in-tile prologue, no target smoothing; tiles_m stays the 16-row block count (loss partial slots)
  REQUIRE(!g.hot.wide || (wide_variant(g.mode, g.epi, g.has_pre) && (g.tn == 64 || g.tn == 32) &&
                          g.hot.wide == g.tn && g.M % 64 == 0 && g.tiles_m * 16 == g.M && !g.noise.t &&
                          g.N % g.tn == 0),
          "gemm: wide tile layout");
  g.inv_tiles_n = 1.f / (float)g.tiles_n;
  GemmHot& h = g.hot;
  h.ks_log = g.ks_log;
  h.tiles_n = g.tiles_n;
  h.tn = g.tn;
  h.N = g.N;
  h.R = g.R;
  h.inv_tiles_n = g.inv_tiles_n;
  h.bias_col = g.epi == EPI_ADAM ? g.adam.bias_col : 0;
  h.nseg_a = g.A.nseg;
  h.nseg_b = g.B.nseg;
  h.a0xs = g.A.seg[0].xs;
  h.a0r0 = g.A.seg[0].r0;
  h.a0r1 = g.A.seg[0].r1;
  h.b0xs = g.B.seg[0].xs;
  h.a0p = g.A.seg[0].p;
  h.b0p = g.B.seg[0].p;
  h.bias = g.epi == EPI_ADAM ? nullptr : g.bias;
  h.tiles = (g.hot.wide ? g.tiles_m / 4 : g.tiles_m) * g.tiles_n;
  xcd_plan(g, xcd);
}

// XCD-aware tile order of a GEMM (GemmHot::xb): each of the 8 XCDs takes ~tiles/8 tiles as
// a band-ordered run.  Band width b (in tiles) minimises the operand blocks one XCD reads:
// ceil(share / b) A row-blocks of 16 rows plus b B column-blocks of tn columns (both x R).
// rle_plan.xcd 0 keeps the plain row-major tile order.
static void xcd_plan(GemmArgs& g, bool xcd) {
  GemmHot& h = g.hot;
  h.xb = 0;
  if (!xcd) return;
  const int tm = g.hot.wide ? g.tiles_m / 4 : g.tiles_m, rh = g.hot.wide ? 64 : 16;  // tile rows, rows per tile
  const int T = tm * g.tiles_n;
  if (T < 16 || g.tiles_n < 2) return;
  const int share = (T + 7) / 8;
  int best = g.tiles_n;
  long long bc = -1;
  for (int b = 1; b <= g.tiles_n; ++b) {
    const long long rows = std::min<long long>(tm, (share + b - 1) / b + 1);  // a run may straddle a row
    const long long cost = rows * rh + (long long)std::min(b, share) * g.tn;
    if (bc < 0 || cost < bc) {
      bc = cost;
      best = b;
    }
  }
  h.xb = best;
  h.tmb = tm * best;
  h.nfull = g.tiles_n / best;
  h.inv_tmb = 1.f / (float)h.tmb;
  h.inv_xb = 1.f / (float)best;
  const int blast = g.tiles_n - h.nfull * best;
  h.inv_blast = blast ? 1.f / (float)blast : 0.f;
  std::vector<char> seen((size_t)T, 0);  // the order must be a permutation of the tiles
  for (int t = 0; t < T; ++t) {
    int it, jt;
    xcd_tile(t, T, g.tiles_n, h.xb, h.tmb, h.nfull, h.inv_tmb, h.inv_xb, h.inv_blast, it, jt);
    const bool ok = it >= 0 && it < tm && jt >= 0 && jt < g.tiles_n && !seen[(size_t)it * g.tiles_n + jt];
    if (!ok) {
      h.xb = 0;
      return;
    }
    seen[(size_t)it * g.tiles_n + jt] = 1;
  }
}


// ---- RLE_AUDIT=1: every byte range a GEMM op's workgroups can touch (the address arithmetic of
// kernels.hip gemm_v / pre_issue / pre_finish, replayed on the host) must lie inside one live
// device allocation.  A debugging aid for new tile layouts; off in production.
// RLE_HAZARD=1 reuses the same address replay to collect each op's byte ranges (Access) instead
// of checking them against the allocations: see level_hazards().
struct Access {
  uintptr_t lo, hi;
  int w;  // 1: the op stores (or atomically updates) these bytes
  const char* what;
  int t = -1;  // (GEMM ranges) the op's workgroup that touches them; -1: the op as a whole
};
static thread_local std::vector<Access>* g_sink = nullptr;
static thread_local int g_tile = -1;  // (audit_gemm: the workgroup whose ranges g_sink receives)

static void audit_range(const void* base, long long lo, long long bytes, const char* what, const GemmArgs& g,
                        int w = 0) {
  if (bytes <= 0) return;
  const uintptr_t a = (uintptr_t)base + (uintptr_t)lo, b = a + (uintptr_t)bytes;
  if (g_sink) {
    g_sink->push_back({a, b, w, what, g_tile});
    return;
  }
  std::lock_guard<std::mutex> lk(live_mu());
  auto& m = live_allocs();
  auto it = m.upper_bound(a);
  bool ok = base != nullptr && lo >= 0 && it != m.begin();
  if (ok) {
    --it;
    ok = a >= it->first && b <= it->first + it->second;
  }
  if (!ok) {
    char msg[256];
    snprintf(msg, sizeof msg, "audit: %s [%lld, +%lld) outside its allocation (gemm mode %d epi %d M %d N %d R %d tn %d)",
             what, lo, bytes, g.mode, g.epi, g.M, g.N, g.R, g.tn);
    throw Error{RLE_EINVAL, msg};
  }
}

static long long h_nblk(int cbn, int r, int c) { return ((long long)(r >> 4) * cbn + (c >> 4)) * 1024; }  // bytes
static long long h_tblk(int rbs, int r, int c) { return ((long long)(c >> 4) * rbs + (r >> 4)) * 1024; }

static void audit_mat(const Mat& m, int r, int c, const char* what, const GemmArgs& g, bool need_n = false,
                      bool need_t = false, int w = 0) {
  if (m.n) audit_range(m.n, h_nblk(m.cbn, r, c), 1024, what, g, w);
  if (m.t) audit_range(m.t, h_tblk(m.rbs, r, c), 1024, what, g, w);
  if (need_n && !m.n) throw Error{RLE_EINVAL, std::string("audit: no N image for ") + what};
  if (need_t && !m.t) throw Error{RLE_EINVAL, std::string("audit: no T image for ") + what};
}

static void audit_norm(const NormRef& nr, int row, int nrows, const GemmArgs& g) {
  if (!nr.part) return;
  for (int p = 0; p < nr.nparts; ++p)
    audit_range(nr.part, ((long long)p * nr.ld + nr.row0 + row) * 4, (long long)nrows * 4, "norm partials", g);
}

static void audit_gemm(const GemmArgs& g0) {
  // (a 64-row tile, kernels.hip gemm_wide: the byte ranges of the four 16-row tn-64 tiles it covers, in row-major
  // order -- its loss partial slots are theirs)
  GemmArgs gw;
  if (g0.hot.wide) {
    gw = g0;
    gw.hot.wide = 0;
    gw.hot.xb = 0;
    gw.hot.tiles = gw.tiles_m * gw.tiles_n;
    gw.ks_log = 0;
  }
  const GemmArgs& g = g0.hot.wide ? gw : g0;
  const GemmHot& h = g.hot;
  // wave w of a 16 x tn tile: column group w >> ks_log, reduction split w & (2^ks_log - 1)
  const int NB = g.tn / 16, T = g.tiles_m * g.tiles_n, ks = 1 << g.ks_log;
  const int nch = g.R / 16, per = (nch + ks - 1) / ks;
  for (int t = 0; t < T; ++t) {
    g_tile = g0.hot.wide ? -1 : t;
    int it, jt;
    if (h.xb) xcd_tile(t, h.tiles, h.tiles_n, h.xb, h.tmb, h.nfull, h.inv_tmb, h.inv_xb, h.inv_blast, it, jt);
    else {
      it = (int)(((float)t + 0.5f) * g.inv_tiles_n);
      jt = t - it * g.tiles_n;
    }
    const int i0 = it * 16, jt0 = jt * g.tn;
    const int bias_col = g.epi == EPI_ADAM ? g.adam.bias_col : 0;
    const bool bias_tile = g.epi == EPI_ADAM && jt0 >= bias_col;
    bool on[4];
    for (int cb = 0; cb < NB; ++cb) on[cb] = bias_tile ? cb == 0 : jt0 + cb * 16 < g.N;
    for (int w = 0; w < 4; ++w) {
      const int cgw = w >> g.ks_log;
      const int c0 = (w & (ks - 1)) * per, c1 = std::min(nch, c0 + per);
      bool mine[4] = {false, false, false, false};  // the wave's column block
      if (cgw < NB) mine[cgw] = on[cgw];
      if (g.mode != GEMM_DW) {
        const bool wabs = g.mode == GEMM_FWD && g.B.nseg == 1;
        for (int q = 0; q < g.A.nseg; ++q) {
          const Seg& sa = g.A.seg[q];
          const Seg& sb = g.B.seg[wabs ? 0 : q];
          const int s0 = sa.r0 / 16, k0 = std::max(c0, s0), k1 = std::min(c1, (sa.r1 + 15) / 16);
          if (k0 >= k1) continue;
          const int kb = wabs ? k0 : k0 - s0;
          if (!mine[0] && !mine[1] && !mine[2] && !mine[3]) continue;  // inactive wave: no loads
          if (!((g.has_pre == 1 || g.has_pre >= 3) && q == g.prea.seg)) {
            audit_range(sa.p, ((long long)(i0 / 16) * sa.xs + (k0 - s0)) * 1024, (long long)(k1 - k0) * 1024, "A", g);
            if (sa.norm.part) audit_norm(sa.norm, i0, 16, g);
          }
          for (int cb = 0; cb < NB; ++cb)
            if (mine[cb])
              audit_range(sb.p, ((long long)(jt0 / 16 + cb) * sb.xs + kb) * 1024, (long long)(k1 - k0) * 1024, "B", g);
        }
        // pre-GEMM operands (pre_issue / pre_finish): 16 rows at i0, both column blocks (has_pre 2,
        // the fused loss head, keeps HeadArgs in the same union: its reads are not audited here)
        if (g.has_pre == 3 || g.has_pre == 4) {  // pre-layer (prelayer_*): every A chunk, the wave's 4 W column
                                                 // blocks, bias (has_pre 4: segment prea2.seg from LDS)
          const PreArgs& p = g.prea;
          for (int k = 0; k < p.R / 16; ++k) {
            int q = 0;
            for (int u = 1; u < p.A.nseg; ++u)
              if (k >= p.A.seg[u].r0 / 16) q = u;
            const Seg& sa = p.A.seg[q];
            if (!(g.has_pre == 4 && q == g.prea2.seg))
              audit_range(sa.p, ((long long)(i0 / 16) * sa.xs + (k - sa.r0 / 16)) * 1024, 1024, "prelayer A", g);
            for (int c = 0; c < 4; ++c)
              if ((w * 4 + c) * 16 < p.N)
                audit_range(p.B.seg[0].p, ((long long)(w * 4 + c) * p.B.seg[0].xs + k) * 1024, 1024, "prelayer W", g);
          }
          for (int c = 0; c < 4; ++c)
            if ((w * 4 + c) * 16 < p.N) {
              if (p.mode == GEMM_FWD)
                audit_range(p.bias, (long long)(w * 4 + c) * 64, (long long)std::min(16, p.N - (w * 4 + c) * 16) * 4,
                            "prelayer bias", g);
              else
                audit_range(p.dsrc.t, h_tblk(p.dsrc.rbs, i0, (w * 4 + c) * 16), 1024, "prelayer dsrc", g);
            }
        }
        if (g.has_pre == 5) {  // sacraw_issue: the wave's 4 chunks of A and of the 3 W column blocks; bias, noise
          const PreArgs& p = g.prea;
          const int nchp = p.R / 16, k0 = std::min(nchp, w * 4), k1 = std::min(nchp, w * 4 + 4);
          if (k1 > k0) {
            const Seg& sa = p.A.seg[0];
            audit_range(sa.p, ((long long)(i0 / 16) * sa.xs + k0) * 1024, (long long)(k1 - k0) * 1024, "sacpre A", g);
            for (int c = 0; c < 3; ++c)
              audit_range(p.B.seg[0].p, ((long long)c * p.B.seg[0].xs + k0) * 1024, (long long)(k1 - k0) * 1024,
                          "sacpre W", g);
          }
          audit_range(p.bias, 0, (long long)p.N * 4, "sacpre bias", g);
          for (int c = 0; c < p.sac_a; c += 16) audit_range(p.noise.t, h_tblk(p.noise.rbs, i0, c), 1024, "sacpre eps", g);
        }
        if (g.has_pre == 1 || g.has_pre == 4) {
          const PreArgs& p = g.has_pre == 4 ? g.prea2 : g.prea;
          const int nchp = p.R / 16, perp = (nchp + 3) / 4;
          const int c0p = w * perp, c1p = std::min(nchp, c0p + perp);
          const bool wp = p.mode == GEMM_FWD && p.B.nseg == 1;
          for (int q = 0; q < p.A.nseg; ++q) {
            const Seg& sa = p.A.seg[q];
            const Seg& sb = p.B.seg[wp ? 0 : q];
            const int s0 = sa.r0 / 16, k0 = std::max(c0p, s0), k1 = std::min(c1p, (sa.r1 + 15) / 16);
            if (k0 >= k1) continue;
            const int kb = wp ? k0 : k0 - s0;
            audit_range(sa.p, ((long long)(i0 / 16) * sa.xs + (k0 - s0)) * 1024, (long long)(k1 - k0) * 1024, "pre A", g);
            audit_range(sb.p, (long long)kb * 1024, (long long)(k1 - k0) * 1024, "pre B", g);
            if (p.N > 16) audit_range(sb.p, ((long long)sb.xs + kb) * 1024, (long long)(k1 - k0) * 1024, "pre B1", g);
          }
          if (w == 0) {
            for (int cb = 0; cb < 2 && cb * 16 < p.N; ++cb) {
              if (p.mode == GEMM_FWD) {
                if (p.bias) audit_range(p.bias, cb * 64, (long long)std::min(16, p.N - cb * 16) * 4, "pre bias", g);
                if (p.noise.t) audit_range(p.noise.t, h_tblk(p.noise.rbs, i0, cb * 16), 1024, "pre noise", g);
              } else {
                audit_range(p.dsrc.t, h_tblk(p.dsrc.rbs, i0, cb * 16), 1024, "pre dsrc", g);
              }
            }
          }
        }
      } else {
        const int nrun = c1 > c0 ? c1 - c0 : 0;
        if (!nrun || !(mine[0] || mine[1] || mine[2] || mine[3])) continue;
        audit_range(h.a0p, ((long long)(i0 / 16) * h.a0xs + c0) * 1024, (long long)nrun * 1024, "DW A", g);
        if (g.act == kDwNb || (g.nbx.t && g.nbm.part))
          audit_range(g.nbx.t, ((long long)(i0 / 16) * g.nbx_xs + c0) * 1024, (long long)nrun * 1024, "DW x", g);
        if (bias_tile) continue;
        for (int cb = 0; cb < NB; ++cb) {
          if (!mine[cb]) continue;
          const int xq = jt0 + cb * 16;
          int qb = 0;
          for (int q = 1; q < g.B.nseg; ++q)
            if (xq >= g.B.seg[q].x0) qb = q;
          const Seg& sb = g.B.seg[qb];
          audit_range(sb.p, ((long long)((xq - sb.x0) / 16) * sb.xs + c0) * 1024, (long long)nrun * 1024, "DW B", g);
        }
      }
    }
    if (g.mode == GEMM_DW)
      for (int q = 0; q < g.B.nseg; ++q)
        if (g.B.seg[q].norm.part) audit_norm(g.B.seg[q].norm, 0, g.B.seg[q].r1 - g.B.seg[q].r0, g);
    // epilogue: column block w of the tile, rows i0..i0+15
    for (int w = 0; w < NB; ++w) {
      const int j0 = jt0 + w * 16;
      const bool active = bias_tile ? w == 0 : j0 < g.N;
      if (!active) continue;
      const int ncol = bias_tile ? 1 : std::min(16, g.N - j0);
      switch (g.epi) {
        case EPI_ADAM: {
          const AdamArgs& ad = g.adam;
          if (bias_tile) {
            for (long long o : {0LL, ad.mo, ad.vo}) audit_range(ad.b, (o + i0) * 4, 64, "adam bias", g, 1);
          } else {
            for (long long o : {0LL, ad.mo, ad.vo})
              audit_range(ad.w.t, o * 4 + h_tblk(ad.w.rbs, i0, j0), 1024, "adam w.t", g, 1);
            audit_range(ad.w.n, h_nblk(ad.w.cbn, i0, j0), 1024, "adam w.n", g, 1);
          }
          if (ad.gsq) {
            if (bias_tile) audit_range(ad.gsq_b, (long long)it * 4, 4, "gsq_b", g, 1);
            else audit_range(ad.gsq, ((long long)it * (g.tiles_n - 1) + jt) * 4, 4, "gsq", g, 1);
          }
          break;
        }
        default: {
          audit_mat(g.out, i0, j0, "out", g, false, false, 1);
          if (g.bias) audit_range(g.bias, (long long)j0 * 4, (long long)ncol * 4, "bias", g);
          if (g.mode == GEMM_FWD && g.pre.t) audit_mat(g.pre, i0, j0, "pre-act", g, false, false, 1);
          if (g.mode == GEMM_DX && g.dact != ACT_NONE) audit_mat(g.dsrc, i0, j0, "dsrc", g, false, true);
          if (g.noise.t && i0 + 15 >= g.noise_row0) {
            const int r0 = std::max(i0, g.noise_row0) - g.noise_row0;
            audit_range(g.noise.t, h_tblk(g.noise.rbs, r0, j0), 1024, "noise", g);
            audit_range(g.noise.t, h_tblk(g.noise.rbs, i0 + 15 - g.noise_row0, j0), 1024, "noise", g);
          }
          if (g.epi == EPI_NBDOT) audit_mat(g.nbx, i0, j0, "nbx", g, false, true);
          if (g.epi == EPI_SACFWD && w == 0) {  // the tile's rows: noise, action, log pi
            const SacFwdArgs& sf = g.sf;
            for (int c : {0, sf.A - 1}) {
              if (i0 < sf.eps_row_split) audit_mat(sf.eps2, i0, c, "sac eps2", g, false, true);
              else audit_mat(sf.eps, i0 - sf.eps_row_split, c, "sac eps", g, false, true);
              audit_mat(sf.act, i0, c, "sac act", g, false, false, 1);
            }
            audit_range(sf.logpi, (long long)i0 * 4, 64, "sac logpi", g, 1);
          }
          if (g.epi == EPI_SACBWD) {  // columns j0 .. j0 + ncol - 1 of the mean and log_std blocks
            const SacBwdArgs& sb = g.sb;
            audit_mat(sb.eps2, i0, j0, "sac eps2", g, false, true);
            for (int off : {sb.mean_off, sb.ls_off})
              for (int c : {off + j0, off + j0 + ncol - 1}) {
                audit_mat(sb.raw, i0, c, "sac raw", g, false, true);
                audit_mat(sb.dout, i0, c, "sac dout", g, false, false, 1);
              }
            audit_range(sb.log_alpha, 0, 4, "sac alpha", g);
          }
          if (g.epi == EPI_MSE) {
            audit_mat(g.tgt, i0, j0, "tgt", g, false, true);
            audit_norm(g.tgt_norm, i0, 16, g);
          }
          if (g.epi == EPI_QHEAD || g.epi == EPI_QDOT) audit_range(g.qw, h_nblk(g.qw_cbn, 0, j0), 1024, "qw", g);
          if (g.epi == EPI_QHEAD && t == 0) audit_range(g.qb, 0, 4, "qb", g);
          if (g.norm_out) audit_range(g.norm_out, ((long long)jt * g.norm_ld + i0) * 4, 64, "norm_out", g, 1);
          if (g.epi == EPI_MSE || g.epi == EPI_QHEAD) audit_range(g.loss_part, (long long)t * 4, 4, "loss_part", g, 1);
        }
      }
    }
  }
  if (g.epi == EPI_ADAM) {  // this step's bias corrections (Ctrl / adamsc1)
    audit_range(g.adam.step, 0, 4, "adam step", g);
    audit_range(g.adam.bc2s, 0, 4, "adam bc2s", g);
  }
  if (g.has_pre == 2) {  // the fused loss head (kernels.hip headdx_reduce), tile rows i0 .. i0 + 15
    const HeadArgs& h = g.hd;
    const int hn = g.head_n;
    audit_range(h.w[hn], 0, (long long)h.w_cbn * 1024, "head w3", g);
    for (int n = 0; n < 2; ++n) {
      audit_range(h.b[n], 0, 4, "head b3", g);
      if (h.tb[n]) audit_range(h.tb[n], 0, 4, "head tb3", g);
    }
    if (h.vt) audit_range(h.vt, 0, 8, "head vt", g);
    if (h.sac) audit_range(h.log_alpha, 0, 4, "head alpha", g);
    for (int it = 0; it < g.tiles_m; ++it) {
      const int i0 = it * 16;
      for (int n = 0; n < 2; ++n) {
        for (int p = 0; p < h.qp_n[n]; ++p) audit_range(h.qp[n], ((long long)p * h.qp_ld + i0) * 4, 64, "head qp", g);
        for (int p = 0; p < h.tp_n[n]; ++p) audit_range(h.tp[n], ((long long)p * h.tp_ld + i0) * 4, 64, "head tp", g);
      }
      if (h.reward) audit_range(h.reward, (long long)i0 * 4, 64, "head reward", g);
      if (h.notdone) audit_range(h.notdone, (long long)i0 * 4, 64, "head notdone", g);
      if (h.sac) audit_range(h.logpi, (long long)i0 * 4, 64, "head logpi", g);
      // tile column 0 stores the head's outputs of its rows
      if (hn == 0 && h.lap) audit_range(h.prio, (long long)i0 * 4, 64, "head prio", g, 1);
      if (h.dq[hn].t) audit_range(h.dq[hn].t, h_tblk(h.dq[hn].rbs, i0, 0), 1024, "head dq", g, 1);
      if (h.dz[hn].n || h.dz[hn].t)
        for (int c = 0; c < g.R; c += 16) audit_mat(h.dz[hn], i0, c, "head dz", g, false, false, 1);
      if (hn == 0) {
        if (h.loss_part) audit_range(h.loss_part, (long long)(i0 / 4) * 16, 64, "head loss", g, 1);
        if (h.vmax_key) audit_range(h.vmax_key, 0, 4, "head vmax", g, 1);
        if (h.vmin_key) audit_range(h.vmin_key, 0, 4, "head vmin", g, 1);
      }
    }
  }
  if (g.mode == GEMM_DW && g.act == kDwNb) {
    audit_norm(g.nbm, 0, g.R, g);
    for (int p = 0; p < g.nbdot_n; ++p) audit_range(g.nbdot, (long long)p * g.nbdot_ld * 4, (long long)g.R * 4, "nbdot", g);
  }
}

// ---- RLE_HAZARD=1: byte-level check of every level's ops against each other.  The scheduler
// orders ops by declared resources; this replays what each op's workgroups actually touch
// (GEMMs: audit_gemm's per-tile address replay; other ops: their descriptor's buffers, a tensor
// image from its pointer to the end of its allocation) and fails the build if a byte one op of a
// level stores is read or stored by another op of the same level -- a race whose outcome would
// depend on workgroup timing.  Ops of one program item (row pieces of one GEMM) are exempt from
// each other: they write disjoint rows by construction.
static uintptr_t alloc_end(const void* p) {
  std::lock_guard<std::mutex> lk(live_mu());
  auto& m = live_allocs();
  auto it = m.upper_bound((uintptr_t)p);
  if (it == m.begin()) return (uintptr_t)p + 4;
  --it;
  const uintptr_t e = it->first + it->second;
  return (uintptr_t)p < e ? e : (uintptr_t)p + 4;
}
static void acc_whole(std::vector<Access>& v, const void* p, int w, const char* what) {
  if (p) v.push_back({(uintptr_t)p, alloc_end(p), w, what});
}
static void acc_bytes(std::vector<Access>& v, const void* p, long long bytes, int w, const char* what) {
  if (p && bytes > 0) v.push_back({(uintptr_t)p, (uintptr_t)p + (uintptr_t)bytes, w, what});
}
static void acc_mat(std::vector<Access>& v, const Mat& m, int w, const char* what) {
  acc_whole(v, m.n, w, what);
  acc_whole(v, m.t, w, what);
}
static void op_accesses(const Op& op, std::vector<Access>& v) {
  switch (op.kind) {
    case OP_GEMM: {
      g_sink = &v;
      audit_gemm(op.gemm);
      g_sink = nullptr;
      g_tile = -1;
      break;
    }
    case OP_NORMBWD: {
      const NormBwdArgs& a = op.nb;
      if (a.fwd == 2) {  // finalize: partials in, one mean per row out
        acc_whole(v, a.norm.part, 0, "nb norm");
        acc_bytes(v, a.mout, (long long)a.rows * 4, 1, "nb mean");
        break;
      }
      acc_mat(v, a.g, 0, "nb g");
      acc_mat(v, a.x, 0, "nb x");
      acc_whole(v, a.norm.part, 0, "nb norm");
      acc_mat(v, a.dx, 1, "nb dx");
      break;
    }
    case OP_SAMPLE_REDUCE:
    case OP_SAMPLE_GATHER:
    case OP_NOISE: {
      const SampleArgs& s = op.sample;
      acc_bytes(v, s.size, 8, 0, "sample size");
      acc_bytes(v, s.tape_mode, 4, 0, "tape mode");
      acc_bytes(v, s.tape_pos, 8, 0, "tape pos");
      acc_bytes(v, s.ctrl_rng, 8, 0, "rng step");
      if (op.kind == OP_NOISE) {
        acc_whole(v, s.tape_eps, 0, "tape eps");
        acc_whole(v, s.tape_eps2, 0, "tape eps2");
        acc_mat(v, s.eps, 1, "eps");
        acc_mat(v, s.eps2, 1, "eps2");
        break;
      }
      acc_whole(v, s.priority, 0, "priority");
      acc_whole(v, s.bsum, op.kind == OP_SAMPLE_REDUCE, "bsum");
      acc_whole(v, s.ssum, op.kind == OP_SAMPLE_REDUCE, "ssum");
      if (op.kind == OP_SAMPLE_REDUCE) break;
      for (const void* r : {(const void*)s.state, (const void*)s.next_state, (const void*)s.action,
                            (const void*)s.reward, (const void*)s.notdone})
        acc_whole(v, r, 0, "replay");
      acc_whole(v, s.tape_u, 0, "tape u");
      acc_whole(v, s.tape_ind, 0, "tape ind");
      if (s.pend_n) {
        acc_bytes(v, s.pend_ind, 8LL * s.pend_n, 0, "pending ind");
        acc_bytes(v, s.pend_p, 4LL * s.pend_n, 0, "pending p");
      }
      acc_mat(v, s.ss, 1, "batch ss");
      acc_mat(v, s.a, 1, "batch a");
      acc_whole(v, s.r, 1, "batch r");
      acc_whole(v, s.nd, 1, "batch nd");
      acc_whole(v, s.ind, 1, "batch ind");
      acc_whole(v, s.u_out, 1, "batch u");
      break;
    }
    case OP_HEAD: {
      const HeadArgs& h = op.head;
      for (int n = 0; n < 2; ++n) {
        acc_mat(v, h.h[n], 0, "head h");
        acc_mat(v, h.dsrc[n], 0, "head dsrc");
        acc_bytes(v, h.w[n], (long long)h.w_cbn * 1024, 0, "head w");
        acc_bytes(v, h.b[n], 4, 0, "head b");
        if (h.tgt_mode >= 0) {
          acc_mat(v, h.th[n], 0, "head th");
          acc_bytes(v, h.tw[n], (long long)h.w_cbn * 1024, 0, "head tw");
          acc_bytes(v, h.tb[n], 4, 0, "head tb");
        }
        acc_whole(v, h.qp[n], 0, "head qp");
        acc_whole(v, h.tp[n], 0, "head tp");
        acc_mat(v, h.dz[n], 1, "head dz");
        acc_mat(v, h.dq[n], 1, "head dq");
      }
      acc_whole(v, h.reward, 0, "head reward");
      acc_whole(v, h.notdone, 0, "head notdone");
      const bool tgt = h.mode == HEAD_TD7_TARGET || h.mode == HEAD_MLP_TARGET;
      acc_whole(v, h.y, tgt || h.tgt_mode >= 0, "head y");
      acc_whole(v, h.logpi, 0, "head logpi");
      acc_bytes(v, h.log_alpha, 4, 0, "head log_alpha");
      acc_bytes(v, h.vt, 8, 0, "head vt");
      acc_whole(v, h.loss_part, 1, "head loss");
      acc_whole(v, h.prio, 1, "head prio");
      if (h.mode == HEAD_TD7_TARGET || h.tgt_mode == HEAD_TD7_TARGET) {
        acc_bytes(v, h.vmax_key, 4, 1, "head vmax");
        acc_bytes(v, h.vmin_key, 4, 1, "head vmin");
      }
      break;
    }
    case OP_PRIORITY: {
      const PriorityArgs& a = op.prio;
      acc_whole(v, a.p, 0, "prio p");
      acc_whole(v, a.ind, 0, "prio ind");
      acc_whole(v, a.priority, 1, "priority");
      acc_whole(v, a.bsum, 1, "bsum");
      acc_whole(v, a.ssum, 1, "ssum");
      acc_bytes(v, a.max_priority, 4, 1, "max priority");
      break;
    }
    case OP_SAC_ACTOR:
    case OP_SAC_ACTOR_BWD: {
      const SacActorArgs& a = op.sac;
      acc_mat(v, a.out, 0, "sac out");
      acc_mat(v, a.eps2, 0, "sac eps2");
      if (op.kind == OP_SAC_ACTOR) {
        acc_mat(v, a.eps, 0, "sac eps");
        acc_mat(v, a.act, 1, "sac act");
        acc_whole(v, a.logpi, 1, "sac logpi");
      } else {
        acc_mat(v, a.da, 0, "sac da");
        acc_bytes(v, a.log_alpha, 4, 0, "sac log_alpha");
        acc_mat(v, a.dout, 1, "sac dout");
      }
      break;
    }
    case OP_STEP_END: {  // (mode 1: counters + temperature; mode 2: the info row; 0: both)
      const StepEndArgs& a = op.end;
      const bool info = a.mode != 1, ctr = a.mode != 2, scr = a.mode == 2 && a.sac_scratch;
      if (info)
        for (int k = 0; k < a.ninfo; ++k)
          if (a.part[k]) acc_bytes(v, a.part[k], (long long)a.npart[k] * a.stride[k] * 4, 0, "info part");
      if (a.logpi_part && !scr) acc_bytes(v, a.logpi_part, (long long)a.nlogpi * 16, 0, "logpi part");
      if (info && a.gsq && a.ngsq_t > 0) acc_bytes(v, a.gsq, (long long)a.gsq_off[a.ngsq_t] * 4, 0, "gsq");
      if (ctr) acc_bytes(v, a.counters, 16 * 8, 1, "counters");
      if (info) acc_bytes(v, a.info_slot, 4, 1, "info slot");
      if (info) acc_whole(v, a.info, 1, "info ring");
      if (a.log_alpha && !scr) acc_bytes(v, a.log_alpha, 4, ctr && a.la_lr > 0.f, "log_alpha");
      if (ctr && a.la_lr > 0.f) {
        acc_bytes(v, a.la_m, 4, 1, "la_m");
        acc_bytes(v, a.la_v, 4, 1, "la_v");
        acc_bytes(v, a.la_t, 8, 1, "la_t");
      }
      if (a.sac_scratch) acc_bytes(v, a.sac_scratch, 8, a.mode == 1, "sac scratch");
      break;
    }
    case OP_POLYAK:
    case OP_COPY: {
      const FlatArgs& f = op.flat;
      acc_bytes(v, f.dst, f.n * 4, 1, "flat dst");
      if (!f.self_alias) acc_bytes(v, f.src, f.n * 4, 0, "flat src");
      break;
    }
    case OP_MAXRED: {
      const FlatArgs& f = op.flat;
      if (f.stage == 0) {
        acc_bytes(v, f.size, 8, 0, "maxred size");
        acc_whole(v, f.src, 0, "maxred src");
        acc_bytes(v, f.partial, (long long)f.nwg * 4, 1, "maxred partial");
      } else {
        acc_bytes(v, f.partial, (long long)f.nwg * 4, 0, "maxred partial");
        acc_bytes(v, f.out, 4, 1, "maxred out");
      }
      break;
    }
    case OP_CTRL: {
      const CtrlArgs& c = op.ctrl;
      if (c.mode == 0) {
        acc_bytes(v, c.vmax_key, 4, 0, "vmax key");
        acc_bytes(v, c.vmin_key, 4, 0, "vmin key");
        acc_bytes(v, c.vt, 8, 1, "vt");
      } else {
        acc_bytes(v, c.counters, 3 * 8, 0, "counters");
        acc_bytes(v, c.adam_step, (c.la_t ? 4 : 3) * 4, 1, "adam step");
        acc_bytes(v, c.adam_bc2s, (c.la_t ? 4 : 3) * 4, 1, "adam bc2s");
        if (c.la_t) acc_bytes(v, c.la_t, 8, 0, "la_t");
      }
      break;
    }
    case OP_FOLDBIAS: {
      const FoldBiasArgs& f = op.fb;
      acc_bytes(v, f.wn, (long long)((f.H + 15) / 16) * f.cbn * 1024, 0, "fold w");
      acc_bytes(v, f.bin, (long long)f.H * 4, 0, "fold bin");
      acc_bytes(v, f.bbase, (long long)f.H * 4, 0, "fold bbase");
      acc_bytes(v, f.bout, (long long)f.H * 4, 1, "fold bout");
      break;
    }
    default:
      throw Error{RLE_EINVAL, "hazard check: unknown op kind " + std::to_string(op.kind)};
  }
}

// ops: one level's ops; item[i]: the program item op i came from.  Throws on a conflict.
static void level_hazards(const std::vector<Op>& ops, const std::vector<int>& item, int level) {
  struct A {
    uintptr_t lo, hi;
    int w, op;
    const char* what;
  };
  std::vector<A> all;
  std::vector<Access> v;
  for (size_t i = 0; i < ops.size(); ++i) {
    v.clear();
    op_accesses(ops[i], v);
    for (const Access& a : v) all.push_back({a.lo, a.hi, a.w, (int)i, a.what});
  }
  std::sort(all.begin(), all.end(), [](const A& x, const A& y) { return x.lo < y.lo; });
  // sweep: active intervals (those whose hi > current lo); report a pair from different items
  // where one side writes
  std::vector<int> act;
  for (size_t k = 0; k < all.size(); ++k) {
    const A& c = all[k];
    size_t keep = 0;
    for (int j : act)
      if (all[j].hi > c.lo) act[keep++] = j;
    act.resize(keep);
    for (int j : act) {
      const A& o = all[j];
      if (o.op == c.op || item[o.op] == item[c.op] || !(o.w || c.w)) continue;
      char msg[320];
      snprintf(msg, sizeof msg, "hazard: level %d op %d (%s, kind %d, %s) and op %d (%s, kind %d, %s) overlap at %#lx", level,
               o.op, o.what, ops[o.op].kind, o.w ? "write" : "read", c.op, c.what, ops[c.op].kind, c.w ? "write" : "read",
               (unsigned long)c.lo);
      throw Error{RLE_EINVAL, msg};
    }
    act.push_back((int)k);
  }
}

// ---- RLE_TRAFFIC=1: the bytes each level must move (the union of its ops' byte ranges, so a range
// several tiles read counts once), by kind: activations read / written, weights read, Adam state
// (p, m, v read and written, N image written).  Graph descriptions carry it (tools/pmc_levels.py
// sets it against the PMC counters: traffic above these bytes is re-reads, e.g. one copy per XCD).
struct LevelTraffic {
  double act_r = 0, act_w = 0, w_r = 0, adam = 0, other = 0;
  // Per-XCD read model: every XCD's L2 fetches its own copy of what its workgroups read (round-robin dispatch:
  // workgroup w of a launch runs on XCD w mod 8, the 8 descriptor-prefetch workgroups first), so a GEMM
  // operand that tiles on several XCDs read is fetched once per XCD; reads of non-GEMM ops count once.
  double xcd_r = 0, adam_w = 0;  // (adam_w: the Adam stores alone -- adam counts its reads and stores)
};
static double union_bytes(std::vector<std::pair<uintptr_t, uintptr_t>>& v) {
  std::sort(v.begin(), v.end());
  double tot = 0;
  uintptr_t lo = 0, hi = 0;
  bool open = false;
  for (auto& r : v) {
    if (!open || r.first > hi) {
      if (open) tot += (double)(hi - lo);
      lo = r.first;
      hi = r.second;
      open = true;
    } else {
      hi = std::max(hi, r.second);
    }
  }
  if (open) tot += (double)(hi - lo);
  return tot;
}
static LevelTraffic level_traffic(const std::vector<Op>& ops, const float* P, size_t nP) {
  LevelTraffic t;
  std::vector<std::pair<uintptr_t, uintptr_t>> ar, aw, wr, ad;
  std::vector<std::pair<uintptr_t, uintptr_t>> xr[8], once;  // (per-XCD model: GEMM reads by XCD, other reads)
  const uintptr_t p0 = (uintptr_t)P, p1 = p0 + 3 * nP * 4;
  std::vector<Access> v;
  for (const Op& op : ops) {
    v.clear();
    if (op.kind == OP_SAMPLE_GATHER) {  // rows of the batch + one path down the LAP sum tree per query
      const SampleArgs& s = op.sample;
      t.other += (double)s.nq * (2.0 * s.Sp + s.Ap + 2) * 4 + (s.lap ? s.nq * (64.0 * 8 + 64 * 4) + s.nblk * 8.0 : 0);
      t.act_w += (double)s.B * ((s.ss.n != nullptr) + (s.ss.t != nullptr)) * 2 * s.Sp * 4 +
                 (double)s.B * ((s.a.n != nullptr) + (s.a.t != nullptr)) * s.Ap * 4 + s.B * 20.0;
      continue;
    }
    if (op.kind == OP_PRIORITY) {  // the scattered rows (a 64-B line each) and their two sums
      t.other += (double)op.prio.B * (8 + 4) + op.prio.B * 64.0 * 3;
      continue;
    }
    if (op.kind == OP_MAXRED && op.flat.stage == 0) {
      t.other += 4.0 * 1e6;  // (the replay size is a device value: the 1M benchmark ring)
      continue;
    }
    op_accesses(op, v);
    for (const Access& a : v) {
      const std::string what = a.what ? a.what : "";
      if (what.rfind("tape", 0) == 0) continue;  // (declared whole; read only in tape mode, one row)
      const bool in_p = a.lo >= p0 && a.hi <= p1;
      // (reads: every range not stored, and Adam's T-image / bias ranges, which hold p, m, v read and then written)
      if (!a.w || what == "adam w.t" || what == "adam bias") {
        if (op.kind == OP_GEMM && a.t >= 0) xr[(op.wg_begin + a.t) & 7].push_back({a.lo, a.hi});
        else once.push_back({a.lo, a.hi});
      }
      if (what.rfind("adam", 0) == 0) {
        if (a.w) t.adam_w += (double)(a.hi - a.lo);
        ad.push_back({a.lo, a.hi});
        if (what == "adam w.t" || what == "adam bias") ad.push_back({a.lo, a.hi});  // (read and written)
      } else if (a.w) {
        aw.push_back({a.lo, a.hi});
      } else if (in_p) {
        wr.push_back({a.lo, a.hi});
      } else {
        ar.push_back({a.lo, a.hi});
      }
    }
  }
  t.act_r += union_bytes(ar);
  t.act_w += union_bytes(aw);
  t.w_r += union_bytes(wr);
  // Adam ranges: each listed range once per direction (reads p, m, v; writes p T, m, v, p N)
  double adam = 0;
  for (auto& r : ad) adam += (double)(r.second - r.first);
  t.adam = adam;
  double xb = union_bytes(once);
  for (auto& r : xr) xb += union_bytes(r);
  t.xcd_r = xb;
  return t;
}

struct Prog {
  struct Item {
    std::vector<Op> ops;  // one op, or a group writing disjoint parts of the same buffers
    std::vector<int> rd, wr;
    int level = 0;
  };
  std::vector<Item> items;
  // ops per level: one launch each (kLevelOps preloaded entries)
  static constexpr int max_ops = kLevelOps;
  // register-blocked wide weight-gradient tiles (rle_plan rb)
  int rb = 0;
  int xcd = 1;  // XCD-aware tile order (rle_plan xcd)
  // (Engine::norm_fin) the finalized AvgL1Norm row means of this program: producer partials -> (means, resource)
  std::map<const float*, std::pair<float*, int>> norm_fins;
  static bool rb_eligible(const GemmArgs& g) {
    bool seg_ok = true;  // (the tile's column blocks lie in one X segment, kernels.hip rb path)
    for (int q = 0; q < g.B.nseg; ++q) seg_ok = seg_ok && g.B.seg[q].x0 % g.tn == 0;
    return g.mode == GEMM_DW && (g.tn == 32 || g.tn == 64) && g.has_pre == 0 && seg_ok;
  }
  void add(const Op& op, std::vector<int> rd, std::vector<int> wr) { add_group({op}, std::move(rd), std::move(wr)); }
  void add_group(std::vector<Op> ops, std::vector<int> rd, std::vector<int> wr) {
    for (Op& op : ops)
      if (op.kind == OP_GEMM) {
        op.gemm.hot.rb = rb && rb_eligible(op.gemm) ? 1 : 0;
        gemm_finalize(op.gemm, xcd != 0);
        check_gemm(op.gemm);
        if (std::getenv("RLE_AUDIT")) audit_gemm(op.gemm);  // (read per op: tests set it per engine)
      }
    Item it;
    it.ops = std::move(ops);
    it.rd = std::move(rd);
    it.wr = std::move(wr);
    items.push_back(std::move(it));
  }
  // Lowest level respecting RAW / WAR / WAW against all earlier ops (program order), and
  // (wg_cap) holding no more workgroups than are resident on the device at once unless
  // the op alone exceeds that: a second dispatch wave costs more than a later level.
  int balance = 0;  // 0 off, 1 any item, 2 no Adam items, 3 no Adam items + only into levels
                    // whose longest op is at least twice as long
  // Relative per-workgroup duration of an item (its longest op): a GEMM workgroup's
  // dependent MFMA chain grows with reduction length x tile width (4 waves share it); Adam
  // epilogues, the loss head and the sampler are long for their size (level traces).
  // weight of the step-end op (RLE_TINY_W, A/B; 0 = no tiny-op moves)
  // (rle_plan tiny_w / uni_w / tiny_wg; A/B tiny_w 0 / 20 / 30: TD7 8021 / 8050 / 8054, SAC 12249 /
  // 12235 / 12328; uni_w 60 as the LAP sampler, 12 with tiny_wg 64: SAC +-0, TD3 -0.5%)
  int tiny_w = 30, uni_w = 60, tiny_wg = 2;
  int pl_w = 0;  // (rle_plan pl_w) added to GEMMs whose workgroups run an in-tile prologue (has_pre 3-5)
  int lap_w = 60, head_w = 60, adam_w = 8;  // (rle_plan lap_w / head_w / adam_w)
  int lpt = 0;                              // (rle_plan lpt: longest-first op order in each level)
  int tiny_weight() const { return tiny_w ? tiny_w : 8; }
  int uniform_weight() const { return uni_w; }
  bool tiny_moves() const { return tiny_w != 0; }
  int op_weight(const Op& op) const {
    int x = 8;
    if (op.kind == OP_GEMM)
      x = op.gemm.R * op.gemm.tn / 1024 + (op.gemm.epi == EPI_ADAM ? adam_w : 0) + (op.gemm.has_pre >= 3 ? pl_w : 0);
    else if (op.kind == OP_HEAD) x = head_w;
    else if (op.kind == OP_SAMPLE_GATHER) x = op.sample.lap ? lap_w : uniform_weight();  // (uniform: a
                                                                                       // ~6 us gather)
    else if (op.kind == OP_STEP_END && op.end.mode != 1) x = tiny_weight();  // (one workgroup, ~4 KB of straight-line
                                                         // code fetched at L2 latency: 7-8 us)
    return x;
  }
  int item_weight(const Item& it) const {
    int w = 0;
    for (const Op& op : it.ops) w = std::max(w, op_weight(op));
    return w;
  }
  // After the ASAP pass: in reverse program order, move each item with slack (every
  // successor at least two levels later) to the lightest level of its window where it is
  // not the longest op, so wide ASAP levels (contended CUs) shed work into thin levels of
  // the critical chain.  Dependencies are the RAW / WAW / WAR edges of the ASAP pass.
  // RAW / WAW / WAR successors of every item (program order)
  std::vector<std::vector<int>> successors() const {
    const int n = (int)items.size();
    std::vector<std::vector<int>> succ(n);
    std::map<int, int> lastw;
    std::map<int, std::vector<int>> readers;
    for (int i = 0; i < n; ++i) {
      const Item& it = items[i];
      auto edge = [&](int from) {
        if (from >= 0) succ[from].push_back(i);
      };
      for (int r : it.rd)
        if (r >= 0 && lastw.count(r)) edge(lastw[r]);
      for (int w : it.wr) {
        if (w < 0) continue;
        if (lastw.count(w)) edge(lastw[w]);
        for (int j : readers[w]) edge(j);
      }
      for (int w : it.wr)
        if (w >= 0) {
          lastw[w] = i;
          readers[w].clear();
        }
      for (int r : it.rd)
        if (r >= 0) readers[r].push_back(i);
    }
    return succ;
  }
  // (describe, RLE_DESC_CRIT=1) items on a longest dependency chain of the ASAP placement: their
  // level + the longest chain after them = the last level (every dependence edge is one level)
  std::vector<char> crit;
  void mark_critical(int maxl) {
    const int n = (int)items.size();
    const auto succ = successors();
    std::vector<int> tail(n, 0);
    for (int i = n - 1; i >= 0; --i)
      for (int s : succ[i]) tail[i] = std::max(tail[i], tail[s] + 1);
    crit.assign(n, 0);
    for (int i = 0; i < n; ++i) crit[i] = items[i].level + tail[i] == maxl;
  }
  void rebalance(int maxl, std::vector<int>& nops, std::vector<int>& nwg, int wg_cap) {
    const int n = (int)items.size();
    const auto succ = successors();
    std::vector<int> wmax(maxl + 1, 0);
    for (auto& it : items) wmax[it.level] = std::max(wmax[it.level], item_weight(it));
    const int cap = std::min(wg_cap, 1024);
    for (int i = n - 1; i >= 0; --i) {
      Item& it = items[i];
      int hi = maxl;
      for (int s : succ[i]) hi = std::min(hi, items[s].level - 1);
      const int cur = it.level;
      if (hi <= cur) continue;
      int wg = 0;
      for (auto& op : it.ops) wg += op.wg_count;
      const int wt = item_weight(it);
      bool adam = false;
      for (auto& op : it.ops) adam = adam || (op.kind == OP_GEMM && op.gemm.epi == EPI_ADAM);
      if (balance >= 2 && adam) continue;
      const int wfac = balance >= 3 ? 2 : 1;
      int best = -1;
      for (int l = cur + 1; l <= hi; ++l) {
        if (nops[l] + (int)it.ops.size() > max_ops || wt * wfac > wmax[l] || nwg[l] + wg > cap) continue;
        if (nwg[l] + wg >= nwg[cur]) continue;
        if (best < 0 || nwg[l] < nwg[best]) best = l;
      }
      // a one-workgroup op (the step end) that is the longest of its level: into the first level
      // of its window that has a longer op, so its time hides there
      if (best < 0 && tiny_moves() && wg <= tiny_wg && wt >= wmax[cur]) {
        for (int l = cur + 1; l <= hi && best < 0; ++l)
          if (wmax[l] > wt && nops[l] + (int)it.ops.size() <= max_ops && nwg[l] + wg <= cap) best = l;
      }
      if (best < 0) continue;
      nops[cur] -= (int)it.ops.size();
      nwg[cur] -= wg;
      nops[best] += (int)it.ops.size();
      nwg[best] += wg;
      it.level = best;
    }
  }
  std::vector<std::vector<char>> crit_lv;  // (describe) per level, per op: on a longest chain
  std::vector<std::vector<Op>> schedule(int wg_cap = 1 << 30) {
    std::map<int, int> lw, lr;
    int maxl = -1;
    std::vector<int> nops, nwg;
    for (auto& it : items) {
      int l = 0;
      for (int r : it.rd)
        if (r >= 0 && lw.count(r)) l = std::max(l, lw[r] + 1);
      for (int w : it.wr) {
        if (w < 0) continue;
        if (lw.count(w)) l = std::max(l, lw[w] + 1);
        if (lr.count(w)) l = std::max(l, lr[w] + 1);
      }
      // a level of more than max_ops ops would take two launches: defer to the next level
      // with room (every dependence is still met at a later level)
      int wg = 0;
      for (auto& op : it.ops) wg += op.wg_count;
      while (l < (int)nops.size() &&
             (nops[l] + (int)it.ops.size() > max_ops || (nwg[l] > 0 && nwg[l] + wg > wg_cap)))
        ++l;
      if (l >= (int)nops.size()) {
        nops.resize(l + 1, 0);
        nwg.resize(l + 1, 0);
      }
      nops[l] += (int)it.ops.size();
      nwg[l] += wg;
      it.level = l;
      for (int w : it.wr)
        if (w >= 0) lw[w] = l;
      for (int r : it.rd)
        if (r >= 0) lr[r] = std::max(lr.count(r) ? lr[r] : -1, l);
      maxl = std::max(maxl, l);
    }
    if (const char* c = std::getenv("RLE_DESC_CRIT"); c && c[0] == '1') mark_critical(maxl);
    if (balance) rebalance(maxl, nops, nwg, wg_cap);
    std::vector<std::vector<Op>> levels(maxl + 1);
    std::vector<std::vector<int>> owner(maxl + 1);
    crit_lv.assign(maxl + 1, {});
    for (size_t i = 0; i < items.size(); ++i)
      for (auto& op : items[i].ops) {
        levels[items[i].level].push_back(op);
        owner[items[i].level].push_back((int)i);
        crit_lv[items[i].level].push_back(crit.empty() ? 0 : crit[i]);
      }
    if (lpt)  // longest first (rle_plan lpt): a stable sort of each level by the estimated workgroup time
      for (size_t l = 0; l < levels.size(); ++l) {
        std::vector<int> ix(levels[l].size());
        for (size_t k = 0; k < ix.size(); ++k) ix[k] = (int)k;
        std::stable_sort(ix.begin(), ix.end(),
                         [&](int a, int b) { return op_weight(levels[l][a]) > op_weight(levels[l][b]); });
        std::vector<Op> lv;
        std::vector<int> ow;
        std::vector<char> cr;
        for (int k : ix) {
          lv.push_back(levels[l][k]);
          ow.push_back(owner[l][k]);
          cr.push_back(crit_lv[l][k]);
        }
        levels[l].swap(lv);
        owner[l].swap(ow);
        crit_lv[l].swap(cr);
      }
    if (const char* hz = std::getenv("RLE_HAZARD"); hz && hz[0] == '1')
      for (size_t l = 0; l < levels.size(); ++l) level_hazards(levels[l], owner[l], (int)l);
    for (auto& lv : levels) {
      int wg = 0;
      for (auto& op : lv) {
        op.wg_begin = wg;
        wg += op.wg_count;
      }
    }
    return levels;
  }
};

// ---- Direct AQL dispatch (default; rle_plan.dispatch 0 for the hipGraph path): the step graphs' level
// launches written as kernel-dispatch packets into the engine's own HSA queue instead of hipGraph
// replays.  Fences as HIP's own: agent-scope acquire and release between dependent levels; the first
// packet of a flush acquires and its last releases at system scope (host-written inputs, host-read
// results).  tools/mbaql.cpp measured the same packets at 3.83 us per level against hipGraph's 4.08.
// One HSA queue of a device, shared by the engines aql_open hands it to (at most kAqlQueuesPerDevice
// per device and process: more user-mode queues than that oversubscribe the device's hardware queue
// slots, and every queue's dispatches slow down -- profiles/r05_seeds_aql.txt, r05_seeds_hwq.txt).
// mu: one burst's packets and doorbells at a time (engines driven from several threads).
struct AqlHw {
  hsa_agent_t agent{};
  hsa_queue_t* q = nullptr;
  uint64_t kobj[KS_COUNT] = {};  // rle_level<false, ks>
  uint32_t gseg[KS_COUNT] = {}, pseg[KS_COUNT] = {};
  std::atomic<bool> failed{false};  // a burst on this queue timed out: every engine sharing it fails fast
  std::mutex mu;
  ~AqlHw() {
    if (q) (void)hsa_queue_destroy(q);
  }
};
constexpr int kAqlQueuesPerDevice = 4;
// An engine's view of its queue: its own completion signal, pending packets and timing.
struct AqlQueue {
  std::shared_ptr<AqlHw> hw;
  hsa_signal_t sig{};
  struct Pending {
    const void* ka;
    unsigned grid;
    int ks;
  };
  std::vector<Pending> pending;
  // a LOWER bound on the time per packet: the fastest burst seen (>= kAqlMinBurst packets) x kAqlBoundFrac, 0 before
  // one was timed.  The wait sleeps only through this bound's share of a burst, so it wakes before the burst ends and
  // spins the rest: a mean-based estimate overslept short bursts (a 20-step bench burst woke 0.5 ms late, -17%).
  double us_per_launch = 0.0;
  bool failed = false;          // a flush timed out: its packets may still be queued, the queue takes no more
  size_t inflight = 0;          // packets submitted since the last aql_complete
  uint64_t last_idx = 0;        // queue index of the last packet this engine submitted
  bool timed_idle = false;      // the oldest burst in flight started on an idle queue (its wall time is its own)
  std::chrono::steady_clock::time_point t0{};  // first doorbell of the oldest burst in flight
  bool closed() const { return failed || (hw && hw->failed.load(std::memory_order_relaxed)); }
  ~AqlQueue() {
    if (sig.handle) (void)hsa_signal_destroy(sig);
  }
};
#define HSACHK(x)                                                                              \
  do {                                                                                         \
    hsa_status_t s_ = (x);                                                                     \
    if (s_ != HSA_STATUS_SUCCESS) throw Error{RLE_EHIP, std::string(#x) + ": hsa status " + std::to_string((int)s_)}; \
  } while (0)

static hsa_status_t aql_find_gpu(hsa_agent_t a, void* data) {
  auto* want = static_cast<std::pair<uint32_t, hsa_agent_t>*>(data);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0;
  if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (bdf == want->first) {
    want->second = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}
struct AqlFind {
  hsa_agent_t agent;
  const char* name;
  uint64_t kobj;
  uint32_t gseg, pseg;
};
static hsa_status_t aql_find_kernel(hsa_executable_t exe, void* data) {
  auto* f = static_cast<AqlFind*>(data);
  hsa_executable_symbol_t sym;
  if (hsa_executable_get_symbol_by_name(exe, f->name, &f->agent, &sym) == HSA_STATUS_SUCCESS) {
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &f->kobj);
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &f->gseg);
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &f->pseg);
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// The queue of device `dev`, after HIP has loaded librle's code object (any rle_level launch).
static std::shared_ptr<AqlHw> aql_hw_create(int dev) {
  auto A = std::make_shared<AqlHw>();
  HSACHK(hsa_init());
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, dev));
  std::pair<uint32_t, hsa_agent_t> want{(uint32_t)((prop.pciBusID << 8) | (prop.pciDeviceID << 3)), {}};
  hsa_iterate_agents(aql_find_gpu, &want);
  REQUIRE(want.second.handle, "aql: no HSA agent for the HIP device");
  A->agent = want.second;
  hsa_ven_amd_loader_1_03_pfn_t tbl;
  HSACHK(hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(tbl), &tbl));
  for (int x = 0; x < KS_COUNT; ++x) {
    AqlFind f{A->agent, level_kernel_symbol(x), 0, 0, 0};
    tbl.hsa_ven_amd_loader_iterate_executables(aql_find_kernel, &f);
    REQUIRE(f.kobj, "aql: rle_level's kernel object is not loaded");
    A->kobj[x] = f.kobj;
    A->gseg[x] = f.gseg;
    A->pseg[x] = f.pseg;
  }
  uint32_t qmax = 0;
  HSACHK(hsa_agent_get_info(A->agent, HSA_AGENT_INFO_QUEUE_MAX_SIZE, &qmax));
  HSACHK(hsa_queue_create(A->agent, std::min<uint32_t>(qmax, 16384), HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr,
                          UINT32_MAX, UINT32_MAX, &A->q));
  return A;
}
// The engine's queue: a new HSA queue while the device has fewer than kAqlQueuesPerDevice live ones,
// else the live one with the fewest engines (its bursts then run in submission order with theirs).
static std::unique_ptr<AqlQueue> aql_open(int dev) {
  static std::mutex pool_mu;
  static std::map<int, std::vector<std::weak_ptr<AqlHw>>> pool;
  auto A = std::make_unique<AqlQueue>();
  {
    std::lock_guard<std::mutex> lk(pool_mu);
    auto& live = pool[dev];
    live.erase(std::remove_if(live.begin(), live.end(), [](const std::weak_ptr<AqlHw>& w) { return w.expired(); }),
               live.end());
    if ((int)live.size() < kAqlQueuesPerDevice) {
      A->hw = aql_hw_create(dev);
      live.push_back(A->hw);
    } else {
      for (auto& w : live) {
        auto h = w.lock();
        if (h && (!A->hw || h.use_count() < A->hw.use_count())) A->hw = h;
      }
    }
  }
  HSACHK(hsa_signal_create(0, 0, nullptr, &A->sig));  // (bursts in flight: aql_submit)
  return A;
}

// How the host waits for a flush without holding its core (MuJoCo stepping runs on the host cores beside
// the engine, north_star): while more than kAqlSpinUs of the expected duration remain it sleeps (slices of
// at most kAqlSliceUs, the signal checked between them), then spins on the signal; past timeout_s it gives
// up.  expected_us = packets still to retire x a lower bound on the queue's time per packet (AqlQueue::us_per_launch).
constexpr double kAqlSpinUs = 150.0, kAqlSliceUs = 2000.0, kAqlTimeoutS = 60.0;
constexpr size_t kAqlMinBurst = 32;   // bursts timed for the per-packet bound (AqlQueue::us_per_launch)
constexpr double kAqlBoundFrac = 0.92;
enum AqlWaitAct : int { AQL_SPIN = 0, AQL_SLEEP = 1, AQL_TIMEOUT = 2 };
static int aql_wait_step(double expected_us, double elapsed_us, double timeout_s, double* sleep_us) {
  *sleep_us = 0.0;
  if (elapsed_us > timeout_s * 1e6) return AQL_TIMEOUT;
  const double left = expected_us - elapsed_us - kAqlSpinUs;
  if (left < 20.0) return AQL_SPIN;
  *sleep_us = std::min(left, kAqlSliceUs);
  return AQL_SLEEP;
}
// Waits until pred() holds, by aql_wait_step's policy; on timeout the engine's queue and the shared
// hardware queue are marked failed (every engine on it then fails fast instead of waiting 60 s again).
template <class Pred>
static void aql_wait(AqlQueue& A, Pred pred, double expected_us, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  while (!pred()) {
    const double el = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    double sl = 0.0;
    const int act = aql_wait_step(expected_us, el, kAqlTimeoutS, &sl);
    if (act == AQL_TIMEOUT) {
      A.failed = true;
      if (A.hw) A.hw->failed = true;
      A.pending.clear();
      A.inflight = 0;
      throw Error{RLE_EHIP, std::string("aql: ") + what + " did not complete within 60 s; the engine's queue is "
                            "closed (every later step fails; destroy the engine)"};
    }
    if (act == AQL_SLEEP) std::this_thread::sleep_for(std::chrono::duration<double, std::micro>(sl));
  }
}
static Error aql_closed_error() { return Error{RLE_EHIP, "aql: the engine's queue is closed after a timed-out dispatch"}; }

// Doorbell batching: the doorbell is rung after a packet whose queue index is the last of an aligned
// group of kAqlDoorbellEvery (and after a burst's last packet).  The groups are aligned to the ABSOLUTE
// index, so the packets one doorbell publishes never straddle the end of the ring (its size is a power
// of two >= kAqlDoorbellEvery).  Queue interceptors (rocprofv3's kernel tracing wraps the queue) copy
// the packets of one doorbell as one contiguous run of the ring: a run that crossed the ring's end read
// past it (profiles/r05_prof_crash.txt: SIGSEGV at the 1 MB ring's end, 16384 x 64 B).
constexpr uint64_t kAqlDoorbellEvery = 64;
static bool aql_doorbell_after(uint64_t idx, bool last) { return last || (idx & (kAqlDoorbellEvery - 1)) == kAqlDoorbellEvery - 1; }

// Writes every pending packet and rings the doorbell; the completion signal counts the submitted bursts
// still in flight (each burst's last packet decrements it), so bursts may be submitted back to back
// (rle_step_async) and aql_complete waits for all of them.  A slot is reserved only once the ring has
// room for it (the wait happens before hsa_queue_add_write_index, under hw.mu, so a timed-out wait never
// leaves a reserved slot unwritten for the packet processor to stall on).
static void aql_submit(AqlQueue& A) {
  const size_t n = A.pending.size();
  if (!n) return;
  if (A.closed()) {
    A.pending.clear();
    throw aql_closed_error();
  }
  AqlHw& hw = *A.hw;
  std::lock_guard<std::mutex> lk(hw.mu);
  hsa_queue_t* q = hw.q;
  const uint64_t mask = q->size - 1;
  if (!A.inflight) {
    A.timed_idle = hsa_queue_load_read_index_scacquire(q) == hsa_queue_load_write_index_relaxed(q);
  }
  hsa_signal_add_relaxed(A.sig, 1);
  bool rung = false;
  uint64_t since_bell = 0;  // packets written since the last doorbell
  auto bell = [&](uint64_t idx) {
    hsa_signal_store_screlease(q->doorbell_signal, idx);
    since_bell = 0;
    if (!A.inflight && !rung) A.t0 = std::chrono::steady_clock::now();
    rung = true;
  };
  for (size_t i = 0; i < n; ++i) {
    const uint64_t next = hsa_queue_load_write_index_relaxed(q);
    if (next - hsa_queue_load_read_index_scacquire(q) >= q->size) {
      // (bursts of > q->size packets) publish what is written, wait until half the queue has drained, then
      // write on: the host sleeps through most of it instead of tracking the device one packet at a time
      if (since_bell) bell(next - 1);
      const uint64_t half = q->size / 2;
      const double ahead = (double)(next - hsa_queue_load_read_index_scacquire(q) - half + 1);
      try {
        aql_wait(A, [&] { return next - hsa_queue_load_read_index_scacquire(q) < half; }, ahead * A.us_per_launch,
                 "a queue slot");
      } catch (...) {
        hsa_signal_subtract_relaxed(A.sig, 1);  // (this burst's last packet will never be written)
        throw;
      }
    }
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
    auto* pk = (hsa_kernel_dispatch_packet_t*)q->base_address + (idx & mask);
    pk->workgroup_size_x = kThreads;
    pk->workgroup_size_y = 1;
    pk->workgroup_size_z = 1;
    pk->reserved0 = 0;
    pk->grid_size_x = A.pending[i].grid * kThreads;
    pk->grid_size_y = 1;
    pk->grid_size_z = 1;
    const int x = A.pending[i].ks;
    pk->private_segment_size = hw.pseg[x];
    pk->group_segment_size = hw.gseg[x];
    pk->kernel_object = hw.kobj[x];
    pk->kernarg_address = const_cast<void*>(A.pending[i].ka);
    pk->reserved2 = 0;
    const bool last = i + 1 == n;
    pk->completion_signal = last ? A.sig : hsa_signal_t{0};
#ifndef RLE_EXP_ACQ  // (timing-only variant builds: make variant-engine; the product uses agent / agent)
#define RLE_EXP_ACQ HSA_FENCE_SCOPE_AGENT
#define RLE_EXP_REL HSA_FENCE_SCOPE_AGENT
#endif
    const int a = i == 0 ? HSA_FENCE_SCOPE_SYSTEM : RLE_EXP_ACQ;
    const int r = last ? HSA_FENCE_SCOPE_SYSTEM : RLE_EXP_REL;
    const uint16_t hdr = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                         (a << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) | (r << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    __atomic_store_n((uint32_t*)pk, (uint32_t)hdr | (1u << 16), __ATOMIC_RELEASE);  // header | setup (1 dim)
    ++since_bell;
    if (last) A.last_idx = idx;
    if (aql_doorbell_after(idx, last)) bell(idx);
  }
  A.inflight += n;
  A.pending.clear();
}
// Waits until every submitted burst has retired (host-side wall time from the first doorbell of the
// oldest burst in flight to completion added to *ms when given).  The sleep estimate counts only the
// packets up to this engine's last one (other engines' later bursts on a pooled queue are not its
// wait), and the per-packet bound is refreshed only from bursts that started on an idle queue.
static void aql_complete(AqlQueue& A, double* ms) {
  if (!A.inflight) return;
  if (A.closed()) {
    A.inflight = 0;
    throw aql_closed_error();
  }
  hsa_queue_t* q = A.hw->q;
  const uint64_t rd = hsa_queue_load_read_index_scacquire(q);
  const double left = A.last_idx + 1 > rd ? (double)(A.last_idx + 1 - rd) : 0.0;
  aql_wait(A, [&] { return hsa_signal_load_scacquire(A.sig) < 1; }, left * A.us_per_launch, "a dispatch");
  const double wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - A.t0).count();
  if (A.inflight >= kAqlMinBurst && A.timed_idle) {
    const double per = kAqlBoundFrac * wall_ms * 1e3 / (double)A.inflight;
    A.us_per_launch = A.us_per_launch > 0.0 ? std::min(A.us_per_launch, per) : per;
  }
  A.inflight = 0;
  if (ms) *ms += wall_ms;
}
static void aql_flush(AqlQueue& A, double* ms) {
  aql_submit(A);
  aql_complete(A, ms);
}

struct Graph {
  hipGraph_t g = nullptr;
  hipGraphExec_t x = nullptr;
  Op* d_ops = nullptr;
  unsigned long long* trace = nullptr;  // [total wg][4] when RLE_TRACE=1
  long long trace_n = 0;
  std::vector<int> nops, nwg, off;
  std::string desc;
  int nlaunch = 0;  // rle_level dispatches per replay (a level of > kLevelOps ops takes several)
  std::vector<std::vector<Op>> host_levels;  // the launches' host op tables (rle_plan dispatch 2)
  std::vector<LevelLaunch> aql;               // (rle_plan dispatch 1) the dispatches' kernel arguments ...
  unsigned char* aql_ka = nullptr;            // ... in device memory, 128 B apart
  int levels() const { return (int)nops.size(); }
};

struct Layer {
  std::string wname, bname;
  int out = 0, K = 0;
  std::vector<int> seg_w, seg_p;  // logical / padded widths of input segments
  int rb = 0, cb = 0;             // 16-blocks of out rows / K columns
  size_t wn_off = 0, wt_off = 0, b_off = 0;  // N image, T image, bias [16 rb]
  int res = -1;
};

struct Net {
  std::string name, kind;  // kind: sale_enc / sale_actor / sale_critic / mlp
  std::vector<Layer> layers;
  size_t off = 0, size = 0;
  int res = -1;  // whole-net resource (polyak / copy)
};

enum Res : int {
  R_CNT = 1,
  R_VKEYS,
  R_VT,
  R_INFO,
  R_LA,
  R_PRIO,
  R_MAXP,
  R_REPLAY,
  R_ADAMSC,  // Ctrl::adam_step / adam_bc2s (Adam bias corrections of this step)
  R_ADAMSC1, // their copy for steps on batch set 1 (two steps in one graph: g_pair)
  R_FIRST_DYNAMIC = 100,
};

// The default plan: every field "default" (resolved per engine by Engine::resolve_plan).
static rle_plan plan_defaults() {
  rle_plan p{};
  p.steps_per_graph = -1;
  p.balance = -1;
  p.tiny_w = p.uni_w = p.tiny_wg = -1;
  p.rb = -1;
  p.pl_w = -1;
  p.lap_w = p.head_w = p.adam_w = -1;
  p.wide = -1;
  p.lpt = -1;
  p.dispatch = p.dpf = p.xcd = -1;
  return p;
}

struct Engine {
  rle_config cfg;
  rle_plan plan = plan_defaults();  // (resolved: no field left "default")
  // Defaults of the fields left at "default" for this engine's algorithm (rle.h rle_plan).
  // The extended kernel instance runs this engine's programs when its plan uses what only that
  // instance compiles: register-blocked weight-gradient tiles, the fused priority sampler.
  // the rle_level instance this engine's programs run on (ops.h KernelSet): the agent's own set, or the
  // extended instance when the plan asks for its opt-in paths
  int kernel_set() const {
    if (!acts_default) return KS_EXT;  // (the activation variants outside the agent's own set)
    if (algo == RLE_TD7 && plan.wide && !(plan.fuse_on & RLE_FUSE_PRIOSAMPLE)) return KS_TD7W;  // (rb compiled in)
    if (plan.rb || (plan.fuse_on & RLE_FUSE_PRIOSAMPLE) || plan.wide) return KS_EXT;
    return algo == RLE_TD7 ? KS_TD7 : KS_MLP;
  }
  void resolve_plan() {
    if (plan.steps_per_graph < 0) plan.steps_per_graph = algo == RLE_TD3 ? 16 : algo == RLE_SAC ? 8 : 6;
    // (SAC's target critics' raw-head pre-GEMM consumers: 32 measured +1.0% over 64, 2 pairs)
    if (plan.pre_tn == 0) plan.pre_tn = algo == RLE_TD3 ? 64 : 32;
    plan.pre_tn = plan.pre_tn == 32 || plan.pre_tn == 64 ? plan.pre_tn : 16;
    // (SAC pl_tn 32: its 64-workgroup actor-DX pre-layer level; with uni_w 30, A/B 2 pairs: 14.40k -> 14.55k;
    // TD3 32: -5%)
    if (plan.pl_tn == 0) plan.pl_tn = algo == RLE_SAC ? 32 : 64;
    plan.pl_tn = plan.pl_tn == 16 || plan.pl_tn == 32 ? plan.pl_tn : 64;
    plan.tn_min = plan.tn_min == 32 || plan.tn_min == 64 ? plan.tn_min : 16;
    if (plan.flat_div <= 0) plan.flat_div = 4;
    // (TD7: mode 3, no Adam items moved and only under a twice-longer op -- interleaved A/B, 4 pairs: TD7 Humanoid
    // 8,295-8,306 -> 8,328-8,341 steps/s, Ant +0.1%, B = 1024 +-0; TD3 -5%, SAC -2% at 3, so they keep 1;
    // profiles/r06_ab_balance.txt)
    // (SAC: mode 2, 4 pairs 14.75k -> 14.78k, profiles/r06_ab_plan_mlp.txt; TD3 keeps 1)
    if (plan.balance < 0) plan.balance = algo == RLE_TD7 ? 3 : algo == RLE_SAC ? 2 : 1;
    if (plan.tiny_w < 0) plan.tiny_w = 30;
    // (uniform sampler weight, A/B 2 pairs, SAC Humanoid uni_w 60 / 45 / 30 / 15 -> 14.10k / 14.13k / 14.40k /
    // 14.39k; TD3 HalfCheetah 60 / 30 / 20 / 15 / 8 / 1 -> 25.40k / 25.42k / 25.30k / 25.81k / 25.84k / 25.76k: a
    // lighter sampler is moved off the level it would bound)
    if (plan.uni_w < 0) plan.uni_w = algo == RLE_SAC ? 30 : algo == RLE_TD3 ? 8 : 60;
    if (plan.tiny_wg < 0) plan.tiny_wg = 2;
    plan.sched_cap = plan.sched_cap ? 1 : 0;
    // (64-row LDS-staged tiles: the 16-row tiles' per-workgroup fixed cost and 2 KB of operand loads per 4
    // MFMAs bound the B >= 512 levels, DESIGN round 5; with them the register-blocked weight-gradient tiles, the
    // batch split over the 4 waves, where a 16 x 64 weight-gradient tile's waves would each reduce all B rows)
    if (plan.wide < 0) plan.wide = 0;  // (opt-in: slower at B = 1024 than the 16-row tiles, DESIGN round 5)
    // (longest first: interleaved A/B on the round-6 tree, TD7 Humanoid +0.5% (4 pairs), Ant +1.1%, B = 1024 +0.2%,
    // TD3 HalfCheetah +1.9%, SAC Humanoid +0.9%; profiles/r06_ab_lpt.txt.  Round 5 measured it at +-0)
    if (plan.lpt < 0) plan.lpt = 1;
    plan.lpt = plan.lpt ? 1 : 0;
    plan.rb = plan.rb < 0 ? (plan.wide ? 1 : 0) : (plan.rb ? 1 : 0);
    // (A/B, 2 pairs: SAC Humanoid pl_w 0 / 8 / 16 / 24 -> 14.09k / 14.09k / 14.11k / 14.15k; TD3 HalfCheetah
    // 25.37k / 25.33k / 25.38k / 25.36k)
    if (plan.pl_w < 0) plan.pl_w = algo == RLE_SAC ? 24 : 0;
    if (plan.lap_w < 0) plan.lap_w = 60;
    if (plan.head_w < 0) plan.head_w = 60;
    // (A/B 2 pairs, SAC Humanoid adam_w 0 / 8 / 12 / 16 / 24 / 32 -> 14.38k / 14.56k / 14.67k / 14.67k / 14.64k /
    // 14.67k; TD3 HalfCheetah 0 / 8 / 16 -> 25.81k / 25.84k / 25.00k; TD7 Humanoid 0 / 8 / 16 -> 8.17k / 8.25k /
    // 8.24k, B = 1024 flat: profiles/r04_ab_weights.txt)
    if (plan.adam_w < 0) plan.adam_w = algo == RLE_SAC ? 16 : 8;
    if (plan.level_cap < 0) plan.level_cap = 0;
    plan.wide = plan.wide == 32 || plan.wide == 0 ? plan.wide : 64;  // (the tile width; 1 = 64)
    plan.dispatch = plan.dispatch < 0 ? 1 : std::min(plan.dispatch, 2);
    plan.dpf = plan.dpf < 0 ? 1 : (plan.dpf ? 1 : 0);
    plan.xcd = plan.xcd < 0 ? 1 : (plan.xcd ? 1 : 0);
  }
  int S, Sp, A, Ap, H, Hp, B;
  int Bv = 0;  // batch rows (rle_config.batch, any 1..1024); B = Bv padded to 16: the padded rows are zero and
               // every mean, loss, priority and value bound counts the Bv batch rows only
  int Z = 0, Zp = 0;    // TD7: SALE embedding width zs_dim (sale.py:23), padded
  std::vector<int> HS;  // TD3 / SAC: hidden widths of make_mlp (mlp.py:10-35), input side first
  // hidden activations (ops.h Act) of the actor, the critics and TD7's encoders (rle_config act_*)
  int actP = ACT_RELU, actC = ACT_ELU, actE = ACT_ELU;
  bool acts_default = true;
  // The derivative source of a hidden activation for an input-gradient GEMM: ELU' = exp(z) reads the pre-activation
  // z (as autograd's elu_backward does), ReLU' the output, identity none.
  static const View* dsrc_of(int act, const View& y, const View& z) {
    return act == ACT_ELU ? &z : act == ACT_RELU ? &y : nullptr;
  }
  int algo;
  hipStream_t stream = nullptr;
  DevMem mem;
  float* P = nullptr;
  size_t nP = 0;
  std::vector<Net> nets;
  Ctrl* ctrl = nullptr;
  float* info = nullptr;
  int info_cap = 4096;
  std::vector<float> info_host;
  Replay* replay = nullptr;
  hipEvent_t done_ev = nullptr;  // recorded after every enqueued step (Replay::users)
  int next_id = R_FIRST_DYNAMIC;
  // Graphs per batch-buffer parity p: g_prime[p] samples batch p (draws of the next
  // step); g_pol[p] / g_pln[p] run a (policy / plain) step on batch p and, once its
  // priority update is done, prefetch the next step's batch into 1 - p.
  Graph g_prime[2], g_pol[2], g_pln[2], g_hard;
  Graph g_slot0;  // info slot := 0 as a level of its own (rle_step_async bursts on the AQL queue)
  // g_pair[p]: multi_k consecutive steps as ONE program, starting on batch p (policy,
  // plain, policy, ... with policy_freq 2; SAC: every step), so the scheduler overlaps
  // each step's early levels (encoder phase, fixed encoders, online critic forward) with
  // the previous step's policy-phase tail and last Adam level.  Steps on the two batch
  // sets keep their own Adam scalars (asc_set) so only true data dependencies order them.
  Graph g_pair[2];
  int multi_k = 0;
  // g_rem[r][p]: kRemK[r] steps as one program (a burst's tail shorter than multi_k: the driver's 20-step bench
  // burst is 3 x 6 + 2), built when kRemK[r] < multi_k
  static constexpr int kRemK[2] = {4, 2};
  Graph g_rem[2][2];
  int asc_set = 0;
  float* adamsc1 = nullptr;  // [step[4], bc2s[4]] of steps built on set 1
  float* adam_step_of(int set) { return set ? adamsc1 : ctrl->adam_step; }
  float* adam_bc2s_of(int set) { return set ? adamsc1 + 4 : ctrl->adam_bc2s; }
  // (diagnostics: the parity that last ran; with policy_freq 2 policy and plain steps
  // alternate, so each kind always runs on the same parity)
  int pol_set = 0, pln_set = 0;
  const Graph& policy_graph() const { return g_pol[pol_set]; }
  const Graph& plain_graph() const { return algo == RLE_SAC ? g_pol[pol_set] : g_pln[pln_set]; }  // SAC: every step
  bool built = false;
  long long n_runs = 0;  // host mirror of the agent's step counter
  int cur_set = 0, last_set = 0;       // batch the next step runs on / the last step ran on
  bool primed = false;                 // batch cur_set holds the next step's draws
  unsigned long long primed_ver = 0;   // replay version it was drawn under
  // step buffers: two batch sets (the running step's and the prefetched next one)
  struct BatchSet {
    View ss, act_in, rw, nd, eps, eps2;
    long long* ind = nullptr;
    float* u_buf = nullptr;
    int ind_id = -1;
  };
  BatchSet bsets[2];
  View ss, act_in, rw, nd, eps, eps2;  // the set a program is being built on (use_set)
  long long* ind = nullptr;
  float* u_buf = nullptr;
  double* bsum = nullptr;
  void use_set(int k) {
    const BatchSet& b = bsets[k];
    ss = b.ss;
    act_in = b.act_in;
    rw = b.rw;
    nd = b.nd;
    eps = b.eps;
    eps2 = b.eps2;
    ind = b.ind;
    u_buf = b.u_buf;
    ind_id = b.ind_id;
  }
  // tapes
  float *t_u = nullptr, *t_eps = nullptr, *t_eps2 = nullptr;
  long long* t_ind = nullptr;
  long long tape_cap = 0, tape_left = 0;
  // act programs (cached per n)
  std::map<int, std::pair<Graph, View>> act_graphs;  // n -> graph, output view
  std::map<int, View> act_inputs;
  // act-sample programs (rle_act_sample): environment action straight into pinned memory
  struct ActSample {
    Graph G;
    View in;
    float* img = nullptr;  // pinned staging of the input image (N image, M rows)
    int* ctl = nullptr;    // pinned: mode, Philox counter lo / hi
    float* eps = nullptr;  // pinned [n][A] noise tape
    float* out = nullptr;  // pinned [n][A] actions
  };
  std::map<int, ActSample> act_samplers;
  // B = 1 act chain (one launch, in-kernel hand-offs): built on first use when it fits
  bool chain_tried = false, chain_ok = false;
  ActChainArgs chain{};
  unsigned chain_tag = 0;
  volatile unsigned* done_host = nullptr;  // pinned [64]: head workgroups' completion tags
  PinMem pin;
  float* act_map = nullptr;  // [scale A | bias A | exploration_noise] (rle_set_action_map)
  unsigned long long act_counter = 0;  // Philox counter of the exploration draws
  // The rle_act_chain program of this engine's actor (ops.h ActChainArgs), or false when it does
  // not fit (observation wider than 384, hidden wider than 256, LDS).
  bool build_chain(const ActArgs& ao) {
    ActChainArgs& c = chain;
    c = ActChainArgs{};
    if (Sp > 384) return false;
    auto layer = [&](const Layer& L, int act, int in0, int in1, int norm, int dst, int sync) {
      ActLayer& x = c.L[c.nl++];
      x.wn = P + L.wn_off;
      x.bias = P + L.b_off;
      x.cbn = L.cb;
      x.rbs = L.rb;
      x.out = L.out;
      x.act = act;
      x.in0 = in0;
      x.in1 = in1;
      x.k0 = L.seg_p.empty() ? 0 : L.seg_p[0];
      x.norm = norm;
      x.dst = dst;
      x.sync = sync;
      return L.K <= kActVec || in1 >= 0;
    };
    bool ok = true;
    if (algo == RLE_TD7) {  // td7.py:158-162: zs = fixed_encoder(s); policy(s, zs)
      Net& fe = net("fixed_encoder");
      Net& pi = net("policy");
      ok &= layer(fe.layers[0], actE, 0, -1, 0, 1, 0);
      ok &= layer(pi.layers[0], ACT_NONE, 0, -1, 1, 2, 1);
      ok &= layer(fe.layers[1], actE, 1, -1, 0, 3, 1);
      ok &= layer(fe.layers[2], ACT_NONE, 3, -1, 1, 4, 1);
      ok &= layer(pi.layers[1], actP, 2, 4, 0, 5, 1);
      ok &= layer(pi.layers[2], actP, 5, -1, 0, 6, 1);
      ok &= layer(pi.layers[3], ACT_TANH, 6, -1, 0, 7, 0);
    } else {  // mlp.py:55-68
      Net& pi = net("policy");
      const int D = (int)HS.size();  // (hidden layer i -> slot i + 1; the output -> slot 7)
      for (int i = 0; i < D; ++i) ok &= layer(pi.layers[i], actP, i, -1, 0, i + 1, 1);
      ok &= layer(pi.layers[D], algo == RLE_SAC ? ACT_NONE : ACT_TANH, D, -1, 0, 7, 0);
      c.sac = algo == RLE_SAC;
    }
    c.nwg = 1;
    for (int l = 0; l < c.nl; ++l) {
      ok &= c.L[l].out <= kActVec && c.L[l].cbn <= 32;  // (kernels.hip act_load: <= 8 blocks per lane)
    ok &= A <= 32;  // ActChainArgs::eps, one output per thread
      if (l < c.nl - 1) c.nwg = std::max(c.nwg, c.L[l].rbs);
    }
    c.heads = c.sac ? 1 : c.L[c.nl - 1].rbs;
    ok &= c.heads <= c.nwg;
    for (int l = 0; l < c.nl - 1; ++l) ok &= c.L[l].rbs == c.nwg;  // (every workgroup in every hidden layer)
    if (!ok) return false;
    c.Sp = Sp;
    c.xbuf = mem.make<unsigned long long>((size_t)kActMaxL * kActVec);
    c.err = const_cast<int*>(ao.ctl) + 8;  // pinned (ActSample::ctl[8], [9]): read by the host directly
    done_host = (volatile unsigned*)pin.alloc(64 * sizeof(unsigned));
    HIPCHK(hipHostGetDevicePointer((void**)&c.done, (void*)done_host, 0));
    c.ao = ao;
    c.min_log_std = cfg.min_log_std;
    c.max_log_std = cfg.max_log_std;
    const char* fw = std::getenv("RLE_ACT_FAIL_WG");  // failure-path test, first call only
    c.fail_wg = fw ? std::atoi(fw) : -1;
    return true;
  }
  void ensure_action_map() {  // default: identity map, exploration_noise 0.1 (td7.py:41, td3.py:40)
    if (act_map) return;
    std::vector<float> m((size_t)2 * A + 1, 0.f);
    for (int j = 0; j < A; ++j) m[j] = 1.f;
    m[2 * A] = 0.1f;
    act_map = mem.make<float>(m.size());
    HIPCHK(hipMemcpy(act_map, m.data(), m.size() * 4, hipMemcpyHostToDevice));
  }

  // ---------------------------------------------------------------- params
  Net& net(const std::string& name) {
    for (auto& n : nets)
      if (n.name == name) return n;
    throw Error{RLE_EINVAL, "unknown net '" + name + "'"};
  }

  void add_layer(Net& n, const std::string& pre, int out, std::vector<int> segw) {
    Layer L;
    L.wname = pre + ".weight";
    L.bname = pre + ".bias";
    L.out = out;
    L.seg_w = segw;
    // every input segment padded to 16 so a 16-wide reduction chunk never straddles two
    for (int w : segw) L.seg_p.push_back(r16(w));
    L.K = 0;
    for (int p : L.seg_p) L.K += p;
    L.res = next_id++;
    n.layers.push_back(L);
  }

  Net make_net(const std::string& name, const std::string& kind) {
    Net n;
    n.name = name;
    n.kind = kind;
    n.res = next_id++;
    if (kind == "sale_enc") {  // rl/nn/sale.py:16-55 (zs_dim Z, hdim H)
      add_layer(n, "zs1", H, {S});
      add_layer(n, "zs2", H, {H});
      add_layer(n, "zs3", Z, {H});
      add_layer(n, "zsa1", H, {Z, A});
      add_layer(n, "zsa2", H, {H});
      add_layer(n, "zsa3", Z, {H});
    } else if (kind == "sale_actor") {  // sale.py:58-83
      add_layer(n, "l0", H, {S});
      add_layer(n, "l1", H, {H, Z});
      add_layer(n, "l2", H, {H});
      add_layer(n, "l3", A, {H});
    } else if (kind == "sale_critic") {  // sale.py:86-121
      add_layer(n, "q01", H, {S, A});
      add_layer(n, "q1", H, {H, Z, Z});
      add_layer(n, "q2", H, {H});
      add_layer(n, "q3", 1, {H});
    } else {  // mlp_actor (mlp.py:38-55) / mlp_critic (mlp.py:75-101): Linear / ReLU pairs, nn.Sequential
      // indices 0, 2, 4, ... (make_mlp, mlp.py:24-35)
      const bool actor = kind == "mlp_actor";
      const int D = (int)HS.size();
      for (int i = 0; i <= D; ++i) {
        const int out = i < D ? HS[i] : !actor ? 1 : algo == RLE_SAC ? 2 * A : A;
        std::vector<int> in{i ? HS[i - 1] : S};
        if (!i && !actor) in.push_back(A);
        add_layer(n, "mlp." + std::to_string(2 * i), out, in);
      }
    }
    return n;
  }

  // Per layer: weight N image | weight T image | bias (padded to 16 rows); the
  // Adam m / v arenas mirror the layout at +nP / +2nP (m, v live at the T offsets).
  void layout_params() {
    size_t off = 0;
    for (auto& n : nets) {
      n.off = off;
      for (auto& L : n.layers) {
        L.rb = cdiv(L.out, 16);
        L.cb = L.K / 16;
        const size_t img = (size_t)L.rb * L.cb * 256;
        L.wn_off = off;
        L.wt_off = off + img;
        L.b_off = off + 2 * img;
        off += 2 * img + (size_t)L.rb * 16;
      }
      n.size = off - n.off;
    }
    nP = off + 4;  // + SAC log_alpha slot
    P = mem.make<float>(3 * nP);  // params | m | v
  }

  Mat wmat(const Layer& L, int which = 0) {
    Mat m{};
    m.n = P + (size_t)which * nP + L.wn_off;
    m.t = P + (size_t)which * nP + L.wt_off;
    m.cbn = L.cb;
    m.rbs = L.rb;
    return m;
  }
  float* bias(const Layer& L) { return P + L.b_off; }

  static size_t h_nidx(int cbn, int r, int c) {
    return ((size_t)(r >> 4) * cbn + (c >> 4)) * 256 + ((c >> 2) & 3) * 64 + (r & 15) * 4 + (c & 3);
  }
  static size_t h_tidx(int rbs, int r, int c) {
    return ((size_t)(c >> 4) * rbs + (r >> 4)) * 256 + ((r >> 2) & 3) * 64 + (c & 15) * 4 + (r & 3);
  }

  // locate (net, torch param name) -> (layer, is_bias)
  std::pair<Layer*, bool> find_param(const std::string& netn, const std::string& name) {
    Net& n = net(netn);
    for (auto& L : n.layers) {
      if (L.wname == name) return {&L, false};
      if (L.bname == name) return {&L, true};
    }
    throw Error{RLE_EINVAL, "unknown param '" + netn + "." + name + "'"};
  }

  long long numel(const std::string& netn, const std::string& name) {
    if (netn == "tmp") return 1;
    auto pr = find_param(netn, name);
    const Layer& L = *pr.first;
    if (pr.second) return L.out;
    long long k = 0;
    for (int w : L.seg_w) k += w;
    return (long long)L.out * k;
  }

  // copy between logical [out][sum seg_w] host layout and padded device layout
  void xfer_param(const std::string& netn, const std::string& name, float* host, long long n, bool to_dev,
                  int which) {
    REQUIRE(n == numel(netn, name), "size mismatch for " + netn + "." + name);
    const size_t base = (size_t)which * nP;
    HIPCHK(hipStreamSynchronize(stream));
    if (to_dev) fold_dirty = true;
    if (netn == "tmp") {
      float* d = P + base + (nP - 4);
      if (to_dev) HIPCHK(hipMemcpy(d, host, 4, hipMemcpyHostToDevice));
      else HIPCHK(hipMemcpy(host, d, 4, hipMemcpyDeviceToHost));
      return;
    }
    auto pr = find_param(netn, name);
    const Layer& L = *pr.first;
    if (pr.second) {
      float* d = P + base + L.b_off;
      if (to_dev) HIPCHK(hipMemcpy(d, host, sizeof(float) * L.out, hipMemcpyHostToDevice));
      else HIPCHK(hipMemcpy(host, d, sizeof(float) * L.out, hipMemcpyDeviceToHost));
      return;
    }
    // weights: both images written from the logical [out][sum seg_w] array (params);
    // read back from the T image (Adam m / v live only there)
    const size_t img = (size_t)L.rb * L.cb * 256;
    std::vector<float> tim(img, 0.f), nim(img, 0.f);
    float* dt = P + base + L.wt_off;
    float* dn = P + base + L.wn_off;
    int klog = 0;
    for (int w : L.seg_w) klog += w;
    if (!to_dev) HIPCHK(hipMemcpy(tim.data(), dt, img * 4, hipMemcpyDeviceToHost));
    for (int o = 0; o < L.out; ++o) {
      int lc = 0, pc = 0;
      for (size_t s = 0; s < L.seg_w.size(); ++s) {
        for (int c = 0; c < L.seg_w[s]; ++c) {
          float& hv = host[(size_t)o * klog + lc + c];
          const size_t ti = h_tidx(L.rb, o, pc + c);
          if (to_dev) {
            tim[ti] = hv;
            nim[h_nidx(L.cb, o, pc + c)] = hv;
          } else {
            hv = tim[ti];
          }
        }
        lc += L.seg_w[s];
        pc += L.seg_p[s];
      }
    }
    if (to_dev) {
      HIPCHK(hipMemcpy(dt, tim.data(), img * 4, hipMemcpyHostToDevice));
      if (which == 0) HIPCHK(hipMemcpy(dn, nim.data(), img * 4, hipMemcpyHostToDevice));
    }
  }

  // ---------------------------------------------------------------- buffers
  // Zero-initialised tensor images (rows and columns padded to 16; padding stays
  // zero, which the GEMM reduction relies on), or a dense vector.
  View buf(int rows, int cols, bool want_n = true, bool want_t = true) {
    View v;
    v.rows = r16(rows);
    v.cols = r16(cols);
    const size_t img = (size_t)v.rows * v.cols;
    v.m.cbn = v.cols / 16;
    v.m.rbs = v.rows / 16;
    if (want_n) v.m.n = mem.make<float>(img);
    if (want_t) v.m.t = mem.make<float>(img);
    v.rows = rows;
    v.id = next_id++;
    return v;
  }
  View vec(int rows) {
    View v;
    v.rows = rows;
    v.cols = 1;
    v.p = mem.make<float>((size_t)rows + 4);
    v.id = next_id++;
    return v;
  }

  // ---------------------------------------------------------------- op builders
  // Operand segments: N image (x = tensor rows, reduction along columns) or
  // T image (x = tensor columns, reduction along rows).
  static Seg seg_n(const View& v, int r0, int r1) {
    Seg s{};
    s.p = v.m.n;
    s.xs = v.m.cbn;
    s.x0 = 0;
    s.x1 = v.rows;
    s.r0 = r0;
    s.r1 = r1;
    s.norm = v.nref();
    return s;
  }
  static Seg seg_t(const View& v, int x0, int r0, int r1) {
    Seg s{};
    s.p = v.m.t;
    s.xs = v.m.rbs;
    s.x0 = x0;
    s.x1 = x0 + v.cols;
    s.r0 = r0;
    s.r1 = r1;
    s.norm = v.nref();
    return s;
  }

  // Y = act(X W^T + b) over concatenated input segments (each a list of row pieces).
  // The GEMM kernel wants every A segment to span the op's whole row range, so
  // row pieces split the op into one sub-op per row range (same level, disjoint
  // output rows).
  // A weight block for fwd(): N image of a [out][segment width] matrix (a column block
  // of a layer's weights, or a folded product) and the resource it belongs to.
  struct WSeg {
    const float* p;
    int xs, res;
  };
  WSeg wblock(const Layer& L, int col0) const {
    return {P + L.wn_off + (size_t)(col0 / 16) * 256, L.cb, L.res};
  }
  // Columns [col0, col0 + width) of a layer's weights as a GEMM A operand (N image).
  View wview_n(const Layer& L, int col0, int width) const {
    View v;
    v.m.n = P + L.wn_off + (size_t)(col0 / 16) * 256;
    v.m.cbn = L.cb;
    v.m.rbs = L.rb;
    v.rows = L.out;
    v.cols = r16(width);
    v.id = L.res;
    return v;
  }

  struct DxTerm {
    View dz;
    const Layer* L;  // weights of a layer (T image) ...
    int col0;
    const View* wv = nullptr;  // ... or of a derived [out][in] matrix (T image) when L is null
  };

  // A pre-GEMM (PreArgs) and the resources it reads, for fwd() / dx(): the consumer's A segment
  // a.seg is computed in-tile, so the view passed for that segment only gives its layout.
  struct PreUse {
    PreArgs a;
    std::vector<int> rd;
    int kind = 1;  // GemmArgs::has_pre: 1 pre-GEMM (actor output layer), 3 pre-layer, 4 pre-layer behind a2
    PreArgs a2{};  // (kind 4) the pre-GEMM computing the pre-layer's input segment a2.seg
  };
  // The critic loss head fused into the DX of critic n's last hidden layer (GemmArgs::has_pre 2)
  struct HeadUse {
    HeadArgs h;
    int n;
    std::vector<int> rd, wr;  // the head's resources (beyond the DX's own)
  };
  // The SAC actor rsample (OP_SAC_ACTOR) as the epilogue of its raw head GEMM (EPI_SACFWD)
  struct SacFwdUse {
    SacFwdArgs a;
    std::vector<int> rd, wr;
  };
  // The SAC actor backward (OP_SAC_ACTOR_BWD) as the epilogue of the DX producing da (EPI_SACBWD)
  struct SacBwdUse {
    SacBwdArgs a;
    std::vector<int> rd, wr;
  };
  // The actor's tanh output layer L over rows x (+ target smoothing noise) as a pre-GEMM
  // (sale.py:77-83 / mlp.py:55-62, td7.py:188-194, td3.py:154-158).
  PreUse pre_actor_fwd(const Layer& L, const View& x, const View* noise, int seg) {
    REQUIRE(L.out <= 32 && L.seg_p.size() == 1 && x.m.n && !x.norm, "pre: actor output layer operands");
    PreUse u{};
    PreArgs& p = u.a;
    p.mode = GEMM_FWD;
    p.A.seg[0] = seg_n(x, 0, L.K);
    p.A.nseg = 1;
    Seg w{};
    w.p = P + L.wn_off;
    w.xs = L.cb;
    w.x1 = L.out;
    w.r1 = L.K;
    p.B.seg[0] = w;
    p.B.nseg = 1;
    p.N = L.out;
    p.R = L.K;
    p.seg = seg;
    p.bias = bias(L);
    u.rd = {x.id, L.res};
    if (noise) {
      p.noise = noise->m;
      p.noise_sigma = cfg.target_policy_noise;
      p.noise_clip = cfg.noise_clip;
      u.rd.push_back(noise->id);
    }
    return u;
  }
  // SAC's raw head L over rows x, then the target rsample a' = tanh(mean + exp(clamp(log_std)) eps)
  // (sac.py:132-152), as a pre-GEMM of the target critics' first layer (GemmArgs::has_pre 5): the target
  // branch does not wait a level for the standalone EPI_SACFWD op, which still runs for the policy rows,
  // log pi and the backward.  Both reduce the raw head in one order (kernels.hip sacraw_*).
  PreUse pre_sac_fwd(const Layer& L, const View& x, const View& eps, int seg) {
    REQUIRE(L.out == 2 * A && L.out <= 48 && L.K <= 256 && L.seg_p.size() == 1 && x.m.n && !x.norm && eps.m.t,
            "pre: SAC raw head operands");
    PreUse u{};
    u.kind = 5;
    PreArgs& p = u.a;
    p.mode = GEMM_FWD;
    p.A.seg[0] = seg_n(x, 0, L.K);
    p.A.nseg = 1;
    Seg w{};
    w.p = P + L.wn_off;
    w.xs = L.cb;
    w.x1 = L.out;
    w.r1 = L.K;
    p.B.seg[0] = w;
    p.B.nseg = 1;
    p.N = L.out;
    p.R = L.K;
    p.seg = seg;
    p.sac_a = A;
    p.bias = bias(L);
    p.noise = eps.m;
    p.noise_sigma = cfg.min_log_std;
    p.noise_clip = cfg.max_log_std;
    u.rd = {x.id, L.res, eps.id};
    return u;
  }
  bool sac_pre() const { return fused(RLE_FUSE_SACPRE) && sac_fwd_fused() && 2 * A <= 48 && H <= 256; }
  // A small-K first layer L0 (ReLU, K <= 48: TD3 / SAC on low-dimensional observations) over the
  // input segments xs, recomputed in-tile by the layer after it (prelayer_fwd): one level fewer on
  // the critic and actor chains.  The standalone L0 output stays for its other readers (the
  // weight gradient, the ReLU mask of the input gradient).  RLE_NO_PRELAYER=1: off (tests, A/B).
  bool pl_src = false;  // (fwd) the layer being built is a pre-layer source
  // minimum tile width of a pre-GEMM consumer: each tile recomputes the actor output layer for its
  // 16 rows, so wider tiles cut that redundant work (A/B, RLE_PRE_TN 16 / 32 / 64: TD3 HalfCheetah
  // 23.37k / 23.79k / 23.91k, TD7 Humanoid 8069 / 8094 / 8060 steps/s)
  int pre_tn() const { return plan.pre_tn; }
  int pl_tn() const { return plan.pl_tn; }
  // (fusions whose in-tile recomputations are compiled for the default activations only; the q-dot partials and the
  // loss head fused into the DX also for ReLU / ELU critics -- the extended instance holds both -- not for identity)
  static constexpr unsigned kActFusions = RLE_FUSE_PRELAYER | RLE_FUSE_PRE | RLE_FUSE_TWOSTAGE | RLE_FUSE_SACPRE;
  static constexpr unsigned kCriticActFusions = RLE_FUSE_QDOT | RLE_FUSE_HEADDX;
  bool fused(unsigned bit) const {
    if (!acts_default && (bit & kActFusions)) return false;
    if (!acts_default && actC == ACT_NONE && (bit & kCriticActFusions)) return false;
    return (bit & RLE_FUSE_OPT_IN) ? (plan.fuse_on & bit) != 0 : !(plan.fuse_off & bit);
  }
  bool prelayer_shape(const Layer& L0, const Layer& L1) const {
    return L0.K <= 48 && L0.out <= 256 && L0.out % 16 == 0 && L1.seg_p.size() == 1 && L1.seg_p[0] == L0.out;
  }
  bool prelayer_ok(const Layer& L0, const Layer& L1) const {
    return fused(RLE_FUSE_PRELAYER) && prelayer_shape(L0, L1);
  }
  bool prelayer_ok_dx(const Layer& L, const Layer& Lprev) const {
    return fused(RLE_FUSE_PRELAYER) && r16(L.out) <= 48 && L.K <= 256 && L.K % 16 == 0 && Lprev.out == L.K &&
           Lprev.out <= 256;
  }
  // (lds_seg >= 0: input segment lds_seg is computed in-tile by a pre-GEMM -- its view gives the layout)
  PreUse pre_layer(const Layer& L0, const std::vector<View>& xs, int lds_seg = -1) {
    REQUIRE(xs.size() == L0.seg_p.size() && L0.K <= 48, "pre-layer: operands");
    PreUse u{};
    u.kind = 3;
    PreArgs& p = u.a;
    p.mode = GEMM_FWD;
    int koff = 0;
    for (size_t q = 0; q < xs.size(); ++q) {
      REQUIRE(xs[q].m.n && xs[q].cols == L0.seg_p[q] && !xs[q].norm, "pre-layer: input segment");
      p.A.seg[q] = seg_n(xs[q], koff, koff + L0.seg_p[q]);
      koff += L0.seg_p[q];
      if ((int)q != lds_seg) u.rd.push_back(xs[q].id);
    }
    p.A.nseg = (int)xs.size();
    Seg w{};
    w.p = P + L0.wn_off;
    w.xs = L0.cb;
    w.x1 = L0.out;
    w.r1 = L0.K;
    p.B.seg[0] = w;
    p.B.nseg = 1;
    p.N = L0.out;
    p.R = L0.K;
    p.seg = 0;
    p.act = ACT_RELU;
    p.bias = bias(L0);
    u.rd.push_back(L0.res);
    return u;
  }
  // The input gradient through layer L (small fan-out: L.out <= 48, e.g. SAC's raw head 2 x action
  // dims) masked by act'(saved), dZ W * act'(saved), recomputed in-tile by the input-gradient GEMM of
  // the layer before (prelayer_fwd, GEMM_DX).  The standalone op stays for the weight gradient.
  PreUse pre_layer_dx(const Layer& L, const View& dz, const View& saved) {
    REQUIRE(r16(L.out) <= 48 && dz.m.n && dz.cols == r16(L.out) && saved.m.t && L.K <= 256, "pre-layer dx: operands");
    PreUse u{};
    u.kind = 3;
    PreArgs& p = u.a;
    p.mode = GEMM_DX;
    p.A.seg[0] = seg_n(dz, 0, L.out);
    p.A.nseg = 1;
    Seg b{};
    b.p = P + L.wt_off;
    b.xs = L.rb;
    b.x1 = L.K;
    b.r1 = L.out;
    p.B.seg[0] = b;
    p.B.nseg = 1;
    p.N = L.K;
    p.R = r16(L.out);
    p.seg = 0;
    p.act = ACT_RELU;
    p.dsrc = saved.m;
    u.rd = {dz.id, L.res, saved.id};
    return u;
  }
  // The gradient wrt the actor's tanh input, sum_t dZ_t W_t[:, col0_t ..] * (1 - a^2), as a
  // pre-GEMM (the DX op dx(terms, ncols, ..., ACT_TANH, &a) would compute).
  PreUse pre_actor_dx(const std::vector<DxTerm>& terms, int ncols, const View& a, int seg) {
    REQUIRE(ncols <= 32 && a.m.t && (int)terms.size() <= kMaxSeg, "pre: actor output gradient operands");
    PreUse u{};
    PreArgs& p = u.a;
    p.mode = GEMM_DX;
    int roff = 0;
    for (size_t t = 0; t < terms.size(); ++t) {
      const DxTerm& tm = terms[t];
      REQUIRE(tm.L && tm.dz.m.n && tm.col0 % 16 == 0, "pre: dx term layout");
      p.A.seg[t] = seg_n(tm.dz, roff, roff + tm.L->out);
      Seg b{};
      b.p = P + tm.L->wt_off + (size_t)(tm.col0 / 16) * tm.L->rb * 256;
      b.xs = tm.L->rb;
      b.x1 = ncols;
      b.r0 = roff;
      b.r1 = roff + tm.L->out;
      p.B.seg[t] = b;
      roff += r16(tm.L->out);
      u.rd.push_back(tm.dz.id);
      u.rd.push_back(tm.L->res);
    }
    p.A.nseg = p.B.nseg = (int)terms.size();
    p.N = ncols;
    p.R = roff;
    p.seg = seg;
    REQUIRE(a.m.t, "pre: the saved tanh output needs a T image");
    p.dsrc = a.m;
    u.rd.push_back(a.id);
    return u;
  }

  View fwd(Prog& pg, const Layer& L, const std::vector<std::vector<View>>& ins, int M, int act, View* pre_out,
           bool normed, const View* noise = nullptr, int noise_row0 = 0, const std::vector<WSeg>* wsegs = nullptr,
           const View* bias_ovr = nullptr, const PreUse* pre = nullptr, const Layer* qdot = nullptr,
           bool pre_n = false, const SacFwdUse* sfu = nullptr) {
    REQUIRE(ins.size() == L.seg_p.size(), "fwd: input segment count mismatch for " + L.wname);
    REQUIRE(M % kTileM == 0, "fwd: rows must be a multiple of 16");
    REQUIRE(!wsegs || wsegs->size() == ins.size(), "fwd: one weight block per input segment");
    std::vector<int> rd{L.res}, wr;
    if (wsegs)
      for (const WSeg& w : *wsegs) rd.push_back(w.res);
    if (bias_ovr) rd.push_back(bias_ovr->id);
    std::vector<int> cuts{0, M};
    for (size_t s = 0; s < ins.size(); ++s) {
      int xo = 0;
      for (const View& v : ins[s]) {
        REQUIRE(v.cols == L.seg_p[s] && v.m.n, "fwd: segment width / image mismatch for " + L.wname);
        xo += v.rows;
        if (xo < M) cuts.push_back(xo);
        if (pre && (int)s == pre->a.seg) continue;  // computed in-tile
        rd.push_back(v.id);
        if (v.norm) rd.push_back(v.norm_id);
      }
      REQUIRE(xo >= M, "fwd: input rows < M");
    }
    std::sort(cuts.begin(), cuts.end());
    cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
    REQUIRE((int)ins.size() <= kMaxSeg, "fwd: too many operand segments");
    if (pre) {
      REQUIRE(cuts.size() == 2 && !noise, "fwd: a pre-GEMM consumer is one row piece");
      rd.insert(rd.end(), pre->rd.begin(), pre->rd.end());
    }
    const auto tq = choose_tn(M, L.out);
    // (EPI_SACFWD: one tile column holds whole rows; a pre-layer consumer recomputes the first layer
    // per tile, so wider tiles cut that redundant work: RLE_PL_TN, default 64)
    // (pl_src: this layer is also recomputed in-tile by a pre-layer consumer -- at most 32-wide tiles
    // keep its reduction split, so the stored output (the ReLU mask of the input gradient, the weight
    // gradient's operand) is the same floats as the consumer's copy, whatever the planner widens)
    // (a pre-GEMM consumer that is also a pre-layer source: at most 32 wide, as any pl_src)
    const int tn = sfu ? 64
                       : (pre && (pre->kind == 3 || pre->kind == 4) ? std::max(tq.first, pl_tn())
                          : pre && (pre->kind == 1 || pre->kind == 5)
                              ? (pl_src ? std::min(std::max(tq.first, pre_tn()), 32) : std::max(tq.first, pre_tn()))
                                                  : (pl_src ? std::min(tq.first, 32) : tq.first));
    // 64-row LDS-staged tiles (rle_plan wide): every row piece whole 64-row blocks, 64-column blocks
    bool wide = plan.wide && !sfu && !pre && !noise && L.out % plan.wide == 0;
    for (size_t ci = 0; wide && ci + 1 < cuts.size(); ++ci) wide = (cuts[ci + 1] - cuts[ci]) % 64 == 0;
    const int tn_w = wide ? plan.wide : tn;
    const int tiles_n = cdiv(L.out, tn_w);
    View out = buf(M, L.out, true, out_t);
    if (sfu) {
      REQUIRE(!pre && !qdot && !normed && !noise && act == ACT_NONE && L.out <= 64, "fwd: SAC forward epilogue");
      rd.insert(rd.end(), sfu->rd.begin(), sfu->rd.end());
      wr.insert(wr.end(), sfu->wr.begin(), sfu->wr.end());
    }
    wr.push_back(out.id);
    if (pre_out) {
      // T: DX epilogue masks; N (pre_n) only where the loss head reads the rows: 4 scattered
      // stores per lane saved everywhere else
      *pre_out = buf(M, L.out, pre_n, true);
      wr.push_back(pre_out->id);
    }
    float* part = nullptr;
    if (normed) {
      part = mem.make<float>((size_t)tiles_n * M);
      out.norm = part;
      out.norm_ld = M;
      out.norm_row0 = 0;
      out.nparts = tiles_n;
      out.width = L.out;
      out.norm_id = next_id++;
      wr.push_back(out.norm_id);
    }
    float* qpart = nullptr;
    if (qdot) {  // EPI_QDOT: row partials of the H -> 1 layer qdot applied to this output
      REQUIRE(!normed && qdot->out == 1 && qdot->K == L.out && (act == ACT_ELU || act == ACT_RELU),
              "fwd: q-dot partial layout");
      qpart = mem.make<float>((size_t)tiles_n * M);
      out.qd = qpart;
      out.qd_ld = M;
      out.qd_n = tiles_n;
      out.qd_id = next_id++;
      wr.push_back(out.qd_id);
      rd.push_back(qdot->res);
    }
    if (noise) rd.push_back(noise->id);
    std::vector<Op> ops;
    for (size_t ci = 0; ci + 1 < cuts.size(); ++ci) {
      const int ra = cuts[ci], rb = cuts[ci + 1], m = rb - ra;
      REQUIRE(ra % kTileM == 0, "fwd: row pieces must be 16-aligned");
      Op op{};
      op.kind = OP_GEMM;
      GemmArgs& g = op.gemm;
      g.mode = GEMM_FWD;
      int koff = 0;
      for (size_t s = 0; s < ins.size(); ++s) {
        int xo = 0;
        for (const View& v : ins[s]) {
          if (ra >= xo && ra < xo + v.rows) {
            g.A.seg[s] = seg_n(v.sub(ra - xo, m), koff, koff + L.seg_p[s]);
            break;
          }
          xo += v.rows;
        }
        koff += L.seg_p[s];
      }
      g.A.nseg = (int)ins.size();
      if (!wsegs) {
        Seg w{};
        w.p = P + L.wn_off;
        w.xs = L.cb;
        w.x0 = 0;
        w.x1 = L.out;
        w.r0 = 0;
        w.r1 = L.K;
        g.B.seg[0] = w;
        g.B.nseg = 1;
      } else {  // one weight block per input segment, paired like a DX operand
        for (size_t q = 0; q < ins.size(); ++q) {
          Seg w{};
          w.p = (*wsegs)[q].p;
          w.xs = (*wsegs)[q].xs;
          w.x0 = 0;
          w.x1 = L.out;
          w.r0 = g.A.seg[q].r0;
          w.r1 = g.A.seg[q].r1;
          g.B.seg[q] = w;
        }
        g.B.nseg = (int)ins.size();
      }
      g.M = m;
      g.N = L.out;
      g.R = L.K;
      g.tn = tn_w;
      g.hot.wide = wide ? plan.wide : 0;
      g.tiles_m = cdiv(m, kTileM);
      g.tiles_n = tiles_n;
      g.epi = EPI_STORE;
      g.act = act;
      g.out = out.sub(ra, m).m;
      g.bias = bias_ovr ? bias_ovr->p : bias(L);
      if (pre_out) g.pre = pre_out->sub(ra, m).m;
      if (normed) {
        g.norm_out = part + ra;
        g.norm_ld = M;
      }
      if (sfu) {
        REQUIRE(cuts.size() == 2, "fwd: SAC forward epilogue over one row piece");
        g.epi = EPI_SACFWD;
        g.sf = sfu->a;
      }
      if (qdot) {
        g.epi = EPI_QDOT;
        g.qw = P + qdot->wn_off;
        g.qw_cbn = qdot->cb;
        g.norm_out = qpart + ra;
        g.norm_ld = M;
      }
      if (noise && rb > noise_row0) {
        const int first = std::max(ra, noise_row0);  // first noised row (global)
        g.noise = noise->sub(first - noise_row0, rb - first).m;
        g.noise_row0 = first - ra;
        g.noise_sigma = cfg.target_policy_noise;
        g.noise_clip = cfg.noise_clip;
      }
      if (pre) {
        g.has_pre = pre->kind;
        g.prea = pre->a;
        if (pre->kind == 4) g.prea2 = pre->a2;
      }
      op.wg_count = (wide ? g.tiles_m / 4 : g.tiles_m) * g.tiles_n;
      op.seq = tq.second;
      ops.push_back(op);
    }
    pg.add_group(std::move(ops), rd, wr);
    return out;
  }


  // dX[:, 0:ncols] = sum_t dZ_t W_t[:, col0_t : col0_t + ncols]  (* act'(saved))
  View dx(Prog& pg, const std::vector<DxTerm>& terms, int ncols, int M, int dact, const View* saved,
          const View* into = nullptr, const View* nb_x = nullptr, const PreUse* pre = nullptr,
          const HeadUse* head = nullptr, const SacBwdUse* sbu = nullptr) {
    if (dact == ACT_NONE && !pre && !head) saved = nullptr;  // (an identity layer's backward reads no derivative)
    Op op{};
    op.kind = OP_GEMM;
    GemmArgs& g = op.gemm;
    g.mode = GEMM_DX;
    std::vector<int> rd, wr;
    REQUIRE((int)terms.size() <= kMaxSeg, "dx: too many terms");
    int roff = 0;
    for (size_t t = 0; t < terms.size(); ++t) {
      const DxTerm& tm = terms[t];
      REQUIRE(tm.dz.m.n && tm.col0 % 16 == 0 && (tm.L || (tm.wv && tm.wv->m.t)), "dx: operand layout");
      const int wout = tm.L ? tm.L->out : tm.wv->rows;
      g.A.seg[t] = seg_n(tm.dz, roff, roff + wout);
      Seg b{};  // W[:, col0 : col0 + ncols] through the T image
      if (tm.L) {
        b.p = P + tm.L->wt_off + (size_t)(tm.col0 / 16) * tm.L->rb * 256;
        b.xs = tm.L->rb;
      } else {
        b.p = tm.wv->m.t + (size_t)(tm.col0 / 16) * tm.wv->m.rbs * 256;
        b.xs = tm.wv->m.rbs;
      }
      b.x0 = 0;
      b.x1 = ncols;
      b.r0 = roff;
      b.r1 = roff + wout;
      g.B.seg[t] = b;
      roff += r16(wout);
      if (!(pre && (int)t == pre->a.seg)) rd.push_back(tm.dz.id);  // (else computed in-tile)
      rd.push_back(tm.L ? tm.L->res : tm.wv->id);
    }
    g.A.nseg = g.B.nseg = (int)terms.size();
    g.M = M;
    g.N = ncols;
    g.R = roff;
    const auto tq = choose_tn(M, ncols);
    g.tn = pre && pre->kind == 3 ? std::max(tq.first, pl_tn())
           : pre && pre->kind == 1 ? std::max(tq.first, pre_tn())
                                   : (pl_src ? std::min(tq.first, 32) : tq.first);
    op.seq = tq.second;
    // 64-row LDS-staged tiles (rle_plan wide): a plain or EPI_NBDOT input gradient over whole 64-row blocks
    const bool wide = plan.wide && !pre && !head && !sbu && M % 64 == 0 && ncols % plan.wide == 0;
    if (wide) g.tn = plan.wide;
    g.hot.wide = wide ? plan.wide : 0;
    g.tiles_m = cdiv(M, kTileM);
    g.tiles_n = cdiv(ncols, g.tn);
    g.epi = EPI_STORE;
    g.act = ACT_NONE;
    View out = into ? *into : buf(M, ncols, out_n, out_t);
    if (nb_x) {  // out = g of AvgL1Norm(x): row partials of sum_j g x for the consuming DW (kDwNb)
      REQUIRE(!saved && nb_x->norm && nb_x->m.t && nb_x->rows == M && nb_x->cols == r16(ncols),
              "dx: deferred AvgL1Norm backward operands");
      g.epi = EPI_NBDOT;
      g.nbx = nb_x->m;
      float* part = mem.make<float>((size_t)cdiv(ncols, kTileM) * M);  // any tile plan fits
      g.norm_out = part;
      g.norm_ld = M;
      out.nbdot = part;
      out.nbdot_ld = M;
      out.nbdot_n = g.tiles_n;
      out.nbdot_id = next_id++;
      wr.push_back(out.nbdot_id);
      rd.push_back(nb_x->id);
    }
    REQUIRE(!into || (into->rows == M && into->cols == r16(ncols)), "dx: output view shape");
    g.out = out.m;
    if (saved) {
      REQUIRE(saved->m.t, "dx: derivative source needs a T image");
      g.dact = dact;
      g.dsrc = saved->m;
      rd.push_back(saved->id);
    }
    wr.push_back(out.id);
    if (pre) {
      g.has_pre = pre->kind;
      g.prea = pre->a;
      rd.insert(rd.end(), pre->rd.begin(), pre->rd.end());
    }
    if (head) {  // A segment 0 is z of critic head->n's last hidden layer, not dZ
      g.has_pre = 2;
      g.hd = head->h;
      g.head_n = head->n;
      rd.insert(rd.end(), head->rd.begin(), head->rd.end());
      wr.insert(wr.end(), head->wr.begin(), head->wr.end());
    }
    if (sbu) {  // the output is sbu->a.dout (d / d(mean | log_std)), not da
      REQUIRE(!head && !pre && !nb_x && !saved, "dx: SAC backward epilogue is a plain DX");
      g.epi = EPI_SACBWD;
      g.out = Mat{};
      g.sb = sbu->a;
      rd.insert(rd.end(), sbu->rd.begin(), sbu->rd.end());
      wr.insert(wr.end(), sbu->wr.begin(), sbu->wr.end());
    }
    op.wg_count = (wide ? g.tiles_m / 4 : g.tiles_m) * g.tiles_n;
    pg.add(op, rd, wr);
    return out;
  }

  // Tile width of the next GEMM op: from the plan of a previous build pass
  // (capture() widens tiles of levels that exceed one resident wave of
  // workgroups), else the per-op default.  Returns the op's creation index too.
  std::vector<int> tn_plan;
  int tn_seq = 0;
  std::pair<int, int> choose_tn(int M, int N) {
    const int seq = tn_seq++;
    const int t = seq < (int)tn_plan.size() ? tn_plan[seq] : pick_tn(M, N);
    return {t, seq};
  }
  // per-tile grad-square partial slots of a dW op (weights at the narrowest tile width,
  // so any plan fits; unused slots stay zero; bias)
  static int dw_gsq_w(const Layer& L) { return cdiv(L.out, kTileM) * cdiv(L.K, 16); }
  static int dw_gsq_b(const Layer& L) { return cdiv(L.out, kTileM); }

  // dW = dZ^T [X], db = sum dZ, fused Adam (torch.optim.Adam law).
  void dw(Prog& pg, const Layer& L, const View& dz, const std::vector<View>& X, int Brows, int cnt, float lr,
          float* gsq = nullptr, float* gsq_b = nullptr, const View* nb_x = nullptr) {
    REQUIRE(X.size() == L.seg_p.size(), "dw: input count mismatch for " + L.wname);
    REQUIRE(dz.m.t, "dw: dZ needs a T image");
    Op op{};
    op.kind = OP_GEMM;
    GemmArgs& g = op.gemm;
    g.mode = GEMM_DW;
    std::vector<int> rd{dz.id, L.res, asc_set ? R_ADAMSC1 : R_ADAMSC}, wr{L.res};
    g.A.seg[0] = seg_t(dz, 0, 0, Brows);
    g.A.nseg = 1;
    int koff = 0;
    for (size_t s = 0; s < X.size(); ++s) {
      const View& v = X[s];
      REQUIRE(v.cols == L.seg_p[s] && v.rows >= Brows && v.m.t, "dw: input view mismatch for " + L.wname);
      g.B.seg[s] = seg_t(v, koff, 0, Brows);
      if (v.norm && fused(RLE_FUSE_NORMFIN)) {  // (the finalized row means, norm_fin)
        const auto f = norm_fin(pg, v);
        g.B.seg[s].norm = f.first;
        rd.push_back(f.second);
      } else if (v.norm) {
        rd.push_back(v.norm_id);
      }
      rd.push_back(v.id);
      koff += L.seg_p[s];
    }
    g.B.nseg = (int)X.size();
    g.M = L.out;
    g.N = L.K;
    g.R = Brows;
    const auto tq = choose_tn(L.out, L.K);
    g.tn = tq.first;
    op.seq = tq.second;
    g.tiles_m = cdiv(L.out, kTileM);
    g.tiles_n = cdiv(L.K, g.tn) + 1;
    g.epi = EPI_ADAM;
    AdamArgs& ad = g.adam;
    ad.w = wmat(L);
    ad.b = bias(L);
    ad.mo = (long long)nP;
    ad.vo = 2LL * (long long)nP;
    ad.step = adam_step_of(asc_set) + cnt;
    ad.bc2s = adam_bc2s_of(asc_set) + cnt;
    ad.lr = lr;
    ad.beta1 = 0.9f;
    ad.beta2 = 0.999f;
    ad.omb1 = (float)(1.0 - 0.9);
    ad.omb2 = (float)(1.0 - 0.999);
    ad.eps = 1e-8f;
    ad.bias_col = cdiv(L.K, g.tn) * g.tn;
    ad.gsq = gsq;
    ad.gsq_b = gsq_b;
    ad.ptau = adam_ptau;
    if (nb_x) {  // dZ = AvgL1Norm backward of (dz = g, x), applied on load (kDwNb)
      REQUIRE(dz.nbdot && nb_x->norm && nb_x->m.t && nb_x->rows >= Brows, "dw: deferred AvgL1Norm backward operands");
      g.act = kDwNb;
      g.nbx = nb_x->m;
      g.nbx_xs = nb_x->m.rbs;
      g.nbm = nb_x->nref();
      g.nbdot = dz.nbdot;
      g.nbdot_ld = dz.nbdot_ld;
      g.nbdot_n = dz.nbdot_n;
      rd.push_back(nb_x->id);
      if (fused(RLE_FUSE_NORMFIN)) {  // (the finalized row means, norm_fin; x's width for the sign term)
        const auto f = norm_fin(pg, *nb_x);
        g.nbm = f.first;
        g.nb_width = nb_x->width;
        rd.push_back(f.second);
      } else {
        rd.push_back(nb_x->norm_id);
      }
      rd.push_back(dz.nbdot_id);
    }
    op.wg_count = g.tiles_m * g.tiles_n;
    pg.add(op, rd, wr);
  }

  // (TD3 policy steps) tau of the self-aliased target-policy Polyak fused into the actor's Adam
  // epilogues (AdamArgs::ptau), 0 elsewhere
  float adam_ptau = 0.f;
  // (plan without RLE_FUSE_PIPOLYAK: the standalone OP_POLYAK over the policy instead, tests, A/B)
  bool pi_polyak_fused() const { return fused(RLE_FUSE_PIPOLYAK); }

  // The AvgL1Norm means of a normed view's rows (sale.py:11-13: mean |x| before the 1e-8 clamp), computed once
  // from its producer's partials by a finalize op (OP_NORMBWD fwd 2, the level after the producer), for the
  // weight gradients: their tables cover every batch row and would otherwise sum every row's partials in every
  // workgroup (B = 1024: 4 rows per thread, 16 partials each, 3-7 us per workgroup).  Returned as a one-partial
  // NormRef of width 1 (the consumer's sum / 1 and clamp are the same floats) and its resource id; one op per
  // producer output per program.
  std::pair<NormRef, int> norm_fin(Prog& pg, const View& v) {
    REQUIRE(v.norm && v.norm_ld > 0, "norm_fin: not a normed view");
    auto it = pg.norm_fins.find(v.norm);
    if (it == pg.norm_fins.end()) {
      Op op{};
      op.kind = OP_NORMBWD;
      NormBwdArgs& a = op.nb;
      a.fwd = 2;
      a.rows = v.norm_ld;  // (the producer's rows: partials are [nparts][norm_ld])
      a.width = v.width;
      a.norm.part = v.norm;
      a.norm.ld = v.norm_ld;
      a.norm.row0 = 0;
      a.norm.nparts = v.nparts;
      a.norm.width = v.width;
      a.mout = mem.make<float>((size_t)v.norm_ld);
      op.wg_count = cdiv(v.norm_ld, kThreads);
      const int id = next_id++;
      pg.add(op, {v.norm_id}, {id});
      it = pg.norm_fins.emplace(v.norm, std::make_pair(a.mout, id)).first;
    }
    NormRef r{};
    r.part = it->second.first;
    r.ld = v.norm_ld;
    r.row0 = v.norm_row0;
    r.nparts = 1;
    r.width = 1;
    return {r, it->second.second};
  }

  View normbwd(Prog& pg, const View& gv, const View& x) {
    REQUIRE(x.norm, "normbwd: x is not a normed view");
    REQUIRE(gv.m.n && x.m.n && gv.rows % 16 == 0, "normbwd: operand layout");
    Op op{};
    op.kind = OP_NORMBWD;
    NormBwdArgs& a = op.nb;
    View out = buf(gv.rows, x.width, out_n, out_t);
    a.g = gv.m;
    a.x = x.m;
    a.dx = out.m;
    a.rows = gv.rows;
    a.width = x.width;
    a.norm = x.nref();
    op.wg_count = cdiv(gv.rows, 4);
    pg.add(op, {gv.id, x.id, x.norm_id}, {out.id});
    return out;
  }

  // AvgL1Norm itself (sale.py:11-13) applied to a normed view: out = x / m (OP_NORMBWD with
  // fwd = 1).  Only diagnostics read a normed tensor explicitly; the step defers the norm.
  View normfwd(Prog& pg, const View& x) {
    REQUIRE(x.norm && x.m.n && x.rows % 16 == 0, "normfwd: x is not a normed view");
    Op op{};
    op.kind = OP_NORMBWD;
    NormBwdArgs& a = op.nb;
    View out = buf(x.rows, x.width);
    a.g = x.m;
    a.x = x.m;
    a.dx = out.m;
    a.rows = x.rows;
    a.width = x.width;
    a.norm = x.nref();
    a.fwd = 1;
    op.wg_count = cdiv(x.rows, 4);
    pg.add(op, {x.id, x.norm_id}, {out.id});
    return out;
  }

  // SALEEncoder.encode_state (sale.py:41-46): a normed view (consumers apply the norm).
  View enc_zs(Prog& pg, Net& E, const View& s, int M) {
    View h1 = fwd(pg, E.layers[0], {{s}}, M, actE, nullptr, false);
    View h2 = fwd(pg, E.layers[1], {{h1}}, M, actE, nullptr, false);
    return fwd(pg, E.layers[2], {{h2}}, M, ACT_NONE, nullptr, true);
  }
  // SALEEncoder.encode_state_action (sale.py:48-55).
  View enc_zsa(Prog& pg, Net& E, const View& zs, const View& a, int M) {
    View a1 = fwd(pg, E.layers[3], {{zs}, {a}}, M, actE, nullptr, false);
    View a2 = fwd(pg, E.layers[4], {{a1}}, M, actE, nullptr, false);
    return fwd(pg, E.layers[5], {{a2}}, M, ACT_NONE, nullptr, false);
  }

  // make_mlp forward (mlp.py:24-35): `act` (action_fn) after every hidden layer, `last` after the output layer.
  View mlp_fwd(Prog& pg, Net& N, const std::vector<std::vector<View>>& in, int M, int last, int act) {
    View h;
    for (size_t i = 0; i < N.layers.size(); ++i)
      h = fwd(pg, N.layers[i], i ? std::vector<std::vector<View>>{{h}} : in, M,
              i + 1 == N.layers.size() ? last : act, nullptr, false);
    return h;
  }

  // Host rows [n][w] into every kept image of v (rows past n and columns past w stay zero).
  void upload(const View& v, const float* host, int n, int w) {
    const size_t img = (size_t)v.m.rbs * 16 * v.m.cbn * 16;
    if (v.m.n) {
      std::vector<float> buf_n(img, 0.f);
      for (int i = 0; i < n; ++i)
        for (int c = 0; c < w; ++c) buf_n[h_nidx(v.m.cbn, i, c)] = host[(size_t)i * w + c];
      HIPCHK(hipMemcpyAsync(v.m.n, buf_n.data(), img * 4, hipMemcpyHostToDevice, stream));
      HIPCHK(hipStreamSynchronize(stream));
    }
    if (v.m.t) {
      std::vector<float> buf_t(img, 0.f);
      for (int i = 0; i < n; ++i)
        for (int c = 0; c < w; ++c) buf_t[h_tidx(v.m.rbs, i, c)] = host[(size_t)i * w + c];
      HIPCHK(hipMemcpyAsync(v.m.t, buf_t.data(), img * 4, hipMemcpyHostToDevice, stream));
      HIPCHK(hipStreamSynchronize(stream));
    }
  }
  // Rows [n][w] of v's T image to the host (syncs the engine stream).
  void download(const View& v, float* host, int n, int w) {
    std::vector<float> res((size_t)v.m.rbs * 16 * v.m.cbn * 16);
    HIPCHK(hipMemcpyAsync(res.data(), v.m.t, res.size() * 4, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    for (int i = 0; i < n; ++i)
      for (int c = 0; c < w; ++c) host[(size_t)i * w + c] = res[h_tidx(v.m.rbs, i, c)];
  }

  // Diagnostic forward programs (rle_eval, rle_sac_rsample), captured once per shape.
  struct EvalGraph {
    Graph G;
    View in0, in1, out;
    float* out_vec = nullptr;
    int width = 0;
  };
  std::map<std::string, EvalGraph> eval_graphs;

  // polyak / copy over a whole net range
  void flat(Prog& pg, int kind, Net& dst, Net* src, float tau, bool self_alias) {
    Op op{};
    op.kind = kind;
    FlatArgs& f = op.flat;
    f.dst = P + dst.off;
    f.src = src ? P + src->off : P + dst.off;
    f.n = (long long)dst.size;
    f.tau = tau;
    f.omt = 1.f - tau;  // fp32(1 - tau) as torch casts the python scalar (Q2)
    f.self_alias = self_alias ? 1 : 0;
    op.wg_count = cdiv(f.n, (long long)kThreads * 4);
    std::vector<int> rd{dst.res}, wr{dst.res};
    for (auto& L : dst.layers) {
      rd.push_back(L.res);
      wr.push_back(L.res);
    }
    if (src) {
      rd.push_back(src->res);
      for (auto& L : src->layers) rd.push_back(L.res);
    }
    pg.add(op, rd, wr);
  }

  // ---------------------------------------------------------------- step programs
  // The previous step's LAP priority update, applied by the sampler (SampleArgs::pend_*)
  struct PendUpd {
    const long long* ind;
    const float* p;
    int ind_id, p_id;
  };
  void add_sampling(Prog& pg, bool sac, int ahead, const PendUpd* pu = nullptr) {
    // LAP block sums are maintained by every priority write (OP_PRIORITY, appends)
    Op op{};
    op.kind = OP_SAMPLE_GATHER;
    fill_sample_args(op.sample, sac);
    op.sample.ahead = ahead;
    op.wg_count = cdiv(Bv, 4);  // one wave per query
    // reads the RNG step / tape position counters -> ordered before STEP_END (WAR)
    std::vector<int> rd{bsum_id, R_PRIO, R_REPLAY, R_CNT};
    if (pu) {
      op.sample.pend_ind = pu->ind;
      op.sample.pend_p = pu->p;
      op.sample.pend_n = Bv;
      rd.push_back(pu->ind_id);
      rd.push_back(pu->p_id);
    }
    pg.add(op, rd, {ss.id, act_in.id, rw.id, nd.id, ind_id});
    Op nz{};
    nz.kind = OP_NOISE;
    fill_sample_args(nz.sample, sac);
    nz.sample.ahead = ahead;
    nz.wg_count = cdiv(Bv * A, kThreads);
    pg.add(nz, {R_CNT}, {eps.id, sac ? eps2.id : -1});
  }
  int bsum_id = -1, ind_id = -1;

  void fill_sample_args(SampleArgs& s, bool sac) {
    Replay& rp = *replay;
    s.state = rp.state;
    s.next_state = rp.next_state;
    s.action = rp.action;
    s.reward = rp.reward;
    s.notdone = rp.notdone;
    s.priority = rp.priority;
    s.S = S;
    s.Sp = Sp;
    s.A = A;
    s.Ap = Ap;
    s.size = rp.size_d;
    s.cap = rp.cap;
    s.lap = rp.lap;
    s.B = B;
    s.nq = Bv;
    s.bsum = rp.bsum;
    s.ssum = rp.ssum;
    s.nblk = rp.nblk;
    s.ss = ss.m;
    s.a = act_in.m;
    s.r = rw.p;
    s.nd = nd.p;
    s.ind = ind;
    s.u_out = u_buf;
    s.eps = eps.m;
    if (sac) s.eps2 = eps2.m;
    s.ctrl_rng = &ctrl->counters[4];
    s.seed = cfg.seed;
    s.tape_mode = &ctrl->tape_mode;
    s.tape_pos = &ctrl->counters[5];
    s.tape_u = t_u;
    s.tape_eps = t_eps;
    s.tape_eps2 = t_eps2;
    s.tape_ind = t_ind;
  }

  Op head_op(int mode, int rows) {
    Op op{};
    op.kind = OP_HEAD;
    HeadArgs& h = op.head;
    h.mode = mode;
    h.rows = rows;
    h.H = H;
    h.gamma = cfg.discount;
    h.inv_b = 1.f / (float)Bv;
    h.nvalid = Bv;
    h.tgt_mode = -1;
    op.wg_count = cdiv(rows, 4);
    return op;
  }

  // The target twins' last layer fused into a *_LOSS head (HeadArgs::tgt_mode).
  void set_head_target(HeadArgs& h, int mode, const View& t1, const View& t2, const Layer& l1, const Layer& l2) {
    REQUIRE(t1.m.n && t2.m.n && l1.out == 1 && l2.out == 1 && l1.cb == h.w_cbn, "head: target operand layout");
    h.tgt_mode = mode;
    h.th[0] = t1.m;
    h.th[1] = t2.m;
    h.tw[0] = P + l1.wn_off;
    h.tw[1] = P + l2.wn_off;
    h.tb[0] = bias(l1);
    h.tb[1] = bias(l2);
  }

  void set_head_twin(HeadArgs& h, const View& h1, const View& h2, const Layer& l1, const Layer& l2) {
    REQUIRE(h1.m.n && h2.m.n && l1.out == 1 && l2.out == 1, "head: operand layout");
    h.h[0] = h1.m;
    h.h[1] = h2.m;
    h.w[0] = P + l1.wn_off;
    h.w[1] = P + l2.wn_off;
    h.w_cbn = l1.cb;
    h.b[0] = bias(l1);
    h.b[1] = bias(l2);
  }

  Op step_end_op() {
    Op op{};
    op.kind = OP_STEP_END;
    StepEndArgs& a = op.end;
    a.counters = ctrl->counters;
    a.info_slot = &ctrl->info_slot;
    a.info = info;
    a.info_cap = info_cap;
    a.inv_b = 1.f / (float)Bv;
    op.wg_count = 1;
    return op;
  }

  void info_sum(StepEndArgs& a, int k, const float* part, int n, int stride, float scale) {
    a.part[k] = part;
    a.npart[k] = n;
    a.stride[k] = stride;
    a.scale[k] = scale;
    a.kind[k] = INFO_SUM;
  }

  // STEP_END writes the info row and bumps the step counters; every reader of a
  // counter (Adam t, RNG step, tape position) is therefore scheduled before it.
  // Split in two (plan without RLE_FUSE_ENDSPLIT: one op): the counters (+ the SAC temperature update), which
  // the next step reads, at the step's end; the info row, which only the host reads, after it,
  // free to sit under a longer op (the rebalance pass's one-workgroup rule).
  float* sac_scr = nullptr;
  int sac_scr_id = -1;
  bool end_split() const { return fused(RLE_FUSE_ENDSPLIT); }
  void add_step_end(Prog& pg, Op op, std::vector<int> rd, const std::vector<int>& counters) {
    StepEndArgs& a = op.end;
    a.cmask = 0;
    for (int c : counters) a.cmask |= 1 << c;
    const std::vector<int> rd_info = rd;  // (the info op does not touch the counters)
    rd.push_back(R_CNT);
    if (!end_split()) {
      std::vector<int> wr{R_INFO, R_CNT};
      if (a.log_alpha) wr.push_back(R_LA);
      pg.add(op, rd, wr);
      return;
    }
    const bool sac_tmp = a.log_alpha && a.la_lr > 0.f;
    if (sac_tmp && !sac_scr) {
      sac_scr = mem.make<float>(4);
      sac_scr_id = next_id++;
    }
    Op c = op, i = op;
    c.end.mode = 1;
    c.end.sac_scratch = sac_tmp ? sac_scr : nullptr;
    std::vector<int> cw{R_CNT};
    if (a.log_alpha) cw.push_back(R_LA);
    if (sac_tmp) cw.push_back(sac_scr_id);
    pg.add(c, rd, cw);
    i.end.mode = 2;
    i.end.cmask = 0;
    i.end.sac_scratch = sac_tmp ? sac_scr : nullptr;
    std::vector<int> ir = rd_info;
    if (sac_tmp) ir.push_back(sac_scr_id);
    else if (a.log_alpha) ir.push_back(R_LA);  // (fixed temperature: read, never written)
    pg.add(i, ir, {R_INFO});
  }

  // TD7 (td7.py:287-332)
  // Next step's batch into the other buffer set, after this step's priority update
  // (RAW on the priorities) and before STEP_END bumps the counters (WAR).
  void add_prefetch(Prog& pg, bool sac, int set, const PendUpd* pu = nullptr) {
    use_set(1 - set);
    add_sampling(pg, sac, 1, pu);
    use_set(set);
  }
  // LAPReplayMemory.update_priority (lap.py:66-69) of this step's batch, then the next step's batch.
  // Fused (RLE_FUSE_PRIOSAMPLE): the sampler applies the update to what its search reads, and the
  // OP_PRIORITY that persists it runs after the sampler, off the step-to-step chain.
  bool prio_sample_fused() const {
    int ns = 64;  // (kernels.hip pend_prepare's LDS layout, within rle_level's 24 KB)
    while (ns < 2 * B) ns <<= 1;
    return fused(RLE_FUSE_PRIOSAMPLE) && replay->lap && B <= 1024 &&
           std::max(8 * ns, 20 * B) + 12 * replay->nblk <= 24 * 1024;
  }
  void add_update_and_prefetch(Prog& pg, bool sac, int set, bool lap, const View& prio) {
    Op op{};
    op.kind = OP_PRIORITY;
    op.prio.priority = replay->priority;
    op.prio.ind = ind;
    op.prio.p = prio.p;
    op.prio.B = Bv;
    op.prio.max_priority = replay->maxp_d;
    op.prio.bsum = replay->lap ? replay->bsum : nullptr;
    op.prio.ssum = replay->ssum;
    op.wg_count = 1;
    const std::vector<int> rd{prio.id, ind_id}, wr{R_PRIO, R_MAXP, bsum_id};
    if (!lap) {
      add_prefetch(pg, sac, set);
    } else if (prio_sample_fused()) {
      const PendUpd pu{ind, prio.p, ind_id, prio.id};
      add_prefetch(pg, sac, set, &pu);
      pg.add(op, rd, wr);
    } else {
      pg.add(op, rd, wr);
      add_prefetch(pg, sac, set);
    }
  }
  void build_prime(Prog& pg, bool sac, int set) {
    use_set(set);
    add_sampling(pg, sac, 0);
  }

  void build_td7(Prog& pg, bool policy, int set) {
    const int B2 = 2 * B;
    Net& enc = net("encoder");
    Net& fe = net("fixed_encoder");
    Net& fet = net("fixed_encoder_target");
    Net& pi = net("policy");
    Net* q[2] = {&net("q1"), &net("q2")};
    Net* tq[2] = {&net("target_q1"), &net("target_q2")};
    const bool lap = cfg.use_lap;
    const bool nbd = td7_nb_defer();
    const bool qpart = td7_qdot();  // the loss head's q from EPI_QDOT partials
    use_set(set);
    asc_set = set;
    add_adam_scalars(pg);
    View s = ss.sub(0, B), s2 = ss.sub(B, B);
    // ---- encoder phase (td7.py:246-257): online encoder on [s; s'] (one GEMM per layer)
    View ez1, ez2;
    View eh1 = fwd(pg, enc.layers[0], {{ss}}, B2, actE, &ez1, false);
    View eh2 = fwd(pg, enc.layers[1], {{eh1}}, B2, actE, &ez2, false);
    View ex3 = fwd(pg, enc.layers[2], {{eh2}}, B2, ACT_NONE, nullptr, true);
    View ezs = ex3.sub(0, B), ezs2 = ex3.sub(B, B);
    View ea1z, ea2z;
    View ea1 = fwd(pg, enc.layers[3], {{ezs}, {act_in}}, B, actE, &ea1z, false);
    View ea2 = fwd(pg, enc.layers[4], {{ea1}}, B, actE, &ea2z, false);
    // zsa3 + MSE gradient vs zs_next (normed) fused
    View ed3;
    float* enc_loss = nullptr;
    int enc_tiles = 0;
    {
      const Layer& L = enc.layers[5];
      Op op{};
      op.kind = OP_GEMM;
      GemmArgs& g = op.gemm;
      g.mode = GEMM_FWD;
      g.A.seg[0] = seg_n(ea2, 0, L.K);
      g.A.nseg = 1;
      Seg w{};
      w.p = P + L.wn_off;
      w.xs = L.cb;
      w.x1 = L.out;
      w.r1 = L.K;
      g.B.seg[0] = w;
      g.B.nseg = 1;
      g.M = B;
      g.N = L.out;
      g.R = L.K;
      const auto tq = choose_tn(B, L.out);
      const bool wide = plan.wide && B % 64 == 0 && L.out % plan.wide == 0;
      g.tn = wide ? plan.wide : tq.first;
      g.hot.wide = wide ? plan.wide : 0;
      op.seq = tq.second;
      g.tiles_m = cdiv(B, kTileM);
      g.tiles_n = cdiv(L.out, g.tn);
      g.epi = EPI_MSE;
      g.bias = bias(L);
      ed3 = buf(B, L.out);
      g.out = ed3.m;
      g.tgt = ezs2.m;
      g.tgt_norm = ezs2.nref();
      enc_tiles = g.tiles_m * g.tiles_n;
      enc_loss = mem.make<float>(enc_tiles);
      g.loss_part = enc_loss;
      g.mse_scale = 1.f / (float)((long long)Bv * Z);  // (mean over the B x zs_dim zsa, td7.py:253)
      g.mvalid = Bv;
      op.wg_count = (wide ? g.tiles_m / 4 : g.tiles_m) * g.tiles_n;
      pg.add(op, {ea2.id, L.res, ezs2.id, ezs2.norm_id}, {ed3.id, loss_id_enc = next_id++});
    }
    // encoder backward + Adam (optim_encoder, lr = policy_lr)
    {
      View d2 = dx(pg, {{ed3, &enc.layers[5], 0}}, H, B, actE, &ea2z);
      dw(pg, enc.layers[5], ed3, {ea2}, B, CNT_ADAM_ENC, cfg.policy_lr);
      View d1 = dx(pg, {{d2, &enc.layers[4], 0}}, H, B, actE, &ea1z);
      dw(pg, enc.layers[4], d2, {ea1}, B, CNT_ADAM_ENC, cfg.policy_lr);
      out_t = false;  // (read by the norm backward only)
      View gzs = dx(pg, {{d1, &enc.layers[3], 0}}, Z, B, ACT_NONE, nullptr);
      out_t = true;
      dw(pg, enc.layers[3], d1, {ezs, act_in}, B, CNT_ADAM_ENC, cfg.policy_lr);
      View dx3 = normbwd(pg, gzs, ex3.sub(0, B));
      View ez2s = ez2.sub(0, B), ez1s = ez1.sub(0, B);
      View dh2 = dx(pg, {{dx3, &enc.layers[2], 0}}, H, B, actE, &ez2s);
      dw(pg, enc.layers[2], dx3, {eh2.sub(0, B)}, B, CNT_ADAM_ENC, cfg.policy_lr);
      View dh1 = dx(pg, {{dh2, &enc.layers[1], 0}}, H, B, actE, &ez1s);
      dw(pg, enc.layers[1], dh2, {eh1.sub(0, B)}, B, CNT_ADAM_ENC, cfg.policy_lr);
      dw(pg, enc.layers[0], dh1, {s}, B, CNT_ADAM_ENC, cfg.policy_lr);
    }
    // ---- fixed encoder on s, fixed target encoder on s'
    out_t = false;  // forward-only outputs (no weight gradient reads them)
    View fh1 = fwd(pg, fe.layers[0], {{s}}, B, actE, nullptr, false);
    View fh2 = fwd(pg, fe.layers[1], {{fh1}}, B, actE, nullptr, false);
    out_t = true;
    View fzs = fwd(pg, fe.layers[2], {{fh2}}, B, ACT_NONE, nullptr, true);
    out_t = false;
    View th1 = fwd(pg, fet.layers[0], {{s2}}, B, actE, nullptr, false);
    View th2 = fwd(pg, fet.layers[1], {{th1}}, B, actE, nullptr, false);
    View tzs = fwd(pg, fet.layers[2], {{th2}}, B, ACT_NONE, nullptr, true);
    View fa1 = fwd(pg, fe.layers[3], {{fzs}, {act_in}}, B, actE, nullptr, false);
    View fa2 = fwd(pg, fe.layers[4], {{fa1}}, B, actE, nullptr, false);
    out_t = true;
    View fzsa = fwd(pg, fe.layers[5], {{fa2}}, B, ACT_NONE, nullptr, false);
    // ---- actor on [s; s'] (target policy aliases the policy, Q1)
    View ap0 = fwd(pg, pi.layers[0], {{ss}}, B2, ACT_NONE, nullptr, true);
    // (an ELU actor keeps its pre-activations for the policy backward: ELU' = exp(z))
    View ap1z, ap2z;
    View ap1 = fwd(pg, pi.layers[1], {{ap0}, {fzs, tzs}}, B2, actP, actP == ACT_ELU ? &ap1z : nullptr, false);
    View ap2 = fwd(pg, pi.layers[2], {{ap1}}, B2, actP, actP == ACT_ELU ? &ap2z : nullptr, false);
    // a' = clamp(pi(s', zs') + noise) only feeds the target branch's first layers, which
    // recompute it in-tile (pre-GEMM): the actor output layer runs on the s rows alone
    const bool prea = actor_pre();
    View actv = prea ? fwd(pg, pi.layers[3], {{ap2.sub(0, B)}}, B, ACT_TANH, nullptr, false)
                     : fwd(pg, pi.layers[3], {{ap2}}, B2, ACT_TANH, nullptr, false, &eps, B);
    View a_pi = actv.sub(0, B), a_next = prea ? a_pi : actv.sub(B, B);  // (pre: layout only)
    const View ap2n = ap2.sub(B, B);
    const PreUse pn1 = prea ? pre_actor_fwd(pi.layers[3], ap2n, &eps, 1) : PreUse{};
    const PreUse* pnext = prea ? &pn1 : nullptr;
    // ---- target: zsa' and target critics (forward only)
    out_t = false;
    View ta1 = fwd(pg, fet.layers[3], {{tzs}, {a_next}}, B, actE, nullptr, false, nullptr, 0, nullptr, nullptr, pnext);
    View ta2 = fwd(pg, fet.layers[4], {{ta1}}, B, actE, nullptr, false);
    // zsa' = zsa3(ta2) only feeds the target critics' first hidden layer, a linear map:
    // with `fold`, tq.q1[:, zsa block] x fet.zsa3 is precomputed (add_target_fold) and the
    // target critics read ta2 directly (one dependent level fewer)
    const bool fold = td7_fold();
    View tzsa;
    if (!fold) tzsa = fwd(pg, fet.layers[5], {{ta2}}, B, ACT_NONE, nullptr, false);
    View th[2];
    for (int n = 0; n < 2; ++n) {
      View t01 = fwd(pg, tq[n]->layers[0], {{s2}, {a_next}}, B, ACT_NONE, nullptr, true, nullptr, 0, nullptr, nullptr,
                     pnext);
      View t1;
      if (fold) {  // fixed_encoder_target.zsa3 folded into the zsa block (tfold_w / tfold_b)
        const Layer& L1 = tq[n]->layers[1];
        const std::vector<WSeg> ws{wblock(L1, 0), {tfold_w[n].m.n, tfold_w[n].m.cbn, tfold_w[n].id},
                                   wblock(L1, L1.seg_p[0] + L1.seg_p[1])};
        t1 = fwd(pg, L1, {{t01}, {ta2}, {tzs}}, B, actC, nullptr, false, nullptr, 0, &ws, &tfold_b[n]);
      } else {
        t1 = fwd(pg, tq[n]->layers[1], {{t01}, {tzsa}, {tzs}}, B, actC, nullptr, false);
      }
      th[n] = fwd(pg, tq[n]->layers[2], {{t1}}, B, actC, nullptr, false, nullptr, 0, nullptr, nullptr, nullptr,
                  qpart ? &tq[n]->layers[3] : nullptr);
    }
    out_t = true;
    // ---- online critics on (s, a, zsa_f, zs_f)
    View c01[2], c1[2], c2[2], c1z[2], c2z[2];
    for (int n = 0; n < 2; ++n) {
      c01[n] = fwd(pg, q[n]->layers[0], {{s}, {act_in}}, B, ACT_NONE, nullptr, true);
      c1[n] = fwd(pg, q[n]->layers[1], {{c01[n]}, {fzsa}, {fzs}}, B, actC, &c1z[n], false);
      c2[n] = fwd(pg, q[n]->layers[2], {{c1[n]}}, B, actC, &c2z[n], false, nullptr, 0, nullptr, nullptr, nullptr,
                  qpart ? &q[n]->layers[3] : nullptr, true);
    }
    const bool hdx = td7_headdx() && qpart;  // (the fused head reads q partials only)
    // (dZ of the critics' last hidden layers: with the fused head only their weight gradients
    // read it, in the T image)
    View dz2[2] = {buf(B, H, !hdx, true), buf(B, H, !hdx, true)},
         dq[2] = {buf(B, 1, false, true), buf(B, 1, false, true)};
    View prio = vec(B);
    const int hw = cdiv(B, 4);
    qloss_part = mem.make<float>((size_t)hw * 4);
    View d1f[2];  // (hdx) dZ of each critic's first hidden layer from the fused head + DX
    {
      // target head (td7.py:211-218) fused: y per row from the target twins, then the loss
      Op op = head_op(HEAD_TD7_LOSS, Bv);
      HeadArgs& h = op.head;
      set_head_twin(h, c2[0], c2[1], q[0]->layers[3], q[1]->layers[3]);
      set_head_target(h, HEAD_TD7_TARGET, th[0], th[1], tq[0]->layers[3], tq[1]->layers[3]);
      h.reward = rw.p;
      h.notdone = nd.p;
      h.vmax_key = &ctrl->vmax_key;
      h.vmin_key = &ctrl->vmin_key;
      h.vt = ctrl->vt;
      h.dsrc[0] = c2z[0].m;
      h.dsrc[1] = c2z[1].m;
      h.dact = actC;
      h.lap = lap;
      h.dz[0] = dz2[0].m;
      h.dz[1] = dz2[1].m;
      h.dq[0] = dq[0].m;
      h.dq[1] = dq[1].m;
      h.loss_part = qloss_part;
      h.prio = prio.p;
      std::vector<int> qrd;
      if (qpart) {
        for (int n = 0; n < 2; ++n) {
          h.qp[n] = c2[n].qd;
          h.tp[n] = th[n].qd;
          h.qp_n[n] = c2[n].qd_n;
          h.tp_n[n] = th[n].qd_n;
          qrd.push_back(c2[n].qd_id);
          qrd.push_back(th[n].qd_id);
        }
        h.qp_ld = c2[0].qd_ld;
        h.tp_ld = th[0].qd_ld;
        REQUIRE(c2[1].qd_ld == h.qp_ld && th[1].qd_ld == h.tp_ld && h.qp_n[0] <= 64 && h.qp_n[1] <= 64 &&
                    h.tp_n[0] <= 64 && h.tp_n[1] <= 64,
                "head: q partial layout");
      }
      qloss_id = next_id++;
      if (!hdx) {
        std::vector<int> rd{c2[0].id, c2[1].id, c2z[0].id, c2z[1].id, q[0]->layers[3].res, q[1]->layers[3].res,
                            th[0].id, th[1].id, tq[0]->layers[3].res, tq[1]->layers[3].res, rw.id, nd.id, R_VT};
        rd.insert(rd.end(), qrd.begin(), qrd.end());
        pg.add(op, rd, {dz2[0].id, dz2[1].id, dq[0].id, dq[1].id, prio.id, qloss_id, R_VKEYS});
      } else {
        // the head runs inside the DX of each critic's second hidden layer (one level fewer on
        // the critic chain); critic 0's op stores the priorities, loss partials and value bounds
        for (int n = 0; n < 2; ++n) {
          HeadUse hu{h, n,
                     {c2[0].id, c2[1].id, q[0]->layers[3].res, q[1]->layers[3].res, th[0].id, th[1].id,
                      tq[0]->layers[3].res, tq[1]->layers[3].res, rw.id, nd.id, R_VT},
                     {dz2[n].id, dq[n].id}};
          if (n == 0) hu.wr.insert(hu.wr.end(), {prio.id, qloss_id, R_VKEYS});
          hu.rd.insert(hu.rd.end(), qrd.begin(), qrd.end());
          d1f[n] = dx(pg, {{c2z[n], &q[n]->layers[2], 0}}, H, B, actC, &c1z[n], nullptr, nullptr, nullptr, &hu);
        }
      }
    }
    add_update_and_prefetch(pg, false, set, lap, prio);
    for (int n = 0; n < 2; ++n) {  // critic backward + Adam (optim_q_fns spans q1 + q2)
      Net& Q = *q[n];
      dw(pg, Q.layers[3], dq[n], {c2[n]}, B, CNT_ADAM_Q, cfg.critic_lr);
      View d1 = hdx ? d1f[n] : dx(pg, {{dz2[n], &Q.layers[2], 0}}, H, B, actC, &c1z[n]);
      dw(pg, Q.layers[2], dz2[n], {c1[n]}, B, CNT_ADAM_Q, cfg.critic_lr);
      (nbd ? out_n : out_t) = false;  // (read by the weight gradient / the norm backward only)
      View g01 = dx(pg, {{d1, &Q.layers[1], 0}}, H, B, ACT_NONE, nullptr, nullptr, nbd ? &c01[n] : nullptr);
      out_n = out_t = true;
      dw(pg, Q.layers[1], d1, {c01[n], fzsa, fzs}, B, CNT_ADAM_Q, cfg.critic_lr);
      if (nbd) {  // AvgL1Norm backward deferred into the weight-gradient GEMM (kDwNb)
        dw(pg, Q.layers[0], g01, {s, act_in}, B, CNT_ADAM_Q, cfg.critic_lr, nullptr, nullptr, &c01[n]);
      } else {
        View dx01 = normbwd(pg, g01, c01[n]);
        dw(pg, Q.layers[0], dx01, {s, act_in}, B, CNT_ADAM_Q, cfg.critic_lr);
      }
    }
    ploss_part = nullptr;
    if (policy) {  // td7.py:259-276 with the updated critics (no weight gradient of these layers)
      View pa1z, pa2z;
      out_t = false;
      View pa1 = fwd(pg, fe.layers[3], {{fzs}, {a_pi}}, B, actE, &pa1z, false);
      View pa2 = fwd(pg, fe.layers[4], {{pa1}}, B, actE, &pa2z, false);
      View pzsa = fwd(pg, fe.layers[5], {{pa2}}, B, ACT_NONE, nullptr, false);
      View p01[2], p1[2], p1z[2], dzp2[2];
      for (int n = 0; n < 2; ++n) {
        p01[n] = fwd(pg, q[n]->layers[0], {{s}, {a_pi}}, B, ACT_NONE, nullptr, true);
        p1[n] = fwd(pg, q[n]->layers[1], {{p01[n]}, {pzsa}, {fzs}}, B, actC, &p1z[n], false);
      }
      out_t = true;
      // q2 + q3 + dL/dQ = -1/(2B) fused (EPI_QHEAD): dZ of q2 straight from the GEMM
      ploss_id = next_id++;  // one loss resource per critic: the two heads share a level
      ploss_id2 = next_id++;
      ploss_part = mem.make<float>((size_t)(qhead_tiles(q[0]->layers[2]) + qhead_tiles(q[1]->layers[2])));
      ploss_n = 0;
      for (int n = 0; n < 2; ++n) {
        int nt = 0;
        dzp2[n] = fwd_qhead(pg, q[n]->layers[2], q[n]->layers[3], p1[n], B, -0.5f / (float)Bv, ploss_part + ploss_n,
                            &nt, n ? ploss_id2 : ploss_id);
        ploss_n += nt;
      }
      View dzp1[2], dxp01[2];
      out_t = false;  // (no weight gradient of the critics or the fixed encoder in the policy pass)
      for (int n = 0; n < 2; ++n) {
        dzp1[n] = dx(pg, {{dzp2[n], &q[n]->layers[2], 0}}, H, B, actC, &p1z[n]);
        View g = dx(pg, {{dzp1[n], &q[n]->layers[1], 0}}, H, B, ACT_NONE, nullptr);
        dxp01[n] = normbwd(pg, g, p01[n]);
      }
      out_t = true;
      // grad wrt zsa from both critics (q1 input columns [H, 2H))
      View dpa2;
      if (fold) {  // d zsa -> d pa2 through zsa3 folded: G_n = q_n.q1[:, zsa block] x fe.zsa3 (updated critics)
        View G[2];
        for (int n = 0; n < 2; ++n)
          G[n] = dx(pg, {{wview_n(q[n]->layers[1], Hp, H), &fe.layers[5], 0}}, H, H, ACT_NONE, nullptr);
        out_t = false;
        dpa2 = dx(pg, {{dzp1[0], nullptr, 0, &G[0]}, {dzp1[1], nullptr, 0, &G[1]}}, H, B, actE, &pa2z);
        out_t = true;
      } else {
        View gzsa = dx(pg, {{dzp1[0], &q[0]->layers[1], Hp}, {dzp1[1], &q[1]->layers[1], Hp}}, Z, B, ACT_NONE,
                       nullptr);
        dpa2 = dx(pg, {{gzsa, &fe.layers[5], 0}}, H, B, actE, &pa2z);
      }
      out_t = false;
      View dpa1 = dx(pg, {{dpa2, &fe.layers[4], 0}}, H, B, actE, &pa1z);
      out_t = true;
      // d action = sum of three paths, then tanh' (actor output)
      const std::vector<DxTerm> t3{
          {dxp01[0], &q[0]->layers[0], Sp}, {dxp01[1], &q[1]->layers[0], Sp}, {dpa1, &fe.layers[3], Zp}};
      View dl3 = dx(pg, t3, A, B, ACT_TANH, &a_pi);
      const PreUse p3 = prea ? pre_actor_dx(t3, A, a_pi, 0) : PreUse{};  // dl2 recomputes dl3 in-tile
      // input-grads through a layer are emitted BEFORE its Adam update so the
      // scheduler orders them against the pre-update weights (as autograd does)
      View ap2s = ap2.sub(0, B), ap1s = ap1.sub(0, B);
      const View ap2zs = actP == ACT_ELU ? ap2z.sub(0, B) : View{}, ap1zs = actP == ACT_ELU ? ap1z.sub(0, B) : View{};
      View dl2 = dx(pg, {{dl3, &pi.layers[3], 0}}, H, B, actP, dsrc_of(actP, ap2s, ap2zs), nullptr, nullptr,
                    prea ? &p3 : nullptr);
      dw(pg, pi.layers[3], dl3, {ap2s}, B, CNT_ADAM_PI, cfg.policy_lr);
      View dl1 = dx(pg, {{dl2, &pi.layers[2], 0}}, H, B, actP, dsrc_of(actP, ap1s, ap1zs));
      dw(pg, pi.layers[2], dl2, {ap1s}, B, CNT_ADAM_PI, cfg.policy_lr);
      const View ap0s = ap0.sub(0, B);
      (nbd ? out_n : out_t) = false;
      View gl0 = dx(pg, {{dl1, &pi.layers[1], 0}}, H, B, ACT_NONE, nullptr, nullptr, nbd ? &ap0s : nullptr);
      out_n = out_t = true;
      dw(pg, pi.layers[1], dl1, {ap0s, fzs}, B, CNT_ADAM_PI, cfg.policy_lr);
      if (nbd) {
        dw(pg, pi.layers[0], gl0, {s}, B, CNT_ADAM_PI, cfg.policy_lr, nullptr, nullptr, &ap0s);
      } else {
        View dl0 = normbwd(pg, gl0, ap0s);
        dw(pg, pi.layers[0], dl0, {s}, B, CNT_ADAM_PI, cfg.policy_lr);
      }
    }
    // ---- step end: info row [encoder, q_fn, policy]
    Op op = step_end_op();
    StepEndArgs& a = op.end;
    info_sum(a, 0, enc_loss, enc_tiles, 1, 1.f / (float)((long long)Bv * Z));
    info_sum(a, 1, qloss_part, hw * 4, 1, (lap ? 1.f : 0.5f) / (float)Bv);
    if (policy) info_sum(a, 2, ploss_part, ploss_n, 1, -0.5f / (float)Bv);
    else a.kind[2] = INFO_NAN;
    a.ninfo = 3;
    std::vector<int> rd{loss_id_enc, qloss_id};
    if (policy) {
      rd.push_back(ploss_id);
      rd.push_back(ploss_id2);
    }
    std::vector<int> cn{CNT_ADAM_Q, CNT_ADAM_ENC, 3, CNT_RNG, CNT_TAPE};
    if (policy) cn.push_back(CNT_ADAM_PI);
    add_step_end(pg, op, rd, cn);
  }
  int loss_id_enc = -1, qloss_id = -1, ploss_id = -1, ploss_id2 = -1, ploss_n = 0;

  // Upper bound on the tiles of a fwd_qhead GEMM over B rows (its loss partial slots).
  int qhead_tiles(const Layer& L) const { return cdiv(B, kTileM) * cdiv(L.out, kTileM); }
  // dZ of a critic's last hidden layer L (input x, activation ELU) under a constant dL/dq
  // through the head layer Lq (H -> 1), and per-tile sums of Q - b3 (+ B b3 on tile 0)
  // into part[0, *ntiles).
  View fwd_qhead(Prog& pg, const Layer& L, const Layer& Lq, const View& x, int M, float dq, float* part,
                 int* ntiles, int loss_id) {
    REQUIRE(L.seg_p.size() == 1 && x.cols == L.seg_p[0] && x.m.n && Lq.out == 1, "qhead: operand layout");
    Op op{};
    op.kind = OP_GEMM;
    GemmArgs& g = op.gemm;
    g.mode = GEMM_FWD;
    g.A.seg[0] = seg_n(x, 0, L.K);
    g.A.nseg = 1;
    Seg w{};
    w.p = P + L.wn_off;
    w.xs = L.cb;
    w.x1 = L.out;
    w.r1 = L.K;
    g.B.seg[0] = w;
    g.B.nseg = 1;
    g.M = M;
    g.N = L.out;
    g.R = L.K;
    const auto tq = choose_tn(M, L.out);
    const bool wide = plan.wide && M % 64 == 0 && L.out % plan.wide == 0;
    g.tn = wide ? plan.wide : tq.first;
    g.hot.wide = wide ? plan.wide : 0;
    op.seq = tq.second;
    g.tiles_m = cdiv(M, kTileM);
    g.tiles_n = cdiv(L.out, g.tn);
    *ntiles = g.tiles_m * g.tiles_n;  // (wide: one loss partial per 16-row block too)
    g.epi = EPI_QHEAD;
    g.act = actC;
    g.bias = bias(L);
    View dz = buf(M, L.out, true, false);  // (read by the input-gradient GEMM only: no weight update here)
    g.out = dz.m;
    g.loss_part = part;
    g.qw = P + Lq.wn_off;
    g.qw_cbn = Lq.cb;
    g.qb = bias(Lq);
    g.qscale = dq;
    g.mvalid = Bv;
    op.wg_count = (wide ? g.tiles_m / 4 : g.tiles_m) * g.tiles_n;
    pg.add(op, {x.id, L.res, Lq.res}, {dz.id, loss_id});
    return dz;
  }
  float* qloss_part = nullptr;
  float* ploss_part = nullptr;
  // fwd outputs get a T image (weight-gradient B operand) unless out_t is cleared around the
  // forward-only layers (fixed and target networks, the policy pass through the critics): one
  // store per lane and the written-back bytes of each such layer saved
  bool out_t = true;
  bool out_n = true;  // (the same for the N image: dx / normbwd outputs only a DW reads)

  // Algebraic folds of TD7's linear zsa3 layer into its consumers (build_td7): on when
  // every block is 16-aligned and zs_dim = hdim (the folded block replaces the zsa block in place).
  // Without RLE_FUSE_FOLD: the unfolded programs (tests).
  bool td7_fold() const {
    return algo == RLE_TD7 && H % 16 == 0 && Z == H && fused(RLE_FUSE_FOLD);
  }
  // The actor's tanh output layer (N = act_dim <= 32) recomputed in-tile by the consumers on
  // the critical path (PreArgs).  Without RLE_FUSE_PRE: separate ops (tests).
  bool actor_pre() const { return A <= 32 && fused(RLE_FUSE_PRE); }
  // The critics' and target critics' last hidden layers emit EPI_QDOT row partials of q, so the
  // loss head reads 2 x 16 floats per row instead of 4 rows of H.  RLE_NO_QDOT=1: row loads (A/B).
  bool td7_qdot() const { return fused(RLE_FUSE_QDOT); }
  // The critic loss head fused into the DX of the critics' second hidden layers (HeadUse):
  // H <= 256, B a multiple of 16.  without RLE_FUSE_HEADDX: the standalone head (tests, A/B).
  bool td7_headdx() const {
    return algo == RLE_TD7 && H <= 256 && H % 16 == 0 && B % 16 == 0 && fused(RLE_FUSE_HEADDX);
  }
  // AvgL1Norm backwards that feed only a weight-gradient GEMM are applied inside it
  // (EPI_NBDOT producer + kDwNb consumer: one level fewer).  RLE_NO_NBDEFER=1: separate
  // OP_NORMBWD (tests).
  bool td7_nb_defer() const { return B <= 1024 && fused(RLE_FUSE_NBDEFER); }
  View tfold_w[2], tfold_b[2];  // per target critic: q1[:, zsa block] x fet.zsa3, folded q1 bias
  bool fold_dirty = true;       // parameters written from the host since the last fold
  Graph g_fold;
  void alloc_folds() {
    if (!td7_fold()) return;
    for (int n = 0; n < 2; ++n) {
      tfold_w[n] = buf(H, H);
      tfold_b[n] = vec(H);
    }
  }
  // tq_n.q1 applied to zsa3(x) = (W1[:, zsa] W3) x + (b1 + W1[:, zsa] b3): the target
  // critics and the fixed target encoder change only at hard updates (and host loads)
  void add_target_fold(Prog& pg) {
    Net& fet = net("fixed_encoder_target");
    for (int n = 0; n < 2; ++n) {
      const Layer& L1 = net(n ? "target_q2" : "target_q1").layers[1];
      const Layer& L3 = fet.layers[5];
      dx(pg, {{wview_n(L1, L1.seg_p[0], H), &L3, 0}}, H, H, ACT_NONE, nullptr, &tfold_w[n]);
      Op op{};
      op.kind = OP_FOLDBIAS;
      FoldBiasArgs& f = op.fb;
      f.wn = P + L1.wn_off;
      f.cbn = L1.cb;
      f.col0 = L1.seg_p[0];
      f.H = H;
      f.bin = bias(L3);
      f.bbase = bias(L1);
      f.bout = tfold_b[n].p;
      op.wg_count = 1;
      pg.add(op, {L1.res, L3.res}, {tfold_b[n].id});
    }
  }

  void build_td7_hard(Prog& pg) {  // td7.py:278-285, 325-331
    flat(pg, OP_COPY, net("target_q1"), &net("q1"), 0.f, false);
    flat(pg, OP_COPY, net("target_q2"), &net("q2"), 0.f, false);
    flat(pg, OP_COPY, net("fixed_encoder_target"), &net("fixed_encoder"), 0.f, false);
    flat(pg, OP_COPY, net("fixed_encoder"), &net("encoder"), 0.f, false);
    if (td7_fold()) add_target_fold(pg);
    Op c{};
    c.kind = OP_CTRL;
    c.ctrl.mode = 0;
    c.ctrl.vmax_key = &ctrl->vmax_key;
    c.ctrl.vmin_key = &ctrl->vmin_key;
    c.ctrl.vt = ctrl->vt;
    c.wg_count = 1;
    pg.add(c, {R_VKEYS}, {R_VT});
    if (cfg.use_lap) add_reset_maxp(pg);
  }

  void add_reset_maxp(Prog& pg) {
    Replay& rp = *replay;
    Op a{};
    a.kind = OP_MAXRED;
    a.flat.src = rp.priority;
    a.flat.size = rp.size_d;
    a.flat.partial = rp.maxred_part;
    a.flat.nwg = rp.maxred_nwg;
    a.flat.stage = 0;
    a.wg_count = rp.maxred_nwg;
    int pid = next_id++;
    pg.add(a, {R_PRIO}, {pid});
    Op b = a;
    b.flat.stage = 1;
    b.flat.out = rp.maxp_d;
    b.wg_count = 1;
    pg.add(b, {pid}, {R_MAXP});
  }

  // MLP critic stack forward (mlp.py:98-101 over make_mlp's layers): hs[i] = hidden layer i's output
  // qd: the last hidden layer also emits EPI_QDOT row partials of q (a fused head reads them)
  // Behind a pre-GEMM (TD3's target critics: a' computed in-tile from the actor's last hidden layer),
  // the first layer is recomputed in-tile by the second too, its a' segment first (two-stage prologue,
  // GemmArgs::has_pre 4, whose epilogue is the q partials: two hidden layers only): the target branch's
  // first layer costs no level of its own.  Without the fusion it is its own level, in at most 32-wide
  // tiles (pl_src), so both give the same floats.
  // hz: the pre-activations too when the backward needs them (ELU critics; the last layer's with an N image,
  // for the loss head's rows)
  void mlp_critic_fwd(Prog& pg, Net& Q, const View& sv, const View& av, std::vector<View>& hs,
                      const PreUse* pre = nullptr, bool last_t = true, bool qd = false, std::vector<View>* hz = nullptr) {
    const int D = (int)Q.layers.size() - 1;
    hs.assign(D, View{});
    if (hz) hz->assign(D, View{});
    auto zp = [&](int i) { return hz && actC == ACT_ELU ? &(*hz)[i] : nullptr; };
    const bool shape = prelayer_shape(Q.layers[0], Q.layers[1]);
    // (the pre-GEMM's a' segment is one column block, kernels.hip PK 4 / gemm_finalize's two-stage REQUIRE)
    const bool two = pre && pre->kind == 1 && pre->a.mode == GEMM_FWD && pre->a.N <= 32 && r16(A) <= 16 && qd &&
                     D == 2 && prelayer_ok(Q.layers[0], Q.layers[1]) && fused(RLE_FUSE_TWOSTAGE);
    // (not behind a pre-GEMM: the first layer's own a segment is recomputed in-tile already)
    const bool use_pl = !pre && prelayer_ok(Q.layers[0], Q.layers[1]);
    if (two) {
      hs[0] = buf(B, Q.layers[0].out, true, false);  // (layout of the consumer's A operand only: never stored)
    } else {
      pl_src = use_pl || (pre && shape);
      hs[0] = fwd(pg, Q.layers[0], {{sv}, {av}}, B, actC, zp(0), false, nullptr, 0, nullptr, nullptr, pre, nullptr,
                  D == 1);
      pl_src = false;
    }
    const bool keep = out_t;
    for (int i = 1; i < D; ++i) {
      const bool last = i == D - 1;
      out_t = keep && (!last || last_t);  // (last_t = false: only the head reads the last layer, in the N image)
      PreUse pl = i == 1 && (use_pl || two) ? pre_layer(Q.layers[0], {sv, av}, two ? pre->a.seg : -1) : PreUse{};
      if (i == 1 && two) {
        pl.kind = 4;
        pl.a2 = pre->a;
        pl.rd.insert(pl.rd.end(), pre->rd.begin(), pre->rd.end());
      }
      hs[i] = fwd(pg, Q.layers[i], {{hs[i - 1]}}, B, actC, zp(i), false, nullptr, 0, nullptr, nullptr,
                  pl.kind >= 3 ? &pl : nullptr, last && qd ? &Q.layers[D] : nullptr, last);
    }
    out_t = keep;
  }
  // TD3 / SAC: the critic loss head and the actor objective's head fused into the DX of each
  // critic's last hidden layer (GemmArgs::has_pre 2; one level fewer on the critic chain and on
  // the policy chain).  without RLE_FUSE_HEADDX: the standalone heads (tests, A/B).
  // SAC: the rsample as the epilogue of the actor's raw head (without RLE_FUSE_SACFWD: OP_SAC_ACTOR, A/B)
  // (kernels.hip sacraw_*: three column blocks over R <= 256, gemm_finalize's REQUIRE; wider heads or larger
  // hidden layers take OP_SAC_ACTOR)
  bool sac_fwd_fused() const { return fused(RLE_FUSE_SACFWD) && 2 * A <= 48 && H <= 256; }
  // SAC: the actor backward as the epilogue of the da DX (without RLE_FUSE_SACBWD: OP_SAC_ACTOR_BWD, A/B)
  bool sac_bwd_fused() const { return fused(RLE_FUSE_SACBWD); }
  bool mlp_headdx() const { return fused(RLE_FUSE_HEADDX) && B % 16 == 0 && H <= 256 && H % 4 == 0; }
  // q partials of the twins (and target twins) into a head fused by headdx
  static void set_head_parts(HeadArgs& h, const View* q, const View* t, std::vector<int>& rd) {
    for (int n = 0; n < 2; ++n) {
      h.qp[n] = q[n].qd;
      h.qp_n[n] = q[n].qd_n;
      rd.push_back(q[n].qd_id);
      if (t) {
        h.tp[n] = t[n].qd;
        h.tp_n[n] = t[n].qd_n;
        rd.push_back(t[n].qd_id);
      }
    }
    h.qp_ld = q[0].qd_ld;
    h.tp_ld = t ? t[0].qd_ld : 0;
    REQUIRE(q[1].qd_ld == h.qp_ld && (!t || t[1].qd_ld == h.tp_ld), "head: q partial layout");
  }

  // SAC temperature operand of the heads and the actor backward: log_alpha (autotune, the
  // trained parameter), or fp32(tmp) itself for a fixed temperature -- the reference multiplies
  // by the Python float (sac.py:189, 227), so exp(log(tmp)) would be an ulp off
  float* alpha_fixed = nullptr;
  const float* alpha_src() {
    if (cfg.tmp < 0.f) return P + (nP - 4);
    if (!alpha_fixed) {
      alpha_fixed = mem.make<float>(1);
      HIPCHK(hipMemcpy(alpha_fixed, &cfg.tmp, 4, hipMemcpyHostToDevice));
    }
    return alpha_fixed;
  }

  // TD3 (td3.py:206-242) and SAC (sac.py:251-295)
  void build_mlp(Prog& pg, bool policy, int set) {
    const bool sac = algo == RLE_SAC;
    const int B2 = 2 * B;
    Net& pi = net("policy");
    Net* q[2] = {&net("q1"), &net("q2")};
    Net* tq[2] = {&net("target_q1"), &net("target_q2")};
    const bool lap = cfg.use_lap && !sac;
    use_set(set);
    asc_set = set;
    add_adam_scalars(pg);
    View s = ss.sub(0, B), s2 = ss.sub(B, B);
    // make_mlp's depth (mlp.py:24-35): D hidden layers, then the output layer Lout
    const int D = (int)HS.size();
    const Layer& Lout = pi.layers[D];
    // actor on [s; s'] (target policy aliases the policy, Q1; SAC policy unchanged until its step)
    pl_src = prelayer_ok(pi.layers[0], pi.layers[1]);
    std::vector<View> h(D), hz(D);  // (hz: an ELU actor's pre-activations, for the policy backward)
    const bool pz = actP == ACT_ELU;
    h[0] = fwd(pg, pi.layers[0], {{ss}}, B2, actP, pz ? &hz[0] : nullptr, false);
    pl_src = false;
    const PreUse pl0 = prelayer_ok(pi.layers[0], pi.layers[1]) ? pre_layer(pi.layers[0], {ss}) : PreUse{};
    for (int i = 1; i < D; ++i)
      h[i] = fwd(pg, pi.layers[i], {{h[i - 1]}}, B2, actP, pz ? &hz[i] : nullptr, false, nullptr, 0, nullptr, nullptr,
                 i == 1 && pl0.kind == 3 ? &pl0 : nullptr);
    const View hl = h[D - 1];  // the last hidden layer's output
    View actv, raw, logpi;
    // TD3: the target critics' first layer recomputes a' in-tile (pre-GEMM, as TD7)
    const bool prea = !sac && actor_pre();
    const View h1n = hl.sub(B, B);
    const PreUse pn1 = prea ? pre_actor_fwd(Lout, h1n, &eps, 1) : PreUse{};
    if (!sac) {
      actv = prea ? fwd(pg, Lout, {{hl.sub(0, B)}}, B, ACT_TANH, nullptr, false)
                  : fwd(pg, Lout, {{hl}}, B2, ACT_TANH, nullptr, false, &eps, B);
    } else if (sac_fwd_fused()) {  // the rsample in the raw head's epilogue (one level fewer)
      actv = buf(B2, A);
      logpi = vec(B2);
      SacFwdUse sfu{};
      SacFwdArgs& a = sfu.a;
      a.eps = eps.m;
      a.eps2 = eps2.m;
      a.act = actv.m;
      a.logpi = logpi.p;
      a.min_log_std = cfg.min_log_std;
      a.max_log_std = cfg.max_log_std;
      a.A = A;
      a.mean_off = 0;
      a.ls_off = A;
      a.eps_row_split = B;
      sfu.rd = {eps.id, eps2.id};
      sfu.wr = {actv.id, logpi.id};
      raw = fwd(pg, Lout, {{hl}}, B2, ACT_NONE, nullptr, false, nullptr, 0, nullptr, nullptr, nullptr, nullptr,
                false, &sfu);
    } else {
      raw = fwd(pg, Lout, {{hl}}, B2, ACT_NONE, nullptr, false);
      actv = buf(B2, A);
      logpi = vec(B2);
      Op op{};
      op.kind = OP_SAC_ACTOR;
      SacActorArgs& a = op.sac;
      a.out = raw.m;
      a.A = A;
      a.rows = B2;
      a.eps = eps.m;
      a.eps2 = eps2.m;
      a.eps_row_split = B;
      a.act = actv.m;
      a.logpi = logpi.p;
      a.min_log_std = cfg.min_log_std;
      a.max_log_std = cfg.max_log_std;
      a.mean_off = 0;
      a.ls_off = A;
      op.wg_count = cdiv(B2, kThreads);
      pg.add(op, {raw.id, eps.id, eps2.id}, {actv.id, logpi.id});
    }
    View a_pi = actv.sub(0, B), a_next = prea ? a_pi : actv.sub(B, B);  // (pre: layout only)
    // SAC: the target critics' first layer recomputes a' in-tile from the raw head (pre-GEMM, has_pre 5)
    const PreUse psac = sac && sac_pre() ? pre_sac_fwd(Lout, h1n, eps, 1) : PreUse{};
    const PreUse* tpre = prea ? &pn1 : (psac.kind == 5 ? &psac : nullptr);
    // target critics + y
    std::vector<View> th[2];
    out_t = false;  // (forward only)
    const bool hdx = mlp_headdx();
    for (int n = 0; n < 2; ++n) mlp_critic_fwd(pg, *tq[n], s2, a_next, th[n], tpre, true, hdx);
    out_t = true;
    // online critics
    std::vector<View> c[2], cz[2];
    for (int n = 0; n < 2; ++n) mlp_critic_fwd(pg, *q[n], s, act_in, c[n], nullptr, true, hdx, &cz[n]);
    // (the loss heads' derivative rows: ELU' reads the pre-activation; ReLU' / identity the output)
    const bool cze = actC == ACT_ELU;
    // (the last hidden layers and the heads' layers)
    const View c1[2] = {c[0][D - 1], c[1][D - 1]}, th1[2] = {th[0][D - 1], th[1][D - 1]};
    const Layer *qo[2] = {&q[0]->layers[D], &q[1]->layers[D]}, *tqo[2] = {&tq[0]->layers[D], &tq[1]->layers[D]};
    // (dZ of the critics' last hidden layers: with the fused head only their weight gradients read
    // it, in the T image)
    View dz1[2] = {buf(B, H, !hdx, true), buf(B, H, !hdx, true)},
         dq[2] = {buf(B, 1, false, true), buf(B, 1, false, true)};
    View d0f[2];  // (hdx) dZ of each critic's first hidden layer from the fused head + DX
    View prio = vec(B);
    const int hw = cdiv(B, 4);
    qloss_part = mem.make<float>((size_t)hw * 4);
    {
      // target head (td3.py:160-164, sac.py:188-193) fused: y per row, then the loss
      Op op = head_op(HEAD_MLP_LOSS, Bv);
      HeadArgs& h = op.head;
      set_head_twin(h, c1[0], c1[1], *qo[0], *qo[1]);
      set_head_target(h, HEAD_MLP_TARGET, th1[0], th1[1], *tqo[0], *tqo[1]);
      h.reward = rw.p;
      h.notdone = nd.p;
      std::vector<int> rd{c1[0].id, c1[1].id, qo[0]->res, qo[1]->res, th1[0].id, th1[1].id,
                          tqo[0]->res, tqo[1]->res, rw.id, nd.id};
      if (sac) {
        h.sac = 1;
        h.logpi = logpi.p + B;  // next-state rows
        h.log_alpha = alpha_src();
        h.alpha_lin = cfg.tmp >= 0.f;
        rd.push_back(logpi.id);
        rd.push_back(R_LA);
      }
      h.dsrc[0] = (cze ? cz[0][D - 1] : c1[0]).m;
      h.dsrc[1] = (cze ? cz[1][D - 1] : c1[1]).m;
      if (cze) rd.insert(rd.end(), {cz[0][D - 1].id, cz[1][D - 1].id});
      h.dact = actC;
      h.lap = lap;
      h.dz[0] = dz1[0].m;
      h.dz[1] = dz1[1].m;
      h.dq[0] = dq[0].m;
      h.dq[1] = dq[1].m;
      h.loss_part = qloss_part;
      h.prio = prio.p;
      qloss_id = next_id++;
      if (!hdx) {
        pg.add(op, rd, {dz1[0].id, dz1[1].id, dq[0].id, dq[1].id, prio.id, qloss_id});
      } else {
        // the head runs inside the DX of each critic's last hidden layer; critic 0's op stores the
        // priorities and loss partials
        set_head_parts(h, c1, th1, rd);
        for (int n = 0; n < 2; ++n) {
          HeadUse hu{h, n, rd, {dz1[n].id, dq[n].id}};
          if (n == 0) hu.wr.insert(hu.wr.end(), {prio.id, qloss_id});
          // (the head forms dZ = dq w act'(segment 0): an ELU critic's pre-activations, a ReLU critic's outputs)
          d0f[n] = dx(pg, {{cze ? cz[n][D - 1] : c1[n], &q[n]->layers[D - 1], 0}}, HS[D - 2], B, actC,
                      dsrc_of(actC, c[n][D - 2], cz[n][D - 2]), nullptr, nullptr, nullptr, &hu);
        }
      }
    }
    add_update_and_prefetch(pg, sac, set, lap, prio);
    for (int n = 0; n < 2; ++n) {  // (input gradients through a layer before its Adam update)
      Net& Q = *q[n];
      dw(pg, Q.layers[D], dq[n], {c1[n]}, B, CNT_ADAM_Q, cfg.critic_lr);
      View d = dz1[n];  // dZ of hidden layer i, from i = D - 1 down
      for (int i = D - 1; i >= 1; --i) {
        const View dp = hdx && i == D - 1 ? d0f[n]
                                           : dx(pg, {{d, &Q.layers[i], 0}}, HS[i - 1], B, actC,
                                                dsrc_of(actC, c[n][i - 1], cz[n][i - 1]));
        dw(pg, Q.layers[i], d, {c[n][i - 1]}, B, CNT_ADAM_Q, cfg.critic_lr);
        d = dp;
      }
      dw(pg, Q.layers[0], d, {s, act_in}, B, CNT_ADAM_Q, cfg.critic_lr);
    }
    ploss_part = nullptr;
    float* gsq = nullptr;
    int ngsq = 0;
    if (policy) {
      std::vector<View> pc[2], pcz[2];
      for (int n = 0; n < 2; ++n) mlp_critic_fwd(pg, *q[n], s, a_pi, pc[n], nullptr, false, hdx, &pcz[n]);
      const View p1[2] = {pc[0][D - 1], pc[1][D - 1]};
      // (no weight gradient of the critics in the policy pass: the gradients keep N images only)
      View dzp1[2];
      if (!hdx) dzp1[0] = buf(B, H, true, false), dzp1[1] = buf(B, H, true, false);
      ploss_part = mem.make<float>((size_t)hw * 4);
      View dzp0[2];
      if (hdx) {  // the objective's head inside the DX of each critic's last hidden layer
        Op op = head_op(HEAD_MLP_POLICY, Bv);
        HeadArgs& h = op.head;
        set_head_twin(h, p1[0], p1[1], *qo[0], *qo[1]);
        h.dact = actC;
        h.loss_part = ploss_part;
        std::vector<int> rd{p1[0].id, p1[1].id, qo[0]->res, qo[1]->res};
        if (sac) {
          h.sac = 1;
          h.logpi = logpi.p;
          h.log_alpha = alpha_src();
          h.alpha_lin = cfg.tmp >= 0.f;
          rd.push_back(logpi.id);
          rd.push_back(R_LA);
        }
        set_head_parts(h, p1, nullptr, rd);
        ploss_id = next_id++;
        out_t = false;
        for (int n = 0; n < 2; ++n) {
          HeadUse hu{h, n, rd, {}};
          if (n == 0) hu.wr.push_back(ploss_id);
          dzp0[n] = dx(pg, {{cze ? pcz[n][D - 1] : p1[n], &q[n]->layers[D - 1], 0}}, HS[D - 2], B, actC,
                       dsrc_of(actC, pc[n][D - 2], pcz[n][D - 2]), nullptr, nullptr, nullptr, &hu);
        }
        out_t = true;
      } else {
        Op op = head_op(HEAD_MLP_POLICY, Bv);
        HeadArgs& h = op.head;
        set_head_twin(h, p1[0], p1[1], *qo[0], *qo[1]);
        h.dsrc[0] = (cze ? pcz[0][D - 1] : p1[0]).m;
        h.dsrc[1] = (cze ? pcz[1][D - 1] : p1[1]).m;
        h.dact = actC;
        h.dz[0] = dzp1[0].m;
        h.dz[1] = dzp1[1].m;
        h.loss_part = ploss_part;
        std::vector<int> rd{p1[0].id, p1[1].id, qo[0]->res, qo[1]->res};
        if (cze) rd.insert(rd.end(), {pcz[0][D - 1].id, pcz[1][D - 1].id});
        if (sac) {
          h.sac = 1;
          h.logpi = logpi.p;
          h.log_alpha = alpha_src();
          h.alpha_lin = cfg.tmp >= 0.f;
          rd.push_back(logpi.id);
          rd.push_back(R_LA);
        }
        pg.add(op, rd, {dzp1[0].id, dzp1[1].id, ploss_id = next_id++});
        out_t = false;
        for (int n = 0; n < 2; ++n)
          dzp0[n] = dx(pg, {{dzp1[n], &q[n]->layers[D - 1], 0}}, HS[D - 2], B, actC,
                       dsrc_of(actC, pc[n][D - 2], pcz[n][D - 2]));
        out_t = true;
      }
      // (deeper critics: on down to the first hidden layer; no weight gradient reads these)
      out_t = false;
      for (int i = D - 2; i >= 1; --i)
        for (int n = 0; n < 2; ++n)
          dzp0[n] = dx(pg, {{dzp0[n], &q[n]->layers[i], 0}}, HS[i - 1], B, actC, dsrc_of(actC, pc[n][i - 1], pcz[n][i - 1]));
      out_t = true;
      View dout;
      PreUse pdout{};  // TD3: d1 recomputes dout in-tile
      if (!sac) {
        dout = dx(pg, {{dzp0[0], &q[0]->layers[0], Sp}, {dzp0[1], &q[1]->layers[0], Sp}}, A, B, ACT_TANH, &a_pi);
        if (prea) pdout = pre_actor_dx({{dzp0[0], &q[0]->layers[0], Sp}, {dzp0[1], &q[1]->layers[0], Sp}}, A, a_pi, 0);
      } else {
        dout = buf(B, 2 * A);
        if (sac_bwd_fused()) {  // the backward in the epilogue of the DX that forms da (one level fewer)
          SacBwdUse sbu{};
          SacBwdArgs& a = sbu.a;
          a.raw = raw.m;
          a.eps2 = eps2.m;
          a.dout = dout.m;
          a.log_alpha = alpha_src();
          a.alpha_lin = cfg.tmp >= 0.f;
          a.inv_b = 1.f / (float)Bv;
          a.nvalid = Bv;
          a.min_log_std = cfg.min_log_std;
          a.max_log_std = cfg.max_log_std;
          a.mean_off = 0;
          a.ls_off = A;
          sbu.rd = {raw.id, eps2.id, R_LA};
          sbu.wr = {dout.id};
          dx(pg, {{dzp0[0], &q[0]->layers[0], Sp}, {dzp0[1], &q[1]->layers[0], Sp}}, A, B, ACT_NONE, nullptr,
             nullptr, nullptr, nullptr, nullptr, &sbu);
        }
      }
      if (sac && !sac_bwd_fused()) {
        View da = dx(pg, {{dzp0[0], &q[0]->layers[0], Sp}, {dzp0[1], &q[1]->layers[0], Sp}}, A, B, ACT_NONE,
                     nullptr);
        Op op{};
        op.kind = OP_SAC_ACTOR_BWD;
        SacActorArgs& a = op.sac;
        a.out = raw.m;
        a.A = A;
        a.rows = Bv;  // (rows of the padded batch past it keep a zero gradient)
        a.eps2 = eps2.m;
        a.min_log_std = cfg.min_log_std;
        a.max_log_std = cfg.max_log_std;
        a.mean_off = 0;
        a.ls_off = A;
        a.da = da.m;
        a.dout = dout.m;
        a.log_alpha = alpha_src();
        a.alpha_lin = cfg.tmp >= 0.f;
        a.inv_b = 1.f / (float)Bv;
        op.wg_count = cdiv(Bv, kThreads);
        pg.add(op, {raw.id, eps2.id, da.id, R_LA}, {dout.id});
      }
      if (!sac) {
        // per-tile grad-square partials for norm/policy (rl/nn/utils.py:13-19)
        for (auto& L : pi.layers) ngsq += dw_gsq_w(L) + dw_gsq_b(L);
        gsq = mem.make<float>(ngsq);
      }
      std::vector<int> tens;
      float* gp = gsq;
      auto gsq_for = [&](const Layer& L, int t_w, int t_b) -> std::pair<float*, float*> {
        if (!gsq) return {nullptr, nullptr};
        int nw = dw_gsq_w(L), nb = dw_gsq_b(L);
        float* w = gp;
        float* b = gp + nw;
        gp += nw + nb;
        for (int i = 0; i < nw; ++i) tens.push_back(t_w);
        for (int i = 0; i < nb; ++i) tens.push_back(t_b);
        return {w, b};
      };
      // actor backward: tensors in parameters() order mlp.0.w, mlp.0.b, mlp.2.w, ...
      std::vector<std::pair<float*, float*>> gl;
      for (int i = 0; i <= D; ++i) gl.push_back(gsq_for(pi.layers[i], 2 * i, 2 * i + 1));
      std::vector<View> hsub(D), hzsub(D);
      for (int i = 0; i < D; ++i) hsub[i] = h[i].sub(0, B);
      if (pz)
        for (int i = 0; i < D; ++i) hzsub[i] = hz[i].sub(0, B);
      // TD3: the aliased target policy's Polyak (td3.py:200-204) in the Adam epilogues: one level
      // fewer between the actor update and the next step's target action
      adam_ptau = !sac && pi_polyak_fused() ? cfg.tau : 0.f;
      // SAC: d1 (the gradient through the raw head, K = 2A <= 48) recomputed in-tile by d0's DX
      const bool pld = sac && sac_bwd_fused() && prelayer_ok_dx(Lout, pi.layers[D - 1]);
      pl_src = pld;
      View d = dx(pg, {{dout, &Lout, 0}}, HS[D - 1], B, actP, dsrc_of(actP, hsub[D - 1], hzsub[D - 1]), nullptr, nullptr,
                  prea ? &pdout : nullptr);
      pl_src = false;
      // (d0 reads the raw head's pre-update weights when it recomputes d1: emitted before that Adam)
      const PreUse pd1 = pld ? pre_layer_dx(Lout, dout, hsub[D - 1]) : PreUse{};
      View dp;
      if (pld) dp = dx(pg, {{d, &pi.layers[D - 1], 0}}, HS[D - 2], B, actP, &hsub[D - 2], nullptr, nullptr, &pd1);
      dw(pg, Lout, dout, {hsub[D - 1]}, B, CNT_ADAM_PI, cfg.policy_lr, gl[D].first, gl[D].second);
      if (!pld) dp = dx(pg, {{d, &pi.layers[D - 1], 0}}, HS[D - 2], B, actP, dsrc_of(actP, hsub[D - 2], hzsub[D - 2]));
      dw(pg, pi.layers[D - 1], d, {hsub[D - 2]}, B, CNT_ADAM_PI, cfg.policy_lr, gl[D - 1].first, gl[D - 1].second);
      d = dp;
      for (int i = D - 2; i >= 1; --i) {  // (deeper actors)
        dp = dx(pg, {{d, &pi.layers[i], 0}}, HS[i - 1], B, actP, dsrc_of(actP, hsub[i - 1], hzsub[i - 1]));
        dw(pg, pi.layers[i], d, {hsub[i - 1]}, B, CNT_ADAM_PI, cfg.policy_lr, gl[i].first, gl[i].second);
        d = dp;
      }
      dw(pg, pi.layers[0], d, {s}, B, CNT_ADAM_PI, cfg.policy_lr, gl[0].first, gl[0].second);
      adam_ptau = 0.f;
      if (gsq) {
        // tensor t owns tiles [gsq_offs[t], gsq_offs[t+1]) (params() order: w0, b0, w1, b1, ...)
        gsq_offs.assign(1, 0);
        for (size_t i = 0; i < tens.size(); ++i)
          if (i + 1 == tens.size() || tens[i + 1] != tens[i]) gsq_offs.push_back((int)i + 1);
      }
    }
    // Polyak (td3.py:194-204 on policy steps incl. aliased policy Q2; sac.py:243-249 every step)
    if (!sac && policy) {
      flat(pg, OP_POLYAK, *tq[0], q[0], cfg.tau, false);
      flat(pg, OP_POLYAK, *tq[1], q[1], cfg.tau, false);
      if (!pi_polyak_fused()) flat(pg, OP_POLYAK, pi, nullptr, cfg.tau, true);
    }
    if (sac) {
      flat(pg, OP_POLYAK, *tq[0], q[0], cfg.tau, false);
      flat(pg, OP_POLYAK, *tq[1], q[1], cfg.tau, false);
    }
    // step end
    Op op = step_end_op();
    StepEndArgs& a = op.end;
    std::vector<int> rd{qloss_id};
    if (policy) rd.push_back(ploss_id);
    if (!sac) {  // [train/q_fn, train/policy, norm/policy]
      info_sum(a, 0, qloss_part, hw * 4, 1, (lap ? 1.f : 0.5f) / (float)Bv);
      if (policy) {
        info_sum(a, 1, ploss_part, hw, 4, -1.f / (float)Bv);
        a.kind[2] = INFO_GNORM;
        a.gsq = gsq;
        a.ngsq_t = (int)gsq_offs.size() - 1;
        for (size_t q = 0; q < gsq_offs.size(); ++q) a.gsq_off[q] = gsq_offs[q];
        for (auto& L : pi.layers) rd.push_back(L.res);
      } else {
        a.kind[1] = INFO_NAN;
        a.kind[2] = INFO_NAN;
      }
      a.ninfo = 3;
    } else if (cfg.tmp < 0.f) {  // [train/q_fn, tmp, norm/tmp, train/policy, train/tmp, entropy]
      info_sum(a, 0, qloss_part, hw * 4, 1, 0.5f / (float)Bv);
      a.kind[1] = INFO_SAC_TMP;
      a.kind[2] = INFO_SAC_NTMP;
      info_sum(a, 3, ploss_part, hw, 4, 1.f / (float)Bv);
      a.kind[3] = INFO_SAC_POL;
      a.kind[4] = INFO_SAC_TMPL;
      a.kind[5] = INFO_SAC_ENT;
      a.ninfo = 6;
      a.log_alpha = P + (nP - 4);
      a.la_m = P + nP + (nP - 4);
      a.la_v = P + 2 * nP + (nP - 4);
      a.la_t = &ctrl->la_t;
      a.la_lr = cfg.policy_lr;
      a.adam_step = adam_step_of(asc_set);  // (slot 3: the temperature's bias corrections, this step's ctrl)
      a.adam_bc2s = adam_bc2s_of(asc_set);
      rd.push_back(asc_set ? R_ADAMSC1 : R_ADAMSC);
      a.target_entropy = -(float)A;
      a.logpi_part = ploss_part;
      a.nlogpi = hw;
    } else {  // fixed temperature: [train/q_fn, train/policy, entropy]
      info_sum(a, 0, qloss_part, hw * 4, 1, 0.5f / (float)Bv);
      info_sum(a, 1, ploss_part, hw, 4, 1.f / (float)Bv);
      a.kind[2] = INFO_SAC_ENT;
      a.ninfo = 3;
      a.logpi_part = ploss_part;
      a.nlogpi = hw;
    }
    std::vector<int> cn{CNT_ADAM_Q, 3, CNT_RNG, CNT_TAPE};
    if (policy) cn.push_back(CNT_ADAM_PI);
    add_step_end(pg, op, rd, cn);
  }
  std::vector<int> gsq_offs;

  // ---------------------------------------------------------------- graphs
  // Workgroup cap of the scheduler's levels: off by default.  Measured on MI355X: neutral at
  // B = 256 (6494 vs 6481 steps/s) and -12% at B = 1024 (2706 vs 3067), where most levels
  // exceed the resident capacity and deferral only adds levels.  RLE_SCHED_CAP=1 enables it.
  int sched_cap() const {
    if (!plan.sched_cap) return 1 << 30;
    return plan.level_cap > 0 ? plan.level_cap : std::max(256, level_capacity());
  }
  Graph capture(Prog& pg) {
    // (rle_plan balance, A/B)
    // measured on MI355X (tools/abk.sh, RLE_BALANCE 0/1/2/3): TD3 HalfCheetah 15481/16050/15911/
    // 15637, SAC Humanoid 7674/8025/7997/7801, TD7 Humanoid 6532/6478/6498/6517 steps/s (round 1);
    // TD7 after the guarded operand rings: 7744/7774/7720/7754 (4-step graphs), and 6-step
    // graphs with mode 1: 7822 (tools/abenv.sh)
    pg.balance = plan.balance;
    pg.tiny_w = plan.tiny_w;
    pg.uni_w = plan.uni_w;
    pg.tiny_wg = plan.tiny_wg;
    pg.pl_w = plan.pl_w;
    pg.lap_w = plan.lap_w;
    pg.head_w = plan.head_w;
    pg.adam_w = plan.adam_w;
    pg.lpt = plan.lpt;
    auto levels = pg.schedule(sched_cap());
    Graph G;
    size_t total = 0;
    for (auto& lv : levels) {
      // (launch_level: ceil(ops / kLevelOps) launches)
      G.nlaunch += (int)((lv.size() + kLevelOps - 1) / kLevelOps);
      G.off.push_back((int)total);
      G.nops.push_back((int)lv.size());
      int wg = 0;
      for (auto& op : lv) wg += op.wg_count;
      G.nwg.push_back(wg);
      total += lv.size();
    }
    static const char* kname[] = {"?", "gemm", "normbwd", "sreduce", "sgather", "head", "prio",
                                  "sacfwd", "sacbwd", "end", "polyak", "copy", "maxred", "ctrl", "noise",
                                  "foldbias"};
    static const bool traffic = [] {
      const char* e = std::getenv("RLE_TRAFFIC");
      return e && e[0] == '1';
    }();
    for (size_t l = 0; l < levels.size(); ++l) {
      G.desc += "L" + std::to_string(l) + " wg=" + std::to_string(G.nwg[l]) + ":";
      if (traffic) {
        const LevelTraffic t = level_traffic(levels[l], P, nP);
        char buf[220];
        snprintf(buf, sizeof buf, " [KB act_r %.0f act_w %.0f w_r %.0f adam %.0f other %.0f xcd_r %.0f adam_w %.0f]",
                 t.act_r / 1024, t.act_w / 1024, t.w_r / 1024, t.adam / 1024, t.other / 1024, t.xcd_r / 1024,
                 t.adam_w / 1024);
        G.desc += buf;
      }
      for (size_t k = 0; k < levels[l].size(); ++k) {
        const Op& op = levels[l][k];
        G.desc += std::string(" ") + (pg.crit_lv[l][k] ? "*" : "") + kname[op.kind];
        if (op.kind == OP_GEMM) {
          static const char* kepi[] = {"st", "adam", "mse", "qhead", "nbdot", "act", "qdot", "sacbwd", "sacfwd"};
          static_assert(sizeof(kepi) / sizeof(kepi[0]) == EPI_SACFWD + 1, "every epilogue has a name");
          const char* ep = op.gemm.mode == GEMM_DW && op.gemm.act == kDwNb ? "adam+nb"
                           : op.gemm.has_pre == 2                         ? "head+dx"
                           : op.gemm.has_pre == 3                         ? (op.gemm.epi == EPI_QDOT ? "qdot+pl" : "st+pl")
                           : op.gemm.has_pre == 4                         ? "qdot+pl2"
                           : op.gemm.has_pre == 5                         ? "st+sacpre"
                                                                           : kepi[op.gemm.epi];
          G.desc += "[" + std::to_string(op.gemm.M) + "x" + std::to_string(op.gemm.N) + "x" +
                    std::to_string(op.gemm.R) + " " + ep + (op.gemm.hot.wide ? ".w" : "") + "]";
        }
        if (std::getenv("RLE_DESC_WG")) G.desc += "/" + std::to_string(op.wg_count);  // trace tools
      }
      G.desc += "\n";
    }
    std::vector<Op> flat_ops;
    flat_ops.reserve(total);
    for (auto& lv : levels)
      for (auto& op : lv) {
        REQUIRE(op.kind != OP_GEMM || gemm_variant_compiled(op.gemm.vid, kernel_set()),
                "capture: a GEMM variant outside the engine's rle_level instance (ops.h RLE_GEMM_VARIANTS sets)");
        flat_ops.push_back(op);
      }
    G.d_ops = mem.make<Op>(total);
    HIPCHK(hipMemcpy(G.d_ops, flat_ops.data(), total * sizeof(Op), hipMemcpyHostToDevice));
    const char* tr_env = std::getenv("RLE_TRACE");
    if (tr_env && tr_env[0] == '1') {
      for (int w : G.nwg) G.trace_n += w;
      G.trace = mem.make<unsigned long long>((size_t)G.trace_n * trace_stride());
    }
    if (plan.dispatch == 1 && !G.trace) g_level_rec = &G.aql;
    HIPCHK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    long long tr_off = 0;
    const bool dpf = plan.dpf != 0;  // (rle_plan dpf: the next level's descriptor prefetch workgroups)
    for (size_t l = 0; l < levels.size(); ++l) {
      // (after the last level: this graph's first, as the next replay is usually of the same graph)
      const size_t ln = l + 1 < levels.size() ? l + 1 : 0;
      hipError_t e = launch_level(G.d_ops + G.off[l], levels[l].data(), G.nops[l], G.nwg[l], stream,
                                  G.trace ? G.trace + tr_off * trace_stride() : nullptr, G.d_ops + G.off[ln],
                                  dpf ? G.nops[ln] : 0, kernel_set());
      tr_off += G.nwg[l];
      if (e != hipSuccess) {
        g_level_rec = nullptr;
        hipGraph_t tmp;
        (void)hipStreamEndCapture(stream, &tmp);
        throw Error{RLE_EHIP, std::string("launch during capture: ") + hipGetErrorString(e)};
      }
    }
    g_level_rec = nullptr;
    HIPCHK(hipStreamEndCapture(stream, &G.g));
    if (!G.aql.empty()) {
      std::vector<unsigned char> ka(G.aql.size() * 128, 0);
      for (size_t i = 0; i < G.aql.size(); ++i) std::memcpy(ka.data() + i * 128, G.aql[i].ka, sizeof G.aql[i].ka);
      G.aql_ka = mem.make<unsigned char>(ka.size());
      HIPCHK(hipMemcpy(G.aql_ka, ka.data(), ka.size(), hipMemcpyHostToDevice));
    }
    HIPCHK(hipGraphInstantiate(&G.x, G.g, nullptr, nullptr, 0));
    G.host_levels = std::move(levels);
    return G;
  }

  void alloc_step_buffers() {
    for (BatchSet& b : bsets) {
      b.ss = buf(2 * B, S);
      b.act_in = buf(B, A);
      b.rw = vec(B);
      b.nd = vec(B);
      b.eps = buf(B, A, false, true);
      b.eps2 = buf(B, A, false, true);
      b.ind = mem.make<long long>(B);
      b.u_buf = mem.make<float>(B);
      b.ind_id = next_id++;
    }
    use_set(0);
    bsum_id = next_id++;
  }

  void ensure_tapes(long long n) {
    if (n <= tape_cap) return;
    // tapes are referenced by captured graphs: allocate once at a generous size
    REQUIRE(!built || n <= tape_cap, "tape larger than the capacity fixed at first use");
    tape_cap = std::max<long long>(n, 1024);
    // + 1 row: the last taped step prefetches (and the host discards) one row past the end
    t_u = mem.make<float>((size_t)(tape_cap + 1) * B);
    t_eps = mem.make<float>((size_t)(tape_cap + 1) * B * A);
    t_eps2 = mem.make<float>((size_t)(tape_cap + 1) * B * A);
    t_ind = mem.make<long long>((size_t)(tape_cap + 1) * B);
  }

  // Builds a step program twice: the first pass fixes the level schedule, then
  // GEMM tiles of any level with more workgroups than fit on the device at once
  // are widened (16 -> 32 -> 64 columns, fewer workgroups, longer reductions per
  // wave) and the program is rebuilt with that tile plan (indexed by the GEMM sequence
  // numbers choose_tn hands out).
  template <class F>
  Prog plan_build(F&& f) {
    tn_plan.clear();
    tn_seq = 0;
    Prog p0;
    p0.rb = plan.rb;
    p0.xcd = plan.xcd;
    f(p0);
    std::vector<int> tplan(tn_seq, 16);
    auto at = [&](int seq) -> int& { return tplan[seq]; };
    auto levels = p0.schedule();
    for (auto& lv : levels)
      for (auto& op : lv)
        if (op.kind == OP_GEMM) at(op.seq) = std::max(op.gemm.tn, plan.tn_min);
    int cap = std::max(256, level_capacity());  // (plan.level_cap 0)
    // TD3 (its first layers folded into 64-wide pre-layer consumers) plans its levels for 7/8 of the
    // resident workgroups: A/B on HalfCheetah, capacity 1024 / 832 / 768 / 640 -> 23.18k / 23.47k /
    // 23.47k / 23.37k steps/s in round 3; with the two-stage prologue and its own kernel instance
    // (round 4, 2 pairs) 1024 / 896 / 768 / 640 -> 25.22k / 25.33k / 25.23k / 24.94k.  TD7 at
    // B >= 1024 plans for 3/2 of them (its levels are over capacity anyway; 2 pairs at B = 1024:
    // 1024 / 1536 / 2048 -> 3564 / 3598 / 3529).  (TD7 B = 256: 1024 best, 896 -1.2%; SAC: 1024 best,
    // 768 -0.8%.)  Round 6, with each level's ops longest first (plan lpt): TD3 at the full capacity again, 4 pairs
    // 896 (7/8) / 960 / 1024 -> 26.53k / 26.55k / 26.62k (profiles/r06_ab_plan_mlp.txt).
    if (algo == RLE_TD3 && !plan.lpt) cap = cap * 7 / 8;
    // (round 6, longest first: TD7 B = 1024 at 5/4, 4 pairs 1,536 / 1,152 / 1,280 / 1,408 -> 3.79k / 3.81k / 3.83k / 3.79k,
    // profiles/r06_ab_b1024_cap.txt)
    if (algo == RLE_TD7 && B >= 1024) cap = plan.lpt ? cap * 5 / 4 : cap * 3 / 2;
    // (plan.level_cap: tuning experiments, and seeds per GPU on streams -- bench.py)
    if (plan.level_cap > 0) cap = plan.level_cap;
    // elementwise ops (Polyak, copies) are short: they free their slots long before the level's
    // GEMMs do, so they count at 1 / flat_div of their workgroups (RLE_FLAT_DIV, A/B; 1 = full)
    const int flat_div = plan.flat_div;  // (A/B 1 / 4 / 1000: SAC 12675 / 13135 / 13122)
    auto wg_of = [&](const Op& op) {
      if (op.kind == OP_POLYAK || op.kind == OP_COPY) return op.wg_count / flat_div;
      if (op.kind != OP_GEMM) return op.wg_count;
      const GemmArgs& g = op.gemm;
      if (g.hot.wide) return op.wg_count;  // (64-row tiles: never widened)
      return g.tiles_m * (cdiv(g.N, at(op.seq)) + (g.epi == EPI_ADAM ? 1 : 0));
    };
    for (auto& lv : levels) {
      while (true) {
        long long total = 0;
        for (auto& op : lv) total += wg_of(op);
        if (total <= cap) break;
        int best = -1, best_wg = 0;
        for (auto& op : lv)
          if (op.kind == OP_GEMM && !op.gemm.hot.wide && at(op.seq) < 64 && wg_of(op) > best_wg) {
            best = op.seq;
            best_wg = wg_of(op);
          }
        if (best < 0) break;
        at(best) *= 2;
      }
    }
    tn_plan = tplan;
    tn_seq = 0;
    Prog p;
    p.rb = plan.rb;
    p.xcd = plan.xcd;
    f(p);
    tn_plan.clear();
    return p;
  }

  // steps per multi-step graph: plan.steps_per_graph (even; 0 = single-step graphs only)
  int pair_k() const {
    // measured on MI355X (tools/abk.sh): TD7 Humanoid K=2/4/6/8 -> 6370/6513/6440/6290
    // steps/s (round 1), K=4/6/8 -> 7744/7785/7789 after the guarded operand rings (with the
    // rebalance pass: K=6/8 -> 7822/7825); TD3 HalfCheetah K=2/4/8/12/16 -> 14072/14885/16066/
    // 16203/16348 and SAC Humanoid K=2/4/8 -> 7874/7977/8052 (with the rebalance pass)
    int k = plan.steps_per_graph;
    if (algo != RLE_SAC && cfg.policy_freq != 2) k = 0;  // the pattern assumes policy_freq 2
    return k >= 2 ? k & ~1 : 0;
  }

  void build() {
    REQUIRE(replay, "no replay bound");
    ensure_tapes(1024);
    const bool sac = algo == RLE_SAC;
    alloc_folds();
    multi_k = pair_k();
    for (int set = 0; set < 2; ++set) {
      Prog pp;
      pp.xcd = plan.xcd;
      build_prime(pp, sac, set);
      g_prime[set] = capture(pp);
      if (algo == RLE_TD7) {
        Prog p1 = plan_build([&](Prog& p) { build_td7(p, true, set); });
        g_pol[set] = capture(p1);
        Prog p2 = plan_build([&](Prog& p) { build_td7(p, false, set); });
        g_pln[set] = capture(p2);
        if (multi_k) {
          Prog p3 = plan_build([&](Prog& p) {
            for (int j = 0; j < multi_k; ++j) build_td7(p, j % 2 == 0, (set + j) % 2);
          });
          g_pair[set] = capture(p3);
          for (int r = 0; r < 2; ++r) {
            if (kRemK[r] >= multi_k) continue;
            Prog p4 = plan_build([&](Prog& p) {
              for (int j = 0; j < kRemK[r]; ++j) build_td7(p, j % 2 == 0, (set + j) % 2);
            });
            g_rem[r][set] = capture(p4);
          }
        }
      } else {
        Prog p1 = plan_build([&](Prog& p) { build_mlp(p, true, set); });
        g_pol[set] = capture(p1);
        if (!sac) {
          Prog p2 = plan_build([&](Prog& p) { build_mlp(p, false, set); });
          g_pln[set] = capture(p2);
        }
        if (multi_k) {  // TD3: policy, plain, ...; SAC: every step is a policy step
          Prog p3 = plan_build([&](Prog& p) {
            for (int j = 0; j < multi_k; ++j) build_mlp(p, sac || j % 2 == 0, (set + j) % 2);
          });
          g_pair[set] = capture(p3);
          for (int r = 0; r < 2; ++r) {
            if (kRemK[r] >= multi_k) continue;
            Prog p4 = plan_build([&](Prog& p) {
              for (int j = 0; j < kRemK[r]; ++j) build_mlp(p, sac || j % 2 == 0, (set + j) % 2);
            });
            g_rem[r][set] = capture(p4);
          }
        }
      }
    }
    if (algo == RLE_TD7) {
      Prog ph;
      ph.xcd = plan.xcd;
      build_td7_hard(ph);
      g_hard = capture(ph);
      if (td7_fold()) {
        Prog pf;
        pf.xcd = plan.xcd;
        add_target_fold(pf);
        g_fold = capture(pf);
      }
    }
    {
      Prog pz;
      Op z{};
      z.kind = OP_COPY;
      z.flat.dst = reinterpret_cast<float*>(&ctrl->info_slot);  // (int 0 = the bits of float 0)
      z.flat.src = mem.make<float>(4);                          // (zero-filled)
      z.flat.n = 1;
      z.wg_count = 1;
      pz.add(z, {}, {next_id++});
      g_slot0 = capture(pz);
    }
    use_set(0);
    built = true;
  }

  // Adam bias-correction scalars of this step from the completed-step counters; the
  // op has no producers, so it runs in level 0 beside the LAP block sums.
  // (SAC autotune: also the temperature optimizer's bias corrections, from la_t, which the previous
  // step end wrote: R_LA)
  bool sac_tmp_auto() const { return algo == RLE_SAC && cfg.tmp < 0.f; }
  void add_adam_scalars(Prog& pg) {
    std::vector<int> rd{R_CNT};
    if (sac_tmp_auto()) rd.push_back(R_LA);
    pg.add(adam_scalars_op(asc_set), rd, {asc_set ? R_ADAMSC1 : R_ADAMSC});
  }
  Op adam_scalars_op(int set) {
    Op op{};
    op.kind = OP_CTRL;
    op.wg_count = 1;
    CtrlArgs& c = op.ctrl;
    c.mode = 1;
    c.counters = ctrl->counters;
    c.adam_step = adam_step_of(set);
    c.adam_bc2s = adam_bc2s_of(set);
    c.adam_lr[CNT_ADAM_Q] = cfg.critic_lr;
    c.adam_lr[CNT_ADAM_PI] = cfg.policy_lr;
    c.adam_lr[CNT_ADAM_ENC] = cfg.policy_lr;
    if (sac_tmp_auto()) {
      c.la_t = &ctrl->la_t;
      c.la_lr = cfg.policy_lr;
    }
    return op;
  }

  // The same computed eagerly (creation / counters set), for readers outside a step.
  void refresh_adam_scalars() {
    if (!adamsc1) adamsc1 = mem.make<float>(8);
    if (!ctrl_op) ctrl_op = mem.make<Op>(2);
    Op ops[2] = {adam_scalars_op(0), adam_scalars_op(1)};
    ops[1].wg_begin = 1;
    HIPCHK(hipMemcpyAsync(ctrl_op, ops, sizeof(ops), hipMemcpyHostToDevice, stream));
    HIPCHK(launch_level(ctrl_op, ops, 2, 2, stream));
    HIPCHK(hipStreamSynchronize(stream));
  }
  Op* ctrl_op = nullptr;

  // ---------------------------------------------------------------- run
  long long launches = 0;  // rle_level dispatches enqueued by step graphs (rle_launch_count)
  std::unique_ptr<AqlQueue> aql;  // (rle_plan dispatch 1) direct dispatch of the step graphs
  bool aql_active = false;        // inside step(): graphs go to the AQL queue
  // Direct AQL dispatch of the step graphs (rle_step / rle_step_timed wait for their bursts; rle_step_async
  // leaves its burst in flight on the engine's own queue -- each seed on a queue of its own, where hipGraph
  // replays on HIP streams share GPU_MAX_HW_QUEUES hardware queues -- and every other entry point, and
  // every replay operation on a replay the engine is bound to, drains it first: aql_drain).  rle_plan
  // dispatch 0 / 2: hipGraph replays / launches on the stream (A/B; the launch path changes no result).
  bool aql_mode() const { return plan.dispatch == 1; }
  void aql_drain(double* ms = nullptr) {
    if (aql) aql_complete(*aql, ms);
  }
  void launch_graph(const Graph& G) {
    const bool eager = plan.dispatch == 2;  // (A/B: level launches on the stream, no graph)
    if (aql_active && !G.aql.empty()) {
      for (size_t i = 0; i < G.aql.size(); ++i) aql->pending.push_back({G.aql_ka + i * 128, G.aql[i].grid, G.aql[i].ks});
      launches += G.nlaunch;
      return;
    }
    if (eager && !G.trace) {
      for (size_t l = 0; l < G.host_levels.size(); ++l)
        HIPCHK(launch_level(G.d_ops + G.off[l], G.host_levels[l].data(), G.nops[l], G.nwg[l], stream, nullptr,
                            nullptr, 0, kernel_set()));
    } else {
      HIPCHK(hipGraphLaunch(G.x, stream));
    }
    launches += G.nlaunch;
  }
  // The next K steps (multi_k, or a remainder program's) may run as one multi-step program: TD7 (counter
  // bumped first, td7.py:295) / TD3 (td3.py:231) when its first step is a policy step (and, TD7, no step
  // of it needs a hard update); SAC any K steps.
  bool pair_window_ok(int K) const {
    if (!K) return false;
    const long long k1 = algo == RLE_TD7 ? n_runs + 1 : n_runs;
    if (algo != RLE_SAC && k1 % 2) return false;
    if (algo == RLE_TD7) {
      const int tur = std::max(1, cfg.target_update_rate);
      for (long long k = k1; k < k1 + K; ++k)
        if (k % tur == 0) return false;
    }
    return true;
  }
  // host state after a K-step program starting on batch set cur_set was enqueued
  void pair_commit(int K) {
    const int p = cur_set;
    n_runs += K;
    pol_set = p;
    if (algo != RLE_SAC) pln_set = 1 - p;
    last_set = 1 - p;
    cur_set = p;
    if (cfg.use_lap && algo != RLE_SAC) replay->version += K;
    primed = true;
    primed_ver = replay->version;
  }

  void step(int n, float* info_out, float* gpu_ms = nullptr, bool async = false) {
    REQUIRE(replay, "no replay bound");
    REQUIRE(replay->size > 0, "replay is empty");
    if (!built) build();
    const int pf = std::max(1, cfg.policy_freq);
    if (fold_dirty && g_fold.x) launch_graph(g_fold);
    fold_dirty = false;
    int done = 0;
    // direct dispatch (rle_plan dispatch 1): the graphs' levels go to the engine's own queue; the HIP
    // stream is drained first and the queue after each chunk (host-side ordering between them; async:
    // the last chunk stays in flight, aql_drain)
    const bool use_aql = aql_mode() && !g_pol[0].aql.empty();
    if (use_aql && !aql) aql = aql_open(cfg.device);
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if (gpu_ms && !use_aql) {  // (AQL: the levels run outside the stream; host wall time instead)
      HIPCHK(hipEventCreate(&ev0));
      HIPCHK(hipEventCreate(&ev1));
      HIPCHK(hipEventRecord(ev0, stream));
    }
    double aql_ms = 0.0;
    while (done < n) {
      const int chunk = std::min(n - done, info_cap);
      if (use_aql) {
        // the info slot reset is the burst's first packet (g_slot0), in order with the bursts still in flight:
        // no host round trip (a 4-byte H2D copy and a stream sync cost ~20 us per burst, 1% of a 20-step burst)
        HIPCHK(hipStreamSynchronize(stream));
        aql_active = true;
        launch_graph(g_slot0);
        launches -= g_slot0.nlaunch;  // (not a step level)
      } else {
        int zero = 0;
        HIPCHK(hipMemcpyAsync(&ctrl->info_slot, &zero, sizeof(int), hipMemcpyHostToDevice, stream));
      }
      for (int i = 0; i < chunk; ++i) {
        if (ctrl_tape_mode_host) {
          REQUIRE(tape_left > 0, "tape exhausted");
          --tape_left;
        }
        // the batch of this step: prefetched by the previous step, unless anything it was
        // drawn from has changed since (appends, other writers of the priorities, tapes)
        if (!primed || primed_ver != replay->version) launch_graph(g_prime[cur_set]);
        const int p = cur_set;
        // multi-step graph (pair_window_ok)
        // (the longest multi-step program that fits the rest of the chunk: multi_k, then the remainder ones)
        const Graph* mg = nullptr;
        int K = 0;
        for (int r = -1; r < 2 && !mg; ++r) {
          const int k = r < 0 ? multi_k : kRemK[r];
          const Graph& g = r < 0 ? g_pair[p] : g_rem[r][p];
          if (k && g.x && i + k - 1 < chunk && (!ctrl_tape_mode_host || tape_left >= k - 1) && pair_window_ok(k)) {
            mg = &g;
            K = k;
          }
        }
        if (mg) {
          if (ctrl_tape_mode_host) tape_left -= K - 1;
          launch_graph(*mg);
          pair_commit(K);
          i += K - 1;
          continue;
        }
        if (algo == RLE_TD7) {
          ++n_runs;  // td7.py:295 (increment first)
          (n_runs % pf == 0 ? pol_set : pln_set) = p;
          launch_graph((n_runs % pf == 0) ? g_pol[p] : g_pln[p]);
          if (n_runs % std::max(1, cfg.target_update_rate) == 0) launch_graph(g_hard);
        } else if (algo == RLE_TD3) {
          (n_runs % pf == 0 ? pol_set : pln_set) = p;
          launch_graph((n_runs % pf == 0) ? g_pol[p] : g_pln[p]);  // td3.py:231
          ++n_runs;
        } else {
          pol_set = p;
          launch_graph(g_pol[p]);
          ++n_runs;
        }
        last_set = p;
        cur_set = 1 - p;
        if (cfg.use_lap && algo != RLE_SAC) ++replay->version;  // this step wrote priorities
        primed = true;
        primed_ver = replay->version;
      }
      if (use_aql) {
        aql_active = false;
        aql_submit(*aql);
        if (!async) aql_complete(*aql, &aql_ms);
      }
      if (info_out) {
        HIPCHK(hipMemcpyAsync(info_out + (size_t)done * kInfoMax, info, (size_t)chunk * kInfoMax * sizeof(float),
                              hipMemcpyDeviceToHost, stream));
      }
      if (!gpu_ms && !async) HIPCHK(hipStreamSynchronize(stream));
      done += chunk;
    }
    HIPCHK(hipEventRecord(done_ev, stream));  // replay operations wait for this (Replay::wait_users)
    if (gpu_ms && use_aql) {
      *gpu_ms = (float)aql_ms;  // (the levels ran outside the stream: host wall time)
    } else if (gpu_ms) {
      HIPCHK(hipEventRecord(ev1, stream));
      HIPCHK(hipEventSynchronize(ev1));
      HIPCHK(hipEventElapsedTime(gpu_ms, ev0, ev1));
      (void)hipEventDestroy(ev0);
      (void)hipEventDestroy(ev1);
    }
  }
  int ctrl_tape_mode_host = 0;
};

void Replay::drain_users() {
  for (auto& u : users) u.first->aql_drain();
}
void Replay::wait_users() {
  drain_users();
  for (auto& u : users) HIPCHK(hipStreamWaitEvent(stream, u.second, 0));
}

}  // namespace rle

// ====================================================================== C ABI

using rle::Engine;
using rle::Error;
using rle::Replay;

struct rle_replay {
  Replay r;
};
struct rle_engine {
  std::unique_ptr<Engine> e;
};
// The engine behind a handle, its rle_step_async burst retired first (Engine::aql_mode)
static Engine& drained(rle_engine* h) {
  h->e->aql_drain();
  return *h->e;
}

template <class F>
static int guard(F&& f) {
  try {
    f();
    return RLE_OK;
  } catch (const Error& err) {
    rle::g_err = err.msg;
    return err.code;
  } catch (const std::exception& ex) {
    rle::g_err = ex.what();
    return RLE_ESTATE;
  }
}

extern "C" {

const char* rle_last_error(void) { return rle::g_err.c_str(); }

int rle_replay_create(int device, long long capacity, int state_dim, int action_dim, int lap, rle_replay** out) {
  return guard([&] {
    REQUIRE(out && capacity > 0 && state_dim > 0 && action_dim > 0, "rle_replay_create: bad args");
    REQUIRE(state_dim <= 1024 && action_dim <= 128, "rle_replay_create: state_dim <= 1024, action_dim <= 128");
    REQUIRE(capacity <= 2048LL * 4096, "rle_replay_create: capacity > 8M transitions");
    HIPCHK(hipSetDevice(device));
    auto* h = new rle_replay();
    Replay& r = h->r;
    r.device = device;
    r.cap = capacity;
    r.S = state_dim;
    r.Sp = rle::r16(state_dim);
    r.A = action_dim;
    r.Ap = rle::r16(action_dim);
    r.lap = lap ? 1 : 0;
    try {
      HIPCHK(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
      r.state = r.mem.make<float>((size_t)capacity * r.Sp);
      r.next_state = r.mem.make<float>((size_t)capacity * r.Sp);
      r.action = r.mem.make<float>((size_t)capacity * r.Ap);
      r.reward = r.mem.make<float>(capacity);
      r.notdone = r.mem.make<float>(capacity);
      r.priority = r.mem.make<float>(capacity);
      r.size_d = r.mem.make<long long>(1);
      r.maxp_d = r.mem.make<float>(1);
      const float one = 1.f;  // lap.py:29 max_priority = 1
      HIPCHK(hipMemcpy(r.maxp_d, &one, 4, hipMemcpyHostToDevice));
      r.nblk = rle::cdiv(capacity, 4096);
      REQUIRE(!lap || capacity <= 64LL * 16 * 4096, "LAP replay capacity above 4M rows");  // (sampler: 16 blocks per lane)
      r.bsum = r.mem.make<double>(r.nblk);
      r.ssum = r.mem.make<double>((size_t)r.nblk * 64);
      r.maxred_part = r.mem.make<float>(r.maxred_nwg);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int rle_replay_destroy(rle_replay* r) {
  return guard([&] {
    if (!r) return;
    try {
      r->r.drain_users();
    } catch (const Error&) {  // (a timed-out burst: the engine's queue is closed; unbind anyway)
    }
    for (auto& u : r->r.users) {  // engines still bound: unbind (their steps now fail: "no replay bound")
      (void)hipEventSynchronize(u.second);
      u.first->replay = nullptr;
    }
    (void)hipStreamSynchronize(r->r.stream);
    (void)hipStreamDestroy(r->r.stream);
    delete r;
  });
}

int rle_replay_append(rle_replay* h, const float* state, const float* action, const float* reward,
                      const float* next_state, const float* notdone, long long count) {
  return guard([&] {
    REQUIRE(h && count >= 0, "append: bad args");
    Replay& r = h->r;
    HIPCHK(hipSetDevice(r.device));
    r.wait_users();
    long long done = 0;
    // a chunk never wraps onto itself (rows i and i+cap would race; the later must win)
    const long long chunk_max = std::min<long long>(65536, r.cap);
    while (done < count) {
      const long long c = std::min(chunk_max, count - done);
      const size_t per = 2 * (size_t)r.Sp + r.Ap + 2;
      if (c > r.stage_rows) {
        r.stage = r.mem.make<float>((size_t)c * per);
        r.stage_rows = c;
      }
      std::vector<float> host((size_t)c * per, 0.f);
      float* hs = host.data();
      float* hns = hs + (size_t)c * r.Sp;
      float* ha = hns + (size_t)c * r.Sp;
      float* hr = ha + (size_t)c * r.Ap;
      float* hd = hr + c;
      for (long long i = 0; i < c; ++i) {
        const long long k = done + i;
        std::memcpy(hs + i * r.Sp, state + k * r.S, sizeof(float) * r.S);
        std::memcpy(hns + i * r.Sp, next_state + k * r.S, sizeof(float) * r.S);
        std::memcpy(ha + i * r.Ap, action + k * r.A, sizeof(float) * r.A);
        hr[i] = reward[k];
        hd[i] = notdone[k];
      }
      float* ds = r.stage;
      HIPCHK(hipMemcpyAsync(ds, hs, host.size() * sizeof(float), hipMemcpyHostToDevice, r.stream));
      HIPCHK(rle::launch_append(r.state, r.next_state, r.action, r.reward, r.notdone, r.priority, ds,
                                ds + (size_t)c * r.Sp, ds + 2 * (size_t)c * r.Sp, ds + 2 * (size_t)c * r.Sp + c * r.Ap,
                                ds + 2 * (size_t)c * r.Sp + c * r.Ap + c, r.ptr, r.cap, (int)c, r.Sp, r.Ap, r.maxp_d,
                                r.lap, r.bsum, r.ssum, r.size, r.stream));
      r.ptr = (r.ptr + c) % r.cap;
      r.size = std::min(r.size + c, r.cap);
      ++r.version;
      HIPCHK(hipMemcpyAsync(r.size_d, &r.size, sizeof(long long), hipMemcpyHostToDevice, r.stream));
      HIPCHK(hipStreamSynchronize(r.stream));
      done += c;
    }
  });
}

int rle_replay_state(rle_replay* h, long long* ptr, long long* size, float* max_priority) {
  return guard([&] {
    REQUIRE(h, "state: null");
    Replay& r = h->r;
    if (ptr) *ptr = r.ptr;
    if (size) *size = r.size;
    if (max_priority) {
      r.drain_users();
      HIPCHK(hipDeviceSynchronize());
      HIPCHK(hipMemcpy(max_priority, r.maxp_d, 4, hipMemcpyDeviceToHost));
    }
  });
}

static void recompute_bsum(Replay& r);

int rle_replay_fill_random(rle_replay* h, long long count, unsigned long long seed) {
  return guard([&] {
    Replay& r = h->r;
    REQUIRE(count > 0 && count <= r.cap, "fill: bad count");
    HIPCHK(hipSetDevice(r.device));
    r.wait_users();
    HIPCHK(rle::launch_fill(r.state, r.next_state, r.action, r.reward, r.notdone, r.priority, count, r.S, r.Sp, r.A,
                            r.Ap, seed, r.stream));
    r.size = std::max(r.size, count);
    r.ptr = count % r.cap;
    ++r.version;
    HIPCHK(hipMemcpyAsync(r.size_d, &r.size, sizeof(long long), hipMemcpyHostToDevice, r.stream));
    HIPCHK(hipStreamSynchronize(r.stream));
    if (r.lap) recompute_bsum(r);
  });
}

int rle_replay_get_priority(rle_replay* h, float* out, long long n) {
  return guard([&] {
    REQUIRE(n <= h->r.cap, "get_priority: n > capacity");
    h->r.drain_users();
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, h->r.priority, n * 4, hipMemcpyDeviceToHost));
  });
}

int rle_replay_set_priority(rle_replay* h, const float* p, long long n, float max_priority) {
  return guard([&] {
    REQUIRE(n <= h->r.cap, "set_priority: n > capacity");
    h->r.drain_users();
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(h->r.priority, p, n * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->r.maxp_d, &max_priority, 4, hipMemcpyHostToDevice));
    if (h->r.lap) recompute_bsum(h->r);
    ++h->r.version;
  });
}

// Runs a small op program eagerly on the replay's stream (test hooks).
static void run_eager(Replay& r, std::vector<std::vector<rle::Op>> levels) {
  for (size_t l = 0; l < levels.size(); ++l) {
    auto& lv = levels[l];
    int wg = 0;
    for (auto& op : lv) {
      op.wg_begin = wg;
      wg += op.wg_count;
    }
    rle::Op* d = r.scratch.get<rle::Op>("ops" + std::to_string(l), lv.size());
    HIPCHK(hipMemcpy(d, lv.data(), lv.size() * sizeof(rle::Op), hipMemcpyHostToDevice));
    HIPCHK(rle::launch_level(d, lv.data(), (int)lv.size(), wg, r.stream));
  }
  HIPCHK(hipStreamSynchronize(r.stream));
}

// Full recompute of the LAP block sums (after bulk priority writes).  In-step and
// eager priority scatters and appends keep them exact incrementally.
static void recompute_bsum(Replay& r) {
  rle::Op a{};
  a.kind = rle::OP_SAMPLE_REDUCE;
  a.sample.priority = r.priority;
  a.sample.size = r.size_d;
  a.sample.bsum = r.bsum;
  a.sample.ssum = r.ssum;
  a.wg_count = r.nblk;
  run_eager(r, {{a}});
}

int rle_replay_sample_indices(rle_replay* h, int n, const float* u, long long* ind_out) {
  return guard([&] {
    Replay& r = h->r;
    REQUIRE(n > 0 && r.size > 0, "sample_indices: bad args / empty replay");
    HIPCHK(hipSetDevice(r.device));
    r.wait_users();
    rle::Scratch& tmp = r.scratch;
    rle::SampleArgs s{};
    s.state = r.state;
    s.next_state = r.next_state;
    s.action = r.action;
    s.reward = r.reward;
    s.notdone = r.notdone;
    s.priority = r.priority;
    s.S = r.S;
    s.Sp = r.Sp;
    s.A = r.A;
    s.Ap = r.Ap;
    s.size = r.size_d;
    s.cap = r.cap;
    s.lap = r.lap;
    s.B = n;
    s.nq = n;
    s.bsum = r.bsum;
    s.ssum = r.ssum;
    s.nblk = r.nblk;
    auto timg = [&](const char* name, int rows, int cols) {  // scratch T image (outputs are not read back)
      rle::Mat m{};
      m.rbs = rle::r16(rows) / 16;
      m.cbn = cols / 16;
      m.t = tmp.get<float>(name, (size_t)rle::r16(rows) * cols);
      return m;
    };
    s.ss = timg("ss", 2 * n, r.Sp);
    s.a = timg("a", n, r.Ap);
    s.r = tmp.get<float>("r", n);
    s.nd = tmp.get<float>("nd", n);
    long long* dind = tmp.get<long long>("ind", n);
    s.ind = dind;
    s.u_out = tmp.get<float>("u_out", n);
    s.eps = timg("eps", n, r.Ap);
    // [0] rng step = 0, [1] tape position = 0 (zero from allocation, only read), [2] tape mode
    long long* cnt = tmp.get<long long>("ctl", 3);
    const long long ctl[3] = {0, 0, rle::kTapeU};
    float* du = tmp.get<float>("u", n);
    HIPCHK(hipMemcpyAsync(cnt, ctl, sizeof ctl, hipMemcpyHostToDevice, r.stream));
    HIPCHK(hipMemcpyAsync(du, u, n * 4, hipMemcpyHostToDevice, r.stream));
    s.ctrl_rng = cnt;
    s.tape_pos = cnt + 1;
    s.tape_mode = (const int*)(cnt + 2);
    s.tape_u = du;
    s.tape_eps = tmp.get<float>("tape_eps", (size_t)n * r.A);
    std::vector<std::vector<rle::Op>> lv;
    rle::Op b{};
    b.kind = rle::OP_SAMPLE_GATHER;
    b.sample = s;
    b.wg_count = rle::cdiv(n, 4);
    lv.push_back({b});
    run_eager(r, lv);
    HIPCHK(hipMemcpy(ind_out, dind, n * sizeof(long long), hipMemcpyDeviceToHost));
  });
}

int rle_replay_update_priority(rle_replay* h, int n, const long long* ind, const float* p) {
  return guard([&] {
    Replay& r = h->r;
    REQUIRE(n > 0 && n <= 1024, "update_priority: 0 < n <= 1024");
    HIPCHK(hipSetDevice(r.device));
    r.wait_users();
    for (int i = 0; i < n; ++i) REQUIRE(ind[i] >= 0 && ind[i] < r.cap, "update_priority: index out of range");
    // The incremental fp64 block-sum update is exact for priorities >= 1 (integer multiples of
    // 2^-23 summing below 2^30); any smaller value -> full recompute of the block sums instead.
    bool small = false;
    for (int i = 0; i < n; ++i) small = small || !(p[i] >= 1.f);
    long long* di = r.scratch.get<long long>("prio_ind", n);
    float* dp = r.scratch.get<float>("prio_p", n);
    HIPCHK(hipMemcpyAsync(di, ind, n * 8, hipMemcpyHostToDevice, r.stream));
    HIPCHK(hipMemcpyAsync(dp, p, n * 4, hipMemcpyHostToDevice, r.stream));
    rle::Op op{};
    op.kind = rle::OP_PRIORITY;
    op.prio.priority = r.priority;
    op.prio.ind = di;
    op.prio.p = dp;
    op.prio.B = n;
    op.prio.max_priority = r.maxp_d;
    op.prio.bsum = r.lap && !small ? r.bsum : nullptr;
    op.prio.ssum = r.ssum;
    op.wg_count = 1;
    run_eager(r, {{op}});
    if (r.lap && small) recompute_bsum(r);
    ++r.version;
  });
}

int rle_replay_reset_max_priority(rle_replay* h) {
  return guard([&] {
    Replay& r = h->r;
    REQUIRE(r.size > 0, "reset_max_priority: empty");
    HIPCHK(hipSetDevice(r.device));
    r.wait_users();
    rle::Op a{};
    a.kind = rle::OP_MAXRED;
    a.flat.src = r.priority;
    a.flat.size = r.size_d;
    a.flat.partial = r.maxred_part;
    a.flat.nwg = r.maxred_nwg;
    a.flat.stage = 0;
    a.wg_count = r.maxred_nwg;
    rle::Op b = a;
    b.flat.stage = 1;
    b.flat.out = r.maxp_d;
    b.wg_count = 1;
    run_eager(r, {{a}, {b}});
  });
}

int rle_replay_gather(rle_replay* h, int n, const long long* ind, float* state, float* action, float* reward,
                      float* next_state, float* notdone) {
  return guard([&] {
    Replay& r = h->r;
    r.drain_users();
    HIPCHK(hipDeviceSynchronize());
    std::vector<float> row(r.Sp);
    for (int i = 0; i < n; ++i) {
      const long long k = ind[i];
      REQUIRE(k >= 0 && k < r.cap, "gather: index out of range");
      if (state) {
        HIPCHK(hipMemcpy(row.data(), r.state + k * r.Sp, r.Sp * 4, hipMemcpyDeviceToHost));
        std::memcpy(state + (size_t)i * r.S, row.data(), r.S * 4);
      }
      if (next_state) {
        HIPCHK(hipMemcpy(row.data(), r.next_state + k * r.Sp, r.Sp * 4, hipMemcpyDeviceToHost));
        std::memcpy(next_state + (size_t)i * r.S, row.data(), r.S * 4);
      }
      if (action) {
        HIPCHK(hipMemcpy(row.data(), r.action + k * r.Ap, r.Ap * 4, hipMemcpyDeviceToHost));
        std::memcpy(action + (size_t)i * r.A, row.data(), r.A * 4);
      }
      if (reward) HIPCHK(hipMemcpy(reward + i, r.reward + k, 4, hipMemcpyDeviceToHost));
      if (notdone) HIPCHK(hipMemcpy(notdone + i, r.notdone + k, 4, hipMemcpyDeviceToHost));
    }
  });
}

int rle_create(const rle_config* cfg, rle_engine** out) {
  return guard([&] {
    REQUIRE(cfg && out, "create: null");
    REQUIRE(cfg->algo >= 0 && cfg->algo <= 2, "create: bad algo");
    REQUIRE(cfg->batch > 0 && cfg->batch <= 1024, "create: batch must be in 1..1024");
    REQUIRE(cfg->state_dim <= 1024 && cfg->action_dim <= 128 && cfg->hidden <= 512,
            "create: state_dim <= 1024, action_dim <= 128, hidden <= 512");
    REQUIRE(cfg->state_dim > 0 && cfg->action_dim > 0 && cfg->hidden > 0 && cfg->hidden % 4 == 0,
            "create: bad dims (hidden must be a multiple of 4)");
    REQUIRE(cfg->zs_dim == 0 || (cfg->algo == RLE_TD7 && cfg->zs_dim > 0 && cfg->zs_dim <= 512 && cfg->zs_dim % 4 == 0),
            "create: zs_dim (TD7 only) must be a multiple of 4, <= 512");
    REQUIRE(cfg->n_hidden == 0 || (cfg->algo != RLE_TD7 && cfg->n_hidden >= 2 && cfg->n_hidden <= RLE_MAX_HIDDEN),
            "create: n_hidden (TD3 / SAC only) must be 2..6");
    for (int i = 0; i < cfg->n_hidden; ++i)
      REQUIRE(cfg->hidden_sizes[i] > 0 && cfg->hidden_sizes[i] <= 512 && cfg->hidden_sizes[i] % 4 == 0,
              "create: hidden_sizes must be multiples of 4, <= 512");
    for (int a : {cfg->act_actor, cfg->act_critic, cfg->act_encoder})
      REQUIRE(a >= RLE_ACT_DEFAULT && a <= RLE_ACT_IDENTITY, "create: activation must be an RLE_ACT_* code");
    REQUIRE(cfg->algo == RLE_TD7 || cfg->act_encoder == RLE_ACT_DEFAULT, "create: act_encoder is TD7's (SALEEncoder)");
    HIPCHK(hipSetDevice(cfg->device));
    auto h = std::make_unique<rle_engine>();
    h->e = std::make_unique<Engine>();
    Engine& e = *h->e;
    e.cfg = *cfg;
    e.algo = cfg->algo;
    e.S = cfg->state_dim;
    e.Sp = rle::r16(e.S);
    e.A = cfg->action_dim;
    e.Ap = rle::r16(e.A);
    // (TD3 / SAC: H is the LAST hidden width -- what the heads and the output layer read; each
    // layer's own width is in HS)
    e.HS.assign(2, cfg->hidden);
    if (cfg->n_hidden) e.HS.assign(cfg->hidden_sizes, cfg->hidden_sizes + cfg->n_hidden);
    e.H = e.algo == RLE_TD7 ? cfg->hidden : e.HS.back();
    e.Hp = rle::r16(e.H);
    e.Z = cfg->zs_dim ? cfg->zs_dim : cfg->hidden;
    e.Zp = rle::r16(e.Z);
    e.Bv = cfg->batch;
    e.B = (cfg->batch + 15) / 16 * 16;  // (padded rows: zero, masked out of every mean, loss and priority)
    // hidden activations (sale.py:25,67,97; mlp.py:13): the reference defaults unless the config names one
    auto act_of = [](int code, int dflt) {
      return code == RLE_ACT_RELU ? rle::ACT_RELU
             : code == RLE_ACT_ELU ? rle::ACT_ELU
             : code == RLE_ACT_IDENTITY ? rle::ACT_NONE
                                        : dflt;
    };
    const bool td7 = e.algo == RLE_TD7;
    e.actP = act_of(cfg->act_actor, rle::ACT_RELU);
    e.actC = act_of(cfg->act_critic, td7 ? rle::ACT_ELU : rle::ACT_RELU);
    e.actE = act_of(cfg->act_encoder, rle::ACT_ELU);
    e.acts_default = e.actP == rle::ACT_RELU && e.actC == (td7 ? rle::ACT_ELU : rle::ACT_RELU) && e.actE == rle::ACT_ELU;
    e.resolve_plan();
    HIPCHK(hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking));
    if (e.algo == RLE_TD7) {
      for (const char* n : {"encoder", "fixed_encoder", "fixed_encoder_target"}) e.nets.push_back(e.make_net(n, "sale_enc"));
      e.nets.push_back(e.make_net("policy", "sale_actor"));
      for (const char* n : {"q1", "q2", "target_q1", "target_q2"}) e.nets.push_back(e.make_net(n, "sale_critic"));
    } else {
      e.nets.push_back(e.make_net("policy", "mlp_actor"));
      for (const char* n : {"q1", "q2", "target_q1", "target_q2"}) e.nets.push_back(e.make_net(n, "mlp_critic"));
    }
    e.layout_params();
    e.ctrl = e.mem.make<rle::Ctrl>(1);
    rle::Ctrl c{};
    c.vmax_key = rle::host_fkey(-1e8f);  // td7.py:84-87
    c.vmin_key = rle::host_fkey(1e8f);
    c.vt[0] = c.vt[1] = 0.f;
    c.max_priority = 1.f;
    HIPCHK(hipMemcpy(e.ctrl, &c, sizeof(c), hipMemcpyHostToDevice));
    if (e.algo == RLE_SAC) {
      const float la = cfg->tmp < 0.f ? 0.f : std::log(cfg->tmp);  // sac.py:56-60
      HIPCHK(hipMemcpy(e.P + (e.nP - 4), &la, 4, hipMemcpyHostToDevice));
    }
    e.info = e.mem.make<float>((size_t)e.info_cap * rle::kInfoMax);
    e.alloc_step_buffers();
    e.refresh_adam_scalars();
    *out = h.release();
  });
}

int rle_plan_default(rle_plan* out) {
  return guard([&] {
    REQUIRE(out, "plan_default: null");
    *out = rle::plan_defaults();
  });
}

int rle_set_plan(rle_engine* h, const rle_plan* plan) {
  return guard([&] {
    REQUIRE(h && plan, "set_plan: null");
    Engine& e = drained(h);
    REQUIRE(!e.built, "set_plan: the engine has already built its step programs (set the plan before the first step)");
    e.plan = *plan;
    e.resolve_plan();
  });
}

int rle_get_plan(rle_engine* h, rle_plan* out) {
  return guard([&] {
    REQUIRE(h && out, "get_plan: null");
    *out = h->e->plan;
  });
}

int rle_destroy(rle_engine* h) {
  return guard([&] {
    if (!h) return;
    Engine& e = *h->e;
    try {
      e.aql_drain();
    } catch (const Error&) {  // (a timed-out burst closed the engine's queue: destroy anyway)
    }
    (void)hipStreamSynchronize(e.stream);
    if (e.replay) {
      auto& us = e.replay->users;
      for (size_t i = 0; i < us.size(); ++i)
        if (us[i].first == &e) {
          us.erase(us.begin() + i);
          break;
        }
    }
    if (e.done_ev) (void)hipEventDestroy(e.done_ev);
    for (rle::Graph* g : {&e.g_prime[0], &e.g_prime[1], &e.g_pol[0], &e.g_pol[1], &e.g_pln[0], &e.g_pln[1],
                          &e.g_pair[0], &e.g_pair[1], &e.g_rem[0][0], &e.g_rem[0][1], &e.g_rem[1][0],
                          &e.g_rem[1][1], &e.g_hard, &e.g_fold, &e.g_slot0}) {
      if (g->x) (void)hipGraphExecDestroy(g->x);
      if (g->g) (void)hipGraphDestroy(g->g);
    }
    for (auto& kv : e.act_graphs) {
      if (kv.second.first.x) (void)hipGraphExecDestroy(kv.second.first.x);
      if (kv.second.first.g) (void)hipGraphDestroy(kv.second.first.g);
    }
    for (auto& kv : e.eval_graphs) {
      if (kv.second.G.x) (void)hipGraphExecDestroy(kv.second.G.x);
      if (kv.second.G.g) (void)hipGraphDestroy(kv.second.G.g);
    }
    (void)hipStreamDestroy(e.stream);
    delete h;
  });
}

int rle_bind_replay(rle_engine* h, rle_replay* r) {
  return guard([&] {
    Engine& e = drained(h);
    REQUIRE(r, "bind: null replay");
    REQUIRE(r->r.S == e.S && r->r.A == e.A, "bind: replay dims differ from agent dims");
    if (e.replay == &r->r) return;
    REQUIRE(!e.built, "bind: engine already bound to another replay");
    if (e.replay) {  // not built yet: move to the new replay
      auto& us = e.replay->users;
      for (size_t i = 0; i < us.size(); ++i)
        if (us[i].first == &e) {
          us.erase(us.begin() + i);
          break;
        }
    }
    e.replay = &r->r;
    e.primed = false;
    if (!e.done_ev) HIPCHK(hipEventCreateWithFlags(&e.done_ev, hipEventDisableTiming));
    r->r.users.push_back({&e, e.done_ev});
  });
}

int rle_param_numel(rle_engine* h, const char* net, const char* name, long long* numel) {
  return guard([&] { *numel = h->e->numel(net, name); });
}
int rle_get_param(rle_engine* h, const char* net, const char* name, float* out, long long n) {
  return guard([&] { drained(h).xfer_param(net, name, out, n, false, 0); });
}
int rle_set_param(rle_engine* h, const char* net, const char* name, const float* in, long long n) {
  return guard([&] { drained(h).xfer_param(net, name, const_cast<float*>(in), n, true, 0); });
}
int rle_get_adam(rle_engine* h, const char* net, const char* name, int which, float* out, long long n) {
  return guard([&] {
    REQUIRE(which == 0 || which == 1, "adam: which in {0,1}");
    drained(h).xfer_param(net, name, out, n, false, 1 + which);
  });
}
int rle_set_adam(rle_engine* h, const char* net, const char* name, int which, const float* in, long long n) {
  return guard([&] {
    REQUIRE(which == 0 || which == 1, "adam: which in {0,1}");
    drained(h).xfer_param(net, name, const_cast<float*>(in), n, true, 1 + which);
  });
}

int rle_get_counters(rle_engine* h, long long* out6) {
  return guard([&] {
    Engine& e = drained(h);
    HIPCHK(hipStreamSynchronize(e.stream));
    rle::Ctrl c;
    HIPCHK(hipMemcpy(&c, e.ctrl, sizeof(c), hipMemcpyDeviceToHost));
    for (int i = 0; i < 5; ++i) out6[i] = c.counters[i];
    out6[3] = e.n_runs;
    out6[5] = c.la_t;
  });
}

int rle_get_act_counter(rle_engine* h, unsigned long long* out) {
  return guard([&] { *out = h->e->act_counter; });
}

int rle_set_act_counter(rle_engine* h, unsigned long long v) {
  return guard([&] { h->e->act_counter = v; });
}

int rle_set_counters(rle_engine* h, const long long* in6) {
  return guard([&] {
    Engine& e = drained(h);
    HIPCHK(hipStreamSynchronize(e.stream));
    rle::Ctrl c;
    HIPCHK(hipMemcpy(&c, e.ctrl, sizeof(c), hipMemcpyDeviceToHost));
    for (int i = 0; i < 5; ++i) c.counters[i] = in6[i];
    c.la_t = in6[5];
    e.n_runs = in6[3];
    e.primed = false;  // the RNG position changed
    HIPCHK(hipMemcpy(e.ctrl, &c, sizeof(c), hipMemcpyHostToDevice));
    e.refresh_adam_scalars();
  });
}

int rle_get_value_bounds(rle_engine* h, float* out4) {
  return guard([&] {
    Engine& e = drained(h);
    HIPCHK(hipStreamSynchronize(e.stream));
    rle::Ctrl c;
    HIPCHK(hipMemcpy(&c, e.ctrl, sizeof(c), hipMemcpyDeviceToHost));
    out4[0] = rle::host_unkey(c.vmax_key);
    out4[1] = rle::host_unkey(c.vmin_key);
    out4[2] = c.vt[0];
    out4[3] = c.vt[1];
  });
}

int rle_set_value_bounds(rle_engine* h, const float* in4) {
  return guard([&] {
    Engine& e = drained(h);
    HIPCHK(hipStreamSynchronize(e.stream));
    rle::Ctrl c;
    HIPCHK(hipMemcpy(&c, e.ctrl, sizeof(c), hipMemcpyDeviceToHost));
    c.vmax_key = rle::host_fkey(in4[0]);
    c.vmin_key = rle::host_fkey(in4[1]);
    c.vt[0] = in4[2];
    c.vt[1] = in4[3];
    HIPCHK(hipMemcpy(e.ctrl, &c, sizeof(c), hipMemcpyHostToDevice));
  });
}

int rle_step(rle_engine* h, int n_steps, float* info_out) {
  return guard([&] {
    REQUIRE(n_steps >= 0, "step: n < 0");
    Engine& e = drained(h);
    HIPCHK(hipSetDevice(e.cfg.device));
    if (e.replay) HIPCHK(hipStreamSynchronize(e.replay->stream));
    e.step(n_steps, info_out);
  });
}

int rle_step_timed(rle_engine* h, int n_steps, float* gpu_ms) {
  return guard([&] {
    REQUIRE(n_steps >= 0 && gpu_ms, "step_timed: bad args");
    Engine& e = drained(h);
    HIPCHK(hipSetDevice(e.cfg.device));
    if (e.replay) HIPCHK(hipStreamSynchronize(e.replay->stream));
    e.step(n_steps, nullptr, gpu_ms);
  });
}

int rle_step_async(rle_engine* h, int n_steps) {
  return guard([&] {
    REQUIRE(n_steps >= 0, "step_async: n < 0");
    Engine& e = *h->e;  // (its earlier bursts stay in flight: the new one queues behind them)
    HIPCHK(hipSetDevice(e.cfg.device));
    if (e.replay) HIPCHK(hipStreamSynchronize(e.replay->stream));
    e.step(n_steps, nullptr, nullptr, true);
  });
}

int rle_set_tapes(rle_engine* h, int n, const float* u, const float* eps, const float* eps_pi, const long long* ind) {
  return guard([&] {
    Engine& e = drained(h);
    HIPCHK(hipStreamSynchronize(e.stream));
    int mode = 0;
    if (n > 0) {
      REQUIRE(n <= 1024, "set_tapes: at most 1024 steps per tape");
      e.ensure_tapes(n);
      const size_t nb = (size_t)n * e.Bv, na = nb * e.A;  // (host tapes: [n][batch rows])
      if (u) HIPCHK(hipMemcpy(e.t_u, u, nb * 4, hipMemcpyHostToDevice));
      if (eps) HIPCHK(hipMemcpy(e.t_eps, eps, na * 4, hipMemcpyHostToDevice));
      if (eps_pi) HIPCHK(hipMemcpy(e.t_eps2, eps_pi, na * 4, hipMemcpyHostToDevice));
      if (ind) {
        const long long size = e.replay ? e.replay->size : 0;
        for (size_t i = 0; i < nb; ++i)
          REQUIRE(ind[i] >= 0 && ind[i] < size, "set_tapes: index outside the bound replay's size");
        HIPCHK(hipMemcpy(e.t_ind, ind, nb * 8, hipMemcpyHostToDevice));
      }
      REQUIRE(u || ind, "set_tapes: need u or ind");
      REQUIRE(e.algo != RLE_SAC || !eps == !eps_pi, "set_tapes: SAC takes eps and eps_pi together");
      mode = (u ? rle::kTapeU : 0) | (ind ? rle::kTapeInd : 0) | (eps ? rle::kTapeEps : 0);
    }
    rle::Ctrl c;
    HIPCHK(hipMemcpy(&c, e.ctrl, sizeof(c), hipMemcpyDeviceToHost));
    c.tape_mode = mode;
    c.counters[5] = 0;
    HIPCHK(hipMemcpy(e.ctrl, &c, sizeof(c), hipMemcpyHostToDevice));
    e.ctrl_tape_mode_host = mode;
    e.tape_left = n;
    e.primed = false;  // a prefetched batch was drawn from the previous draws
  });
}

int rle_last_indices(rle_engine* h, long long* out) {
  return guard([&] {
    Engine& e = drained(h);
    HIPCHK(hipStreamSynchronize(e.stream));
    HIPCHK(hipMemcpy(out, e.bsets[e.last_set].ind, e.Bv * sizeof(long long), hipMemcpyDeviceToHost));
  });
}

int rle_act(rle_engine* h, const float* obs, int n, float* out) {
  return guard([&] {
    Engine& e = drained(h);
    REQUIRE(n > 0 && n <= 1024, "act: 0 < n <= 1024");
    HIPCHK(hipSetDevice(e.cfg.device));
    auto it = e.act_graphs.find(n);
    if (it == e.act_graphs.end()) {
      rle::Prog pg;
      const int M = rle::r16(n);  // image rows; rows n..M-1 are padding
      rle::View in = e.buf(M, e.S, true, false);
      rle::View o;
      if (e.algo == RLE_TD7) {  // td7.py:158-162
        rle::Net& fe = e.net("fixed_encoder");
        rle::Net& pi = e.net("policy");
        rle::View h1 = e.fwd(pg, fe.layers[0], {{in}}, M, e.actE, nullptr, false);
        rle::View h2 = e.fwd(pg, fe.layers[1], {{h1}}, M, e.actE, nullptr, false);
        rle::View zs = e.fwd(pg, fe.layers[2], {{h2}}, M, rle::ACT_NONE, nullptr, true);
        rle::View p0 = e.fwd(pg, pi.layers[0], {{in}}, M, rle::ACT_NONE, nullptr, true);
        rle::View p1 = e.fwd(pg, pi.layers[1], {{p0}, {zs}}, M, e.actP, nullptr, false);
        rle::View p2 = e.fwd(pg, pi.layers[2], {{p1}}, M, e.actP, nullptr, false);
        o = e.fwd(pg, pi.layers[3], {{p2}}, M, rle::ACT_TANH, nullptr, false);
      } else {
        o = e.mlp_fwd(pg, e.net("policy"), {{in}}, M, rle::ACT_NONE, e.actP);
      }
      rle::Graph G = e.capture(pg);
      it = e.act_graphs.emplace(n, std::make_pair(G, o)).first;
      e.act_inputs[n] = in;
    }
    rle::View in = e.act_inputs[n];
    rle::View o = it->second.second;
    const int W = e.algo == RLE_SAC ? 2 * e.A : e.A;
    const int M = rle::r16(n);
    std::vector<float> img((size_t)M * in.cols, 0.f);
    for (int i = 0; i < n; ++i)
      for (int c = 0; c < e.S; ++c) img[Engine::h_nidx(in.m.cbn, i, c)] = obs[(size_t)i * e.S + c];
    HIPCHK(hipMemcpyAsync(in.m.n, img.data(), img.size() * 4, hipMemcpyHostToDevice, e.stream));
    HIPCHK(hipGraphLaunch(it->second.first.x, e.stream));
    std::vector<float> res((size_t)M * o.cols);
    HIPCHK(hipMemcpyAsync(res.data(), o.m.t, res.size() * 4, hipMemcpyDeviceToHost, e.stream));
    HIPCHK(hipStreamSynchronize(e.stream));
    for (int i = 0; i < n; ++i)
      for (int c = 0; c < W; ++c) out[(size_t)i * W + c] = res[Engine::h_tidx(o.m.rbs, i, c)];
  });
}

int rle_set_action_map(rle_engine* h, const float* scale, const float* bias, float exploration_noise) {
  return guard([&] {
    Engine& e = drained(h);
    REQUIRE(scale && bias, "set_action_map: null scale / bias");
    HIPCHK(hipSetDevice(e.cfg.device));
    e.ensure_action_map();
    std::vector<float> m((size_t)2 * e.A + 1);
    std::copy(scale, scale + e.A, m.begin());
    std::copy(bias, bias + e.A, m.begin() + e.A);
    m[2 * e.A] = exploration_noise;
    HIPCHK(hipStreamSynchronize(e.stream));
    HIPCHK(hipMemcpy(e.act_map, m.data(), m.size() * 4, hipMemcpyHostToDevice));
  });
}

int rle_act_sample(rle_engine* h, const float* obs, int n, int mode, const float* eps, float* out) {
  return guard([&] {
    Engine& e = drained(h);
    REQUIRE(n > 0 && n <= 1024 && obs && out, "act_sample: 0 < n <= 1024, obs and out");
    REQUIRE(mode >= 0 && mode <= 2 && (mode != 2 || eps), "act_sample: mode 0 / 1 / 2 (2 needs eps)");
    HIPCHK(hipSetDevice(e.cfg.device));
    e.ensure_action_map();
    auto it = e.act_samplers.find(n);
    if (it == e.act_samplers.end()) {
      Engine::ActSample as;
      const int M = rle::r16(n);
      as.in = e.buf(M, e.S, true, false);
      as.img = (float*)e.pin.alloc((size_t)M * as.in.cols * 4);
      as.ctl = (int*)e.pin.alloc(64);
      as.eps = (float*)e.pin.alloc((size_t)n * e.A * 4);
      as.out = (float*)e.pin.alloc((size_t)n * e.A * 4);
      rle::ActArgs ao{};
      HIPCHK(hipHostGetDevicePointer((void**)&ao.out, as.out, 0));
      HIPCHK(hipHostGetDevicePointer((void**)&ao.ctl, as.ctl, 0));
      HIPCHK(hipHostGetDevicePointer((void**)&ao.eps, as.eps, 0));
      ao.scale = e.act_map;
      ao.bias = e.act_map + e.A;
      ao.sigma = e.act_map + 2 * e.A;
      ao.n = n;
      ao.A = e.A;
      ao.seed = e.cfg.seed * 0x9E3779B97F4A7C15ull + 0x5851F42D4C957F2Dull;  // own stream, not the step's
      rle::Prog pg;
      rle::View in = as.in;
      auto tanh_act = [&](rle::Prog& p) {  // the last GEMM becomes the act epilogue (EPI_ACT)
        rle::Op& op = p.items.back().ops[0];
        op.gemm.epi = rle::EPI_ACT;
        op.gemm.ao = ao;
        rle::gemm_finalize(op.gemm);
      };
      if (e.algo == RLE_TD7) {  // td7.py:141-162
        rle::Net& fe = e.net("fixed_encoder");
        rle::Net& pi = e.net("policy");
        rle::View h1 = e.fwd(pg, fe.layers[0], {{in}}, M, e.actE, nullptr, false);
        rle::View h2 = e.fwd(pg, fe.layers[1], {{h1}}, M, e.actE, nullptr, false);
        rle::View zs = e.fwd(pg, fe.layers[2], {{h2}}, M, rle::ACT_NONE, nullptr, true);
        rle::View p0 = e.fwd(pg, pi.layers[0], {{in}}, M, rle::ACT_NONE, nullptr, true);
        rle::View p1 = e.fwd(pg, pi.layers[1], {{p0}, {zs}}, M, e.actP, nullptr, false);
        rle::View p2 = e.fwd(pg, pi.layers[2], {{p1}}, M, e.actP, nullptr, false);
        e.fwd(pg, pi.layers[3], {{p2}}, M, rle::ACT_TANH, nullptr, false);
        tanh_act(pg);
      } else if (e.algo == RLE_TD3) {  // td3.py:114-135
        e.mlp_fwd(pg, e.net("policy"), {{in}}, M, rle::ACT_TANH, e.actP);
        tanh_act(pg);
      } else {  // sac.py:132-159
        rle::View raw = e.mlp_fwd(pg, e.net("policy"), {{in}}, M, rle::ACT_NONE, e.actP);
        rle::Op op{};
        op.kind = rle::OP_SAC_ACTOR;
        rle::SacActorArgs& sa = op.sac;
        sa.ao = ao;
        sa.out = raw.m;
        sa.A = e.A;
        sa.rows = n;
        sa.min_log_std = e.cfg.min_log_std;
        sa.max_log_std = e.cfg.max_log_std;
        sa.mean_off = 0;
        sa.ls_off = e.A;
        op.wg_count = rle::cdiv(n, rle::kThreads);
        pg.add(op, {raw.id}, {});
      }
      as.G = e.capture(pg);
      it = e.act_samplers.emplace(n, as).first;
    }
    Engine::ActSample& as = it->second;
    if (n == 1 && !e.chain_tried) {
      e.chain_tried = true;
      static const bool no_chain = std::getenv("RLE_NO_ACT_CHAIN") != nullptr;  // A/B
      rle::ActArgs ao{};
      HIPCHK(hipHostGetDevicePointer((void**)&ao.out, as.out, 0));
      HIPCHK(hipHostGetDevicePointer((void**)&ao.ctl, as.ctl, 0));
      HIPCHK(hipHostGetDevicePointer((void**)&ao.eps, as.eps, 0));
      ao.scale = e.act_map;
      ao.bias = e.act_map + e.A;
      ao.sigma = e.act_map + 2 * e.A;
      ao.n = 1;
      ao.A = e.A;
      ao.seed = e.cfg.seed * 0x9E3779B97F4A7C15ull + 0x5851F42D4C957F2Dull;
      e.chain_ok = !no_chain && e.build_chain(ao);
    }
    if (n == 1 && e.chain_ok) {  // one launch, in-kernel hand-offs (kernels.hip rle_act_chain)
      rle::ActChainArgs& c = e.chain;
      std::memset(c.obs, 0, sizeof c.obs);
      std::memcpy(c.obs, obs, (size_t)e.S * 4);
      if (++e.chain_tag >= 0x80000000u) e.chain_tag = 1;  // (bit 31 marks poisoned granules)
      c.tag = e.chain_tag;
      as.ctl[8] = 0;  // the error flag of this call (set by a head workgroup whose hand-off failed)
      c.mode = mode;
      c.ctr_lo = (unsigned)e.act_counter;
      c.ctr_hi = (unsigned)(e.act_counter >> 32);
      if (mode == 1) ++e.act_counter;
      if (mode == 2) std::memcpy(c.eps, eps, (size_t)e.A * 4);
      static const bool cprof = std::getenv("RLE_ACT_PROF") != nullptr;
      static double cp[3] = {0, 0, 0};
      static long long ccalls = 0;
      static hipEvent_t ce0 = nullptr, ce1 = nullptr;
      static std::vector<double> sacc;
      if (cprof && !ce0) {
        HIPCHK(hipEventCreate(&ce0));
        HIPCHK(hipEventCreate(&ce1));
        c.stamps = e.mem.make<unsigned long long>((size_t)c.nwg * 16);
        sacc.assign(16, 0.0);
      }
      const auto t0 = std::chrono::steady_clock::now();
      if (cprof) HIPCHK(hipEventRecord(ce0, e.stream));
      HIPCHK(rle::launch_act_chain(c, e.stream));
      c.fail_wg = -1;
      if (cprof) HIPCHK(hipEventRecord(ce1, e.stream));
      const auto t1 = std::chrono::steady_clock::now();
      // the head workgroups' completion tags (system-scope release after their action stores):
      // poll pinned memory instead of waiting for the stream; a failed launch ends the poll
      for (int hw = 0; hw < c.heads; ++hw) {
        for (long long k = 1; e.done_host[hw] != c.tag; ++k) {
          if ((k & 4095) == 0 && hipStreamQuery(e.stream) != hipErrorNotReady) {
            HIPCHK(hipStreamSynchronize(e.stream));
            REQUIRE(e.done_host[hw] == c.tag, "act chain: the kernel ended without its completion tag");
            break;
          }
        }
      }
      std::atomic_thread_fence(std::memory_order_acquire);
      const auto t2 = std::chrono::steady_clock::now();
      if (cprof) HIPCHK(hipStreamSynchronize(e.stream));
      REQUIRE(((volatile int*)as.ctl)[8] == 0, "act chain: a workgroup hand-off failed");
      std::memcpy(out, as.out, (size_t)e.A * 4);
      if (cprof) {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, ce0, ce1));
        cp[0] += std::chrono::duration<double, std::micro>(t1 - t0).count();
        cp[1] += std::chrono::duration<double, std::micro>(t2 - t1).count();
        cp[2] += ms * 1e3;
        std::vector<unsigned long long> sv((size_t)c.nwg * 16);
        HIPCHK(hipMemcpy(sv.data(), c.stamps, sv.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0s = ~0ull;
        for (int q = 0; q < c.nwg; ++q) t0s = std::min(t0s, sv[(size_t)q * 16]);
        for (int k = 1; k < 16; ++k) {  // latest workgroup to reach stamp k, after the first start
          unsigned long long mx = 0;
          for (int q = 0; q < c.nwg; ++q) mx = std::max(mx, sv[(size_t)q * 16 + k]);
          sacc[k] += mx > t0s ? (double)(mx - t0s) * 0.01 : 0.0;  // 100 MHz ticks -> us
        }
        HIPCHK(hipMemset(c.stamps, 0, sv.size() * 8));
        if (++ccalls % 2000 == 0) {
          fprintf(stderr, "act chain (us/call): launch %.2f  sync %.2f  kernel (events) %.2f\n", cp[0] / 2000,
                  cp[1] / 2000, cp[2] / 2000);
          fprintf(stderr, "  stamps (us after first start, latest wg): load %.2f", sacc[1] / 2000);
          for (int k = 2; k < 15; ++k)
            if (sacc[k] > 0) fprintf(stderr, " | hand-off %d %.2f", k - 1, sacc[k] / 2000);
          fprintf(stderr, " | head %.2f\n", sacc[15] / 2000);
          cp[0] = cp[1] = cp[2] = 0;
          std::fill(sacc.begin(), sacc.end(), 0.0);
        }
      }
      return;
    }
    const int M = rle::r16(n);
    static const bool prof = std::getenv("RLE_ACT_PROF") != nullptr;  // phase times, tools/act_bench.py
    static double tp[4] = {0, 0, 0, 0};
    static long long calls = 0;
    auto now = [] { return std::chrono::steady_clock::now(); };
    const auto t0 = now();
    for (int i = 0; i < n; ++i)
      for (int c = 0; c < e.S; ++c) as.img[Engine::h_nidx(as.in.m.cbn, i, c)] = obs[(size_t)i * e.S + c];
    as.ctl[0] = mode;
    as.ctl[1] = (int)(unsigned)e.act_counter;
    as.ctl[2] = (int)(unsigned)(e.act_counter >> 32);
    if (mode == 1) ++e.act_counter;
    if (mode == 2) std::memcpy(as.eps, eps, (size_t)n * e.A * 4);
    HIPCHK(hipMemcpyAsync(as.in.m.n, as.img, (size_t)M * as.in.cols * 4, hipMemcpyHostToDevice, e.stream));
    const auto t1 = now();
    e.launch_graph(as.G);
    const auto t2 = now();
    HIPCHK(hipStreamSynchronize(e.stream));
    const auto t3 = now();
    std::memcpy(out, as.out, (size_t)n * e.A * 4);
    if (prof) {
      tp[0] += std::chrono::duration<double, std::micro>(t1 - t0).count();
      tp[1] += std::chrono::duration<double, std::micro>(t2 - t1).count();
      tp[2] += std::chrono::duration<double, std::micro>(t3 - t2).count();
      if (++calls % 2000 == 0) {
        fprintf(stderr, "act_sample phases (us/call): stage+H2D %.2f  graph launch %.2f  sync %.2f\n", tp[0] / 2000,
                tp[1] / 2000, tp[2] / 2000);
        tp[0] = tp[1] = tp[2] = 0;
      }
    }
  });
}

int rle_launch_count(rle_engine* h, long long* n) {
  return guard([&] {
    REQUIRE(n, "launch_count: null out");
    *n = h->e->launches;
  });
}

int rle_graph_stats(rle_engine* h, int* lp, int* lplain) {
  return guard([&] {
    Engine& e = drained(h);
    if (!e.built) e.build();
    if (lp) *lp = e.policy_graph().levels();
    if (lplain) *lplain = e.plain_graph().levels();
  });
}

int rle_graph_describe(rle_engine* h, int which, char* buf, int len) {
  return guard([&] {
    Engine& e = drained(h);
    if (!e.built) e.build();
    const rle::Graph& G = which == 0 ? e.policy_graph()
                          : which == 1 ? e.plain_graph()
                          : which == 3 ? e.g_pair[e.pol_set]
                                       : e.g_hard;
    REQUIRE(buf && len > 0, "describe: bad buffer");
    std::snprintf(buf, (size_t)len, "%s", G.desc.c_str());
  });
}

int rle_graph_trace(rle_engine* h, int which, unsigned long long* out, long long cap, long long* n_out) {
  return guard([&] {
    Engine& e = drained(h);
    REQUIRE(n_out, "trace: null n_out");
    if (!e.built) e.build();
    const rle::Graph& G = which == 0 ? e.policy_graph()
                          : which == 1 ? e.plain_graph()
                          : which == 3 ? e.g_pair[e.pol_set]
                                       : e.g_hard;
    *n_out = G.trace ? G.trace_n : 0;
    if (!G.trace || !out) return;
    const int st = rle::trace_stride();
    REQUIRE(cap >= G.trace_n * st, "trace: buffer too small");
    HIPCHK(hipStreamSynchronize(e.stream));
    HIPCHK(hipMemcpy(out, G.trace, (size_t)G.trace_n * st * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    *n_out = G.trace_n;
  });
}

int rle_trace_stride(void) { return rle::trace_stride(); }

// The failed-queue state machine of the AQL path without a device (no HSA call is reached): a closed
// queue refuses new bursts and completes at once, for the engine that timed out and for every engine
// sharing its hardware queue; doorbell groups never straddle the ring's end.
int rle_aql_selftest(void) {
  return guard([&] {
    using namespace rle;
    auto hw = std::make_shared<AqlHw>();
    AqlQueue a, b;
    a.hw = hw;
    b.hw = hw;
    REQUIRE(!a.closed() && !b.closed(), "selftest: fresh queues closed");
    a.failed = true;
    hw->failed = true;  // (as aql_wait's timeout leaves them)
    a.pending.push_back({nullptr, 1, 0});
    a.inflight = 7;
    int refused = 0;
    try {
      aql_submit(a);
    } catch (const Error&) {
      ++refused;
    }
    REQUIRE(refused == 1 && a.pending.empty(), "selftest: a closed queue took a burst");
    try {
      aql_complete(a, nullptr);
    } catch (const Error&) {
      ++refused;
    }
    REQUIRE(refused == 2 && a.inflight == 0, "selftest: a closed queue waited for its burst");
    aql_complete(a, nullptr);  // (nothing in flight: returns)
    b.pending.push_back({nullptr, 1, 0});
    try {
      aql_submit(b);
    } catch (const Error&) {
      ++refused;
    }
    REQUIRE(refused == 3, "selftest: an engine sharing a failed hardware queue took a burst");
    // doorbell groups: for every start index, the packets between two doorbells lie in one pass of the ring
    for (uint64_t size : {64ull, 1024ull, 16384ull})
      for (uint64_t start = size - 130; start < size + 130; ++start)
        for (uint64_t n : {1ull, 5ull, 64ull, 200ull}) {
          uint64_t first = start;
          for (uint64_t i = start; i < start + n; ++i)
            if (aql_doorbell_after(i, i + 1 == start + n)) {
              REQUIRE(first / size == i / size, "selftest: a doorbell group straddles the ring's end");
              first = i + 1;
            }
          REQUIRE(first == start + n, "selftest: packets left without a doorbell");
        }
    a.hw.reset();
    b.hw.reset();
  });
}

int rle_aql_wait_plan(double expected_us, double elapsed_us, double timeout_s, double* sleep_us) {
  double sl = 0.0;
  const int act = rle::aql_wait_step(expected_us, elapsed_us, timeout_s, &sl);
  if (sleep_us) *sleep_us = sl;
  return act;
}

int rle_copy_state(rle_engine* dst, rle_engine* src) {
  return guard([&] {
    Engine& d = drained(dst);
    Engine& s = drained(src);
    REQUIRE(d.nP == s.nP && d.algo == s.algo, "copy_state: config mismatch");
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(d.P, s.P, 3 * d.nP * sizeof(float), hipMemcpyDeviceToDevice));
    rle::Ctrl c;
    HIPCHK(hipMemcpy(&c, s.ctrl, sizeof(c), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(d.ctrl, &c, sizeof(c), hipMemcpyHostToDevice));
    d.n_runs = s.n_runs;
    d.primed = false;
    d.fold_dirty = true;
  });
}

int rle_eval(rle_engine* h, int what, const char* net, const char* enc, const float* s, const float* a, int n,
             float* out) {
  return guard([&] {
    REQUIRE(h && net && s && out && n > 0 && n <= 1024, "eval: bad args (0 < n <= 1024)");
    REQUIRE(what == RLE_EVAL_Q || what == RLE_EVAL_ZS || what == RLE_EVAL_ZSA, "eval: bad `what`");
    REQUIRE(what == RLE_EVAL_ZS || a, "eval: needs actions");
    Engine& e = drained(h);
    const bool td7 = e.algo == RLE_TD7;
    REQUIRE(what == RLE_EVAL_Q || td7, "eval: encoder outputs exist for TD7 only");
    REQUIRE(!(td7 && what == RLE_EVAL_Q) || enc, "eval: TD7 critics need the encoder of their embeddings");
    HIPCHK(hipSetDevice(e.cfg.device));
    const std::string key = std::to_string(what) + "|" + net + "|" + (enc ? enc : "") + "|" + std::to_string(n);
    auto it = e.eval_graphs.find(key);
    if (it == e.eval_graphs.end()) {
      rle::Net& N = e.net(net);
      rle::Prog pg;
      const int M = rle::r16(n);
      Engine::EvalGraph eg;
      eg.in0 = e.buf(M, e.S, true, false);
      eg.in1 = e.buf(M, e.A, true, false);
      if (what == RLE_EVAL_Q) {
        if (td7) {  // SALECritic.estimate_q_value (sale.py:106-121) on (s, a, zsa, zs) of `enc`
          rle::Net& E = e.net(enc);
          REQUIRE(N.kind == "sale_critic" && E.kind == "sale_enc", "eval: Q needs a critic net and an encoder");
          rle::View zs = e.enc_zs(pg, E, eg.in0, M);
          rle::View zsa = e.enc_zsa(pg, E, zs, eg.in1, M);
          rle::View c01 = e.fwd(pg, N.layers[0], {{eg.in0}, {eg.in1}}, M, rle::ACT_NONE, nullptr, true);
          rle::View c1 = e.fwd(pg, N.layers[1], {{c01}, {zsa}, {zs}}, M, e.actC, nullptr, false);
          rle::View c2 = e.fwd(pg, N.layers[2], {{c1}}, M, e.actC, nullptr, false);
          eg.out = e.fwd(pg, N.layers[3], {{c2}}, M, rle::ACT_NONE, nullptr, false);
        } else {  // MLPCritic.estimate_q_value (mlp.py:98-101)
          REQUIRE(N.kind == "mlp_critic", "eval: Q needs a critic net");
          eg.out = e.mlp_fwd(pg, N, {{eg.in0}, {eg.in1}}, M, rle::ACT_NONE, e.actC);
        }
        eg.width = 1;
      } else {
        REQUIRE(N.kind == "sale_enc", "eval: ZS / ZSA need an encoder net");
        rle::View zs = e.enc_zs(pg, N, eg.in0, M);
        eg.out = what == RLE_EVAL_ZS ? e.normfwd(pg, zs) : e.enc_zsa(pg, N, zs, eg.in1, M);
        eg.width = e.Z;
      }
      eg.G = e.capture(pg);
      it = e.eval_graphs.emplace(key, eg).first;
    }
    Engine::EvalGraph& eg = it->second;
    e.upload(eg.in0, s, n, e.S);
    if (a) e.upload(eg.in1, a, n, e.A);
    HIPCHK(hipGraphLaunch(eg.G.x, e.stream));
    e.download(eg.out, out, n, eg.width);
  });
}

int rle_sac_rsample(rle_engine* h, const float* mean, const float* log_std, const float* eps, int n, float* action,
                    float* log_pi) {
  return guard([&] {
    REQUIRE(h && mean && log_std && eps && action && log_pi && n > 0 && n <= 1024, "sac_rsample: bad args");
    Engine& e = drained(h);
    REQUIRE(e.algo == RLE_SAC, "sac_rsample: SAC engines only");
    HIPCHK(hipSetDevice(e.cfg.device));
    const int A = e.A;
    const std::string key = "rsample|" + std::to_string(n);
    auto it = e.eval_graphs.find(key);
    if (it == e.eval_graphs.end()) {
      rle::Prog pg;
      const int M = rle::r16(n);
      Engine::EvalGraph eg;
      eg.in0 = e.buf(M, 2 * A);              // raw head output: mean | log_std (as mlp.4's output)
      eg.in1 = e.buf(M, A, false, true);     // eps
      eg.out = e.buf(M, A);                  // tanh action
      rle::View lp = e.vec(M);
      eg.out_vec = lp.p;
      rle::Op op{};
      op.kind = rle::OP_SAC_ACTOR;
      rle::SacActorArgs& sa = op.sac;
      sa.out = eg.in0.m;
      sa.A = A;
      sa.rows = n;
      sa.eps = eg.in1.m;
      sa.eps2 = eg.in1.m;
      sa.eps_row_split = 0;  // every row draws from eps
      sa.act = eg.out.m;
      sa.logpi = lp.p;
      sa.min_log_std = e.cfg.min_log_std;
      sa.max_log_std = e.cfg.max_log_std;
      sa.mean_off = 0;
      sa.ls_off = A;
      op.wg_count = rle::cdiv(n, rle::kThreads);
      pg.add(op, {eg.in0.id, eg.in1.id}, {eg.out.id, lp.id});
      eg.width = A;
      eg.G = e.capture(pg);
      it = e.eval_graphs.emplace(key, eg).first;
    }
    Engine::EvalGraph& eg = it->second;
    std::vector<float> raw((size_t)n * 2 * A);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < A; ++j) {
        raw[(size_t)i * 2 * A + j] = mean[(size_t)i * A + j];
        raw[(size_t)i * 2 * A + A + j] = log_std[(size_t)i * A + j];
      }
    e.upload(eg.in0, raw.data(), n, 2 * A);
    e.upload(eg.in1, eps, n, A);
    HIPCHK(hipGraphLaunch(eg.G.x, e.stream));
    e.download(eg.out, action, n, A);
    HIPCHK(hipMemcpy(log_pi, eg.out_vec, (size_t)n * 4, hipMemcpyDeviceToHost));
  });
}

int rle_get_info(rle_engine* h, int n, float* out) {
  return guard([&] {
    Engine& e = drained(h);
    REQUIRE(out && n >= 0 && n <= e.info_cap, "get_info: 0 <= n <= info capacity (4096)");
    HIPCHK(hipStreamSynchronize(e.stream));
    HIPCHK(hipMemcpy(out, e.info, (size_t)n * rle::kInfoMax * sizeof(float), hipMemcpyDeviceToHost));
  });
}

int rle_synchronize(rle_engine* h) {
  return guard([&] { HIPCHK(hipStreamSynchronize(drained(h).stream)); });
}

}  // extern "C"
