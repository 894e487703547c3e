// Device side of the MI355X off-policy update engine (gfx950 / CDNA4).
//
// A gradient step is a DAG of ops scheduled into dependency levels on the
// host (engine.cpp).  Each level is ONE launch of `rle_level`, whose
// workgroups are partitioned over that level's ops (Op::wg_begin); every
// workgroup is 256 threads (4 waves of 64).  The whole step is captured into
// a hipGraph, so one gradient step = one graph launch, no host sync.
//
// Memory-access discipline (what makes a level fast on CDNA4): op descriptors
// are read through the constant address space (scalar loads into SGPRs, no
// per-field latency chains) and every tensor access goes through the global
// address space (global_load/store, counted on vmcnt only) -- plain C++
// pointers loaded from a descriptor would compile to flat loads that force
// `s_waitcnt vmcnt(0) lgkmcnt(0)` after every access.
//
// Op kinds (reference rows they implement):
//   GEMM          Linear forward / input-grad / weight-grad+Adam for every layer
//                 of rl/nn/{sale,mlp}.py (a6-a11, a24), v_mfma_f32_16x16x4_f32
//   NORMBWD       AvgL1Norm backward (sale.py:11-13)
//   SAMPLE_*      LAPReplayMemory.sample / SimpleReplayMemory.sample (a2, a3)
//   HEAD          critic heads + TD target / losses / priority (a13, a14, a17,
//                 a18, a21, a22)
//   PRIORITY      LAPReplayMemory.update_priority (a4)
//   SAC_ACTOR*    SAC._inference/_rsample forward/backward (a20)
//   POLYAK/COPY   target updates (a15, a19, a23); MAXRED reset_max_priority (a5)
//   STEP_END      info row, optimizer/RNG counters, SAC temperature Adam
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <cstring>
#include <type_traits>
#include <vector>

#include "ops.h"

#define CAS __attribute__((address_space(4)))
#define GAS __attribute__((address_space(1)))

namespace rle {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <class T>
__device__ __forceinline__ const GAS T* G(const T* p) {
  return (const GAS T*)p;
}
template <class T>
__device__ __forceinline__ GAS T* GW(T* p) {
  return (GAS T*)p;
}
// Uniform control value written by an earlier launch: scalar load (s_load, issued
// with the other descriptor loads) instead of a vector load and its round trip.
template <class T>
__device__ __forceinline__ T sload(const T* p) {
  return *(const CAS T*)p;
}

// ---------------------------------------------------------------- utilities

__device__ __forceinline__ float4 ld4g(const GAS float* p) {
  const f32x4 v = *(const GAS f32x4*)p;
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st4g(GAS float* p, const float4& v) {
  f32x4 w;
  w.x = v.x; w.y = v.y; w.z = v.z; w.w = v.w;
  *(GAS f32x4*)p = w;
}
// Write-through store (sc1): the bytes leave the XCD's L2 during the kernel instead of staying dirty for the
// launch's end-of-kernel release (its L2 write-back costs ~bytes / 6 TB/s at every level boundary).  For data
// nothing reads again soon (Adam moments, the weights' T image).  (s_nop 1: the asm store's data registers
// must not be overwritten right behind it.)
__device__ __forceinline__ void st4wt(GAS float* p, const f32x4& w) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
}

// Cross-lane reductions through DPP (register-to-register, a few cycles per step)
// instead of ds_bpermute shuffles (an LDS round trip each).  Fixed order:
// quad butterflies, row rotations, then row broadcasts into lane 63.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_f(float v) {  // lanes outside ROW_MASK read 0
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf, false));
}
// Sum over each row of 16 lanes, result in every lane of the row.
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xb1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4e>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x124>(v);  // row_ror:4
  v += dpp_f<0x128>(v);  // row_ror:8
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
  v = row16_sum(v);
  v += dpp_f<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_f<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROW_MASK, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum_d(double v) {
  v += dpp_d<0xb1>(v);
  v += dpp_d<0x4e>(v);
  v += dpp_d<0x124>(v);
  v += dpp_d<0x128>(v);
  v += dpp_d<0x142, 0xa>(v);
  v += dpp_d<0x143, 0xc>(v);
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// Deterministic per-workgroup sum (tree inside waves, fixed wave order).
__device__ __forceinline__ float wg_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return r;
}

// Ordered-int key of a float: monotone under signed int comparison.
__device__ __forceinline__ int fkey(float f) {
  int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float unkey(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7FFFFFFF); }

// Philox4x32-10 counter-based RNG.
__device__ __forceinline__ uint4 philox(uint2 key, uint4 c) {
#pragma unroll 1
  for (int i = 0; i < 10; ++i) {
    unsigned hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    unsigned hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ key.x, lo1, hi0 ^ c.w ^ key.y, lo0);
    key.x += 0x9E3779B9u;
    key.y += 0xBB67AE85u;
  }
  return c;
}
__device__ __forceinline__ float u01(unsigned x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
__device__ __forceinline__ float normal_from(unsigned a, unsigned b) {
  // Box-Muller on the hardware transcendental units (no range reduction needed:
  // v_cos_f32 takes revolutions): sqrt(-2 ln u1) * cos(2 pi u2), u1 in (0, 1]
  const float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);
  const float u2 = (float)(b >> 8) * (1.0f / 16777216.0f);
  const float l = __builtin_amdgcn_logf(u1) * -1.3862943611198906f;  // -2 ln u1 = -2 ln2 log2 u1
  return __builtin_sqrtf(l) * __builtin_amdgcn_cosf(u2);
}

// AvgL1Norm mean |x| of a row from column-tile partial |x| sums (sequential order);
// the partials are loaded 16 at a time (clamped, independent) so a row costs one
// memory round trip per 16 partials.
__device__ __attribute__((noinline)) float norm_mean(const float* part, int ld, int row, int nparts, int width) {
  const GAS float* p = G(part) + row;
  float s = 0.f;
  for (int q0 = 0; q0 < nparts; q0 += 16) {
    float v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = p[(size_t)min(q0 + q, nparts - 1) * ld];
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (q0 + q < nparts) s += v[q];
  }
  return s / (float)width;
}
// Inline copy for operand scaling that must overlap loads already in flight (a call would
// make the caller wait for them).
__device__ __forceinline__ float norm_mean_i(const float* part, int ld, int row, int nparts, int width) {
  const GAS float* p = G(part) + row;
  float s = 0.f;
  for (int q0 = 0; q0 < nparts; q0 += 16) {
    float v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = p[(size_t)min(q0 + q, nparts - 1) * ld];
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (q0 + q < nparts) s += v[q];
  }
  return s / (float)width;
}
// Denominator m = clamp(mean, min=1e-8) (rl/nn/sale.py:11-13).
__device__ __forceinline__ float norm_m(const float* part, int ld, int row, int nparts, int width) {
  const float m = norm_mean(part, ld, row, nparts, width);
  return m < 1e-8f ? 1e-8f : m;
}

__device__ __forceinline__ float act_fwd(int act, float v) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_ELU: return v > 0.f ? v : expm1f(v);
    case ACT_TANH: return tanhf(v);
    default: return v;
  }
}

// Derivative mask given the saved tensor: ReLU/tanh from the output H,
// ELU from the pre-activation Z (torch elu_backward uses the input).
__device__ __forceinline__ float act_bwd(int act, float saved) {
  switch (act) {
    case ACT_RELU: return saved > 0.f ? 1.f : 0.f;
    case ACT_ELU: return saved > 0.f ? 1.f : expf(saved);
    case ACT_TANH: return 1.f - saved * saved;
    default: return 1.f;
  }
}

__device__ __forceinline__ float norm_inv(const CAS NormRef& nr, int row) {
  return 1.f / norm_m(nr.part, nr.ld, row + nr.row0, nr.nparts, nr.width);
}
__device__ __forceinline__ float norm_inv_i(const CAS NormRef& nr, int row) {
  const float m = norm_mean_i(nr.part, nr.ld, row + nr.row0, nr.nparts, nr.width);
  return 1.f / (m < 1e-8f ? 1e-8f : m);
}

// Sums of the first nparts (<= PMAX) row partials, in partial order as norm_mean adds them, of rows
// tid + kThreads r (r < RPT, clamped to n - 1) of a partial array: every load issued together, clamped instead
// of branched, so a thread pays one memory round trip for all its rows.  (The weight gradients' AvgL1Norm
// tables cover the whole batch: 4 rows per thread at B = 1024, where one round trip per row cost 7-12 us per
// workgroup, DESIGN round 5.)
template <int RPT, int PMAX>
__device__ __forceinline__ void row_sums(const float* part, int ld, int row0, int nparts, int n, float (&s)[RPT]) {
  const GAS float* p = G(part) + row0;
  float v[RPT][PMAX];
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int i = min((int)threadIdx.x + r * kThreads, n - 1);
#pragma unroll
    for (int q = 0; q < PMAX; ++q) v[r][q] = p[(size_t)min(q, nparts - 1) * ld + i];
  }
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < PMAX; ++q)
      if (q < nparts) a += v[r][q];
    s[r] = a;
  }
}

// LDS table of 1/m for n consecutive rows of a normed tensor (16-padded with 0).
template <int RPT, int PMAX>
__device__ __forceinline__ void norm_tab_batched(const CAS NormRef& nr, int n, float* dst) {
  float sm[RPT];
  row_sums<RPT, PMAX>(nr.part, nr.ld, nr.row0, nr.nparts, n, sm);
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int i = threadIdx.x + r * kThreads;
    const float m = sm[r] / (float)nr.width;
    if (i < n) dst[i] = 1.f / (m < 1e-8f ? 1e-8f : m);  // (norm_inv_i's floats)
  }
}
__device__ __forceinline__ void build_norm_tab(const CAS NormRef& nr, int n, float* dst) {
  if (n <= kThreads && nr.nparts == 1) {  // (finalized means, engine.cpp norm_fin)
    norm_tab_batched<1, 1>(nr, n, dst);
  } else if (n <= 4 * kThreads && nr.nparts == 1) {
    norm_tab_batched<4, 1>(nr, n, dst);
  } else if (n <= kThreads && nr.nparts <= 16) {
    norm_tab_batched<1, 16>(nr, n, dst);
  } else if (n <= 4 * kThreads && nr.nparts <= 8) {
    norm_tab_batched<4, 8>(nr, n, dst);
  } else {
#pragma unroll 1
    for (int i = threadIdx.x; i < n; i += kThreads) dst[i] = norm_inv_i(nr, i);
  }
#pragma unroll 1
  for (int i = n + threadIdx.x; i < ((n + 15) & ~15); i += kThreads) dst[i] = 0.f;
}

// ---------------------------------------------------------------- tensor images (ops.h "tensor images")
__device__ __forceinline__ size_t nidx(int cbn, int r, int c) {
  return ((size_t)(r >> 4) * cbn + (c >> 4)) * 256 + ((c >> 2) & 3) * 64 + (r & 15) * 4 + (c & 3);
}
__device__ __forceinline__ size_t tidx(int rbs, int r, int c) {
  return ((size_t)(c >> 4) * rbs + (r >> 4)) * 256 + ((r >> 2) & 3) * 64 + (c & 15) * 4 + (r & 3);
}
// Element read (T image preferred, else N) / write (every kept image).
__device__ __forceinline__ float mat_ld(const CAS Mat& m, int r, int c) {
  return m.t ? G(m.t)[tidx(m.rbs, r, c)] : G(m.n)[nidx(m.cbn, r, c)];
}
__device__ __forceinline__ void mat_st(const CAS Mat& m, int r, int c, float v) {
  if (m.t) GW(m.t)[tidx(m.rbs, r, c)] = v;
  if (m.n) GW(m.n)[nidx(m.cbn, r, c)] = v;
}
// Columns c..c+3 (c % 4 == 0) of row r: one float4 of the N image.
__device__ __forceinline__ float4 mat_ldr4(const CAS Mat& m, int r, int c) { return ld4g(G(m.n) + nidx(m.cbn, r, c)); }
// Store columns c..c+3 of row r into every kept image (T: 4 floats 16 B apart).
__device__ __forceinline__ void mat_str4(const CAS Mat& m, int r, int c, float4 v) {
  if (m.n) st4g(GW(m.n) + nidx(m.cbn, r, c), v);
  if (m.t) {
    GAS float* q = GW(m.t) + tidx(m.rbs, r, c);
    q[0] = v.x;
    q[4] = v.y;
    q[8] = v.z;
    q[12] = v.w;
  }
}
// Four consecutive rows r..r+3 (r % 4 == 0) of column c: one float4 of the T image.
__device__ __forceinline__ float4 mat_ld4(const CAS Mat& m, int r, int c) {
  return ld4g(G(m.t) + tidx(m.rbs, r, c));
}
__device__ __forceinline__ void mat_st4(const CAS Mat& m, int r, int c, float4 v) {
  if (m.t) st4g(GW(m.t) + tidx(m.rbs, r, c), v);
  if (m.n) {
    GAS float* q = GW(m.n) + nidx(m.cbn, r, c);  // rows r..r+3 are 4 floats apart in the N image
    q[0] = v.x;
    q[4] = v.y;
    q[8] = v.z;
    q[12] = v.w;
  }
}

// Phase timestamps of one workgroup (wave 0, lane 0): [0] entry, [1] main loop
// start, [2] main loop end (GEMM only), [3] exit.
__device__ __forceinline__ void trace_mark(unsigned long long* tr, int slot) {
  if (tr && threadIdx.x == 0) tr[slot] = __builtin_amdgcn_s_memrealtime();
}
// Diagnostics builds (-DRLE_TRACE_FINE, tools only): 12 more stamps per workgroup
// in the same trace buffer (SGPR pointer: a stamp never waits on a load).
#ifdef RLE_TRACE_FINE
constexpr int kTraceStride = 16;
#define FINE_MARK(slot) trace_mark(tr, 4 + (slot))
#else
constexpr int kTraceStride = 4;
#define FINE_MARK(slot) \
  do {                  \
  } while (0)
#endif

// ---------------------------------------------------------------- act graph output
// Exploration draw e (row-major index row * A + j) of an act call (ActArgs::ctl).
__device__ __forceinline__ float act_noise(unsigned long long seed, int e, unsigned lo, unsigned hi) {
  const uint2 key = make_uint2((unsigned)seed, (unsigned)(seed >> 32));
  const uint4 r = philox(key, make_uint4((unsigned)e, 7u, lo, hi));
  return normal_from(r.x, r.y);
}
template <class AO>  // (ActArgs in the constant address space, or a kernel argument)
__device__ __forceinline__ float act_eps(const AO& ao, int mode, int e) {
  if (mode == 2) return G(ao.eps)[e];
  return act_noise(ao.seed, e, (unsigned)G(ao.ctl)[1], (unsigned)G(ao.ctl)[2]);
}
// out = a * scale + bias (numpy float32: two rounded ops)
template <class AO>
__device__ __forceinline__ void act_store(const AO& ao, int row, int j, float a) {
  GW(ao.out)[(size_t)row * ao.A + j] = __fadd_rn(__fmul_rn(a, G(ao.scale)[j]), G(ao.bias)[j]);
}

// ---------------------------------------------------------------- GEMM
//
// One workgroup = one 16 x tn output tile (tn in {16, 32, 64}); its 4 waves are
// tn/16 column groups x 64/tn reduction splits, split partials summed through
// LDS in a fixed order.  Both operands are fragment images (ops.h), so each
// 16-wide reduction chunk is one lane-linear 16-byte buffer load per lane per
// operand (whole 1 KB blocks per wave), 4 chunks in flight.
//
// Code size is the first-order cost here: the instruction cache is invalidated
// at every dispatch and a wave fetches code at ~0.4 us per KB (tools/mbic.hip),
// while a level's arithmetic is ~1 us.  So every op runs a compile-time
// specialised variant (mode, epilogue, activation, norm: GemmArgs::vid) whose
// straight-line path contains only what that op does: no per-element
// activation switch, no segment bookkeeping inside the chunk loop (segments
// are walked by an outer loop), and no normalisation code in the plain case.

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x16 __attribute__((ext_vector_type(16)));
constexpr int kOOB = 0x7ffffff0;  // voffset beyond num_records: the load returns 0

__device__ __forceinline__ float4 as_f4(u32x4 v) {
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, 0x7fff0000, 0x00020000);
}
__device__ __forceinline__ float4 bload(__amdgpu_buffer_rsrc_t r, int off) {
  return as_f4(__builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ f32x4 mfma4(const float4& a, const float4& b, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  return acc;
}
__device__ __forceinline__ float4 scale4(float4 v, float s) { return make_float4(v.x * s, v.y * s, v.z * s, v.w * s); }
__device__ __forceinline__ float4 mul4(float4 v, float4 s) {
  return make_float4(v.x * s.x, v.y * s.y, v.z * s.z, v.w * s.w);
}

template <int ACT>
__device__ __forceinline__ float act_f(float v) {
  if constexpr (ACT == ACT_RELU) return v > 0.f ? v : 0.f;
  else if constexpr (ACT == ACT_ELU) return v > 0.f ? v : expm1f(v);
  else if constexpr (ACT == ACT_TANH) return tanhf(v);
  else return v;
}
template <int ACT>
__device__ __forceinline__ float act_b(float saved) {  // see act_bwd
  if constexpr (ACT == ACT_RELU) return saved > 0.f ? 1.f : 0.f;
  else if constexpr (ACT == ACT_ELU) return saved > 0.f ? 1.f : expf(saved);
  else if constexpr (ACT == ACT_TANH) return 1.f - saved * saved;
  else return 1.f;
}

// Reduction over chunks [k0, k1) of one operand pair: A from (ra, va), B from
// (rb, vb) (byte offsets of chunk k0, +1 KB per chunk); kRing chunks in flight.
// SA / SB: per-chunk scaling (deferred AvgL1Norm) by a lane constant (N image)
// or an LDS table of 4 rows (T image, tab = float offset of chunk k0's rows).
#ifndef RLE_RING
#define RLE_RING 4
#endif
constexpr int kRing = RLE_RING;  // chunks in flight per wave

// The ring in two halves, so that work with its own memory round trip (AvgL1Norm scalars
// and tables) can run between issuing the first kRing chunks and consuming them.
// (RG: ring depth; the weight-gradient variants may run a deeper one, RLE_DW_RING.  An even RG
// keeps chunk k on accumulator k & 1 in order, so the sums do not depend on it.)
#ifndef RLE_DW_RING
#define RLE_DW_RING 4
#endif
constexpr int kRingDW = RLE_DW_RING;
template <int RG = kRing>
__device__ __forceinline__ void ring_issue(float4 (&a)[RG], float4 (&b)[RG], __amdgpu_buffer_rsrc_t ra, int va,
                                           __amdgpu_buffer_rsrc_t rb, int vb, int n, bool bias_ones) {
#pragma unroll
  for (int r = 0; r < RG; ++r) {
    if (r >= n) break;  // (uniform: no load past the last chunk)
    a[r] = bload(ra, va + r * 1024);
    b[r] = bias_ones ? make_float4(1.f, 1.f, 1.f, 1.f) : bload(rb, vb + r * 1024);
  }
}
template <int SA, int SB, int RG = kRing>
__device__ __forceinline__ f32x4 ring_run(float4 (&a)[RG], float4 (&b)[RG], __amdgpu_buffer_rsrc_t ra, int va,
                                          __amdgpu_buffer_rsrc_t rb, int vb, int n, f32x4 acc, float inva,
                                          const float* taba, const float* tabb, bool bias_ones) {
  const int rl = ((threadIdx.x & 63) >> 4) << 2;
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int c = 0; c < n; c += RG) {
#pragma unroll
    for (int r = 0; r < RG; ++r) {
      // (uniform branches: no MFMA of a chunk past the last and no load past it -- an
      // out-of-range load still occupies the memory pipeline and the in-order load counter:
      // +2.9% steps/s over loading zeros)
      if (c + r >= n) break;
      float4 x = a[r], y = b[r];
      if constexpr (SA == 1) x = scale4(x, inva);
      // (table rows past n are not built: clamp; their chunks load as zeros anyway)
      if constexpr (SA == 2) x = mul4(x, *(const float4*)(taba + min(c + r, n - 1) * 16 + rl));
      if constexpr (SB == 2) y = mul4(y, *(const float4*)(tabb + min(c + r, n - 1) * 16 + rl));
      if (r & 1) acc1 = mfma4(x, y, acc1);
      else acc = mfma4(x, y, acc);
      const int nx = c + r + RG;
      if (nx >= n) continue;
      a[r] = bload(ra, va + nx * 1024);
      if (!bias_ones) b[r] = bload(rb, vb + nx * 1024);
    }
  }
  return acc + acc1;
}
template <int SA, int SB>
__device__ __forceinline__ f32x4 chunk_loop(__amdgpu_buffer_rsrc_t ra, int va, __amdgpu_buffer_rsrc_t rb, int vb,
                                            int n, f32x4 acc, float inva, const float* taba, const float* tabb,
                                            bool bias_ones) {
  float4 a[kRing], b[kRing];
  ring_issue(a, b, ra, va, rb, vb, n, bias_ones);
  return ring_run<SA, SB>(a, b, ra, va, rb, vb, n, acc, inva, taba, tabb, bias_ones);
}

__device__ __forceinline__ float sgnf(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

// DW reduction whose A operand (dZ, T image) is an AvgL1Norm backward applied on load
// (kDwNb, sale.py:11-13): a = g * inv[r] + sign(x) * gm[r] for the chunk's rows r, with
// x read from (rx, vx) in the same T-image layout as g and inv / gm from LDS tables
// (ti / tg: float offset of chunk k0's first row).  Same ring as chunk_loop.
// (x ring issued by the caller together with ring_issue for a / b, ahead of the tables)
template <int RG = kRing>
__device__ __forceinline__ f32x4 ring_run_nb(float4 (&a)[RG], float4 (&x)[RG], float4 (&b)[RG],
                                             __amdgpu_buffer_rsrc_t ra, int va, __amdgpu_buffer_rsrc_t rx, int vx,
                                             __amdgpu_buffer_rsrc_t rb, int vb, int n, f32x4 acc, const float* ti,
                                             const float* tg, bool bias_ones) {
  const int rl = ((threadIdx.x & 63) >> 4) << 2;
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int c = 0; c < n; c += RG) {
#pragma unroll
    for (int r = 0; r < RG; ++r) {
      if (c + r >= n) break;  // (as ring_run)
      const int k = c + r;
      const float4 iv = *(const float4*)(ti + k * 16 + rl), gv = *(const float4*)(tg + k * 16 + rl);
      const float4 y = make_float4(a[r].x * iv.x + sgnf(x[r].x) * gv.x, a[r].y * iv.y + sgnf(x[r].y) * gv.y,
                                   a[r].z * iv.z + sgnf(x[r].z) * gv.z, a[r].w * iv.w + sgnf(x[r].w) * gv.w);
      if (r & 1) acc1 = mfma4(y, b[r], acc1);
      else acc = mfma4(y, b[r], acc);
      const int nx = c + r + RG;
      if (nx >= n) continue;
      a[r] = bload(ra, va + nx * 1024);
      x[r] = bload(rx, vx + nx * 1024);
      if (!bias_ones) b[r] = bload(rb, vb + nx * 1024);
    }
  }
  return acc + acc1;
}

// kDwNb tables for the n reduction rows: 1/m and the sign coefficient
// gm = -(sum_j g x) / (n_x m^2) (0 when m is clamped), exactly as op_normbwd.
// (rows r0 .. r0 + n - 1 into ti / tg [0, n); PM / PD: the mean's and the dot's partial bounds)
template <int RPT, int PM, int PD>
__device__ __forceinline__ void nb_tab_batched(const CAS GemmArgs& g, int n, float* ti, float* tg, float xw, int r0 = 0) {
  float sm[RPT], sd[RPT];
  row_sums<RPT, PM>(g.nbm.part, g.nbm.ld, g.nbm.row0 + r0, g.nbm.nparts, n, sm);
  row_sums<RPT, PD>(g.nbdot, g.nbdot_ld, r0, g.nbdot_n, n, sd);
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int i = threadIdx.x + r * kThreads;
    const float mean = sm[r] / (float)g.nbm.width, dot = sd[r] / 1.f;  // (norm_mean_i's floats)
    const bool clamped = mean < 1e-8f;
    const float inv = 1.f / (clamped ? 1e-8f : mean);
    if (i < n) {
      ti[i] = inv;
      tg[i] = clamped ? 0.f : (-dot * inv * inv) / xw;
    }
  }
}
__device__ __forceinline__ void build_nb_tab(const CAS GemmArgs& g, int n, float* ti, float* tg) {
  // (x's width: the mean may come finalized, engine.cpp norm_fin, as one partial of width 1)
  const float xw = (float)(g.nb_width ? g.nb_width : g.nbm.width);
  const int pm = g.nbm.nparts, pd = g.nbdot_n;
  if (n <= kThreads && pm <= 16 && pd <= 16) {
    nb_tab_batched<1, 16, 16>(g, n, ti, tg, xw);
    return;
  }
  if (n <= 4 * kThreads && pm == 1 && pd <= 8) {
    nb_tab_batched<4, 1, 8>(g, n, ti, tg, xw);
    return;
  }
  if (n <= 4 * kThreads && pm <= 4 && pd <= 4) {
    nb_tab_batched<4, 4, 4>(g, n, ti, tg, xw);
    return;
  }
  if (n <= 4 * kThreads && pm == 1 && pd <= 16) {  // (two rows per thread per round trip)
    nb_tab_batched<2, 1, 16>(g, min(n, 2 * kThreads), ti, tg, xw);
    if (n > 2 * kThreads) nb_tab_batched<2, 1, 16>(g, n - 2 * kThreads, ti + 2 * kThreads, tg + 2 * kThreads, xw, 2 * kThreads);
    return;
  }
#pragma unroll 1
  for (int i = threadIdx.x; i < n; i += kThreads) {
    const float mean = norm_mean_i(g.nbm.part, g.nbm.ld, i + g.nbm.row0, g.nbm.nparts, g.nbm.width);
    const float dot = norm_mean_i(g.nbdot, g.nbdot_ld, i, g.nbdot_n, 1);
    const bool clamped = mean < 1e-8f;
    const float inv = 1.f / (clamped ? 1e-8f : mean);
    ti[i] = inv;
    tg[i] = clamped ? 0.f : (-dot * inv * inv) / xw;
  }
}

// chunk_loop over one A stream and two B streams (two 16-column blocks sharing A).
__device__ __forceinline__ void chunk_loop2(__amdgpu_buffer_rsrc_t ra, int va, __amdgpu_buffer_rsrc_t rb, int vb0,
                                            int vb1, int n, f32x4& acc0, f32x4& acc1) {
  float4 a[kRing], b0[kRing], b1[kRing];
#pragma unroll
  for (int r = 0; r < kRing; ++r) {
    if (r >= n) break;  // (uniform, as ring_run)
    a[r] = bload(ra, va + r * 1024);
    b0[r] = bload(rb, vb0 + r * 1024);
    b1[r] = bload(rb, vb1 + r * 1024);
  }
#pragma unroll 1
  for (int c = 0; c < n; c += kRing) {
#pragma unroll
    for (int r = 0; r < kRing; ++r) {
      if (c + r >= n) break;
      acc0 = mfma4(a[r], b0[r], acc0);
      acc1 = mfma4(a[r], b1[r], acc1);
      const int nx = c + r + kRing;
      if (nx >= n) continue;
      a[r] = bload(ra, va + nx * 1024);
      b0[r] = bload(rb, vb0 + nx * 1024);
      b1[r] = bload(rb, vb1 + nx * 1024);
    }
  }
}

// ---- register-blocked wide weight-gradient tiles (GemmHot::rb, tn = 16 NB): the 4 waves split the
// reduction (batch rows) in quarters and each wave accumulates all NB column blocks of the tile on NB
// independent chains, so one A chunk (and, kDwNb, its AvgL1Norm-backward transform) serves NB MFMA
// groups and a wave's operand ring covers its whole quarter in one or two rounds; the quarters are
// summed through LDS in wave order (rb_exchange).  B block cb of chunk k at (rbr, vbv[cb] + k KB) (the
// tile's blocks lie in one X segment: engine.cpp rb_eligible); blocks cb >= nb are outside the tile
// (no load, no MFMA).  tabb: B scaled per reduction row from an LDS table (deferred AvgL1Norm of X);
// NBX: A = g * ti + sgn(x) * tg per reduction row (kDwNb), x from (rx, vx).
// LDS floats: [4 waves][NB][64 lanes][4] partials, over the tables (rb_exchange waits for every
// wave's loop first)
constexpr int kRbOff = 2048;
template <int NB, int RG>
struct RbRing {
  float4 a[RG], x[RG], b[RG][NB];
};
template <int NB, int RG, bool NBX>
__device__ __forceinline__ void rb_issue(RbRing<NB, RG>& R, __amdgpu_buffer_rsrc_t ra, int va,
                                         __amdgpu_buffer_rsrc_t rbr, const int (&vbv)[NB], int nb, int n,
                                         __amdgpu_buffer_rsrc_t rx, int vx, bool bias_ones) {
  const float4 ones = make_float4(1.f, 1.f, 1.f, 1.f);
#pragma unroll
  for (int r = 0; r < RG; ++r) {
    if (r >= n) break;  // (uniform)
    R.a[r] = bload(ra, va + r * 1024);
    if constexpr (NBX) R.x[r] = bload(rx, vx + r * 1024);
#pragma unroll
    for (int cb = 0; cb < NB; ++cb)
      if (cb < nb) R.b[r][cb] = bias_ones ? ones : bload(rbr, vbv[cb] + r * 1024);
  }
}
template <int NB, int RG, bool NBX>
__device__ __forceinline__ void rb_run(RbRing<NB, RG>& R, __amdgpu_buffer_rsrc_t ra, int va,
                                       __amdgpu_buffer_rsrc_t rbr, const int (&vbv)[NB], int nb, int n,
                                       f32x4 (&acc)[NB], const float* tabb, __amdgpu_buffer_rsrc_t rx, int vx,
                                       const float* ti, const float* tg, bool bias_ones) {
  const int rl = ((threadIdx.x & 63) >> 4) << 2;
#pragma unroll 1
  for (int c = 0; c < n; c += RG) {
#pragma unroll
    for (int r = 0; r < RG; ++r) {
      const int k = c + r;
      if (k >= n) break;  // (uniform)
      float4 y = R.a[r];
      if constexpr (NBX) {
        const float4 iv = *(const float4*)(ti + k * 16 + rl), gv = *(const float4*)(tg + k * 16 + rl);
        const float4 xv = R.x[r];
        y = make_float4(y.x * iv.x + sgnf(xv.x) * gv.x, y.y * iv.y + sgnf(xv.y) * gv.y,
                        y.z * iv.z + sgnf(xv.z) * gv.z, y.w * iv.w + sgnf(xv.w) * gv.w);
      }
#pragma unroll
      for (int cb = 0; cb < NB; ++cb) {
        if (cb >= nb) break;
        float4 bb = R.b[r][cb];
        if (tabb) bb = mul4(bb, *(const float4*)(tabb + k * 16 + rl));
        acc[cb] = mfma4(y, bb, acc[cb]);
      }
      const int nx = k + RG;
      if (nx >= n) continue;
      R.a[r] = bload(ra, va + nx * 1024);
      if constexpr (NBX) R.x[r] = bload(rx, vx + nx * 1024);
#pragma unroll
      for (int cb = 0; cb < NB; ++cb)
        if (cb < nb && !bias_ones) R.b[r][cb] = bload(rbr, vbv[cb] + nx * 1024);
    }
  }
}
// The quarters of column block cg summed in wave order (q = 0..3) into the lead wave of cg.
template <int NB>
__device__ __forceinline__ f32x4 rb_exchange(const f32x4 (&acc)[NB], float* smem, int cg, bool lead) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* xr = smem + kRbOff;
  __syncthreads();  // (every wave is done with the tables this region overlaps)
#pragma unroll
  for (int cb = 0; cb < NB; ++cb) *(f32x4*)(xr + ((wave * NB + cb) * 64 + lane) * 4) = acc[cb];
  __syncthreads();
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (lead) {
#pragma unroll
    for (int q = 0; q < 4; ++q) s += *(const f32x4*)(xr + ((q * NB + cg) * 64 + lane) * 4);
  }
  return s;
}

// A chunks from an LDS fragment image (pre-GEMM output), B from memory.
__device__ __forceinline__ f32x4 chunk_loop_lds(const float* la, __amdgpu_buffer_rsrc_t rb, int vb, int n, f32x4 acc) {
  const int lane = threadIdx.x & 63;
  for (int c = 0; c < n; ++c) acc = mfma4(*(const float4*)(la + c * 256 + lane * 4), bload(rb, vb + c * 1024), acc);
  return acc;
}

// ... with the chunks on two accumulators by parity, as ring_run sums a segment read from memory (the
// consumer's floats equal those of reading the standalone op's output)
__device__ __forceinline__ f32x4 chunk_loop_lds_par(const float* la, __amdgpu_buffer_rsrc_t rb, int vb, int n,
                                                    f32x4 acc) {
  const int lane = threadIdx.x & 63;
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < n; ++c) {
    const float4 x = *(const float4*)(la + c * 256 + lane * 4);
    if (c & 1) acc1 = mfma4(x, bload(rb, vb + c * 1024), acc1);
    else acc = mfma4(x, bload(rb, vb + c * 1024), acc);
  }
  return acc + acc1;
}

// Pre-GEMM (PreArgs): the actor's tanh output layer for the 16 rows at i0 into pimg[2][256]
// (N-image fragment blocks, columns >= N zero).  Each wave reduces a quarter of the chunks
// for both column blocks; the quarters are summed in fixed wave order by wave 0, which
// also runs the epilogue.  Two phases, so that one memory round trip serves both the
// pre-GEMM and the consumer's own segments: pre_issue puts the wave's first kPreRing chunks
// and the epilogue operands in flight; pre_finish (after the consumer's other segments)
// reduces, applies the epilogue and publishes pimg.
#ifndef RLE_PRE_RING
#define RLE_PRE_RING 4  // MI355X A/B (K=4 step graphs): 2/3/4 -> 6509/6476/6540 steps/s; 125 VGPRs, no spills
#endif
// pre-GEMM chunks prefetched per wave, i.e. all of a wave's quarter of K = 256: registers held
// across the consumer's own segments (within the 4-waves/SIMD budget)
constexpr int kPreRing = RLE_PRE_RING;
struct PreRing {
  float4 a[kPreRing], b0[kPreRing], b1[kPreRing];
  float4 e[2];   // FWD: noise, DX: saved tanh output (4 rows, per column block)
  float bj[2];   // FWD: bias per column block
  int c0, c1, cp;
};

// (LITE: the host guarantees N <= 16 and one A and one B segment -- one column block, no registers
// for a second, no segment lookup; GemmArgs::has_pre 4)
template <int MODE, bool LITE = false>
__device__ __forceinline__ void pre_issue(const CAS PreArgs& p, int i0, PreRing& R) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nch = p.R >> 4, per = (nch + 3) >> 2;
  R.c0 = wave * per;
  R.c1 = min(nch, R.c0 + per);
  R.cp = min(R.c1, R.c0 + kPreRing);
  const bool wabs = MODE == GEMM_FWD && (LITE || p.B.nseg == 1);
  const int lb = lane * 16;
#pragma unroll
  for (int r = 0; r < kPreRing; ++r) {
    const int k = R.c0 + r;
    int q = 0;  // segment of chunk k (wave-uniform)
#pragma unroll
    for (int u = 1; u < (LITE ? 1 : kMaxSeg); ++u)
      if (u < p.A.nseg && k >= (p.A.seg[u].r0 >> 4)) q = u;
    const CAS Seg& sa = p.A.seg[q];
    const CAS Seg& sb = p.B.seg[wabs ? 0 : q];
    const int s0 = sa.r0 >> 4, kb = wabs ? k : k - s0;
    if (k >= R.cp) break;  // (uniform)
    R.a[r] = bload(rsrc(sa.p), ((i0 >> 4) * sa.xs + (k - s0)) * 1024 + lb);
    R.b0[r] = bload(rsrc(sb.p), kb * 1024 + lb);
    if (!LITE && p.N > 16) R.b1[r] = bload(rsrc(sb.p), (sb.xs + kb) * 1024 + lb);
  }
  // (buffer loads at an out-of-range offset return 0: no branch, so no register merge that would
  // wait for every load in flight)
  const int rb = (lane >> 4) << 2;
  if (wave != 0) return;  // (wave 0 runs the epilogue: no loads for the others)
#pragma unroll
  for (int cb = 0; cb < (LITE ? 1 : 2); ++cb) {
    const int j = cb * 16 + (lane & 15);
    const bool jok = j < p.N;
    if constexpr (MODE == GEMM_FWD) {
      R.bj[cb] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc(p.bias), jok && p.bias ? j * 4 : kOOB, 0, 0));
      R.e[cb] = bload(rsrc(p.noise.t), jok && p.noise.t ? (int)tidx(p.noise.rbs, i0 + rb, j) * 4 : kOOB);
    } else {
      R.bj[cb] = 0.f;
      R.e[cb] = bload(rsrc(p.dsrc.t), jok ? (int)tidx(p.dsrc.rbs, i0 + rb, j) * 4 : kOOB);
    }
  }
}

template <int MODE, bool LITE = false>
__device__ __forceinline__ void pre_finish(const CAS PreArgs& p, int i0, PreRing& R, float* part, float* part2,
                                           float* pimg) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool two = !LITE && p.N > 16, wabs = MODE == GEMM_FWD && (LITE || p.B.nseg == 1);
  const int lb = lane * 16;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
  for (int r = 0; r < kPreRing; ++r) {  // (chunks past cp are not loaded)
    if (R.c0 + r >= R.cp) break;
    acc0 = mfma4(R.a[r], R.b0[r], acc0);
    if (two) acc1 = mfma4(R.a[r], R.b1[r], acc1);
  }
  for (int q = 0; q < (LITE ? 1 : p.A.nseg); ++q) {  // the rest of the wave's chunks
    const CAS Seg& sa = p.A.seg[q];
    const CAS Seg& sb = p.B.seg[wabs ? 0 : q];
    const int s0 = sa.r0 >> 4;
    const int k0 = max(R.cp, s0), k1 = min(R.c1, (sa.r1 + 15) >> 4);
    if (k0 >= k1) continue;
    const int va = ((i0 >> 4) * sa.xs + (k0 - s0)) * 1024 + lb;
    const int kb = wabs ? k0 : k0 - s0;
    if (two) chunk_loop2(rsrc(sa.p), va, rsrc(sb.p), kb * 1024 + lb, (sb.xs + kb) * 1024 + lb, k1 - k0, acc0, acc1);
    else acc0 = chunk_loop<0, 0>(rsrc(sa.p), va, rsrc(sb.p), kb * 1024 + lb, k1 - k0, acc0, 1.f, nullptr, nullptr, false);
  }
  if (wave) {
    *(f32x4*)(part + (wave * 64 + lane) * 4) = acc0;
    if (!LITE) *(f32x4*)(part2 + (wave * 64 + lane) * 4) = acc1;
  }
  __syncthreads();
  if (wave == 0) {
    for (int w = 1; w < 4; ++w) {
      acc0 += *(const f32x4*)(part + (w * 64 + lane) * 4);
      if (!LITE) acc1 += *(const f32x4*)(part2 + (w * 64 + lane) * 4);
    }
    const int rb = (lane >> 4) << 2;
#pragma unroll
    for (int cb = 0; cb < (LITE ? 1 : 2); ++cb) {
      const f32x4 acc = cb ? acc1 : acc0;
      const int j = cb * 16 + (lane & 15);
      const bool jok = j < p.N;
      const float ev[4] = {R.e[cb].x, R.e[cb].y, R.e[cb].z, R.e[cb].w};
      float y[4];
      if constexpr (MODE == GEMM_FWD) {  // tanh (+ target smoothing), as the EPI_STORE tanh path
#pragma unroll
        for (int q = 0; q < 4; ++q) y[q] = act_f<ACT_TANH>(acc[q] + R.bj[cb]);
        if (p.noise.t) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float nz = fminf(fmaxf(ev[q] * p.noise_sigma, -p.noise_clip), p.noise_clip);
            y[q] = fminf(fmaxf(y[q] + nz, -1.f), 1.f);
          }
        }
      } else {  // grad wrt the tanh input: * (1 - a^2)
#pragma unroll
        for (int q = 0; q < 4; ++q) y[q] = acc[q] * act_b<ACT_TANH>(ev[q]);
      }
      float* dst = pimg + cb * 256 + ((lane & 15) >> 2) * 64 + rb * 4 + (lane & 3);
#pragma unroll
      for (int q = 0; q < 4; ++q) dst[q * 4] = jok ? y[q] : 0.f;
    }
  }
  __syncthreads();
}

// Pre-layer (GemmArgs::has_pre 3, PreArgs with N = the consumer's whole A width <= 256, R <= 48):
// the consumer's A operand, act(X W^T + b) for the tile's 16 rows, computed in the workgroup into
// pimg[N / 16][256] (N-image fragment blocks) -- a small-K first layer (TD3 / SAC on low-dimensional
// observations: K = state (+ action) dims) folded into the layer after it, one level fewer on the
// chain.  Wave w computes output column blocks 4w .. 4w + 3 over all (<= 3) reduction chunks; each
// chunk's sum is a separate MFMA chain and the chunks are added in order, as the standalone op
// reduces them split-K over its waves (tn 16 / 32): the same floats.
// (GEMM_DX: the same over dZ (N image) and W's T image, no bias, the output scaled by act'(saved)
// (p.dsrc, T image) -- SAC's gradient through the actor's raw head, K = 2 x action dims.)
// (prelayer_issue puts every operand in flight; prelayer_finish reduces and publishes pimg.  TWO: the
// input has two segments and the chunks of segment 1 come from lds_a, an LDS fragment image --
// GemmArgs::has_pre 4, whose pre-GEMM computed them -- instead of memory)
struct PlRing {
  float4 a[3], b[3][4];
  float bj[4];
  float4 ev[4];  // (DX) act'(saved) sources: 4 rows of column j per lane
};
template <int MODE, bool TWO = false>
__device__ __forceinline__ void prelayer_issue(const CAS PreArgs& p, int i0, PlRing& R) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nch = p.R >> 4;
  const int lb = lane * 16;
  const CAS Seg& sb = p.B.seg[0];
  const auto rw = rsrc(sb.p);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k >= nch) break;  // (uniform)
    if constexpr (TWO) {  // (segment 0 starts at chunk 0)
      const CAS Seg& sa = p.A.seg[0];
      if (k < (p.A.seg[1].r0 >> 4)) R.a[k] = bload(rsrc(sa.p), ((i0 >> 4) * sa.xs + k) * 1024 + lb);
    } else {
      int q = 0;
#pragma unroll
      for (int u = 1; u < kMaxSeg; ++u)
        if (u < p.A.nseg && k >= (p.A.seg[u].r0 >> 4)) q = u;
      const CAS Seg& sa = p.A.seg[q];
      R.a[k] = bload(rsrc(sa.p), ((i0 >> 4) * sa.xs + (k - (sa.r0 >> 4))) * 1024 + lb);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)  // (column blocks past N: no load, zeros)
      R.b[k][c] = (wave * 4 + c) * 16 < p.N ? bload(rw, ((wave * 4 + c) * sb.xs + k) * 1024 + lb)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int rb = (lane >> 4) << 2;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int j = (wave * 4 + c) * 16 + (lane & 15);
    if constexpr (MODE == GEMM_FWD) {
      R.bj[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc(p.bias), j < p.N ? j * 4 : kOOB, 0, 0));
      R.ev[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      R.bj[c] = 0.f;
      R.ev[c] = bload(rsrc(p.dsrc.t), j < p.N ? (int)tidx(p.dsrc.rbs, i0 + rb, j) * 4 : kOOB);
    }
  }
}
template <int MODE, int ACT, bool TWO = false>
__device__ __forceinline__ void prelayer_finish(const CAS PreArgs& p, PlRing& R, float* pimg, const float* lds_a) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nch = p.R >> 4;
  if constexpr (TWO) {
    const int s1 = p.A.seg[1].r0 >> 4;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k >= nch) break;
      if (k >= s1) R.a[k] = *(const float4*)(lds_a + (k - s1) * 256 + lane * 4);
    }
  }
  const int rb = (lane >> 4) << 2;
  f32x4 s[4];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k >= nch) break;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const f32x4 pk = mfma4(R.a[k], R.b[k][c], z);
      s[c] = k ? s[c] + pk : pk;
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int cb = wave * 4 + c;
    float* dst = pimg + cb * 256 + ((lane & 15) >> 2) * 64 + rb * 4 + (lane & 3);
    const bool jok = cb * 16 + (lane & 15) < p.N;
    const float e4[4] = {R.ev[c].x, R.ev[c].y, R.ev[c].z, R.ev[c].w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float y;
      if constexpr (MODE == GEMM_FWD) y = act_f<ACT>(s[c][q] + R.bj[c]);
      else y = s[c][q] * act_b<ACT>(e4[q]);
      dst[q * 4] = jok ? y : 0.f;
    }
  }
  __syncthreads();
}
template <int MODE, int ACT>
__device__ __forceinline__ void prelayer_fwd(const CAS PreArgs& p, int i0, float* pimg) {
  PlRing R;
  prelayer_issue<MODE>(p, i0, R);
  prelayer_finish<MODE, ACT>(p, R, pimg, nullptr);
}

// SAC's raw head [mean | log_std] (sac.py:132-152; N = 2A <= 48, three column blocks, R <= 256) for the
// 16 rows at i0: wave w reduces chunks 4w .. 4w + 3 for every column block, and wave 0 sums the partials
// in wave order.  Both the standalone EPI_SACFWD op and the target critics' in-tile copy (GemmArgs::has_pre
// 5) reduce this way, so their floats agree.  sacraw_issue puts the operands in flight; sacraw_finish
// returns the sums in wave 0 (part: [3 blocks][4 waves][256] floats of LDS).
struct SacRing {
  float4 a[4], b[3][4];
};
__device__ __forceinline__ void sacraw_issue(const float* ap, int axs, const float* bp, int bxs, int nch, int i0,
                                             SacRing& R) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lb = lane * 16;
  const auto ra = rsrc(ap), rb = rsrc(bp);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k = wave * 4 + r;
    if (k >= nch) break;  // (uniform)
    R.a[r] = bload(ra, ((i0 >> 4) * axs + k) * 1024 + lb);
#pragma unroll
    for (int c = 0; c < 3; ++c) R.b[c][r] = bload(rb, (c * bxs + k) * 1024 + lb);
  }
}
__device__ __forceinline__ void sacraw_finish(const SacRing& R, int nch, float* part, f32x4 (&s)[3]) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int c = 0; c < 3; ++c) s[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (wave * 4 + r >= nch) break;
#pragma unroll
    for (int c = 0; c < 3; ++c) s[c] = mfma4(R.a[r], R.b[c][r], s[c]);
  }
  if (wave) {
#pragma unroll
    for (int c = 0; c < 3; ++c) *(f32x4*)(part + (c * 4 + wave) * 256 + lane * 4) = s[c];
  }
  __syncthreads();
  if (wave == 0) {
    for (int w = 1; w < 4; ++w) {
#pragma unroll
      for (int c = 0; c < 3; ++c) s[c] += *(const f32x4*)(part + (c * 4 + w) * 256 + lane * 4);
    }
  }
}

// max(|td|, 1)^0.4 rounded from double (torch's float pow is correctly rounded).  The double pow
// is ~1.3 us of dependent FP64 work on the loss head's critical path, so: a float seed, two
// Newton steps on y^5 = x^2 in double (relative error ~1e-15), rounded to float; the exact
// pow runs only when that double lies within 1e-13 (relative) of a float rounding boundary,
// where the two could round differently -- otherwise both round to the same float.
__device__ __attribute__((noinline)) float lap_priority_pow(float x) { return (float)pow((double)x, 0.4); }
__device__ __forceinline__ float lap_priority(float d) {
  const float x = fmaxf(d, 1.f);
  const double x2 = (double)x * (double)x;
  double y = (double)exp2f(0.4f * log2f(x));
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double y2 = y * y;
    y = 0.2 * (4.0 * y + x2 / (y2 * y2));
  }
  const float f = (float)y;
  const float nb = __int_as_float(__float_as_int(f) + (y > (double)f ? 1 : -1));  // (f >= 1)
  const double mid = 0.5 * ((double)f + (double)nb);  // the rounding boundary on y's side of f
  if (!(fabs(y - mid) > 1e-13 * y)) return lap_priority_pow(x);
  return f;
}

// ---- fused loss head (GemmArgs::has_pre 2): a critic head for the tile's 16 rows, one per
// lane, from EPI_QDOT partials of q -- HEAD_TD7_LOSS / HEAD_MLP_LOSS (op_head_t with the target
// twins fused) or HEAD_MLP_POLICY (TD3 / SAC actor objective, min of the twins) -- then the DX
// reduction of critic head_n whose A operand dZ = (dq * w) * act'(z) is formed from z (segment
// 0) as op_head_t formed dz.  own_wg: this workgroup stores the head's outputs of its rows (tile
// column 0); own_dz: this wave also stores its dZ chunks (column group 0), when dz has an image.
template <int DACT>
__device__ __forceinline__ f32x4 headdx_reduce(const CAS GemmArgs& g, int i0, int j0, bool active, bool own_wg,
                                               bool own_dz, int c0, int c1, int nch, const float* a0p, int a0xs,
                                               const float* b0p, int b0xs, float* smem, f32x4 acc) {
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const CAS HeadArgs& h = g.hd;
  const int hn = g.head_n;
  const bool pol = h.mode == HEAD_MLP_POLICY, td7 = h.mode == HEAD_TD7_LOSS;  // (uniform)
  // the DX operand ring issued before the head (z and W do not depend on it): A/B +0.2% TD7,
  // +0.5% SAC, +1.1% TD3
  const bool run = active && c0 < c1;
  const int lb = lane * 16, n = c1 - c0, cq = 4 * (lane >> 4);
  const int va = ((i0 >> 4) * a0xs + c0) * 1024 + lb;
  const int vb = ((j0 >> 4) * b0xs + c0) * 1024 + lb;
  const __amdgpu_buffer_rsrc_t ra = rsrc(a0p), rb = rsrc(b0p);
  float4 xa[kRing], xb[kRing];
  if (run) ring_issue(xa, xb, ra, va, rb, vb, n, false);
  float* dqs = smem + 64 + 1024;  // [16] dq of critic hn per tile row (the tabs region)
  float* w3s = dqs + 16;          // [H] critic hn's last-layer weights
  for (int c = 4 * tid; c < h.H; c += 4 * kThreads) *(float4*)(w3s + c) = ld4g(G(h.w[hn]) + nidx(h.w_cbn, 0, c));
  // q of the twins and (loss heads) of the target twins for the tile's 16 rows from their
  // EPI_QDOT row partials: wave w sums quantity w (0 / 1: q of critic 0 / 1, 2 / 3: the target
  // critics' q), lane l adds partials 16 (l / 16) .. +15 of row l % 16 in order, then the 4 lane
  // groups
  float* qv = w3s + 256;        // [4][16] the quantities (+ bias)
  float* acs = qv + 64;         // [2][16] loss terms
  int* kq = (int*)(acs + 32);   // [16] value keys
  const int row = lane & 15, grp = lane >> 4;
  const bool tw = wave >= 2;    // a target twin's quantity (none in the policy head)
  const float* src = wave == 0 ? h.qp[0] : (wave == 1 ? h.qp[1] : (wave == 2 ? h.tp[0] : h.tp[1]));
  const int np = (pol && tw) ? 0 : (wave == 0 ? h.qp_n[0] : (wave == 1 ? h.qp_n[1] : (wave == 2 ? h.tp_n[0] : h.tp_n[1])));
  const int ld = wave < 2 ? h.qp_ld : h.tp_ld;
  float pv[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int p = grp * 16 + k;
    pv[k] = p < np ? G(src)[(size_t)p * ld + i0 + row] : 0.f;
  }
  float rw = 0.f, ndn = 0.f, lpv = 0.f;
  if (wave == 0 && lane < 16) {
    if (h.reward) rw = G(h.reward)[i0 + lane];
    if (h.notdone) ndn = G(h.notdone)[i0 + lane];
    if (h.sac) lpv = G(h.logpi)[i0 + lane];
  }
  const float bq = (pol && tw) ? 0.f : sload(wave == 0 ? h.b[0] : (wave == 1 ? h.b[1] : (wave == 2 ? h.tb[0] : h.tb[1])));
  const float vtmax = h.vt ? sload(h.vt) : 0.f, vtmin = h.vt ? sload(h.vt + 1) : 0.f;
  const float alpha = h.sac ? (h.alpha_lin ? sload(h.log_alpha) : expf(sload(h.log_alpha))) : 0.f;
  float sm = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) sm += pv[k];
  sm += __shfl_xor(sm, 16);
  sm += __shfl_xor(sm, 32);
  if (lane < 16) qv[wave * 16 + lane] = sm + bq;
  __syncthreads();
  if (wave == 0 && lane < 16) {  // one row per lane (op_head_t, target fused)
    const int b = i0 + lane;
    const bool ok = b < h.nvalid;  // (rows of the padded batch past it: no loss, no gradient, no priority)
    const float q[2] = {qv[lane], qv[16 + lane]};
    float dq[2], ac[2] = {0.f, 0.f}, dmax = 0.f;
    if (pol) {  // HEAD_MLP_POLICY: td3.py:191, sac.py:227-229
      const float mn = fminf(q[0], q[1]);
      const float gq = -h.inv_b;  // torch.minimum backward: ties split the gradient
      dq[0] = q[0] < q[1] ? gq : (q[0] == q[1] ? 0.5f * gq : 0.f);
      dq[1] = q[1] < q[0] ? gq : (q[0] == q[1] ? 0.5f * gq : 0.f);
      if (h.sac) {
        ac[0] = -mn + lpv * alpha;
        ac[1] = lpv;
      } else {
        ac[0] = mn;
      }
      kq[lane] = 0;
    } else {
      float v = fminf(qv[32 + lane], qv[48 + lane]);
      if (td7) v = fminf(fmaxf(v, vtmin), vtmax);  // td7.py:211-218
      else if (h.sac) v = v - alpha * lpv;         // sac.py:188-193 (td3.py:160-164: neither)
      const float yv = rw + (h.gamma * v) * ndn;
#pragma unroll
      for (int n = 0; n < 2; ++n) {  // td7.py:231-244, td3.py:169-182
        const float diff = q[n] - yv;
        if (h.lap) {
          const float d = fabsf(diff);
          ac[n] = d < 1.f ? 0.5f * (d * d) : d;
          const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
          dq[n] = (d < 1.f ? d : 1.f) * sg * h.inv_b;
          dmax = fmaxf(dmax, d);
        } else {
          const float e = yv - q[n];
          ac[n] = e * e;
          dq[n] = -e * h.inv_b;
        }
      }
      if (own_wg && hn == 0 && h.lap && ok) GW(h.prio)[b] = lap_priority(dmax);
      kq[lane] = fkey(yv);
    }
    if (!ok) dq[0] = dq[1] = ac[0] = ac[1] = 0.f;
    const float dqn = hn ? dq[1] : dq[0];
    if (own_wg && h.dq[hn].t) GW(h.dq[hn].t)[tidx(h.dq[hn].rbs, b, 0)] = dqn;
    dqs[lane] = dqn;
    acs[lane] = ac[0];
    acs[16 + lane] = ac[1];
  }
  __syncthreads();
  if (own_wg && hn == 0 && wave == 0) {
    if (lane < 4 && h.loss_part) {  // op_head_t's partials: its workgroups of 4 rows
      GAS float* lp = GW(h.loss_part) + (size_t)((i0 >> 2) + lane) * 4;
      const int r4 = 4 * lane;
      lp[0] = (acs[r4] + acs[r4 + 1]) + (acs[r4 + 2] + acs[r4 + 3]);
      lp[1] = (acs[16 + r4] + acs[16 + r4 + 1]) + (acs[16 + r4 + 2] + acs[16 + r4 + 3]);
      lp[2] = 0.f;
      lp[3] = 0.f;
    }
    if (lane == 0 && td7) {  // value_max / value_min (td7.py:217-218)
      int kmax = kq[0], kmin = kq[0];
      const int nr = min(16, h.nvalid - i0);  // (>= 1: the batch pads fewer than 16 rows)
      for (int r = 1; r < nr; ++r) {
        kmax = max(kmax, kq[r]);
        kmin = min(kmin, kq[r]);
      }
      atomicMax(h.vmax_key, kmax);
      atomicMin(h.vmin_key, kmin);
    }
  }
  own_dz = own_dz && (h.dz[hn].n != nullptr || h.dz[hn].t != nullptr);
  __syncthreads();
  // ---- the DX reduction over this wave's chunks [c0, c1) of the single A segment
  if (!active || c0 >= c1) return acc;
  const float dqr = dqs[lane & 15];
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int c = 0; c < n; c += kRing) {
#pragma unroll
    for (int r = 0; r < kRing; ++r) {
      if (c + r >= n) break;  // (uniform, as ring_run)
      const int k = c0 + c + r;  // absolute chunk
      const float4 z = xa[r], w = *(const float4*)(w3s + k * 16 + cq);
      const float4 y = make_float4((dqr * w.x) * act_b<DACT>(z.x), (dqr * w.y) * act_b<DACT>(z.y),
                                   (dqr * w.z) * act_b<DACT>(z.z), (dqr * w.w) * act_b<DACT>(z.w));
      if (own_dz) mat_str4(h.dz[hn], i0 + (lane & 15), k * 16 + cq, y);
      if (r & 1) acc1 = mfma4(y, xb[r], acc1);
      else acc = mfma4(y, xb[r], acc);
      const int nx = c + r + kRing;
      if (nx >= n) continue;
      xa[r] = bload(ra, va + nx * 1024);
      xb[r] = bload(rb, vb + nx * 1024);
    }
  }
  return acc + acc1;
}

// ---------------------------------------------------------------- 64-row LDS-staged tiles (GemmHot::wide)
//
// One workgroup = a 64 x (16 NBW) output tile of a FWD / DX GEMM over >= 512 batch rows (rle_plan wide, the
// KS_TD7W instance): wave w owns rows 16w .. 16w + 15 and the tile's NBW column blocks (NBW = 4: 64 columns, 2:
// 32).  Each 16-wide reduction chunk's operands -- the tile's 4 A row blocks and its NBW W column blocks -- are
// copied into one slot of an LDS ring by LDS-DMA (global_load_lds_dwordx4, 1 KB per wave instruction: wave w
// copies its own A block and, w < NBW, W column block w), so each W block is fetched once per workgroup and
// feeds all four row blocks, and the ring holds no VGPRs: R - 1 chunks are in flight while one is reduced
// (R = wide_ring<NBW>, 40 KB of LDS).  Every wave keeps NBW independent accumulator chains, each split by chunk
// parity relative to its segment exactly as ring_run sums a segment, so at NBW = 4 the sums are the floats of
// the 16-row tn-64 tile; the epilogues combine column blocks in that tile's wave order.
// Protocol per chunk k: wait for this wave's DMAs of chunk k (counted vmcnt: the DMAs are inline asm, outside
// the compiler's wait bookkeeping, and no other vector-memory instruction is issued inside the loop), s_barrier
// (every wave's DMAs of chunk k landed; every wave is done reading chunk k - 1's slot), issue chunk k + R - 1
// into that freed slot, read chunk k's fragments, MFMA.
constexpr int kWideSmem = 10240;  // floats (40 KB: 4 workgroups per CU, as the 127 VGPRs allow)
template <int NBW>
constexpr int wide_slot() {
  return (4 + NBW) * 256;
}
template <int NBW>
constexpr int wide_ring() {
  return kWideSmem / wide_slot<NBW>() > 6 ? 6 : kWideSmem / wide_slot<NBW>();
}

__device__ __forceinline__ unsigned lds_off(const float* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)p;
}
// one 1 KB fragment block (this lane's 16 bytes at src) -> LDS bytes [lds, lds + 1 KB), lane l at lds + 16 l
__device__ __forceinline__ void glds_block(const float* src, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds)
               : "memory");
}
// this wave's DMAs of a chunk landed, with n younger DMAs still in flight (n <= 10)
__device__ __forceinline__ void wide_wait(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
  }
}
__device__ __forceinline__ void wide_barrier() { asm volatile("s_barrier" ::: "memory"); }

template <int MODE, int EPI, int ACT, bool NORM, int NBW>
__device__ __forceinline__ void gemm_wide(const CAS GemmArgs& g, int t, float* smem, unsigned long long* tr,
                                          int tiles_n, int gN, int gR, float inv_tn, int nseg_a, int nseg_b,
                                          int tiles, int xb, int tmb, int nfull, float inv_tmb, float inv_xb,
                                          float inv_blast, const float* biasp) {
  constexpr int R = wide_ring<NBW>(), SLOT = wide_slot<NBW>();
  static_assert(R >= 3 && R * SLOT <= kWideSmem, "wide ring");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int it, jt;
  if (xb) {
    xcd_tile(t, tiles, tiles_n, xb, tmb, nfull, inv_tmb, inv_xb, inv_blast, it, jt);
  } else {
    it = (int)(((float)t + 0.5f) * inv_tn);
    jt = t - it * tiles_n;
  }
  const int i0 = (it << 6) + (wave << 4);  // this wave's 16 rows
  const int jc0 = jt * (16 * NBW);         // the tile's first column
  const int ib = i0 + ((lane >> 4) << 2);
  const int nch = gR >> 4;
  const bool wabs = MODE == GEMM_FWD && nseg_b == 1;
  const int nbv = min(NBW, (gN - jc0 + 15) >> 4);  // column blocks of this tile inside the output
  const int per = wave < NBW ? 2 : 1;              // DMAs this wave issues per chunk
  // ---- epilogue operands, issued before any LDS-DMA (ordinary loads older than the ring)
  float pb[NBW], qwj[NBW];
  float4 ev[NBW];
#pragma unroll
  for (int c = 0; c < NBW; ++c) {
    const int j = jc0 + c * 16 + (lane & 15);
    const bool jok = j < gN;
    pb[c] = qwj[c] = 0.f;
    ev[c] = make_float4(1.f, 1.f, 1.f, 1.f);
    if (jok && biasp) pb[c] = G(biasp)[j];
    if constexpr (EPI == EPI_QHEAD || EPI == EPI_QDOT) {
      if (jok) qwj[c] = G(g.qw)[nidx(g.qw_cbn, 0, j)];
    }
    if constexpr (MODE == GEMM_DX && ACT != ACT_NONE && EPI == EPI_STORE) {
      if (jok) ev[c] = mat_ld4(g.dsrc, ib, j);
    }
    if constexpr (EPI == EPI_MSE) {
      if (jok) ev[c] = mat_ld4(g.tgt, ib, j);
    }
    if constexpr (EPI == EPI_NBDOT) {
      if (jok) ev[c] = mat_ld4(g.nbx, ib, j);
    }
  }
  // EPI_MSE: |zs'| partials of the wave's 16 rows, partial p = lane / 16 + 4 m (<= 16 partials: a row table)
  float tnv[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (EPI == EPI_MSE) {
    const CAS NormRef& nr = g.tgt_norm;
    if (nr.part && nr.nparts <= 16) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int p = (lane >> 4) + 4 * m;
        if (p < nr.nparts) tnv[m] = G(nr.part)[(size_t)p * nr.ld + nr.row0 + i0 + (lane & 15)];
      }
    }
  }
  // deferred AvgL1Norm of each A segment: 1 / m of this lane's row (as inv_of in gemm_v)
  float inv[kMaxSeg] = {1.f, 1.f, 1.f, 1.f};
  if constexpr (NORM) {
#pragma unroll
    for (int q = 0; q < kMaxSeg; ++q)
      if (q < nseg_a && g.A.seg[q].norm.part) inv[q] = norm_inv_i(g.A.seg[q].norm, i0 + (lane & 15));
  }
  trace_mark(tr, 1);
  // ---- DMA issue: chunk by chunk in reduction order, the segment pointers advanced at segment starts
  const unsigned ring = lds_off(smem);
  const int bcol = (jc0 >> 4) + min(wave, nbv - 1);  // (blocks past the output: a valid block, never used)
  int iq = 0, inext = nseg_a > 1 ? (g.A.seg[1].r0 >> 4) : nch;
  const float* ia = g.A.seg[0].p + ((size_t)((i0 >> 4) * g.A.seg[0].xs) * 256 + lane * 4);
  const float* ibp = g.B.seg[0].p + ((size_t)(bcol * g.B.seg[0].xs) * 256 + lane * 4);
  int ik = 0;  // the next chunk to issue
  auto issue_next = [&]() {
    if (ik == inext) {  // (uniform) the next A segment; W: its own segment (DX / folded), or the same (wabs)
      ++iq;
      const CAS Seg& sa = g.A.seg[iq];
      ia = sa.p + ((size_t)((i0 >> 4) * sa.xs) * 256 + lane * 4);
      if (!wabs) {
        const CAS Seg& sb = g.B.seg[iq];
        ibp = sb.p + ((size_t)(bcol * sb.xs) * 256 + lane * 4);
      }
      inext = iq + 1 < nseg_a ? (g.A.seg[iq + 1].r0 >> 4) : nch;
    }
    const unsigned slot = ring + (unsigned)((ik % R) * SLOT * 4);
    glds_block(ia, slot + wave * 1024);
    if (wave < NBW) glds_block(ibp, slot + 4096 + wave * 1024);
    ia += 256;
    ibp += 256;
    ++ik;
  };
#pragma unroll
  for (int k = 0; k < R - 1; ++k)
    if (k < nch) issue_next();
  // ---- the chunk loop, segment by segment, chunks in pairs (even / odd accumulators, as ring_run); one wait,
  // barrier and issue round per pair, so the per-step synchronisation is paid once per 32 reduction rows
  f32x4 ac[NBW], ac1[NBW];
#pragma unroll
  for (int c = 0; c < NBW; ++c) ac[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](int k, f32x4(&acc)[NBW], float sinv) {
    const float* slot = smem + (k % R) * SLOT;
    float4 a = *(const float4*)(slot + wave * 256 + lane * 4);
    if constexpr (NORM) a = scale4(a, sinv);
    float4 b[NBW];
#pragma unroll
    for (int c = 0; c < NBW; ++c) b[c] = *(const float4*)(slot + 1024 + c * 256 + lane * 4);
#pragma unroll
    for (int c = 0; c < NBW; ++c) acc[c] = mfma4(a, b[c], acc[c]);
  };
#pragma unroll 1
  for (int q = 0; q < nseg_a; ++q) {
    const int k0 = g.A.seg[q].r0 >> 4, k1 = q + 1 < nseg_a ? (g.A.seg[q + 1].r0 >> 4) : nch;
    const float sinv = NORM ? (q == 0 ? inv[0] : q == 1 ? inv[1] : q == 2 ? inv[2] : inv[3]) : 1.f;
#pragma unroll
    for (int c = 0; c < NBW; ++c) ac1[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int k = k0; k < k1; k += 2) {
      const bool two = k + 1 < k1;
      wide_wait(per * (ik - k - (two ? 2 : 1)));  // (chunks k, k + 1 landed: ik - k - n younger ones in flight)
      wide_barrier();
      if (ik < nch && ik < k + R) issue_next();  // (the slots of chunks < k are free: up to chunk k + R - 1)
      if (ik < nch && ik < k + R) issue_next();
      mma(k, ac, sinv);
      if (two) mma(k + 1, ac1, sinv);
    }
#pragma unroll
    for (int c = 0; c < NBW; ++c) ac[c] = ac[c] + ac1[c];  // (ring_run's "return acc + acc1")
  }
  trace_mark(tr, 2);
  __syncthreads();  // (every wave is done with the ring: the epilogue reuses the LDS)
  // ---- epilogue, column block by column block; the tile's row sums in the 16-row tile's wave order
  // (NBW 4: (s0 + s1) + (s2 + s3), s_c the row16_sum of column block c; NBW 2: s0 + s1), loss partials one per
  // 16-row block (wave_sum per column block, the same order) at the 16-row tile's row-major index
  float rsa[4] = {0.f, 0.f, 0.f, 0.f}, rsb[4] = {0.f, 0.f, 0.f, 0.f};
  float lsa = 0.f, lsb = 0.f;
  float* tabw = smem + wave * 256;  // (EPI_MSE: this wave's row table of norm partials)
  if constexpr (EPI == EPI_MSE) {
#pragma unroll
    for (int m = 0; m < 4; ++m) tabw[((lane >> 4) + 4 * m) * 16 + (lane & 15)] = tnv[m];
  }
#pragma unroll
  for (int c = 0; c < NBW; ++c) {
    const int j = jc0 + c * 16 + (lane & 15);
    const bool jok = j < gN;
    const f32x4 acc = ac[c];
    const float e4[4] = {ev[c].x, ev[c].y, ev[c].z, ev[c].w};
    float rv[4] = {0.f, 0.f, 0.f, 0.f};
    float lv = 0.f;
    if constexpr (EPI == EPI_STORE || EPI == EPI_QDOT) {
      if (jok) {
        float y[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) y[qq] = acc[qq] + pb[c];
        if constexpr (MODE == GEMM_FWD) {
          if (g.pre.t) mat_st4(g.pre, ib, j, make_float4(y[0], y[1], y[2], y[3]));
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) y[qq] = act_f<ACT>(y[qq]);
        } else {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) y[qq] *= act_b<ACT>(e4[qq]);
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) rv[qq] = EPI == EPI_QDOT ? y[qq] * qwj[c] : fabsf(y[qq]);
        mat_st4(g.out, ib, j, make_float4(y[0], y[1], y[2], y[3]));
      }
    } else if constexpr (EPI == EPI_NBDOT) {
      if (jok) {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) rv[qq] = acc[qq] * e4[qq];
        mat_st4(g.out, ib, j, make_float4(acc[0], acc[1], acc[2], acc[3]));
      }
    } else if constexpr (EPI == EPI_QHEAD) {  // td7.py:268-275
      if (jok) {
        float dz[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const float z = acc[qq] + pb[c], y = act_f<ACT>(z);
          const bool rv = ib + qq < g.mvalid;  // (rows of the padded batch past it add nothing)
          lv += rv ? y * qwj[c] : 0.f;
          dz[qq] = rv ? (g.qscale * qwj[c]) * act_b<ACT>(ACT == ACT_RELU ? y : z) : 0.f;
        }
        mat_st4(g.out, ib, j, make_float4(dz[0], dz[1], dz[2], dz[3]));
      }
    } else if constexpr (EPI == EPI_MSE) {  // td7.py:256
      const CAS NormRef& nr = g.tgt_norm;
      if (jok) {
        float gr[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          float iv;
          if (nr.part && nr.nparts <= 16) {  // the sum order, clamp and reciprocal of norm_inv
            float sm = 0.f;
            for (int p = 0; p < nr.nparts; ++p) sm += tabw[p * 16 + (ib - i0) + qq];
            const float m = sm / (float)nr.width;
            iv = 1.f / (m < 1e-8f ? 1e-8f : m);
          } else {
            iv = norm_inv(nr, ib + qq);
          }
          const float d = ib + qq < g.mvalid ? (acc[qq] + pb[c]) - e4[qq] * iv : 0.f;  // (padded rows: 0)
          gr[qq] = (2.f * d) * g.mse_scale;
          lv += d * d;
        }
        mat_st4(g.out, ib, j, make_float4(gr[0], gr[1], gr[2], gr[3]));
      }
    }
    if constexpr (EPI == EPI_QDOT || EPI == EPI_NBDOT || (EPI == EPI_STORE && MODE == GEMM_FWD)) {
      if (EPI != EPI_STORE || g.norm_out) {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const float s = row16_sum(rv[qq]);
          if (c == 0) rsa[qq] = s;
          else if (c == 1) rsa[qq] += s;
          else if (c == 2) rsb[qq] = s;
          else rsb[qq] += s;
        }
      }
    }
    if constexpr (EPI == EPI_QHEAD || EPI == EPI_MSE) {
      const float s = wave_sum(lv);
      if (c == 0) lsa = s;
      else if (c == 1) lsa += s;
      else if (c == 2) lsb = s;
      else lsb += s;
    }
  }
  if constexpr (EPI == EPI_QDOT || EPI == EPI_NBDOT || (EPI == EPI_STORE && MODE == GEMM_FWD)) {
    if ((EPI != EPI_STORE || g.norm_out) && (lane & 15) == 0) {
      GAS float* dst = GW(g.norm_out) + (size_t)jt * g.norm_ld + ib;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) dst[qq] = NBW == 4 ? rsa[qq] + rsb[qq] : rsa[qq];
    }
  }
  if constexpr (EPI == EPI_QHEAD || EPI == EPI_MSE) {
    if (lane == 0) {
      const int t16 = (i0 >> 4) * tiles_n + jt;  // (the 16-row tile's row-major index: the partial count is unchanged)
      float v = NBW == 4 ? lsa + lsb : lsa;
      if constexpr (EPI == EPI_QHEAD) v = t16 == 0 ? v + (float)g.mvalid * sload(g.qb) : v;
      GW(g.loss_part)[t16] = v;
    }
  }
}

// EXT: the register-blocked weight-gradient tiles are compiled in (the extended and the KS_TD7W instances); the
// production instances compile without them, so their registers do not shape their allocation
// WIDE: the variant also runs 64-row LDS-staged tiles (GemmHot::wide, gemm_wide; the KS_TD7W and extended instances)
template <int MODE, int EPI, int ACT, bool NORM, int PK = 0, bool EXT = false, bool WIDE = false>  // PK: 1 pre-GEMM, 2 fused loss head, 3 pre-layer, 4 pre-layer behind a pre-GEMM, 5 SAC raw head + rsample pre-GEMM
__device__ __forceinline__ void gemm_v(const CAS GemmArgs& g, int t, float* smem, unsigned long long* tr) {
  FINE_MARK(10);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // ---- every descriptor field the prologue and the first operand segment need (GemmHot)
  // in ONE batch of scalar loads.  Left to the compiler, each load is issued next to its
  // use, behind branches: one dependent round trip each, ~6 before the first operand load.
  // The same batch also touches (one dword each) every other 64-byte line of the descriptor
  // this variant reads later (segments, epilogue, Adam, pre-GEMM fields), so those loads hit
  // the scalar cache instead of each paying a dependent L2/MALL round trip (+2% steps/s).
  // Early-clobber outputs: the base must not share SGPRs with a load still being issued.
  u32x16 h0, h1;
  unsigned dsink;
#define RLE_HOT_ASM(TOUCH)                                  \
  asm volatile("s_load_dwordx16 %0, %3, 0x0\n\t"            \
               "s_load_dwordx16 %1, %3, 0x40\n\t" TOUCH     \
               "s_waitcnt lgkmcnt(0)"                       \
               : "=&s"(h0), "=&s"(h1), "=&s"(dsink)         \
               : "s"(&g.hot))
#define TL(off) "s_load_dword %2, %3, " #off "\n\t"
#define TL_A TL(0xb0) TL(0xf0) TL(0x130) TL(0x170)
#define TL_B TL(0x1b0) TL(0x1f0) TL(0x230) TL(0x270)
#define TL_S TL(0x2b0)
#define TL_N TL(0x2f0) TL(0x330)
#define TL_X TL(0x370)
#define TL_P TL(0x3b0) TL(0x3f0) TL(0x430) TL(0x470) TL(0x4b0) TL(0x4f0) TL(0x530) TL(0x570) TL(0x5b0) TL(0x5f0)
#define TL_D TL(0x5f0) TL(0x630)
#define TL_O TL(0x670)
#define TL_Q TL(0x6b0) TL(0x770) TL(0x7b0) TL(0x870) TL(0x8b0)
  if constexpr (MODE == GEMM_DW) {
    if constexpr (ACT == kDwNb) RLE_HOT_ASM(TL_B TL_D TL_X);
    else RLE_HOT_ASM(TL_B TL_D);
  } else if constexpr (PK == 4) {
    RLE_HOT_ASM(TL_A TL_B TL_S TL_N TL_P TL_Q);
  } else if constexpr (PK != 0) {
    if constexpr (MODE == GEMM_FWD && (ACT == ACT_TANH || EPI == EPI_QDOT)) RLE_HOT_ASM(TL_A TL_B TL_S TL_N TL_P);
    else RLE_HOT_ASM(TL_A TL_B TL_S TL_P);
  } else if constexpr (EPI == EPI_NBDOT) {
    RLE_HOT_ASM(TL_A TL_B TL_S TL_X);
  } else if constexpr (EPI == EPI_ACT) {
    RLE_HOT_ASM(TL_A TL_B TL_S TL_O);
  } else if constexpr (EPI == EPI_MSE || EPI == EPI_QHEAD || EPI == EPI_QDOT || (MODE == GEMM_FWD && ACT == ACT_TANH)) {
    RLE_HOT_ASM(TL_A TL_B TL_S TL_N);
  } else {
    RLE_HOT_ASM(TL_A TL_B TL_S);
  }
#undef RLE_HOT_ASM
#undef TL
#undef TL_A
#undef TL_B
#undef TL_S
#undef TL_N
#undef TL_X
#undef TL_P
#undef TL_D
#undef TL_O
#undef TL_Q
  (void)dsink;
  auto ptr = [](unsigned lo, unsigned hi) { return (const float*)(((unsigned long long)hi << 32) | lo); };
  const int ksl = (int)h0[0], tiles_n = (int)h0[1], tn = (int)h0[2], gN = (int)h0[3], gR = (int)h0[4];
  const float inv_tn = __uint_as_float(h0[5]);
  const int bias_col = (int)h0[6], nseg_a = (int)h0[7], nseg_b = (int)h0[8];
  const int a0xs = (int)h0[9], a0r0 = (int)h0[10], a0r1 = (int)h0[11], b0xs = (int)h0[12];
  const float* a0p = ptr(h0[14], h0[15]);
  const float* b0p = ptr(h1[0], h1[1]);
  const float* biasp = ptr(h1[2], h1[3]);
  if constexpr (WIDE) {
    if (h1[11]) {  // (GemmHot::wide: 64 -> 64-column tiles, 32 -> 32-column tiles)
      if (h1[11] == 64)
        gemm_wide<MODE, EPI, ACT, NORM, 4>(g, t, smem, tr, tiles_n, gN, gR, inv_tn, nseg_a, nseg_b, (int)h0[13],
                                           (int)h1[4], (int)h1[5], (int)h1[9], __uint_as_float(h1[6]),
                                           __uint_as_float(h1[7]), __uint_as_float(h1[8]), biasp);
      else
        gemm_wide<MODE, EPI, ACT, NORM, 2>(g, t, smem, tr, tiles_n, gN, gR, inv_tn, nseg_a, nseg_b, (int)h0[13],
                                           (int)h1[4], (int)h1[5], (int)h1[9], __uint_as_float(h1[6]),
                                           __uint_as_float(h1[7]), __uint_as_float(h1[8]), biasp);
      return;
    }
  }
  const int cg = wave >> ksl, kp = wave & ((1 << ksl) - 1);
  // register-blocked wide weight-gradient tile (GemmHot::rb; the host sets it only for tn 32 / 64)
  constexpr bool RBOK = EXT && PK == 0 && MODE == GEMM_DW;
  const bool rbm = RBOK && h1[10] != 0;
  int it, jt;
  if (h1[4]) {  // XCD-aware order (GemmHot::xb): residue class t % 8 -> a contiguous run p
    xcd_tile(t, (int)h0[13], tiles_n, (int)h1[4], (int)h1[5], (int)h1[9], __uint_as_float(h1[6]),
             __uint_as_float(h1[7]), __uint_as_float(h1[8]), it, jt);
  } else {
    it = (int)(((float)t + 0.5f) * inv_tn);
    jt = t - it * tiles_n;
  }
  const int i0 = it << 4, j0 = jt * tn + (cg << 4);
  // the 16 x 64 weight-gradient + Adam tiles are the longest ops of their levels: their waves win
  // instruction arbitration over the shorter ops sharing a CU (A/B: +0.2-0.3%; also raising the
  // pre-GEMM and fused-head consumers: no further gain)
  if constexpr (MODE == GEMM_DW) {
    if (tn == 64) __builtin_amdgcn_s_setprio(3);
  }
  const bool bias_tile = EPI == EPI_ADAM && jt * tn >= bias_col;
  const bool lead = kp == 0;
  const bool active = bias_tile ? cg == 0 : j0 < gN;  // wave-uniform
  const int j = j0 + (lane & 15), ib = i0 + ((lane >> 4) << 2);
  const bool jok = active && lead && (bias_tile ? j == bias_col : j < gN);
  float* red = smem;               // [64] reduction scratch
  float* part = smem + 64;         // [4 waves][64][4] split-K partials
  float* tabs = smem + 64 + 1024;  // AvgL1Norm 1/m tables (T-image operands)
  const int nch = gR >> 4;
  const int per = (nch + (1 << ksl) - 1) >> ksl;
  const int c0 = kp * per, c1 = min(nch, c0 + per);
  FINE_MARK(8);

  // ---- epilogue operands fetched ahead of the main loop
  float pre_b = 0.f;
  float4 ds = make_float4(1.f, 1.f, 1.f, 1.f), pp = make_float4(0.f, 0.f, 0.f, 0.f), mm = pp, vv = pp;
  size_t wt = 0;
  float qwj = 0.f;
  if constexpr (EPI == EPI_QHEAD || EPI == EPI_QDOT) {
    if (jok) qwj = G(g.qw)[nidx(g.qw_cbn, 0, j)];
  }
  // EPI_MSE: the target tile and the |zs'| partials of its 16 rows (thread t: part t / 16, row
  // t % 16), so the epilogue does not wait on 4 dependent norm fetches after the loop
  float4 tgv = make_float4(0.f, 0.f, 0.f, 0.f);
  float tnv = 0.f;
  if constexpr (EPI == EPI_MSE) {
    if (jok) tgv = mat_ld4(g.tgt, ib, j);
    const CAS NormRef& nr = g.tgt_norm;
    if (nr.part && (tid >> 4) < nr.nparts && nr.nparts <= 16)
      tnv = G(nr.part)[(size_t)(tid >> 4) * nr.ld + nr.row0 + i0 + (tid & 15)];
  }
  float4 nbxv = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (EPI == EPI_NBDOT) {
    if (jok) nbxv = mat_ld4(g.nbx, ib, j);
  }
  // EPI_SACFWD: the rsample noise of this thread's (row, column) items of the epilogue (16 A <= 2
  // kThreads of them), fetched before the main loop
  float sfe[2] = {0.f, 0.f};
  if constexpr (EPI == EPI_SACFWD) {
    const CAS SacFwdArgs& s = g.sf;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int it2 = tid + k * kThreads, r = it2 / s.A, jj = it2 - r * s.A, b = i0 + r;
      if (it2 < 16 * s.A && b < g.M)
        sfe[k] = b < s.eps_row_split ? mat_ld(s.eps2, b, jj) : mat_ld(s.eps, b - s.eps_row_split, jj);
    }
  }
  if constexpr (EPI != EPI_ADAM) {
    if (jok && biasp) pre_b = G(biasp)[j];
    if constexpr (MODE == GEMM_DX && ACT != ACT_NONE) {
      if (jok) ds = mat_ld4(g.dsrc, ib, j);
    }
  } else {
    if (jok) {
      const CAS AdamArgs& ad = g.adam;
      if (bias_tile) {
        pp = ld4g(G(ad.b) + ib);
        mm = ld4g(G(ad.b) + ib + ad.mo);
        vv = ld4g(G(ad.b) + ib + ad.vo);
      } else {
        wt = tidx(ad.w.rbs, ib, j);
        pp = ld4g(G(ad.w.t) + wt);
        mm = ld4g(G(ad.w.t) + wt + ad.mo);
        vv = ld4g(G(ad.w.t) + wt + ad.vo);
      }
    }
  }
  trace_mark(tr, 1);

  // ---- reduction
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f32x4 sac1 = acc, sac2 = acc;  // (EPI_SACFWD: column blocks 1, 2 of the raw tile, wave 0)
  const int lb = lane * 16;
  if constexpr (MODE != GEMM_DW) {
    // A: N image, segments along the reduction; B: W (FWD: N image, one segment over
    // the whole reduction; DX: T image, one segment per A segment)
    // (segment 0 from the hot header; later segments load their own fields)
    // FWD with one W segment: W spans the whole reduction (absolute chunk index);
    // DX, or FWD with one W segment per A segment (folded weight blocks): each W
    // segment starts at its own reduction offset (relative chunk index)
    const bool wabs = MODE == GEMM_FWD && nseg_b == 1;
    auto inv_of = [&](int q) {
      float inva = 1.f;
      if constexpr (NORM) {
        if (g.A.seg[q].norm.part) inva = norm_inv_i(g.A.seg[q].norm, i0 + (lane & 15));
      }
      return inva;
    };
    // (the segment's deferred-AvgL1Norm scale is fetched while its first chunks are in flight)
    auto seg = [&](const float* sap, int sxs, int sr0, int sr1, const float* sbp, int bxs, int q) {
      const int s0 = sr0 >> 4;
      const int k0 = max(c0, s0), k1 = min(c1, (sr1 + 15) >> 4);
      if (!active || k0 >= k1) return;
      const int va = ((i0 >> 4) * sxs + (k0 - s0)) * 1024 + lb;
      const int vb = ((j0 >> 4) * bxs + (wabs ? k0 : k0 - s0)) * 1024 + lb;
      float4 ra[kRing], rb[kRing];
      ring_issue(ra, rb, rsrc(sap), va, rsrc(sbp), vb, k1 - k0, false);
      const float inva = inv_of(q);
      acc = ring_run<NORM ? 1 : 0, 0>(ra, rb, rsrc(sap), va, rsrc(sbp), vb, k1 - k0, acc, inva, nullptr, nullptr, false);
    };
    if constexpr (PK == 2) {  // fused loss head: one A segment, dZ of the critic's last hidden layer
      acc = headdx_reduce<ACT>(g, i0, j0, active, jt == 0, jt == 0 && cg == 0, c0, c1, nch, a0p, a0xs, b0p, b0xs,
                               smem, acc);
    } else if constexpr (PK == 3 || PK == 4) {  // the whole A operand from the pre-layer in LDS (prelayer_*)
      float* pimg = smem + 64 + 1024;
      const int nrun = active && c0 < c1 ? c1 - c0 : 0;
      const int vb = ((j0 >> 4) * b0xs + c0) * 1024 + lb;
      const auto rbw = rsrc(b0p);
      float4 rbq[4];  // the wave's first W chunks in flight with the pre-layer's operands
      auto issue_rbq = [&]() {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (r < nrun) rbq[r] = bload(rbw, vb + r * 1024);
      };
      if constexpr (PK == 3) issue_rbq();
      // (A/B, TD3: issuing 8 more chunks once the pre-layer's MFMAs free their registers measured
      // -1.2% against this one-group-ahead loop)
      if constexpr (PK == 4) {
        // two-stage prologue: the pre-GEMM (target action, N <= 16) and the pre-layer's memory operands in
        // flight together; the pre-GEMM's output (pimg2, after the pre-layer image) is the pre-layer's input
        // segment 1 (host-checked: prea2.seg == 1 of 2)
        float* pimg2 = smem + 64 + 1024 + 4096;
        PreRing pr;
        PlRing pl;
        pre_issue<GEMM_FWD, true>(g.prea2, i0, pr);
        prelayer_issue<MODE, true>(g.prea, i0, pl);
        pre_finish<GEMM_FWD, true>(g.prea2, i0, pr, part, nullptr, pimg2);
        issue_rbq();  // (in the pre-GEMM ring's registers, in flight through the pre-layer's MFMAs)
        prelayer_finish<MODE, ACT, true>(g.prea, pl, pimg, pimg2);
      } else {
        prelayer_fwd<MODE, ACT>(g.prea, i0, pimg);
      }
      f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};  // (chunks on two accumulators by parity, as ring_run)
#pragma unroll 1
      for (int c = 0; c < nrun; c += 4) {
        float4 nx[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (c + 4 + r < nrun) nx[r] = bload(rbw, vb + (c + 4 + r) * 1024);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (c + r >= nrun) break;
          const float4 x = *(const float4*)(pimg + (c0 + c + r) * 256 + lane * 4);
          if (r & 1) acc1 = mfma4(x, rbq[r], acc1);
          else acc = mfma4(x, rbq[r], acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) rbq[r] = nx[r];
      }
      acc = acc + acc1;
    } else if constexpr (PK == 5) {
      // segment g.prea.seg is SAC's target action a' = tanh(mean + exp(clamp(log_std)) eps) of the tile's
      // rows, from the raw head recomputed in-tile (sacraw_*, the standalone EPI_SACFWD's order and
      // arithmetic); its operands are in flight with the consumer's own segments
      const CAS PreArgs& p = g.prea;
      float* pimg = smem + 64 + 3072;  // a' (N-image fragment blocks, columns >= A zero)
      float* rt = pimg + 512;          // [16][48] raw rows
      const int nchp = p.R >> 4, A = p.sac_a;
      SacRing sr;
      sacraw_issue(p.A.seg[0].p, p.A.seg[0].xs, p.B.seg[0].p, p.B.seg[0].xs, nchp, i0, sr);
      float bj[3], ev[2];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int jj = c * 16 + (lane & 15);
        bj[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc(p.bias), jj < p.N ? jj * 4 : kOOB, 0, 0));
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int it = tid + k * kThreads, r = it >> 5, jj = it & 31;
        ev[k] = jj < A ? mat_ld(p.noise, i0 + r, jj) : 0.f;
      }
      const int pseg = p.seg;
      if (pseg != 0) seg(a0p, a0xs, a0r0, a0r1, b0p, b0xs, 0);
      for (int q = 1; q < nseg_a; ++q) {
        if (q == pseg) continue;
        const CAS Seg& sa = g.A.seg[q];
        const CAS Seg& sb = g.B.seg[wabs ? 0 : q];
        seg(sa.p, sa.xs, sa.r0, sa.r1, sb.p, sb.xs, q);
      }
      f32x4 sv[3];
      sacraw_finish(sr, nchp, part, sv);
      if (wave == 0) {
        const int rb = (lane >> 4) << 2;
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
          for (int q = 0; q < 4; ++q) rt[(rb + q) * 48 + c * 16 + (lane & 15)] = sv[c][q] + bj[c];
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 2; ++k) {  // (as the standalone epilogue's rsample)
        const int it = tid + k * kThreads, r = it >> 5, jj = it & 31;
        float v = 0.f;
        if (jj < A) {
          const float mu = rt[r * 48 + jj];
          const float ls = fminf(fmaxf(rt[r * 48 + A + jj], p.noise_sigma), p.noise_clip);
          const float sd = expf(ls);
          v = tanhf(mu + ev[k] * sd);
        }
        pimg[(jj >> 4) * 256 + ((jj & 15) >> 2) * 64 + r * 4 + (jj & 3)] = v;
      }
      __syncthreads();
      const CAS Seg& sa = g.A.seg[pseg];
      const CAS Seg& sb = g.B.seg[wabs ? 0 : pseg];
      const int s0 = sa.r0 >> 4;
      const int k0 = max(c0, s0), k1 = min(c1, (sa.r1 + 15) >> 4);
      if (active && k0 < k1)
        acc = chunk_loop_lds_par(pimg + (k0 - s0) * 256, rsrc(sb.p),
                                 ((j0 >> 4) * sb.xs + (wabs ? k0 : k0 - s0)) * 1024 + lb, k1 - k0, acc);
    } else if constexpr (EPI == EPI_SACFWD) {  // the raw head in sacraw order (see PK 5), whole rows per tile
      SacRing sr;
      sacraw_issue(a0p, a0xs, b0p, b0xs, nch, i0, sr);
      f32x4 sv[3];
      sacraw_finish(sr, nch, part, sv);
      if (wave == 0) {
        acc = sv[0];
        sac1 = sv[1];
        sac2 = sv[2];
      }
    } else if constexpr (PK == 1) {  // segment g.prea.seg comes from the pre-GEMM in LDS
      float* pimg = smem + 64 + 2048;
      PreRing pr;
      pre_issue<MODE>(g.prea, i0, pr);
      FINE_MARK(0);
      const int pseg = g.prea.seg;
      // segment 0 from the hot header, outside the loop: a loop header would wait for every
      // load in flight (the pre-GEMM's included) before the segment's first load is issued
      if (pseg != 0) seg(a0p, a0xs, a0r0, a0r1, b0p, b0xs, 0);
      for (int q = 1; q < nseg_a; ++q) {
        if (q == pseg) continue;
        const CAS Seg& sa = g.A.seg[q];
        const CAS Seg& sb = g.B.seg[wabs ? 0 : q];
        seg(sa.p, sa.xs, sa.r0, sa.r1, sb.p, sb.xs, q);
      }
      FINE_MARK(1);
      pre_finish<MODE>(g.prea, i0, pr, part, smem + 64 + 1024, pimg);
      FINE_MARK(2);
      const CAS Seg& sa = g.A.seg[pseg];
      const CAS Seg& sb = g.B.seg[wabs ? 0 : pseg];
      const int s0 = sa.r0 >> 4;
      const int k0 = max(c0, s0), k1 = min(c1, (sa.r1 + 15) >> 4);
      if (active && k0 < k1)
        acc = chunk_loop_lds(pimg + (k0 - s0) * 256, rsrc(sb.p), ((j0 >> 4) * sb.xs + (wabs ? k0 : k0 - s0)) * 1024 + lb,
                             k1 - k0, acc);
    } else {
      seg(a0p, a0xs, a0r0, a0r1, b0p, b0xs, 0);
      for (int q = 1; q < nseg_a; ++q) {
        const CAS Seg& sa = g.A.seg[q];
        // FWD: one W segment over the whole reduction; DX: W segment q pairs with A segment q
        const CAS Seg& sb = g.B.seg[wabs ? 0 : q];
        seg(sa.p, sa.xs, sa.r0, sa.r1, wabs ? b0p : sb.p, wabs ? b0xs : sb.xs, q);
      }
    }
  } else if (RBOK && rbm) {
    // DW, register-blocked: every wave reduces its quarter of the batch rows for all tn / 16 column
    // blocks; the bias tile is one block of ones
    auto rbw = [&](auto nbt) {
      constexpr int NB = decltype(nbt)::value, RG = NB == 4 ? 2 : 4;
      constexpr bool NBX = ACT == kDwNb;
      const int nq = (nch + 3) >> 2, q0 = wave * nq, q1 = min(nch, q0 + nq), nrun = max(0, q1 - q0);
      const int jc0 = jt * tn;
      int nb = 0;
#pragma unroll
      for (int cb = 0; cb < NB; ++cb) nb = jc0 + cb * 16 < gN ? cb + 1 : nb;
      if (bias_tile) nb = 1;
      // (the tile's column blocks lie in one X segment: every segment starts at a multiple of tn)
      int qb = 0;
#pragma unroll
      for (int q = 1; q < kMaxSeg; ++q)
        if (q < nseg_b && min(jc0, gN - 1) >= g.B.seg[q].x0) qb = q;
      const CAS Seg& sbq = g.B.seg[qb];
      int vbv[NB];
#pragma unroll
      for (int cb = 0; cb < NB; ++cb) vbv[cb] = ((((jc0 - sbq.x0) >> 4) + cb) * sbq.xs + q0) * 1024 + lb;
      const int va = ((i0 >> 4) * a0xs + q0) * 1024 + lb;
      const int vx = NBX ? ((i0 >> 4) * g.nbx_xs + q0) * 1024 + lb : 0;
      const auto rx = NBX ? rsrc(g.nbx.t) : rsrc(a0p);
      RbRing<NB, RG> R;
      rb_issue<NB, RG, NBX>(R, rsrc(a0p), va, rsrc(sbq.p), vbv, nb, nrun, rx, vx, bias_tile);
      const float* tabb = nullptr;
      if constexpr (NORM) {  // 1/m of the reduction rows of the tile's X segment
        if (sbq.norm.part) build_norm_tab(sbq.norm, sbq.r1 - sbq.r0, tabs);
        __syncthreads();
        if (sbq.norm.part && !bias_tile) tabb = tabs + q0 * 16;
      }
      int tgo = 0;
      if constexpr (NBX) {
        tgo = (gR + 15) & ~15;
        build_nb_tab(g, gR, tabs, tabs + tgo);
        __syncthreads();
      }
      f32x4 ac[NB];
#pragma unroll
      for (int cb = 0; cb < NB; ++cb) ac[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
      rb_run<NB, RG, NBX>(R, rsrc(a0p), va, rsrc(sbq.p), vbv, nb, nrun, ac, tabb, rx, vx, tabs + q0 * 16,
                          tabs + tgo + q0 * 16, bias_tile);
      acc = rb_exchange<NB>(ac, smem, cg, lead);
    };
    if (tn == 64) rbw(std::integral_constant<int, 4>{});
    else rbw(std::integral_constant<int, 2>{});
  } else {
    // DW: A = dZ (T image, x = output row), B = X (T image, x = output column; the
    // wave's 16 columns lie in one column segment); both reduce over batch rows
    int qb = 0;
#pragma unroll
    for (int q = 1; q < kMaxSeg; ++q)
      if (q < nseg_b && j0 >= g.B.seg[q].x0) qb = q;
    const CAS Seg& sb = g.B.seg[qb];
    // first chunks in flight before the AvgL1Norm tables are built (their loads overlap)
    const bool run = active && c0 < c1;
    const int va = ((i0 >> 4) * a0xs + c0) * 1024 + lb;
    const int vb = (((j0 - sb.x0) >> 4) * sb.xs + c0) * 1024 + lb;
    const int vx = ACT == kDwNb ? ((i0 >> 4) * g.nbx_xs + c0) * 1024 + lb : 0;
    const int nrun = run ? c1 - c0 : 0;
    constexpr int RGD = ACT == kDwNb ? kRing : kRingDW;  // (the kDwNb ring carries a third operand)
    float4 ra[RGD], rb[RGD], rx[RGD];
    ring_issue<RGD>(ra, rb, rsrc(a0p), va, rsrc(sb.p), vb, nrun, bias_tile);
    if constexpr (ACT == kDwNb) {
#pragma unroll
      for (int r = 0; r < RGD; ++r)
        if (r < nrun) rx[r] = bload(rsrc(g.nbx.t), vx + r * 1024);
    }
    FINE_MARK(0);
    const float* tb = nullptr;
    if constexpr (NORM) {
      // 1/m of every reduction row of every normed B segment, segment by segment
      int off = 0, mine = -1;
      for (int q = 0; q < nseg_b; ++q) {
        const CAS Seg& s = g.B.seg[q];
        if (!s.norm.part) continue;
        build_norm_tab(s.norm, s.r1 - s.r0, tabs + off);
        if (q == qb) mine = off;
        off += (s.r1 - s.r0 + 15) & ~15;
      }
      __syncthreads();
      if (mine >= 0) tb = tabs + mine + c0 * 16;
    }
    int tgo = 0;
    if constexpr (ACT == kDwNb) {
      tgo = (gR + 15) & ~15;
      build_nb_tab(g, gR, tabs, tabs + tgo);
      __syncthreads();
    }
    FINE_MARK(1);
    if (run) {
      if constexpr (ACT == kDwNb) {
        acc = ring_run_nb<RGD>(ra, rx, rb, rsrc(a0p), va, rsrc(g.nbx.t), vx, rsrc(sb.p), vb, nrun, acc,
                               tabs + c0 * 16, tabs + tgo + c0 * 16, bias_tile);
      } else if (NORM && tb && !bias_tile)  // the bias column's B is ones: never scaled
        acc = ring_run<0, 2, RGD>(ra, rb, rsrc(a0p), va, rsrc(sb.p), vb, nrun, acc, 1.f, nullptr, tb, bias_tile);
      else
        acc = ring_run<0, 0, RGD>(ra, rb, rsrc(a0p), va, rsrc(sb.p), vb, nrun, acc, 1.f, nullptr, nullptr, bias_tile);
    }
  }
  trace_mark(tr, 2);
  if (ksl && !rbm) {  // split-K: partials of splits 1.. through LDS, summed by split 0 in fixed order
    if (!lead) *(f32x4*)(part + (wave * 64 + lane) * 4) = acc;
    __syncthreads();
    if (lead) {
      for (int q = 1; q < (1 << ksl); ++q) acc += *(const f32x4*)(part + ((wave + q) * 64 + lane) * 4);
    }
  }
  FINE_MARK(9);

  // ---- epilogue
  if constexpr (EPI == EPI_STORE || EPI == EPI_QDOT) {
    auto epi_store = [&](const f32x4 acc, const int i0, const int ib, const float4 ds, float* red) {
      float rowabs[4] = {0.f, 0.f, 0.f, 0.f};
      if (jok) {
        float y[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) y[q] = acc[q] + pre_b;
        if constexpr (MODE == GEMM_FWD) {
          if (g.pre.t) mat_st4(g.pre, ib, j, make_float4(y[0], y[1], y[2], y[3]));
#pragma unroll
          for (int q = 0; q < 4; ++q) y[q] = act_f<ACT>(y[q]);
          if constexpr (ACT == ACT_TANH) {
            if (g.noise.t && ib >= g.noise_row0) {  // target policy smoothing (td7.py:188-194)
              const float4 e = mat_ld4(g.noise, ib - g.noise_row0, j);
              const float ev[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const float nz = fminf(fmaxf(ev[q] * g.noise_sigma, -g.noise_clip), g.noise_clip);
                y[q] = fminf(fmaxf(y[q] + nz, -1.f), 1.f);
              }
            }
          }
        } else {  // DX: derivative mask
          const float dv[4] = {ds.x, ds.y, ds.z, ds.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) y[q] *= act_b<ACT>(dv[q]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) rowabs[q] = EPI == EPI_QDOT ? y[q] * qwj : fabsf(y[q]);
        mat_st4(g.out, ib, j, make_float4(y[0], y[1], y[2], y[3]));
      }
      if constexpr (MODE == GEMM_FWD) {
        if (EPI == EPI_QDOT || g.norm_out) {  // |y| (EPI_QDOT: y w) summed over the tile's tn columns, per row
#pragma unroll
          for (int q = 0; q < 4; ++q) rowabs[q] = row16_sum(rowabs[q]);
          if ((lane & 15) == 0) *(float4*)(red + wave * 16 + ((lane >> 4) << 2)) =
              make_float4(rowabs[0], rowabs[1], rowabs[2], rowabs[3]);
          __syncthreads();
          if (tid < 16)
            GW(g.norm_out)[(size_t)jt * g.norm_ld + i0 + tid] =
                (red[tid] + red[16 + tid]) + (red[32 + tid] + red[48 + tid]);
        }
      }
    };
    epi_store(acc, i0, ib, ds, red);
  } else if constexpr (EPI == EPI_SACFWD) {  // op_sac_actor for the tile's 16 rows (sac.py:132-152)
    const CAS SacFwdArgs& s = g.sf;
    float* rt = smem;                // [16][64] the tile's raw rows
    float* lpt = smem + 1024;        // [16][32] log-density terms
    float* crt = lpt + 512;          // [16][32] tanh corrections
    __syncthreads();  // (the reduction scratch is free)
    if (wave == 0) {  // (sacraw_finish: every column block's sums in wave 0)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const f32x4 a4 = c == 0 ? acc : (c == 1 ? sac1 : sac2);
        const int jc = c * 16 + (lane & 15);
        const float bc = jc < gN && biasp ? G(biasp)[jc] : 0.f;
        float y[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) y[q] = a4[q] + bc;
        if (jc < gN) mat_st4(g.out, ib, jc, make_float4(y[0], y[1], y[2], y[3]));  // raw (the backward reads it)
#pragma unroll
        for (int q = 0; q < 4; ++q) rt[(ib - i0 + q) * 64 + jc] = jc < gN ? y[q] : 0.f;
      }
    }
    __syncthreads();
    const float c = (float)0.9189385332046727;  // log(sqrt(2*pi))
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int it = tid + k * kThreads, r = it / s.A, jj = it - r * s.A, b = i0 + r;
      if (it >= 16 * s.A || b >= g.M) continue;
      const float mu = rt[r * 64 + s.mean_off + jj];
      const float ls = fminf(fmaxf(rt[r * 64 + s.ls_off + jj], s.min_log_std), s.max_log_std);
      const float sd = expf(ls);
      const float ej = sfe[k];
      const float u = mu + ej * sd;
      const float a = tanhf(u);
      const float var = sd * sd;
      const float d = u - mu;
      lpt[r * 32 + jj] = -(d * d) / (2.f * var) - logf(sd) - c;
      crt[r * 32 + jj] = logf((1.f - a * a) + 1e-6f);
      mat_st(s.act, b, jj, a);
    }
    __syncthreads();
    if (tid < 16 && i0 + tid < g.M) {  // the row sums in op_sac_actor's order
      float lp = 0.f, corr = 0.f;
      for (int jj = 0; jj < s.A; ++jj) {
        lp += lpt[tid * 32 + jj];
        corr += crt[tid * 32 + jj];
      }
      GW(s.logpi)[i0 + tid] = lp - corr;
    }
  } else if constexpr (EPI == EPI_SACBWD) {  // sac.py:227-229 through rsample, tanh and log pi (op_sac_actor_bwd)
    if (jok) {
      const CAS SacBwdArgs& s = g.sb;
      const float w = (s.alpha_lin ? sload(s.log_alpha) : expf(sload(s.log_alpha))) * s.inv_b;  // d obj / d logpi_b
      const float4 mu4 = mat_ld4(s.raw, ib, s.mean_off + j), ls4 = mat_ld4(s.raw, ib, s.ls_off + j),
                   e4 = mat_ld4(s.eps2, ib, j);
      const float muv[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, lsv[4] = {ls4.x, ls4.y, ls4.z, ls4.w},
                  ev[4] = {e4.x, e4.y, e4.z, e4.w};
      float gm[4], gl[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float mu = muv[q], lsr = lsv[q], ej = ev[q];
        const float ls = fminf(fmaxf(lsr, s.min_log_std), s.max_log_std);
        const float sd = expf(ls);
        const float u = mu + ej * sd;
        const float a = tanhf(u);
        const float var = sd * sd;
        const float d = u - mu;
        const float ga = acc[q] + (w / ((1.f - a * a) + 1e-6f)) * (2.f * a);
        float gu = ga * (1.f - a * a);
        gu += -(w / (2.f * var)) * (2.f * d);
        float gmu = (w / (2.f * var)) * (2.f * d);
        const float gvar = (w * (d * d)) / ((2.f * var) * (2.f * var)) * 2.f;
        float gsd = gvar * (2.f * sd) - w / sd;
        gmu += gu;
        gsd += gu * ej;
        float gls = gsd * sd;
        if (!(lsr >= s.min_log_std && lsr <= s.max_log_std)) gls = 0.f;
        const bool rv = ib + q < s.nvalid;  // (rows of the padded batch past it: no gradient)
        gm[q] = rv ? gmu : 0.f;
        gl[q] = rv ? gls : 0.f;
      }
      mat_st4(s.dout, ib, s.mean_off + j, make_float4(gm[0], gm[1], gm[2], gm[3]));
      mat_st4(s.dout, ib, s.ls_off + j, make_float4(gl[0], gl[1], gl[2], gl[3]));
    }
  } else if constexpr (EPI == EPI_QHEAD) {  // td7.py:268-275: Q = w3 . act(z) + b3, L = -mean(cat Q)
    float ls = 0.f;
    if (jok) {
      float dz[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float z = acc[q] + pre_b, y = act_f<ACT>(z);
        const bool rv = ib + q < g.mvalid;  // (rows of the padded batch past it add nothing)
        ls += rv ? y * qwj : 0.f;
        dz[q] = rv ? (g.qscale * qwj) * act_b<ACT>(ACT == ACT_RELU ? y : z) : 0.f;
      }
      mat_st4(g.out, ib, j, make_float4(dz[0], dz[1], dz[2], dz[3]));
    }
    ls = wg_sum(ls, red);
    // (partials by tile, not by workgroup: the sum's order does not follow the XCD tile order)
    const int tix = it * tiles_n + jt;
    if (tid == 0) GW(g.loss_part)[tix] = tix == 0 ? ls + (float)g.mvalid * sload(g.qb) : ls;
  } else if constexpr (EPI == EPI_NBDOT) {  // sale.py:11-13 backward, first half (the rest: kDwNb)
    auto epi_nbdot = [&](const f32x4 acc, const int i0, const int ib, const float4 nbxv, float* red) {
      float rd[4] = {0.f, 0.f, 0.f, 0.f};
      if (jok) {
        const float xq[4] = {nbxv.x, nbxv.y, nbxv.z, nbxv.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) rd[q] = acc[q] * xq[q];
        mat_st4(g.out, ib, j, make_float4(acc[0], acc[1], acc[2], acc[3]));
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) rd[q] = row16_sum(rd[q]);
      if ((lane & 15) == 0) *(float4*)(red + wave * 16 + ((lane >> 4) << 2)) = make_float4(rd[0], rd[1], rd[2], rd[3]);
      __syncthreads();
      if (tid < 16)
        GW(g.norm_out)[(size_t)jt * g.norm_ld + i0 + tid] = (red[tid] + red[16 + tid]) + (red[32 + tid] + red[48 + tid]);
    };
    epi_nbdot(acc, i0, ib, nbxv, red);
  } else if constexpr (EPI == EPI_ACT) {  // td7.py:141-156 / td3.py:114-129: env action of the act graph
    if (jok) {
      const CAS ActArgs& ao = g.ao;
      const int mode = G(ao.ctl)[0];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = ib + q;
        if (row >= ao.n) continue;
        float a = act_f<ACT>(acc[q] + pre_b);
        if (mode) {  // action += randn * exploration_noise; clip(-1, 1)
          const float nz = __fmul_rn(act_eps(ao, mode, row * ao.A + j), sload(ao.sigma));
          a = fminf(fmaxf(__fadd_rn(a, nz), -1.f), 1.f);
        } else {
          a = fminf(fmaxf(a, -1.f), 1.f);
        }
        act_store(ao, row, j, a);
      }
    }
  } else if constexpr (EPI == EPI_MSE) {  // td7.py:256 encoder loss, grad wrt zsa
    float d2 = 0.f;
    const CAS NormRef& nr = g.tgt_norm;
    const bool tab = nr.part && nr.nparts <= 16;  // row norms from the prefetched partials
    if (tab) {
      tabs[tid] = tnv;
      __syncthreads();
    }
    if (jok) {
      const float tq[4] = {tgv.x, tgv.y, tgv.z, tgv.w};
      float gr[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float inv;
        if (tab) {  // the sum order, clamp and reciprocal of norm_inv
          float sm = 0.f;
          for (int p = 0; p < nr.nparts; ++p) sm += tabs[p * 16 + (ib - i0) + q];
          const float m = sm / (float)nr.width;
          inv = 1.f / (m < 1e-8f ? 1e-8f : m);
        } else {
          inv = norm_inv(nr, ib + q);
        }
        const float d = ib + q < g.mvalid ? (acc[q] + pre_b) - tq[q] * inv : 0.f;  // (padded rows: 0)
        gr[q] = (2.f * d) * g.mse_scale;  // mse_scale = 1/n
        d2 += d * d;
      }
      mat_st4(g.out, ib, j, make_float4(gr[0], gr[1], gr[2], gr[3]));
    }
    d2 = wg_sum(d2, red);
    if (tid == 0) GW(g.loss_part)[it * tiles_n + jt] = d2;  // (by tile: see EPI_QHEAD)
  } else {  // EPI_ADAM (torch.optim.Adam single-tensor law, see oracle/agents.py)
    const CAS AdamArgs& ad = g.adam;
    float gg = 0.f;
    if (jok) {
      const float step_size = sload(ad.step), bc2s = sload(ad.bc2s);  // this step's (level-0 CTRL op)
      const float p4[4] = {pp.x, pp.y, pp.z, pp.w}, m4[4] = {mm.x, mm.y, mm.z, mm.w}, v4[4] = {vv.x, vv.y, vv.z, vv.w};
      float po[4], mo[4], vo[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float gv = acc[q];
        const float m = m4[q] + ad.omb1 * (gv - m4[q]);
        const float v2 = v4[q] * ad.beta2 + (ad.omb2 * gv) * gv;
        const float denom = sqrtf(v2) / bc2s + ad.eps;
        const bool ok = ib + q < g.M;  // weight rows past out stay untouched (zero)
        po[q] = ok ? p4[q] + (-step_size * m) / denom : p4[q];
        mo[q] = ok ? m : m4[q];
        vo[q] = ok ? v2 : v4[q];
        gg += ok ? gv * gv : 0.f;
      }
      if (ad.ptau != 0.f) {  // TD3 policy step: the Polyak of the aliased target policy (op_polyak's law)
        const float omt = 1.f - ad.ptau;
#pragma unroll
        for (int q = 0; q < 4; ++q) po[q] = __fadd_rn(__fmul_rn(ad.ptau, po[q]), __fmul_rn(po[q], omt));
      }
      GAS float* pw = bias_tile ? GW(ad.b) + ib : GW(ad.w.t) + wt;
      // The weights' T image (+ bias) and the Adam moments: read again only a step later (the moments by this
      // tile's next Adam, the T image by the next step's input-gradient GEMMs), so write-through stores (round 6;
      // they were nontemporal stores, +0.45% / +0.3% over plain in round 3): the bytes leave the XCD's L2 during
      // the kernel instead of waiting dirty for the launch's release.  A/B against the nontemporal stores: TD7
      // Humanoid B = 256 8,341 / 8,338 steps/s (3 pairs), B = 1024 3,809 / 3,789 (2 pairs)
      {
        f32x4 w;
        w.x = po[0]; w.y = po[1]; w.z = po[2]; w.w = po[3];
        st4wt(pw, w);
        w.x = mo[0]; w.y = mo[1]; w.z = mo[2]; w.w = mo[3];
        st4wt(pw + ad.mo, w);
        w.x = vo[0]; w.y = vo[1]; w.z = vo[2]; w.w = vo[3];
        st4wt(pw + ad.vo, w);
      }
      if (!bias_tile) {
        GAS float* qn = GW(ad.w.n) + nidx(ad.w.cbn, ib, j);
        qn[0] = po[0];
        qn[4] = po[1];
        qn[8] = po[2];
        qn[12] = po[3];
      }
    }
    if (ad.gsq) {
      gg = wg_sum(gg, red);
      if (tid == 0) {
        if (bias_tile) GW(ad.gsq_b)[it] = gg;
        else GW(ad.gsq)[it * (tiles_n - 1) + jt] = gg;
      }
    }
  }
}

template <int KS>
__device__ __forceinline__ void op_gemm(const CAS GemmArgs& g, int vid, int t, float* smem, unsigned long long* tr) {
  // (ops.h RLE_GEMM_VARIANTS, those of kernel set KS; the host refuses any other id.  PK 4 / 5 take an id
  // with the norm bit their consumers never set, so their NORM is false)
#define RLE_VX(mode, epi, act, norm, pre, pk, sets)                                                       \
  case gemm_vid(mode, epi, act, norm, pre):                                                               \
    if constexpr (KS == KS_EXT || (((sets) >> ks_family(KS)) & 1)) {                                     \
      asm volatile("; gemm variant " #mode " " #epi " " #act " norm " #norm " pk " #pk ::);               \
      gemm_v<mode, epi, act, (norm) != 0 && (pk) <= 3, pk, KS == KS_EXT || KS == KS_TD7W,                 \
             (KS == KS_TD7W || KS == KS_EXT) && wide_variant(mode, epi, pk)>(g, t, smem, tr);             \
    }                                                                                                     \
    break;
  switch (vid) {
    RLE_GEMM_VARIANTS(RLE_VX)
    default: break;
  }
#undef RLE_VX
}

// ---------------------------------------------------------------- AvgL1Norm backward

// One row per wave (4 per workgroup): lane l holds columns 4l..4l+3 (+256 per
// pass) as float4s of the N images; the row dot product is one wave reduction.
__device__ __forceinline__ void op_normbwd(const CAS NormBwdArgs& a, int t) {
  if (a.fwd == 2) {  // finalize (NormBwdArgs::mout): the mean of each row's partials, one thread per row
    const int row = t * kThreads + (int)threadIdx.x;
    if (row < a.rows) GW(a.mout)[row] = norm_mean_i(a.norm.part, a.norm.ld, row + a.norm.row0, a.norm.nparts, a.width);
    return;
  }
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row = t * 4 + wave;
  if (row >= a.rows) return;
  const float mean = norm_mean(a.norm.part, a.norm.ld, row + a.norm.row0, a.norm.nparts, a.width);
  const bool clamped = mean < 1e-8f;  // m recomputed exactly as the forward consumers did (norm_m)
  const float inv = 1.f / (clamped ? 1e-8f : mean);
  const int c0 = 4 * lane, c1 = c0 + 256;
  const bool in0 = c0 < a.width, in1 = c1 < a.width;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 x0 = mat_ldr4(a.x, row, in0 ? c0 : 0), g0 = mat_ldr4(a.g, row, in0 ? c0 : 0);
  const float4 x1 = in1 ? mat_ldr4(a.x, row, c1) : z, g1 = in1 ? mat_ldr4(a.g, row, c1) : z;
  float dot = in0 ? (g0.x * x0.x + g0.y * x0.y) + (g0.z * x0.z + g0.w * x0.w) : 0.f;
  if (in1) dot += (g1.x * x1.x + g1.y * x1.y) + (g1.z * x1.z + g1.w * x1.w);
  dot = wave_sum(dot);
  // y = x / m: dy/dx path g/m ; dm path -(sum g x)/m^2 * sign(x)/n (unless clamped)
  const float gm = (clamped || a.fwd) ? 0.f : (-dot * inv * inv) / (float)a.width;
  auto sgn = [](float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); };
  auto f = [&](float4 gv, float4 xv) {
    return make_float4(gv.x * inv + sgn(xv.x) * gm, gv.y * inv + sgn(xv.y) * gm, gv.z * inv + sgn(xv.z) * gm,
                       gv.w * inv + sgn(xv.w) * gm);
  };
  if (in0) mat_str4(a.dx, row, c0, f(g0, x0));
  if (in1) mat_str4(a.dx, row, c1, f(g1, x1));
}

// ---------------------------------------------------------------- critic heads


// Last critic layer (H -> 1) as a dot product fused with the TD target / loss /
// priority / policy objective and the gradient into the last hidden layer.  One
// row per wave (4 per workgroup): lane l holds columns 4l..4l+3 (+256 per pass)
// as float4s of the N images, so every operand of the row -- both twins' hidden
// layer, weights and derivative source -- is loaded in one round trip.
template <int DACT>
__device__ __forceinline__ void op_head_t(const CAS HeadArgs& h, int t, float* smem, unsigned long long* tr) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = t * 4 + wave;  // wave-uniform: per-row scalars come through s_load
  float acc0 = 0.f, acc1 = 0.f;  // this row's loss terms
  int kmax = (int)0x80000000, kmin = 0x7FFFFFFF;
  if (b < h.rows) {
    const int c0 = 4 * lane, c1 = c0 + 256;
    const bool in0 = c0 < h.H, in1 = c1 < h.H;
    const int k0 = in0 ? c0 : 0, k1 = in1 ? c1 : 0;
    const bool dz = h.mode != HEAD_TD7_TARGET && h.mode != HEAD_MLP_TARGET;
    const bool fused = h.tgt_mode >= 0;  // target twins in this op too (wave-uniform)
    const bool qpart = h.qp[0] != nullptr, tpart = fused && h.tp[0] != nullptr;  // EPI_QDOT partials
    float4 hv[2][2], wv[2][2], dv[2][2], tv[2][2], twv[2][2];
    float qpv[2] = {0.f, 0.f}, tpv[2] = {0.f, 0.f};
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      if (qpart) {
        if (lane < h.qp_n[n]) qpv[n] = G(h.qp[n])[(size_t)lane * h.qp_ld + b];
      } else {
        hv[n][0] = mat_ldr4(h.h[n], b, k0);
        hv[n][1] = mat_ldr4(h.h[n], b, k1);
      }
      wv[n][0] = ld4g(G(h.w[n]) + nidx(h.w_cbn, 0, k0));
      wv[n][1] = ld4g(G(h.w[n]) + nidx(h.w_cbn, 0, k1));
      if (dz) {
        dv[n][0] = mat_ldr4(h.dsrc[n], b, k0);
        dv[n][1] = mat_ldr4(h.dsrc[n], b, k1);
      }
      if (tpart) {
        if (lane < h.tp_n[n]) tpv[n] = G(h.tp[n])[(size_t)lane * h.tp_ld + b];
      } else if (fused) {
        tv[n][0] = mat_ldr4(h.th[n], b, k0);
        tv[n][1] = mat_ldr4(h.th[n], b, k1);
        twv[n][0] = ld4g(G(h.tw[n]) + nidx(h.w_cbn, 0, k0));
        twv[n][1] = ld4g(G(h.tw[n]) + nidx(h.w_cbn, 0, k1));
      }
    }
    FINE_MARK(0);
    const float rw = h.reward ? sload(h.reward + b) : 0.f, ndn = h.notdone ? sload(h.notdone + b) : 0.f;
    float yv = ((h.mode == HEAD_TD7_LOSS || h.mode == HEAD_MLP_LOSS) && !fused) ? sload(h.y + b) : 0.f;
    const float lp = h.sac ? sload(h.logpi + b) : 0.f;
    const float alpha = h.sac ? (h.alpha_lin ? sload(h.log_alpha) : expf(sload(h.log_alpha))) : 0.f;
    const float bias0 = sload(h.b[0]), bias1 = sload(h.b[1]);
    const float vtmax = h.vt ? sload(h.vt) : 0.f, vtmin = h.vt ? sload(h.vt + 1) : 0.f;
    auto dot2 = [&](const float4 (&x)[2], const float4 (&w)[2]) {
      float s = 0.f;
      if (in0) s += (x[0].x * w[0].x + x[0].y * w[0].y) + (x[0].z * w[0].z + x[0].w * w[0].w);
      if (in1) s += (x[1].x * w[1].x + x[1].y * w[1].y) + (x[1].z * w[1].z + x[1].w * w[1].w);
      return wave_sum(s);
    };
    float q[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) q[n] = (qpart ? wave_sum(qpv[n]) : dot2(hv[n], wv[n])) + (n ? bias1 : bias0);
    FINE_MARK(1);
    if (fused) {  // the TD target of this row (as HEAD_TD7_TARGET / HEAD_MLP_TARGET below)
      const float qt0 = (tpart ? wave_sum(tpv[0]) : dot2(tv[0], twv[0])) + sload(h.tb[0]);
      const float qt1 = (tpart ? wave_sum(tpv[1]) : dot2(tv[1], twv[1])) + sload(h.tb[1]);
      float v = fminf(qt0, qt1);
      if (h.tgt_mode == HEAD_TD7_TARGET) v = fminf(fmaxf(v, vtmin), vtmax);
      else if (h.sac) v = v - alpha * lp;
      yv = rw + (h.gamma * v) * ndn;
      if (h.y && lane == 0) GW(h.y)[b] = yv;
      if (h.tgt_mode == HEAD_TD7_TARGET) kmax = kmin = fkey(yv);
    }
    trace_mark(tr, 1);
    float dq[2] = {0.f, 0.f};
    switch (h.mode) {
      case HEAD_TD7_TARGET: {  // td7.py:211-218
        float v = fminf(q[0], q[1]);
        v = fminf(fmaxf(v, vtmin), vtmax);
        const float y = rw + (h.gamma * v) * ndn;
        if (lane == 0) GW(h.y)[b] = y;
        kmax = kmin = fkey(y);
        break;
      }
      case HEAD_MLP_TARGET: {  // td3.py:160-164, sac.py:188-193
        float v = fminf(q[0], q[1]);
        if (h.sac) v = v - alpha * lp;
        const float y = rw + (h.gamma * v) * ndn;
        if (lane == 0) GW(h.y)[b] = y;
        break;
      }
      case HEAD_TD7_LOSS:
      case HEAD_MLP_LOSS: {  // td7.py:231-244, td3.py:169-182
        float dmax = 0.f;
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const float diff = q[n] - yv;
          if (h.lap) {
            const float d = fabsf(diff);
            const float hub = d < 1.f ? 0.5f * (d * d) : d;
            if (n == 0) acc0 = hub; else acc1 = hub;
            const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
            dq[n] = (d < 1.f ? d : 1.f) * sg * h.inv_b;
            dmax = fmaxf(dmax, d);
          } else {
            const float e = yv - q[n];
            if (n == 0) acc0 = e * e; else acc1 = e * e;
            dq[n] = -e * h.inv_b;
          }
        }
        FINE_MARK(2);
        if (h.lap && lane == 0) GW(h.prio)[b] = lap_priority(dmax);
        FINE_MARK(3);
        break;
      }
      case HEAD_TD7_POLICY:  // td7.py:274-275
        acc0 = q[0] + q[1];
        dq[0] = dq[1] = -0.5f * h.inv_b;
        break;
      default: {  // HEAD_MLP_POLICY: td3.py:191, sac.py:227-229
        const float mn = fminf(q[0], q[1]);
        // torch.minimum backward: ties split the gradient
        const float gq = -h.inv_b;
        dq[0] = q[0] < q[1] ? gq : (q[0] == q[1] ? 0.5f * gq : 0.f);
        dq[1] = q[1] < q[0] ? gq : (q[0] == q[1] ? 0.5f * gq : 0.f);
        if (h.sac) {
          acc0 = -mn + lp * alpha;
          acc1 = lp;
        } else {
          acc0 = mn;
        }
      }
    }
    trace_mark(tr, 2);
    if (dz) {  // dz = dq * w * act'(dsrc); dq stored for the last layer's dW
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        if (lane == 0 && h.dq[n].t) GW(h.dq[n].t)[tidx(h.dq[n].rbs, b, 0)] = dq[n];
        auto g4 = [&](float4 w, float4 d) {
          return make_float4((dq[n] * w.x) * act_b<DACT>(d.x), (dq[n] * w.y) * act_b<DACT>(d.y),
                             (dq[n] * w.z) * act_b<DACT>(d.z), (dq[n] * w.w) * act_b<DACT>(d.w));
        };
        if (in0) mat_str4(h.dz[n], b, c0, g4(wv[n][0], dv[n][0]));
        if (in1) mat_str4(h.dz[n], b, c1, g4(wv[n][1], dv[n][1]));
      }
    }
    FINE_MARK(4);
  }
  // workgroup partials (fixed order) + value tracking
  float* red = smem;
  int* ired = reinterpret_cast<int*>(smem + 16);
  if (lane == 0) {
    red[wave * 2 + 0] = acc0;
    red[wave * 2 + 1] = acc1;
    ired[wave * 2 + 0] = kmax;
    ired[wave * 2 + 1] = kmin;
  }
  __syncthreads();
  FINE_MARK(5);
  if (threadIdx.x == 0) {
    if (h.loss_part) {
      GAS float* lp = GW(h.loss_part);
      lp[t * 4 + 0] = (red[0] + red[2]) + (red[4] + red[6]);
      lp[t * 4 + 1] = (red[1] + red[3]) + (red[5] + red[7]);
      lp[t * 4 + 2] = 0.f;
      lp[t * 4 + 3] = 0.f;
    }
    if (h.mode == HEAD_TD7_TARGET || h.tgt_mode == HEAD_TD7_TARGET) {  // value_max / value_min (td7.py:217-218)
      int mx = ired[0], mn = ired[1];
      for (int w = 1; w < 4; ++w) {
        mx = max(mx, ired[2 * w]);
        mn = min(mn, ired[2 * w + 1]);
      }
      atomicMax(h.vmax_key, mx);
      atomicMin(h.vmin_key, mn);
    }
  }
}

__device__ __forceinline__ void op_head(const CAS HeadArgs& h, int t, float* smem, unsigned long long* tr) {
  if (h.dact == ACT_ELU) op_head_t<ACT_ELU>(h, t, smem, tr);
  else if (h.dact == ACT_RELU) op_head_t<ACT_RELU>(h, t, smem, tr);
  else op_head_t<ACT_NONE>(h, t, smem, tr);
}

// ---------------------------------------------------------------- replay sampling

constexpr int kBlk = 4096;  // priorities per block-sum

// Exact fp64 block sums of the priorities (lap.py:47; Q8: any-order fp64 is exact), and the
// 64-priority sub-block sums of the same block.  Thread tid sums 16 consecutive priorities (rows
// past the replay size count as 0); 4 threads make a sub-block.
constexpr int kSub = 64;  // priorities per sub-block sum
__device__ __forceinline__ void op_sample_reduce(const CAS SampleArgs& s, int t, float* smem) {
  const long long size = sload(s.size);
  const long long e0 = (long long)t * kBlk + (long long)threadIdx.x * 16;
  double acc = 0.0;
#pragma unroll
  for (int q = 0; q < 16; ++q)
    if (e0 + q < size) acc += (double)G(s.priority)[e0 + q];
  double sub = acc + dpp_d<0xb1>(acc);  // quad_perm [1,0,3,2]
  sub += dpp_d<0x4e>(sub);              // quad_perm [2,3,0,1]: the quad's 64 priorities
  if ((threadIdx.x & 3) == 0 && s.ssum) GW(s.ssum)[(size_t)t * (kBlk / kSub) + (threadIdx.x >> 2)] = sub;
  acc = wave_sum_d(acc);
  double* dred = reinterpret_cast<double*>(smem);
  if ((threadIdx.x & 63) == 0) dred[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) GW(s.bsum)[t] = (dred[0] + dred[1]) + (dred[2] + dred[3]);
}

// Inclusive scan of a double over the 64 lanes (DPP: row shifts, then row broadcasts).
__device__ __forceinline__ double wave_scan_incl_d(double v) {
  v += dpp_d<0x111>(v);  // row_shr:1
  v += dpp_d<0x112>(v);  // row_shr:2
  v += dpp_d<0x114>(v);  // row_shr:4
  v += dpp_d<0x118>(v);  // row_shr:8
  v += dpp_d<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_d<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
  return v;
}
// Exclusive scan of one double per thread over the workgroup (fixed order; the
// priority sums are exact in fp64, so the order does not change a value, Q8).
__device__ __forceinline__ double wg_scan_excl_d(double v, double* wtot, double& total) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const double inc = wave_scan_incl_d(v);
  if (lane == 63) wtot[wave] = inc;
  __syncthreads();
  const double w0 = wtot[0], w1 = wtot[1], w2 = wtot[2], w3 = wtot[3];
  const double before = (wave > 0 ? w0 : 0.0) + (wave > 1 ? w1 : 0.0) + (wave > 2 ? w2 : 0.0);
  total = ((w0 + w1) + w2) + w3;
  return before + (inc - v);
}

// Noise of the batch (its own op so that the sampler's search does not wait on it):
// element e = (b, j) of the [B][A] target-smoothing noise (td7.py:188, td3.py:154) or
// SAC next-state rsample noise, and the SAC policy rsample noise in eps2.
__device__ __forceinline__ void op_noise(const CAS SampleArgs& s, int t) {
  const int e = t * kThreads + threadIdx.x;
  if (e >= s.nq * s.A) return;  // (rows of the padded batch past nq keep zero noise)
  const int b = e / s.A, j = e - b * s.A;
  const int tape = sload(s.tape_mode);
  const long long pos = sload(s.tape_pos) + s.ahead;
  const unsigned long long step = (unsigned long long)sload(s.ctrl_rng) + s.ahead;
  float v, v2 = 0.f;
  if (tape & kTapeEps) {
    v = G(s.tape_eps)[(size_t)pos * s.nq * s.A + e];
    if (s.eps2.t) v2 = G(s.tape_eps2)[(size_t)pos * s.nq * s.A + e];
  } else {
    const uint2 key = make_uint2((unsigned)s.seed, (unsigned)(s.seed >> 32));
    const uint4 r = philox(key, make_uint4((unsigned)e, 1u, (unsigned)step, (unsigned)(step >> 32)));
    v = normal_from(r.x, r.y);
    v2 = normal_from(r.z, r.w);
  }
  mat_st(s.eps, b, j, v);
  if (s.eps2.t) mat_st(s.eps2, b, j, v2);
}

// One WAVE per query (4 per workgroup): uniform / LAP index search (searchsorted left over the
// fp32-rounded exact prefix), then the coalesced row gather.  The LAP search descends three
// levels of exact fp64 sums: the 4096-priority block sums (each lane owns a run of blocks), the
// 64 sub-block sums of the chosen block (one per lane), the 64 priorities of the chosen sub-block
// (one per lane) -- about 0.8 KB read per query instead of a whole 16 KB block.  At each level the
// answer lies in the first unit whose rounded inclusive prefix is >= v: prefixes are monotone, so
// an element qualifying in an earlier unit would make that unit qualify (the last unit if none).
__device__ __forceinline__ int first_lane(bool p) {
  const unsigned long long bal = __ballot(p);
  return bal ? __builtin_ffsll((long long)bal) - 1 : -1;
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}
// The previous step's priority update applied in LDS by every sampler workgroup (SampleArgs::pend_n;
// its OP_PRIORITY persists it one level later, off the chain): duplicates resolved as op_priority
// (LDS hash, last writer wins), each winner's fp64 delta added to its 4096-block's delta (exact in
// any order, as the block sums are: SURVEY Q8) and pushed on its block's list, so a query patches the
// block sums it scans, the sub-block sums of its block and the priorities of its sub-block with the
// values the search would read after the update.  LDS (bytes): [0, r0) the hash (2 ns ints), then
// the winner records by batch row (key, next, new value, delta); at r0 the block deltas, then the
// block list heads (engine.cpp prio_sample_fused checks the sizes).
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its global
// loads in flight (__syncthreads' workgroup fences would wait for those too).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
struct PendTab {
  const int* wkey; const int* wnext; const float* wnew; const double* wdel; const double* bdel; const int* bhead;
};
__device__ __forceinline__ PendTab pend_prepare(const CAS SampleArgs& s, float* smem) {
  const int tid = threadIdx.x, n = s.pend_n;
  int ns = 64;
  while (ns < 2 * n) ns <<= 1;  // hash slots: load factor <= 1/2
  const int r0 = max(8 * ns, 20 * n);
  char* L = (char*)smem;
  int* keys = (int*)L;
  int* last = keys + ns;
  int* wkey = (int*)L;  // (records: after the hash is dead)
  int* wnext = wkey + n;
  float* wnew = (float*)(wnext + n);
  double* wdel = (double*)(L + 12 * n);  // (12 n: 8-aligned, n a multiple of 16)
  const int nbc = (int)((s.cap + kBlk - 1) / kBlk);
  double* bdel = (double*)(L + r0);
  int* bhead = (int*)(bdel + nbc);
  int key[4];
  float pn[4], po[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {  // (B <= 1024: at most 4 updates per thread)
    const int b = tid + u * kThreads;
    key[u] = b < n ? (int)G(s.pend_ind)[b] : 0;
    pn[u] = b < n ? G(s.pend_p)[b] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) po[u] = tid + u * kThreads < n ? G(s.priority)[key[u]] : 0.f;  // (every update's)
  for (int i = tid; i < ns; i += kThreads) {
    keys[i] = -1;
    last[i] = -1;
  }
  for (int i = tid; i < nbc; i += kThreads) {
    bdel[i] = 0.0;
    bhead[i] = -1;
  }
  lds_barrier();
  int slot[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int b = tid + u * kThreads;
    slot[u] = 0;
    if (b >= n) continue;
    int h = (int)(((unsigned)key[u] * 2654435761u) >> 21) & (ns - 1);
    while (true) {
      const int old = atomicCAS(&keys[h], -1, key[u]);
      if (old == -1 || old == key[u]) break;
      h = (h + 1) & (ns - 1);
    }
    atomicMax(&last[h], b);
    slot[u] = h;
  }
  lds_barrier();
  bool win[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) win[u] = tid + u * kThreads < n && last[slot[u]] == tid + u * kThreads;
  lds_barrier();  // (the hash is dead)
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (win[u]) {
      const int b = tid + u * kThreads, blk = key[u] / kBlk;
      const double d = (double)pn[u] - (double)po[u];
      atomicAdd(&bdel[blk], d);
      wkey[b] = key[u];
      wnew[b] = pn[u];
      wdel[b] = d;
      wnext[b] = atomicExch(&bhead[blk], b);  // (list order: any -- every use below is exact in any order)
    }
  lds_barrier();
  return PendTab{wkey, wnext, wnew, wdel, bdel, bhead};
}

template <bool EXT>  // (EXT: the fused priority update, SampleArgs::pend_n)
__device__ __forceinline__ void op_sample_gather(const CAS SampleArgs& s, int t, float* smem, unsigned long long* tr) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = t * 4 + wave;  // query (wave-uniform)
  const int tape = sload(s.tape_mode);
  // (uniform over the workgroup: every wave takes part in the fused update's LDS phases)
  const bool pend = EXT && s.pend_n > 0 && s.lap && !(tape & kTapeInd);
  if (!pend && b >= s.nq) return;
  const bool live = b < s.nq;  // (wave-uniform; a wave past the batch only helps with the update)
  const long long size = sload(s.size);
  const long long pos = sload(s.tape_pos) + s.ahead;
  const uint2 key = make_uint2((unsigned)s.seed, (unsigned)(s.seed >> 32));
  const unsigned long long step = (unsigned long long)sload(s.ctrl_rng) + s.ahead;
  FINE_MARK(0);
  const bool tind = tape & kTapeInd;
  // LAP block sums: lane l owns blocks [l * per, l * per + per) of the CAPACITY's blocks (per <= 16,
  // capacity <= 4M), loaded with the control values; blocks past the replay size are zeroed below
  const int nb = (int)((size + kBlk - 1) / kBlk);
  const int nbc = (int)((s.cap + kBlk - 1) / kBlk);
  const int per = (nbc + 63) >> 6;
  double bs[16];
  if (s.lap && !tind) {
#pragma unroll
    for (int q = 0; q < 16; ++q) bs[q] = q < per ? G(s.bsum)[min(lane * per + q, nbc - 1)] : 0.0;  // (per: uniform)
  }
  float u = 0.f;
  if (!tind && live) {
    if (tape & kTapeU) u = sload(s.tape_u + (size_t)pos * s.nq + b);
    else u = u01(philox(key, make_uint4((unsigned)b, 0u, (unsigned)step, (unsigned)(step >> 32))).x);
  }
  PendTab pt{};
  if (pend) {  // (after the block-sum loads and u: they stay in flight through its LDS phases)
    pt = pend_prepare(s, smem);
    if (!live) return;
#pragma unroll
    for (int q = 0; q < 16; ++q) bs[q] += q < per ? pt.bdel[min(lane * per + q, nbc - 1)] : 0.0;
  }
  FINE_MARK(1);
  long long ind;
  if (tind) {
    // (host-checked in range; the clamp only guards a prefetch past a tape's end, whose batch
    // the host discards)
    ind = sload(s.tape_ind + (size_t)pos * s.nq + b);
    ind = ind < 0 ? 0 : (ind > size - 1 ? size - 1 : ind);
  } else {
    if (lane == 0) GW(s.u_out)[b] = u;
    if (!s.lap) {
      // searchsorted(cumsum(ones(size)), u*size): first j in 1..size with j >= v
      const float v = u * (float)size;
      const long long k = (long long)ceilf(v) - 1;
      ind = k < 0 ? 0 : (k > size - 1 ? size - 1 : k);
    } else {
      // level 1: the blocks (exact fp64 prefix, rounded to fp32 per unit: Q8)
      double loc = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (q >= per || lane * per + q >= nb) bs[q] = 0.0;
        loc += bs[q];
      }
      double inc = wave_scan_incl_d(loc);
      const double total = readlane_d(inc, 63);
      const float v = u * (float)total;
      double run = inc - loc;
      int mine = -1;
      double mbase = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int k = lane * per + q;
        if (q < per && k < nb && mine < 0) {
          if ((float)(run + bs[q]) >= v || k == nb - 1) {
            mine = k;
            mbase = run;
          }
          run += bs[q];
        }
      }
      const int l1 = first_lane(mine >= 0);  // (nb >= 1: some lane holds the last block)
      const int blk = __builtin_amdgcn_readlane(mine, l1);
      double base = readlane_d(mbase, l1);
      FINE_MARK(2);
      // level 2: the block's 64 sub-blocks, one per lane
      const int nsub = (int)min((long long)(kBlk / kSub), (size - (long long)blk * kBlk + kSub - 1) / kSub);
      double sv = lane < nsub ? G(s.ssum)[(size_t)blk * (kBlk / kSub) + lane] : 0.0;
      const int pj0 = pend ? pt.bhead[blk] : -1;
      for (int j = pj0; j >= 0; j = pt.wnext[j])  // (the update's rows in this block: ~B / blocks of them)
        if (((pt.wkey[j] & (kBlk - 1)) >> 6) == lane) sv += pt.wdel[j];
      inc = wave_scan_incl_d(sv);
      const int l2 = first_lane(lane < nsub && ((float)(base + inc) >= v || lane == nsub - 1));
      const int sub = max(l2, 0);
      base += readlane_d(inc - sv, sub);
      FINE_MARK(3);
      // level 3: the sub-block's 64 priorities, one per lane
      // (a two-tier search -- the chosen block's 4096 priorities in one round trip, the sub-block sums formed
      // from them -- measured slower in round 6: standalone 9.6 against 7.1 us, TD7 Humanoid -1.7%)
      const long long e = (long long)blk * kBlk + (long long)sub * kSub + lane;
      float pv = e < size ? G(s.priority)[e] : 0.f;
      for (int j = pj0; j >= 0; j = pt.wnext[j])
        if (pt.wkey[j] == (int)e) pv = pt.wnew[j];
      inc = wave_scan_incl_d((double)pv);
      const int l3 = first_lane(e < size && (float)(base + inc) >= v);
      ind = l3 < 0 ? size - 1 : (long long)blk * kBlk + (long long)sub * kSub + l3;
      if (ind >= size) ind = size - 1;
    }
  }
  trace_mark(tr, 2);
  // gather the transition into the batch images (rows b and B + b of ss): lane l moves columns
  // 4 l .. 4 l + 3 (+ 256 per pass; rows are 16-float aligned); every load is issued before any
  // store (one memory round trip)
  float4 v0[2], v1[2];
  float4 va = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int c = 4 * lane + 256 * p;
    v0[p] = v1[p] = va;
    if (c < s.Sp) {
      v0[p] = ld4g(G(s.state) + (size_t)ind * s.Sp + c);
      v1[p] = ld4g(G(s.next_state) + (size_t)ind * s.Sp + c);
    }
  }
  if (4 * lane < s.Ap) va = ld4g(G(s.action) + (size_t)ind * s.Ap + 4 * lane);
  float rv = 0.f, dv = 0.f;
  if (lane == 0) {
    rv = G(s.reward)[ind];
    dv = G(s.notdone)[ind];
  }
  // (B % 4 == 0, every batch the engine draws: the workgroup's four rows b = 4 t .. 4 t + 3 are one
  // float4 of each T-image column -- mat_ld4's layout -- so they meet in LDS and each thread stores
  // whole float4s, instead of every wave storing its row as four scattered floats per column quad.
  // A/B: TD7 Humanoid +0.4%, SAC Humanoid +0.4%, TD7 B = 1024 +0.8%; rows of <= 64 floats (TD3
  // HalfCheetah) -0.3%: they keep the per-wave stores.)
  const bool quad = (s.nq & 3) == 0 && s.Sp >= 128;  // (uniform; a partial last quad of queries: per-wave stores)
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int c = 4 * lane + 256 * p;
    if (c < s.Sp) {
      if (quad) {
        if (s.ss.n) {
          st4g(GW(s.ss.n) + nidx(s.ss.cbn, b, c), v0[p]);
          st4g(GW(s.ss.n) + nidx(s.ss.cbn, s.B + b, c), v1[p]);
        }
      } else {
        mat_str4(s.ss, b, c, v0[p]);
        mat_str4(s.ss, s.B + b, c, v1[p]);
      }
    }
  }
  if (4 * lane < s.Ap) {
    if (!quad) mat_str4(s.a, b, 4 * lane, va);
    else if (s.a.n) st4g(GW(s.a.n) + nidx(s.a.cbn, b, 4 * lane), va);
  }
  if (lane == 0) {
    GW(s.r)[b] = rv;
    GW(s.nd)[b] = dv;
    GW(s.ind)[b] = ind;
  }
  if (quad && (s.ss.t || s.a.t)) {
    const int RW = 2 * s.Sp + s.Ap;  // (<= 800 floats: four rows in 12.5 KB of LDS)
    float* rows = smem;
    if (pend) __syncthreads();  // (the priority update's LDS tables are dead)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int c = 4 * lane + 256 * p;
      if (c < s.Sp) {
        *(float4*)(rows + wave * RW + c) = v0[p];
        *(float4*)(rows + wave * RW + s.Sp + c) = v1[p];
      }
    }
    if (4 * lane < s.Ap) *(float4*)(rows + wave * RW + 2 * s.Sp + 4 * lane) = va;
    __syncthreads();
    const int r0 = t * 4;
    for (int i = threadIdx.x; i < RW; i += kThreads) {
      const float4 v = make_float4(rows[i], rows[RW + i], rows[2 * RW + i], rows[3 * RW + i]);
      if (i < s.Sp) {
        if (s.ss.t) st4g(GW(s.ss.t) + tidx(s.ss.rbs, r0, i), v);
      } else if (i < 2 * s.Sp) {
        if (s.ss.t) st4g(GW(s.ss.t) + tidx(s.ss.rbs, s.B + r0, i - s.Sp), v);
      } else if (s.a.t) {
        st4g(GW(s.a.t) + tidx(s.a.rbs, r0, i - 2 * s.Sp), v);
      }
    }
  }
  FINE_MARK(6);
}

// LAPReplayMemory.update_priority (lap.py:66-69): last duplicate wins (Q9).
// Duplicates are resolved with an LDS hash table (open addressing, 2048 slots,
// load factor <= 1/2): slot value = largest batch position holding that index.
__device__ __forceinline__ void op_priority(const CAS PriorityArgs& a, float* smem) {
  constexpr int kSlots = 2048;
  int* keys = reinterpret_cast<int*>(smem);
  int* last = keys + kSlots;
  float* red = smem + 2 * kSlots;
  for (int i = threadIdx.x; i < kSlots; i += kThreads) {
    keys[i] = -1;
    last[i] = -1;
  }
  __syncthreads();
  auto slot0 = [](int key) { return (int)(((unsigned)key * 2654435761u) >> 21); };  // 11 bits
  int mine[4], myslot[4];
  const int per = (a.B + kThreads - 1) / kThreads;  // B <= 1024
  for (int u = 0; u < per; ++u) {
    const int b = threadIdx.x + u * kThreads;
    mine[u & 3] = -1;
    if (b >= a.B) continue;
    const int key = (int)G(a.ind)[b];
    int h = slot0(key);
    while (true) {
      const int old = atomicCAS(&keys[h], -1, key);
      if (old == -1 || old == key) break;
      h = (h + 1) & (kSlots - 1);
    }
    atomicMax(&last[h], b);
    mine[u & 3] = key;
    myslot[u & 3] = h;
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int u = 0; u < per; ++u) {
    const int b = threadIdx.x + u * kThreads;
    if (b >= a.B) continue;
    const float pv = G(a.p)[b];
    if (last[myslot[u & 3]] == b) {
      // the block sums follow every priority write exactly: fp64 differences of fp32
      // priorities (>= 1, lap.py) and their sums are exact, so any order gives the sums
      // a full recompute would (op_sample_reduce)
      const int key = mine[u & 3];
      if (a.bsum) {
        const double d = (double)pv - (double)G(a.priority)[key];
        atomicAdd(&a.bsum[key / kBlk], d);
        atomicAdd(&a.ssum[key / kSub], d);
      }
      GW(a.priority)[key] = pv;
    }
    mx = fmaxf(mx, pv);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    GW(a.max_priority)[0] = fmaxf(m, G(a.max_priority)[0]);
  }
}

// ---------------------------------------------------------------- SAC Gaussian-tanh

__device__ __forceinline__ void op_sac_actor(const CAS SacActorArgs& s, int t) {
  const int b = t * kThreads + threadIdx.x;
  if (s.ao.out) {  // act graph (sac.py:132-152): tanh(mean) or tanh(rsample), env map
    const CAS ActArgs& ao = s.ao;
    if (b >= ao.n) return;
    const int mode = G(ao.ctl)[0];
    for (int j = 0; j < ao.A; ++j) {
      const float mu = mat_ld(s.out, b, s.mean_off + j);
      float u = mu;
      if (mode) {
        const float ls = fminf(fmaxf(mat_ld(s.out, b, s.ls_off + j), s.min_log_std), s.max_log_std);
        u = __fadd_rn(mu, __fmul_rn(act_eps(ao, mode, b * ao.A + j), expf(ls)));  // Normal.rsample
      }
      act_store(ao, b, j, tanhf(u));
    }
    return;
  }
  if (b >= s.rows) return;
  const bool pol = b < s.eps_row_split;  // rows < split use eps2 (policy), else eps (target)
  const int eb = pol ? b : b - s.eps_row_split;
  const float c = (float)0.9189385332046727;  // log(sqrt(2*pi))
  float lp = 0.f, corr = 0.f;
  for (int j = 0; j < s.A; ++j) {
    const float mu = mat_ld(s.out, b, s.mean_off + j);
    const float ls = fminf(fmaxf(mat_ld(s.out, b, s.ls_off + j), s.min_log_std), s.max_log_std);
    const float sd = expf(ls);
    const float ej = pol ? mat_ld(s.eps2, eb, j) : mat_ld(s.eps, eb, j);
    const float u = mu + ej * sd;
    const float a = tanhf(u);
    const float var = sd * sd;
    const float d = u - mu;
    lp += -(d * d) / (2.f * var) - logf(sd) - c;
    corr += logf((1.f - a * a) + 1e-6f);
    mat_st(s.act, b, j, a);
  }
  GW(s.logpi)[b] = lp - corr;
}

__device__ __forceinline__ void op_sac_actor_bwd(const CAS SacActorArgs& s, int t) {
  const int b = t * kThreads + threadIdx.x;
  if (b >= s.rows) return;
  const float w = (s.alpha_lin ? G(s.log_alpha)[0] : expf(G(s.log_alpha)[0])) * s.inv_b;  // d obj / d logpi_b
  for (int j = 0; j < s.A; ++j) {
    const float mu = mat_ld(s.out, b, s.mean_off + j);
    const float lsr = mat_ld(s.out, b, s.ls_off + j);
    const float ls = fminf(fmaxf(lsr, s.min_log_std), s.max_log_std);
    const float sd = expf(ls);
    const float ej = mat_ld(s.eps2, b, j);
    const float u = mu + ej * sd;
    const float a = tanhf(u);
    const float var = sd * sd;
    const float d = u - mu;
    // logpi = sum(-d^2/(2 var) - log sd - c) - sum log(1 - a^2 + 1e-6)
    const float ga = mat_ld(s.da, b, j) + (w / ((1.f - a * a) + 1e-6f)) * (2.f * a);
    float gu = ga * (1.f - a * a);
    gu += -(w / (2.f * var)) * (2.f * d);       // d(-d^2/(2var))/du
    float gmu = (w / (2.f * var)) * (2.f * d);  // via d = u - mu
    const float gvar = (w * (d * d)) / ((2.f * var) * (2.f * var)) * 2.f;
    float gsd = gvar * (2.f * sd) - w / sd;
    gmu += gu;
    gsd += gu * ej;
    float gls = gsd * sd;
    if (!(lsr >= s.min_log_std && lsr <= s.max_log_std)) gls = 0.f;
    mat_st(s.dout, b, s.mean_off + j, gmu);
    mat_st(s.dout, b, s.ls_off + j, gls);
  }
}

// ---------------------------------------------------------------- step end

// torch.optim.Adam bias corrections of the step after t completed ones (double, as
// the Python scalars of the reference): step = lr / (1 - 0.9^(t+1)), bc2s = sqrt(1 - 0.999^(t+1)).
__device__ __attribute__((noinline)) float2 adam_bias(long long t, float lr) {
  const double tt = (double)(t + 1);
  return make_float2((float)((double)lr / (1.0 - pow(0.9, tt))), (float)sqrt(1.0 - pow(0.999, tt)));
}
__device__ __forceinline__ void adam_scalars(long long t, float lr, GAS float* step, GAS float* bc2s) {
  const float2 r = adam_bias(t, lr);
  *step = r.x;
  *bc2s = r.y;
}

// All partial-sum reductions of the step end in one pass: every thread loads its
// elements of every sum (independent loads, one memory round trip), parks its
// per-sum partials in LDS, then wave w reduces sums w, w+4, ... (fixed order).
// (SAC: the temperature terms, compiled into the TD3 / SAC and extended instances only)
template <bool SAC>
__device__ __forceinline__ void op_step_end(const CAS StepEndArgs& a, float* smem, unsigned long long* tr) {
  constexpr int kSums = kInfoMax + 1 + kGsqT;  // info sums, logpi, grad-norm tensors
  float* res = smem + kSums * kThreads;    // [kSums]
  float* vals = res + kSums;               // [kInfoMax]
  const float nanv = __int_as_float(0x7FC00000);
  const int tid = threadIdx.x;
  // tail operands loaded up front (independent of the sums: one round trip overall)
  const bool w0 = tid < 64;
  const long long cnt = (w0 && tid < 16 && a.mode != 2) ? G(a.counters)[tid] : 0;
  const int slot0 = (w0 && a.info_slot && a.mode != 1) ? G(a.info_slot)[0] : 0;
  const int mode = a.mode;
  const bool scr = SAC && mode == 2 && a.sac_scratch;  // (alpha and the logpi sum from the counters op)
  const bool sac_tmp = SAC && a.log_alpha && a.la_lr > 0.f && mode != 2;
  const float la = SAC && a.log_alpha && !scr ? G(a.log_alpha)[0] : 0.f;
  const float la_m = sac_tmp ? G(a.la_m)[0] : 0.f, la_v = sac_tmp ? G(a.la_v)[0] : 0.f;
  const long long la_t = sac_tmp ? G(a.la_t)[0] : 0;
  // (the temperature's bias corrections: from the step's control op when it computed them, slot 3)
  const bool la_pre = sac_tmp && a.adam_step;
  const float la_bx = la_pre ? G(a.adam_step)[3] : 0.f, la_by = la_pre ? G(a.adam_bc2s)[3] : 0.f;
  const float scr_alpha = scr ? G(a.sac_scratch)[0] : 0.f, scr_slp = scr ? G(a.sac_scratch)[1] : 0.f;
  FINE_MARK(0);
  // sum list: j < ninfo -> info k (if summed); kInfoMax -> logpi; kInfoMax+1+q -> gsq tensor q
  auto sum_src = [&](int j, const float*& p, int& n, int& stride) {
    p = nullptr;
    n = 0;
    stride = 1;
    if (j < kInfoMax) {
      if (j < a.ninfo && (a.kind[j] == INFO_SUM || a.kind[j] == INFO_SAC_POL)) {
        p = a.part[j];
        n = a.npart[j];
        stride = a.stride[j];
      }
    } else if (j == kInfoMax) {
      if (a.logpi_part) {
        p = a.logpi_part + 1;
        n = a.nlogpi;
        stride = 4;
      }
    } else {
      const int q = j - kInfoMax - 1;
      if (a.gsq && q < a.ngsq_t) {
        p = a.gsq + a.gsq_off[q];
        n = a.gsq_off[q + 1] - a.gsq_off[q];
      }
    }
  };
  // each wave sums every 4th list entry: lane l adds the entry's elements l + 64 k (k = 0..3,
  // + 256 m) in the order thread 64 k + l of the former one-pass layout did, then the 4 quarters
  // and the wave as that layout's LDS reduction did -- the same float operations, with the 4
  // quarters' first loads in flight together and 4 lists at once (one list at a time paid one
  // dependent round trip per list: 3-4 us of the op's ~7, the longest op of its level)
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nsums = kInfoMax + 1 + (a.gsq ? a.ngsq_t : 0);  // (the lists in use)
  for (int j = wave; j < nsums; j += 4) {
    // (mode 1 sums only the logpi list; mode 2 takes it from the scratch when there is one)
    if ((mode == 1 && j != kInfoMax) || (scr && j == kInfoMax)) continue;
    const float* p;
    int n, stride;
    sum_src(j, p, n, stride);
    float x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = lane + 64 * k;
      x[k] = i < n ? G(p)[(size_t)i * stride] : 0.f;
    }
    float q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float v = 0.f + x[k];
      for (int i = lane + 64 * k + kThreads; i < n; i += kThreads) v += G(p)[(size_t)i * stride];
      q[k] = v;
    }
    float v = (q[0] + q[1]) + (q[2] + q[3]);
    v = wave_sum(v);
    if (lane == 0) res[j] = v;
  }
  FINE_MARK(1);
  __syncthreads();
  FINE_MARK(3);
  if (!w0) return;
  // wave 0, every lane (uniform values from LDS); lane-parallel stores
  if (tid < 16 && (a.cmask & (1 << tid))) GW(a.counters)[tid] = cnt + 1;
  const float slp = scr ? scr_slp : res[kInfoMax];
  const float alpha = scr ? scr_alpha : expf(la);
  if (mode == 1) {
    if (a.sac_scratch && tid == 0) {  // (for the info op)
      GW(a.sac_scratch)[0] = alpha;
      GW(a.sac_scratch)[1] = slp;
    }
  } else {
    for (int k = 0; k < a.ninfo; ++k) {
      float v = res[k];
      if (a.kind[k] == INFO_GNORM) {
        // per-tensor sum of squares -> sqrt -> sum (rl/nn/utils.py:13-19)
        v = 0.f;
        for (int q = 0; q < a.ngsq_t; ++q) v += sqrtf(res[kInfoMax + 1 + q]);
      }
      vals[k] = v;
    }
  }
  // mean_b(-lp_b - target_entropy); d/dla mean(exp(la) * c) = exp(la) * mean(c)
  const float gmean = (-slp) * a.inv_b - a.target_entropy;
  const float tmp_obj = alpha * gmean;
  float mine = 0.f;  // lane k < ninfo: info value k
  for (int k = 0; k < (mode == 1 ? 0 : a.ninfo); ++k) {
    float v = vals[k];
    switch (a.kind[k]) {
      case INFO_SUM: v *= a.scale[k]; break;
      case INFO_NAN: v = nanv; break;
      case INFO_GNORM: break;
      case INFO_SAC_TMP: v = alpha; break;
      case INFO_SAC_NTMP: v = tmp_obj; break;
      case INFO_SAC_POL: v = v * a.scale[k] + tmp_obj; break;
      case INFO_SAC_TMPL: v = tmp_obj; break;
      case INFO_SAC_ENT: v = -slp * a.inv_b; break;
    }
    if (tid == k) mine = v;
  }
  FINE_MARK(4);
  if (sac_tmp && tid == 0) {  // optim_tmp.step (sac.py:283)
    const float g = tmp_obj;
    const float2 bc = la_pre ? make_float2(la_bx, la_by) : adam_bias(la_t, a.la_lr);
    float m = la_m, v2 = la_v;
    m = m + (float)(1.0 - 0.9) * (g - m);
    v2 = v2 * 0.999f + ((float)(1.0 - 0.999) * g) * g;
    const float denom = sqrtf(v2) / bc.y + 1e-8f;
    GW(a.la_m)[0] = m;
    GW(a.la_v)[0] = v2;
    GW(a.log_alpha)[0] = la + (-bc.x * m) / denom;
    GW(a.la_t)[0] = la_t + 1;
  }
  if (a.info_slot && mode != 1) {
    const int slot = slot0 >= a.info_cap ? a.info_cap - 1 : slot0;
    if (tid < a.ninfo) GW(a.info)[(size_t)slot * kInfoMax + tid] = mine;
    if (tid == 0) GW(a.info_slot)[0] = slot + 1;
  }
}

// ---------------------------------------------------------------- flat ops

__device__ __forceinline__ void op_polyak(const CAS FlatArgs& f, int t) {
  const long long i0 = ((long long)t * kThreads + threadIdx.x) * 4;
  GAS float* d = GW(f.dst);
  const GAS float* src = G(f.src);
  for (long long i = i0; i < i0 + 4 && i < f.n; ++i) {
    const float s = f.self_alias ? d[i] : src[i];
    // tau*src + dst*(1-tau), each product rounded separately (Q2, no FMA)
    d[i] = __fadd_rn(__fmul_rn(f.tau, s), __fmul_rn(d[i], f.omt));
  }
}

__device__ __forceinline__ void op_copy(const CAS FlatArgs& f, int t) {
  const long long i0 = ((long long)t * kThreads + threadIdx.x) * 4;
  for (long long i = i0; i < i0 + 4 && i < f.n; ++i) GW(f.dst)[i] = G(f.src)[i];
}

__device__ __forceinline__ void op_maxred(const CAS FlatArgs& f, int t, float* smem) {
  float mx = -INFINITY;
  if (f.stage == 0) {
    const long long size = *G(f.size);
    const long long per = (size + f.nwg - 1) / f.nwg;
    const long long b0 = (long long)t * per, b1 = min(size, b0 + per);
    for (long long i = b0 + threadIdx.x; i < b1; i += kThreads) mx = fmaxf(mx, G(f.src)[i]);
  } else {
    for (int i = threadIdx.x; i < f.nwg; i += kThreads) mx = fmaxf(mx, G(f.partial)[i]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) smem[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(smem[0], smem[1]), fmaxf(smem[2], smem[3]));
    if (f.stage == 0) GW(f.partial)[t] = m;
    else GW(f.out)[0] = m;
  }
}

template <bool SAC>  // (SAC: the temperature's bias corrections; not compiled into the TD7 instance)
__device__ __forceinline__ void op_ctrl(const CAS CtrlArgs& c) {
  const int k = threadIdx.x;
  if (c.mode == 0) {
    if (k != 0) return;
    GW(c.vt)[0] = unkey(G(c.vmax_key)[0]);
    GW(c.vt)[1] = unkey(G(c.vmin_key)[0]);
  } else if (k < 3) {  // (one lane per optimizer: the fp64 pow pairs side by side, not one after another)
    adam_scalars(G(c.counters)[k], c.adam_lr[k], GW(c.adam_step) + k, GW(c.adam_bc2s) + k);
  } else if (SAC && k == 3 && c.la_t) {
    adam_scalars(G(c.la_t)[0], c.la_lr, GW(c.adam_step) + 3, GW(c.adam_bc2s) + 3);
  }
}

// ---------------------------------------------------------------- folded bias
// (runs at hard updates / parameter loads only: plain loads, one thread per output)
__device__ __forceinline__ void op_foldbias(const CAS FoldBiasArgs& f) {
  for (int o = threadIdx.x; o < f.H; o += kThreads) {
    float acc = 0.f;
    for (int z = 0; z < f.H; ++z) acc += f.wn[nidx(f.cbn, o, f.col0 + z)] * f.bin[z];
    f.bout[o] = f.bbase[o] + acc;
  }
}

// ---------------------------------------------------------------- dispatch

// TRACE: compiled with the phase stamps (RLE_TRACE=1 runs); the production instance has
// none, so nothing but the op table is read before the op body starts.
// The op table entries and the op array pointer are the first 14 dwords of the kernel
// arguments, scalar arguments that the command processor preloads into SGPRs
// (-mllvm -amdgpu-kernarg-preload-count=14, Makefile): a workgroup knows its op without
// a kernel-argument load; its first memory access is its op's descriptor.
static_assert(kLevelOps == 12, "rle_level takes the op table as 12 scalar arguments");

template <bool TRACE, int KS>  // KS: KernelSet (ops.h)
#ifndef RLE_WAVES
#define RLE_WAVES 4  // waves per SIMD the register allocation must allow (4 workgroups per CU)
#endif
__global__ __launch_bounds__(kThreads, RLE_WAVES) void rle_level(unsigned e0, unsigned e1, unsigned e2, unsigned e3,
                                                                  unsigned e4, unsigned e5, unsigned e6, unsigned e7,
                                                                  unsigned e8, unsigned e9, unsigned e10, unsigned e11,
                                                                  const Op* ops_arg, unsigned long long* trace_arg,
                                                                  const Op* next_arg, unsigned next_lines) {
  // 24 KB (the wide instances: the 40 KB LDS ring of gemm_wide)
  constexpr int kSmemF = (KS == KS_TD7W || KS == KS_EXT) && kWideSmem > 6144 ? kWideSmem : 6144;  // (40 KB)
  static_assert(kSmemF >= kRbOff + 4096, "LDS for the register-blocked exchange");
  __shared__ __attribute__((aligned(16))) float smem[kSmemF];
  // op of this workgroup from the (preloaded) entry table: straight-line selects over SGPRs
  const unsigned long long t_in = TRACE ? __builtin_amdgcn_s_memrealtime() : 0ull;  // before any load
  // Entry 0 bit 31: the launch leads with 8 workgroups that only load the next launch's
  // descriptors into L2, one per XCD (round-robin dispatch).  Between two uses of a descriptor
  // (one graph replay) tens of MB pass through every L2, so without them the next launch's
  // first scalar batch goes to the memory-side cache.  They are dispatched first and finish
  // well within the level; only they read the two (not preloaded) kernel arguments.
  if ((e0 >> 31) && blockIdx.x < 8) {
    const unsigned nl = next_lines;
    const char* nb = (const char*)next_arg;
    unsigned v0 = 0, v1 = 0;
    const unsigned l0 = threadIdx.x, l1 = threadIdx.x + kThreads;
    if (l0 < nl) asm volatile("global_load_dword %0, %1, off" : "=v"(v0) : "v"(nb + l0 * 64) : "memory");
    if (l1 < nl) asm volatile("global_load_dword %0, %1, off" : "=v"(v1) : "v"(nb + l1 * 64) : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(v0), "v"(v1) : "memory");
    return;
  }
  const unsigned entry[kLevelOps] = {e0 & 0x7fffffffu, e1, e2, e3, e4, e5, e6, e7, e8, e9, e10, e11};
  const int wg = (int)blockIdx.x - (int)(e0 >> 31) * 8;
  int k = 0;
  unsigned e = entry[0];
#pragma unroll
  for (int q = 1; q < kLevelOps; ++q) {
    const unsigned x = entry[q];
    const bool in = (int)(x & 0xffffu) <= wg;
    e = in ? x : e;
    k = in ? q : k;
  }
  const int kind = (e >> 16) & 0xf, vid = e >> 20;
  const CAS Op* ops = (const CAS Op*)ops_arg;
  const int wb = (int)(e & 0xffffu);
  const CAS Op& op = ops[k];
  const int t = wg - wb;
  // (stamp 0 is taken on entry, before the kernel-argument loads)
  unsigned long long* tr = TRACE ? trace_arg + (size_t)wg * kTraceStride : nullptr;
  if (TRACE && threadIdx.x == 0) tr[0] = t_in;
  // Non-GEMM ops (head, sampler, norm backward, priority, step end, ...): their descriptors
  // are at most 8 lines; touching them all in one batch makes every later descriptor load a
  // scalar-cache hit instead of a chain of dependent misses.  (GEMM variants touch their own
  // line sets together with the hot header: gemm_v.)
  if (kind != OP_GEMM) {
    unsigned dsink;
    asm volatile(
        "s_load_dword %0, %1, 0x0\n\t"
        "s_load_dword %0, %1, 0x40\n\t"
        "s_load_dword %0, %1, 0x80\n\t"
        "s_load_dword %0, %1, 0xc0\n\t"
        "s_load_dword %0, %1, 0x100\n\t"
        "s_load_dword %0, %1, 0x140\n\t"
        "s_load_dword %0, %1, 0x180\n\t"
        "s_load_dword %0, %1, 0x1c0\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(dsink)
        : "s"(&op));
    (void)dsink;
  }
  FINE_MARK(7);
  switch (kind) {
#define RLE_OP(K, call)                       \
  case K:                                     \
    asm volatile("; op case " #K ::);         \
    call;                                     \
    break;
    RLE_OP(OP_GEMM, op_gemm<KS>(op.gemm, vid, t, smem, tr))
    RLE_OP(OP_NORMBWD, op_normbwd(op.nb, t))
    RLE_OP(OP_SAMPLE_REDUCE, op_sample_reduce(op.sample, t, smem))
    RLE_OP(OP_SAMPLE_GATHER, op_sample_gather<KS == KS_EXT>(op.sample, t, smem, tr))
    RLE_OP(OP_HEAD, op_head(op.head, t, smem, tr))
    RLE_OP(OP_PRIORITY, op_priority(op.prio, smem))
    RLE_OP(OP_SAC_ACTOR, op_sac_actor(op.sac, t))
    RLE_OP(OP_SAC_ACTOR_BWD, op_sac_actor_bwd(op.sac, t))
    RLE_OP(OP_STEP_END, op_step_end<ks_family(KS) != KS_TD7>(op.end, smem, tr))
    RLE_OP(OP_POLYAK, op_polyak(op.flat, t))
    RLE_OP(OP_COPY, op_copy(op.flat, t))
    RLE_OP(OP_MAXRED, op_maxred(op.flat, t, smem))
    RLE_OP(OP_CTRL, op_ctrl<ks_family(KS) != KS_TD7>(op.ctrl))
    RLE_OP(OP_NOISE, op_noise(op.sample, t))
    RLE_OP(OP_FOLDBIAS, op_foldbias(op.fb))
#undef RLE_OP
    default: break;
  }
  trace_mark(tr, 3);
}


// ---------------------------------------------------------------- B = 1 act chain (ops.h ActChainArgs)
// Row block rb of layer L in registers: column block cb = wave + 4 i of the [16][K] strip, lane l
// holding row l % 16, columns 4 (l / 16) .. +3 of each 1 KB block (K <= 512: at most 8 per lane),
// and (threads 0..15) the row's bias.
constexpr int kActPre = 8;
struct ActW {
  float4 v[kActPre];
  float b;
};
__device__ __forceinline__ void act_load(const ActLayer& L, int rb, ActW& W) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < kActPre; ++i) {
    const int cb = wave + 4 * i;
    W.v[i] = cb < L.cbn ? ld4g(G(L.wn) + ((size_t)rb * L.cbn + cb) * 256 + lane * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int row = rb * 16 + (int)threadIdx.x;
  W.b = threadIdx.x < 16 && row < L.out ? G(L.bias)[row] : 0.f;
}
// The 16 rows against the LDS vectors; the 4 lane groups and the 4 waves summed in fixed order.
// Result (bias, activation) for row r in red[64 + r].
__device__ __forceinline__ void act_rows(const ActLayer& L, const ActW& W, const float* vec, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < kActPre; ++i) {
    const int cb = wave + 4 * i;
    if (cb >= L.cbn) break;
    const int c = cb * 16 + (lane >> 4) * 4;  // reduction column of v[i].x
    const float* x = (L.in1 >= 0 && c >= L.k0) ? vec + L.in1 * kActVec + (c - L.k0) : vec + L.in0 * kActVec + c;
    acc += W.v[i].x * x[0] + W.v[i].y * x[1] + W.v[i].z * x[2] + W.v[i].w * x[3];
  }
  acc += __shfl_xor(acc, 16);
  acc += __shfl_xor(acc, 32);
  if (lane < 16) red[wave * 16 + lane] = acc;
  __syncthreads();
  if (threadIdx.x < 16) {
    const int r = threadIdx.x;
    const float y = (red[r] + red[16 + r]) + (red[32 + r] + red[48 + r]) + W.b;
    red[64 + r] = act_fwd(L.act, y);
  }
  __syncthreads();
}

// Reads the granules of layer q (this call's tag) into vector slot Q.dst, then AvgL1Norm.
// Returns true (every thread) when the hand-off failed: a granule never arrived (~0.1 s), or it
// arrived poisoned (kActPoison: its producer had failed before it).  A failed workgroup keeps
// going, so the grid drains, but publishes poisoned granules from then on: the failure reaches
// the head workgroups, which report it before their completion tag.
constexpr unsigned kActPoison = 0x80000000u;  // tag bit 31 (the host's call tags stay below it)
__device__ __forceinline__ bool act_receive(const ActChainArgs& a, int q, float* vec, float* red) {
  const ActLayer& Q = a.L[q];
  bool fail = false;
  for (int i = threadIdx.x; i < Q.out; i += kThreads) {
    unsigned long long g = 0;
    int spins = 0;
    while (true) {
      g = __hip_atomic_load(a.xbuf + (size_t)q * kActVec + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned gt = (unsigned)(g >> 32);
      if (gt == a.tag) break;
      if (gt == (a.tag | kActPoison) || ++spins > (1 << 20)) {  // (fail, do not hang)
        fail = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    vec[Q.dst * kActVec + i] = __uint_as_float((unsigned)g);
  }
  fail = __syncthreads_or(fail);
  if (Q.norm) {  // AvgL1Norm: x / max(mean |x|, 1e-8), the same fixed-order sum in every workgroup
    float sabs = 0.f;
    for (int i = threadIdx.x; i < Q.out; i += kThreads) sabs += fabsf(vec[Q.dst * kActVec + i]);
    sabs = wg_sum(sabs, red);
    const float m = fmaxf(sabs / (float)Q.out, 1e-8f);
    for (int i = threadIdx.x; i < Q.out; i += kThreads) vec[Q.dst * kActVec + i] /= m;
    __syncthreads();
  }
  return fail;
}

// One row block of an exchanged layer: compute from W, publish as {value, tag} granules.
__device__ __forceinline__ void act_publish(const ActChainArgs& a, int l, int w, const ActW& W, const float* vec,
                                            float* red, bool bad) {
  const ActLayer& L = a.L[l];
  act_rows(L, W, vec, red);
  const unsigned tag = bad ? (a.tag | kActPoison) : a.tag;
  if (l == 0 && w == a.fail_wg) return;  // (failure-path test: these granules never arrive)
  if (threadIdx.x < 16 && w * 16 + (int)threadIdx.x < L.out)  // one 8-byte sc1 store per row
    __hip_atomic_store(a.xbuf + (size_t)l * kActVec + w * 16 + threadIdx.x,
                       ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(red[64 + threadIdx.x]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The act chain as straight-line code (TD7: 6 hidden layers, MLP: 2), so the compiler sees every
// weight load's place in the in-order load counter: each layer's weights load one hand-off ahead
// into one of two register sets, and computing a layer waits only for its own set.  Every
// workgroup owns row block w of every hidden layer (all are H wide: nwg = H / 16).
template <bool TD7>
__global__ __launch_bounds__(kThreads, 1) void rle_act_chain(const ActChainArgs a) {
  __shared__ __attribute__((aligned(16))) float vec[8 * kActVec];  // vector slots (0: observation, 7: head)
  __shared__ float red[128];
  const int tid = threadIdx.x, w = blockIdx.x;
  unsigned long long* st = a.stamps ? a.stamps + (size_t)w * 16 : nullptr;
  auto stamp = [&](int k) {
    if (st && tid == 0) st[k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  const int last = a.nl - 1;
  const ActLayer& H = a.L[last];
  const ActArgs& ao = a.ao;
  // head row blocks of this workgroup: TD7 / TD3 row block w (if any), SAC all in workgroup 0
  const int hr0 = a.sac ? 0 : w, hr1 = a.sac ? (w == 0 ? H.rbs : 0) : (w < H.rbs ? w + 1 : 0);
  const bool head = hr1 > hr0;
  const int j0 = a.sac ? 0 : w * 16;  // head outputs of this workgroup: [j0, j1), one per thread
  const int j1 = a.sac ? ao.A : min(ao.A, w * 16 + 16);
  float sc = 0.f, bi = 0.f;           // their action map, prefetched
  const float sg = sload(ao.sigma);
  if (j0 + tid < j1) {
    sc = G(ao.scale)[j0 + tid];
    bi = G(ao.bias)[j0 + tid];
  }
  ActW W, X;
  act_load(a.L[0], w, W);
  act_load(a.L[1], w, X);
  for (int i = tid; i < 8 * kActVec; i += kThreads) vec[i] = i < a.Sp ? a.obs[i] : 0.f;
  __syncthreads();
  stamp(1);
  bool bad = false;  // a hand-off of this call failed (workgroup-uniform)
  if constexpr (TD7) {  // 0 fe0 | 1 pi0 (norm) || 2 fe1 || 3 fe2 (norm) || 4 pi1 || 5 pi2 || 6 head
    act_publish(a, 0, w, W, vec, red, bad);
    act_load(a.L[2], w, W);
    act_publish(a, 1, w, X, vec, red, bad);
    act_load(a.L[3], w, X);
    stamp(2);
    bad |= act_receive(a, 0, vec, red);
    bad |= act_receive(a, 1, vec, red);
    stamp(3);
    act_publish(a, 2, w, W, vec, red, bad);
    act_load(a.L[4], w, W);
    bad |= act_receive(a, 2, vec, red);
    stamp(4);
    act_publish(a, 3, w, X, vec, red, bad);
    act_load(a.L[5], w, X);
    bad |= act_receive(a, 3, vec, red);
    stamp(5);
    act_publish(a, 4, w, W, vec, red, bad);
    if (head) act_load(H, hr0, W);
    bad |= act_receive(a, 4, vec, red);
    stamp(6);
    act_publish(a, 5, w, X, vec, red, bad);
    if (!head) return;
    if (hr0 + 1 < hr1) act_load(H, hr0 + 1, X);
    bad |= act_receive(a, 5, vec, red);
    stamp(7);
  } else {  // 0 h0 || 1 h1 || 2 head
    act_publish(a, 0, w, W, vec, red, bad);
    if (head) act_load(H, hr0, W);
    bad |= act_receive(a, 0, vec, red);
    stamp(2);
    act_publish(a, 1, w, X, vec, red, bad);
    if (!head) return;
    if (hr0 + 1 < hr1) act_load(H, hr0 + 1, X);
    bad |= act_receive(a, 1, vec, red);
    stamp(3);
  }
  // ---- the head: env action (td7.py:141-156, td3.py:114-129, sac.py:132-152)
  for (int rb = hr0; rb < hr1; ++rb) {
    if (rb == hr0) act_rows(H, W, vec, red);
    else if (rb == hr0 + 1) act_rows(H, X, vec, red);
    else {  // (SAC, a third row block: 2A > 32)
      act_load(H, rb, W);
      act_rows(H, W, vec, red);
    }
    if (tid < 16) vec[7 * kActVec + rb * 16 + tid] = red[64 + tid];
    __syncthreads();
  }
  const float* h = vec + 7 * kActVec;
  const int mode = a.mode;
  const int j = j0 + tid;
  if (j < j1) {
    const float e = mode == 2 ? a.eps[j] : (mode ? act_noise(ao.seed, j, a.ctr_lo, a.ctr_hi) : 0.f);
    float act;
    if (a.sac) {
      const float mu = h[j];
      float u = mu;
      if (mode) {
        const float ls = fminf(fmaxf(h[ao.A + j], a.min_log_std), a.max_log_std);
        u = __fadd_rn(mu, __fmul_rn(e, expf(ls)));  // Normal.rsample: loc + eps * scale
      }
      act = tanhf(u);
    } else {
      act = h[j];  // tanh applied by act_rows (L.act); + exploration_noise * eps, clip
      if (mode) act = __fadd_rn(act, __fmul_rn(e, sg));
      act = fminf(fmaxf(act, -1.f), 1.f);
    }
    GW(ao.out)[j] = __fadd_rn(__fmul_rn(act, sc), bi);
  }
  // completion for the host's poll: this workgroup's action stores, then its slot := tag with a
  // system-scope release (a plain store, no PCIe atomic)
  __syncthreads();
  stamp(15);
  // (a failed hand-off is reported by the same thread before the tag: the release orders it)
  if (tid == 0) {
    if (bad) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(a.done + w, a.tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---------------------------------------------------------------- standalone kernels

// Scatter `count` staged transitions into the ring at ptr (wrapping).
__global__ void rle_append_kernel(float* state, float* next_state, float* action, float* reward, float* notdone,
                                  float* priority, const float* st_s, const float* st_ns, const float* st_a,
                                  const float* st_r, const float* st_d, long long ptr, long long cap, int count,
                                  int Sp, int Ap, const float* max_priority, int lap, double* bsum, double* ssum,
                                  long long size_before) {
  const int i = blockIdx.x;
  if (i >= count) return;
  const long long row = (ptr + i) % cap;
  for (int k = threadIdx.x; k < Sp; k += blockDim.x) {
    state[row * Sp + k] = st_s[(size_t)i * Sp + k];
    next_state[row * Sp + k] = st_ns[(size_t)i * Sp + k];
  }
  for (int k = threadIdx.x; k < Ap; k += blockDim.x) action[row * Ap + k] = st_a[(size_t)i * Ap + k];
  if (threadIdx.x == 0) {
    reward[row] = st_r[i];
    notdone[row] = st_d[i];
    if (lap) {  // lap.py:41, with the block sum following the write (rows past size count as 0)
      const float nv = *max_priority;
      const float old = row < size_before ? priority[row] : 0.f;
      priority[row] = nv;
      atomicAdd(&bsum[row / kBlk], (double)nv - (double)old);
      atomicAdd(&ssum[row / kSub], (double)nv - (double)old);
    }
  }
}

// Synthetic replay for the benchmark: s, s' ~ N(0,1),
// a ~ U(-1,1), r ~ N(0,1), notdone ~ Bernoulli(0.99), priority = 1.
__global__ void rle_fill_kernel(float* state, float* next_state, float* action, float* reward, float* notdone,
                                float* priority, long long n, int S, int Sp, int A, int Ap, unsigned long long seed) {
  const long long row = blockIdx.x;
  if (row >= n) return;
  const uint2 key = make_uint2((unsigned)seed, (unsigned)(seed >> 32));
  for (int k = threadIdx.x; k < Sp; k += blockDim.x) {
    const uint4 r = philox(key, make_uint4((unsigned)row, (unsigned)k, 7u, (unsigned)(row >> 32)));
    state[row * Sp + k] = k < S ? normal_from(r.x, r.y) : 0.f;
    next_state[row * Sp + k] = k < S ? normal_from(r.z, r.w) : 0.f;
  }
  for (int k = threadIdx.x; k < Ap; k += blockDim.x) {
    const uint4 r = philox(key, make_uint4((unsigned)row, (unsigned)k, 8u, (unsigned)(row >> 32)));
    action[row * Ap + k] = k < A ? 2.f * u01(r.x) - 1.f : 0.f;
  }
  if (threadIdx.x == 0) {
    const uint4 r = philox(key, make_uint4((unsigned)row, 0u, 9u, (unsigned)(row >> 32)));
    reward[row] = normal_from(r.x, r.y);
    notdone[row] = u01(r.z) < 0.99f ? 1.f : 0.f;
    priority[row] = 1.f;
  }
}

// ---------------------------------------------------------------- host launchers

// Workgroups of rle_level resident at once on the current device.
// Timestamps per workgroup in trace buffers (4; 16 in -DRLE_TRACE_FINE builds).
int trace_stride() { return kTraceStride; }

int level_capacity() {
  int per_cu = 0, cus = 0, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 1024;
  int p1 = 0, p2 = 0, p3 = 0;  // (every instance: the planner's capacity must hold for the one an engine runs)
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rle_level<false, KS_TD7>, kThreads, 0) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&p1, rle_level<false, KS_MLP>, kThreads, 0) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&p2, rle_level<false, KS_EXT>, kThreads, 0) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&p3, rle_level<false, KS_TD7W>, kThreads, 0) != hipSuccess)
    return 1024;
  per_cu = per_cu < p1 ? per_cu : p1;
  per_cu = per_cu < p2 ? per_cu : p2;
  per_cu = per_cu < p3 ? per_cu : p3;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 1024;
  return per_cu * cus;
}

// (host) when set, launch_level also appends each dispatch's kernel arguments here (capture of the
// AQL launch lists; traced launches are never recorded)
std::vector<LevelLaunch>* g_level_rec = nullptr;
// the production kernel's HSA symbol name (AQL dispatch)
const char* level_kernel_symbol(int ks) {
  return ks == KS_EXT    ? "_ZN3rle9rle_levelILb0ELi2EEEvjjjjjjjjjjjjPKNS_2OpEPyS3_j.kd"
         : ks == KS_MLP  ? "_ZN3rle9rle_levelILb0ELi1EEEvjjjjjjjjjjjjPKNS_2OpEPyS3_j.kd"
         : ks == KS_TD7W ? "_ZN3rle9rle_levelILb0ELi3EEEvjjjjjjjjjjjjPKNS_2OpEPyS3_j.kd"
                         : "_ZN3rle9rle_levelILb0ELi0EEEvjjjjjjjjjjjjPKNS_2OpEPyS3_j.kd";
}

hipError_t launch_level(const Op* d_ops, const Op* h_ops, int nops, int nwg, hipStream_t st,
                        unsigned long long* trace, const Op* next_ops, int next_nops, int ks) {
  // a level of more than kLevelOps ops: consecutive launches of kLevelOps (its ops are
  // independent, so any split is correct)
  for (int q0 = 0; q0 < nops; q0 += kLevelOps) {
    const int n = nops - q0 < kLevelOps ? nops - q0 : kLevelOps;
    const int w0 = h_ops[q0].wg_begin;
    const int w1 = q0 + n < nops ? h_ops[q0 + n].wg_begin : nwg;
    if (w1 - w0 + 8 > kMaxLevelWG) return hipErrorInvalidValue;
    LevelArgs la{};
    la.ops = d_ops + q0;
    la.trace = trace ? trace + (size_t)w0 * kTraceStride : nullptr;
    // the following launch's ops: the rest of this level, then the next level's
    const bool last = q0 + n >= nops;
    const int nn = !last ? (nops - q0 - n < kLevelOps ? nops - q0 - n : kLevelOps)
                         : (next_nops <= kLevelOps ? next_nops : kLevelOps);
    const Op* next = !last ? d_ops + q0 + n : next_ops;
    const unsigned next_lines = (unsigned)(nn * (int)(sizeof(Op) / 64) < 2 * kThreads ? nn * (int)(sizeof(Op) / 64) : 2 * kThreads);
    const int npf = next_lines ? 8 : 0;  // leading prefetch workgroups (entry 0 bit 31)
    for (int q = 0; q < kLevelOps; ++q) {
      if (q < n) {
        const Op& o = h_ops[q0 + q];
        const unsigned vid = o.kind == OP_GEMM ? (unsigned)o.gemm.vid : 0u;
        la.entry[q] = (unsigned)(o.wg_begin - w0) | ((unsigned)o.kind << 16) | (vid << 20);
      } else {
        la.entry[q] = 0xffffu;
      }
    }
    if (npf) la.entry[0] |= 0x80000000u;
    if (g_level_rec && !trace) {  // (traced launches are never recorded)
      LevelLaunch L{};
      std::memcpy(L.ka, la.entry, sizeof la.entry);
      std::memcpy(L.ka + 48, &la.ops, 8);
      std::memcpy(L.ka + 56, &la.trace, 8);
      std::memcpy(L.ka + 64, &next, 8);
      std::memcpy(L.ka + 72, &next_lines, 4);
      L.grid = (unsigned)(w1 - w0 + npf);
      L.ks = ks;
      g_level_rec->push_back(L);
    }
#define RLE_LEVEL_ARGS                                                                                         \
  la.entry[0], la.entry[1], la.entry[2], la.entry[3], la.entry[4], la.entry[5], la.entry[6], la.entry[7], \
      la.entry[8], la.entry[9], la.entry[10], la.entry[11], la.ops, la.trace, next, next_lines
    const dim3 grid(w1 - w0 + npf);
    if (trace) {
      if (ks == KS_TD7) hipLaunchKernelGGL((rle_level<true, KS_TD7>), grid, dim3(kThreads), 0, st, RLE_LEVEL_ARGS);
      else if (ks == KS_MLP) hipLaunchKernelGGL((rle_level<true, KS_MLP>), grid, dim3(kThreads), 0, st, RLE_LEVEL_ARGS);
      else if (ks == KS_TD7W) hipLaunchKernelGGL((rle_level<true, KS_TD7W>), grid, dim3(kThreads), 0, st, RLE_LEVEL_ARGS);
      else hipLaunchKernelGGL((rle_level<true, KS_EXT>), grid, dim3(kThreads), 0, st, RLE_LEVEL_ARGS);
    } else {
      if (ks == KS_TD7) hipLaunchKernelGGL((rle_level<false, KS_TD7>), grid, dim3(kThreads), 0, st, RLE_LEVEL_ARGS);
      else if (ks == KS_MLP) hipLaunchKernelGGL((rle_level<false, KS_MLP>), grid, dim3(kThreads), 0, st, RLE_LEVEL_ARGS);
      else if (ks == KS_TD7W) hipLaunchKernelGGL((rle_level<false, KS_TD7W>), grid, dim3(kThreads), 0, st, RLE_LEVEL_ARGS);
      else hipLaunchKernelGGL((rle_level<false, KS_EXT>), grid, dim3(kThreads), 0, st, RLE_LEVEL_ARGS);
    }
#undef RLE_LEVEL_ARGS
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
hipError_t launch_append(float* state, float* next_state, float* action, float* reward, float* notdone,
                         float* priority, const float* st_s, const float* st_ns, const float* st_a,
                         const float* st_r, const float* st_d, long long ptr, long long cap, int count, int Sp,
                         int Ap, const float* max_priority, int lap, double* bsum, double* ssum, long long size_before,
                         hipStream_t st) {
  hipLaunchKernelGGL(rle_append_kernel, dim3(count), dim3(256), 0, st, state, next_state, action, reward, notdone,
                     priority, st_s, st_ns, st_a, st_r, st_d, ptr, cap, count, Sp, Ap, max_priority, lap, bsum, ssum,
                     size_before);
  return hipGetLastError();
}
hipError_t launch_act_chain(const ActChainArgs& a, hipStream_t st) {
  if (a.nl == 7) hipLaunchKernelGGL(rle_act_chain<true>, dim3(a.nwg), dim3(kThreads), 0, st, a);
  else hipLaunchKernelGGL(rle_act_chain<false>, dim3(a.nwg), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_fill(float* state, float* next_state, float* action, float* reward, float* notdone,
                       float* priority, long long n, int S, int Sp, int A, int Ap, unsigned long long seed,
                       hipStream_t st) {
  hipLaunchKernelGGL(rle_fill_kernel, dim3((unsigned)n), dim3(128), 0, st, state, next_state, action, reward,
                     notdone, priority, n, S, Sp, A, Ap, seed);
  return hipGetLastError();
}

}  // namespace rle
