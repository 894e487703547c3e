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

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
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
#pragma unroll
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
  float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
  float u2 = (float)(b >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// AvgL1Norm denominator from column-tile partial |x| sums (fixed order).
__device__ __forceinline__ float norm_m(const float* part, int ld, int row, int nparts, int width) {
  const GAS float* p = G(part);
  float s = 0.f;
  for (int q = 0; q < nparts; ++q) s += p[(size_t)q * ld + row];
  const float m = s / (float)width;
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

// LDS table of 1/m for n consecutive rows of a normed tensor (16-padded with 0).
__device__ __forceinline__ void build_norm_tab(const CAS NormRef& nr, int n, float* dst) {
#pragma unroll 1
  for (int i = threadIdx.x; i < n; i += kThreads) dst[i] = norm_inv(nr, i);
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

// ---------------------------------------------------------------- GEMM
//
// One workgroup = one 16 x 64 output tile; wave w owns columns [16w, 16w+16)
// and the FULL reduction.  Both operands are fragment images (ops.h), so each
// 16-wide reduction chunk is one lane-linear 16-byte buffer load per lane per
// operand -- the wave reads whole 1 KB blocks (8 full cache lines) instead of
// 16 row pieces.  A load cursor per operand walks the reduction block by block
// and segment by segment; 4 chunks are kept in flight in a register ring.
// AvgL1Norm scales (deferred normalisation) are applied when a chunk is
// consumed.  Epilogue operands (bias, derivative source, Adam w/m/v) are
// fetched before the main loop; the accumulator fragment (rows 4*(l>>4)+q,
// column l&15) is exactly one float4 of a T image, so T-image traffic in the
// epilogue is one 16-byte access per lane.

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
static_assert(kMaxSeg == 4, "LaneOp holds 4 segments");
constexpr int kRing = 4;  // GEMM main-loop chunks in flight per wave

struct LaneOp {
  f32x4 inv;  // N-image operand + normed: 1/m of the lane's row, per segment (vector, not
              // array: a per-chunk select must stay in registers)
  i32x4 tab;  // T-image operand + normed: LDS offset of the segment's 1/m table, -1 = none
  bool norm;  // any normed segment
};

// v[q] for a wave-uniform q as a select chain (a variable extract is lowered to scratch).
template <class V>
__device__ __forceinline__ auto pick(const V& v, int q) -> decltype(v[0] + 0) {
  return q == 0 ? v[0] : q == 1 ? v[1] : q == 2 ? v[2] : v[3];
}

__device__ __forceinline__ void lane_op(const CAS Operand& op, bool T, int x, LaneOp& L, float* tabs, int& used) {
  L.inv = f32x4{1.f, 1.f, 1.f, 1.f};
  L.tab = i32x4{-1, -1, -1, -1};
  L.norm = false;
#pragma unroll
  for (int s = 0; s < kMaxSeg; ++s) {
    if (s < op.nseg) {
      const CAS Seg& sg = op.seg[s];
      if (sg.norm.part) {
        L.norm = true;
        if (!T) {
          if (x >= sg.x0 && x < sg.x1) L.inv[s] = norm_inv(sg.norm, x - sg.x0);
        } else {
          const int n = sg.r1 - sg.r0;
          L.tab[s] = used;
          build_norm_tab(sg.norm, n, tabs + used);
          used += (n + 15) & ~15;
        }
      }
    }
  }
}

__device__ __forceinline__ float4 as_f4(u32x4 v) {
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

// Load cursor of one operand: lane-linear 1 KB block per chunk, segment after segment.
struct Cursor {
  __amdgpu_buffer_rsrc_t rs;  // current segment (wave-uniform)
  int voff;                   // this lane's byte offset of the next chunk
  int left;                   // chunks left in the segment
  int s;                      // segment index (>= nseg: past the end, reads 0)
  int toff;                   // T image + normed: LDS 1/m table offset of the next chunk (-1: none)
  float inv;                  // N image + normed: lane row's 1/m in the segment

  __device__ __forceinline__ void open(const CAS Operand& op, const LaneOp& L, int xw, int q) {
    s = q;
    if (q >= op.nseg) {
      rs = __builtin_amdgcn_make_buffer_rsrc((void*)nullptr, 0, 0, 0x00020000);
      left = 1 << 30;
      voff = 0;
      toff = -1;
      inv = 1.f;
      return;
    }
    const CAS Seg& sg = op.seg[q];
    rs = __builtin_amdgcn_make_buffer_rsrc((void*)sg.p, 0, 0x7fff0000, 0x00020000);
    left = (sg.r1 - sg.r0 + 15) >> 4;
    voff = ((xw - sg.x0) >> 4) * sg.xs * 1024 + (threadIdx.x & 63) * 16;
    inv = pick(L.inv, q);
    toff = pick(L.tab, q);
  }
  __device__ __forceinline__ float4 next(const CAS Operand& op, const LaneOp& L, int xw, float& inv_out,
                                         int& toff_out) {
    if (left == 0) open(op, L, xw, s + 1);
    const float4 v = as_f4(__builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0));
    inv_out = inv;
    toff_out = toff;
    if (toff >= 0) toff += 16;
    voff += 1024;
    --left;
    return v;
  }
};

// Deferred AvgL1Norm of a consumed chunk.
template <bool T>
__device__ __forceinline__ float4 chunk_scale(float4 v, float inv, int toff, int rl, const float* tabs) {
  if (!T) {
    v.x *= inv; v.y *= inv; v.z *= inv; v.w *= inv;
  } else if (toff >= 0) {
    const float4 w = *(const float4*)(tabs + toff + rl);
    v.x *= w.x; v.y *= w.y; v.z *= w.z; v.w *= w.w;
  }
  return v;
}

__device__ __forceinline__ f32x4 mfma4(const float4& a, const float4& b, f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  return acc;
}

// Main loop, one instantiation per operand image pair (FWD <N,N>, DX <N,T>,
// DW <T,T>, DW bias column <T,-> with B = ones).  xa_w / xb_w: the wave's first
// A row / B column (wave-uniform).
template <bool TA, bool TB, bool BIAS>
__device__ __forceinline__ f32x4 gemm_mainloop(const CAS GemmArgs& g, int xa, int xb, int xa_w, int xb_w,
                                               bool active, float* tabs) {
  const int lane = threadIdx.x & 63;
  LaneOp la, lb;
  int used = 0;
  lane_op(g.A, TA, xa, la, tabs, used);
  if (!BIAS) lane_op(g.B, TB, xb, lb, tabs, used);
  if (used) __syncthreads();
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  if (!active) return acc0;
  const bool b_ok = BIAS ? (xb == g.adam.bias_col) : true;
  const int rl = 4 * (lane >> 4);
  const int nch = (g.R + 15) >> 4;
  const bool an = la.norm, bn = !BIAS && lb.norm;
  // DW B: the segments split the columns; the wave's 16 columns lie in one of them
  int qb = 0;
  if (TA && TB && !BIAS) {
#pragma unroll
    for (int q = 1; q < kMaxSeg; ++q)
      if (q < g.B.nseg && xb_w >= g.B.seg[q].x0) qb = q;
  }
  Cursor ca, cb;
  ca.open(g.A, la, xa_w, 0);
  if (!BIAS) cb.open(g.B, lb, xb_w, qb);
  const int nb_end = (TA && TB) ? qb + 1 : g.B.nseg;  // DW: one B segment only
  const float4 ones = b_ok ? make_float4(1.f, 1.f, 1.f, 1.f) : make_float4(0.f, 0.f, 0.f, 0.f);
  auto ldA = [&](float& i, int& t) { return ca.next(g.A, la, xa_w, i, t); };
  auto ldB = [&](float& i, int& t) {
    if constexpr (BIAS) return ones;  // db = sum_r dZ(r, n); A is zero past R
    else {
      if (cb.left == 0 && cb.s + 1 >= nb_end) cb.s = kMaxSeg;  // DW: never walk into another column block
      return cb.next(g.B, lb, xb_w, i, t);
    }
  };
  auto use = [&](float4 a, float4 b, float ia, int ta, float ib, int tb, f32x4 acc) {
    if (an) a = chunk_scale<TA>(a, ia, ta, rl, tabs);
    if (bn) b = chunk_scale<TB>(b, ib, tb, rl, tabs);
    return mfma4(a, b, acc);
  };
  float4 ra[kRing], rb[kRing];
  float ia[kRing], ib[kRing];
  int ta[kRing], tb[kRing];
#pragma unroll
  for (int k = 0; k < kRing; ++k) {
    ra[k] = ldA(ia[k], ta[k]);
    rb[k] = ldB(ib[k], tb[k]);
  }
#pragma unroll 1
  for (int c = 0; c < nch; c += kRing) {
#pragma unroll
    for (int k = 0; k < kRing; ++k) {
      if (k & 1) acc1 = use(ra[k], rb[k], ia[k], ta[k], ib[k], tb[k], acc1);
      else acc0 = use(ra[k], rb[k], ia[k], ta[k], ib[k], tb[k], acc0);
      ra[k] = ldA(ia[k], ta[k]);
      rb[k] = ldB(ib[k], tb[k]);
    }
  }
  return acc0 + acc1;
}

__device__ __forceinline__ void op_gemm(const CAS GemmArgs& g, int t, float* smem) {
  // wave index via readfirstlane: the compiler then treats every wave-derived
  // condition as uniform (scalar branches)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int it = t / g.tiles_n, jt = t - it * g.tiles_n;
  const int i0 = it * kTileM, j0 = jt * kTileN + wave * 16;
  const bool bias_tile = (g.epi == EPI_ADAM) && (jt * kTileN >= g.adam.bias_col);
  float* red = smem;            // [64] reduction scratch
  float* tabs = smem + 64;      // normalisation tables
  const int xa = i0 + (lane & 15), xb = j0 + (lane & 15);
  const int j = xb;                       // output column of this lane
  const int ib = i0 + 4 * (lane >> 4);    // first of this lane's 4 output rows
  const bool jok = bias_tile ? (j == g.adam.bias_col) : (j < g.N);
  const bool active = bias_tile ? (wave == 0) : (j0 < g.N);  // wave-uniform

  // ---- epilogue operands fetched ahead of the main loop
  float pre_b = 0.f;
  float4 ds = make_float4(1.f, 1.f, 1.f, 1.f), pp = make_float4(0.f, 0.f, 0.f, 0.f), mm = pp, vv = pp;
  size_t wt = 0;  // T-image element offset of (ib, j) in the weight (EPI_ADAM)
  if (g.epi != EPI_ADAM) {
    if (g.bias && jok) pre_b = G(g.bias)[j];
    if (g.dsrc.t && jok) ds = mat_ld4(g.dsrc, ib, j);
  } else if (active) {
    const CAS AdamArgs& ad = g.adam;
    if (bias_tile) {
      if (jok) {
        pp = ld4g(G(ad.b) + ib);
        mm = ld4g(G(ad.b) + ib + ad.mo);
        vv = ld4g(G(ad.b) + ib + ad.vo);
      }
    } else {
      wt = tidx(ad.w.rbs, ib, j);
      pp = ld4g(G(ad.w.t) + wt);
      mm = ld4g(G(ad.w.t) + wt + ad.mo);
      vv = ld4g(G(ad.w.t) + wt + ad.vo);
    }
  }

  const int xa_w = i0, xb_w = j0;  // wave-uniform operand origins
  // The distinct empty asm statements head each arm so the compiler cannot hoist
  // the arms' common descriptor loads above the branch.
  f32x4 acc;
  if (g.mode == GEMM_FWD) {
    asm volatile("; gemm fwd" ::);
    acc = gemm_mainloop<false, false, false>(g, xa, xb, xa_w, xb_w, active, tabs);
  } else if (g.mode == GEMM_DX) {
    asm volatile("; gemm dx" ::);
    acc = gemm_mainloop<false, true, false>(g, xa, xb, xa_w, xb_w, active, tabs);
  } else if (!bias_tile) {
    asm volatile("; gemm dw" ::);
    acc = gemm_mainloop<true, true, false>(g, xa, xb, xa_w, xb_w, active, tabs);
  } else {
    asm volatile("; gemm db" ::);
    acc = gemm_mainloop<true, true, true>(g, xa, xb, xa_w, xb_w, active, tabs);
  }

  if (g.epi == EPI_STORE) {
    float rowabs[4] = {0.f, 0.f, 0.f, 0.f};
    if (jok) {
      float v[4] = {acc[0] + pre_b, acc[1] + pre_b, acc[2] + pre_b, acc[3] + pre_b};
      if (g.pre.t) mat_st4(g.pre, ib, j, make_float4(v[0], v[1], v[2], v[3]));
      float4 e = make_float4(0.f, 0.f, 0.f, 0.f);
      const bool noised = g.noise.t && ib >= g.noise_row0;  // target policy smoothing (td7.py:188-194)
      if (noised) e = mat_ld4(g.noise, ib - g.noise_row0, j);
      const float ev[4] = {e.x, e.y, e.z, e.w}, dv[4] = {ds.x, ds.y, ds.z, ds.w};
      float y[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        y[q] = act_fwd(g.act, v[q]);
        if (noised) {
          const float nz = fminf(fmaxf(ev[q] * g.noise_sigma, -g.noise_clip), g.noise_clip);
          y[q] = fminf(fmaxf(y[q] + nz, -1.f), 1.f);
        }
        if (g.dsrc.t) y[q] *= act_bwd(g.dact, dv[q]);
        rowabs[q] = fabsf(y[q]);
      }
      mat_st4(g.out, ib, j, make_float4(y[0], y[1], y[2], y[3]));
    }
    if (g.norm_out) {  // |y| summed over the tile's 64 columns, per row
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) rowabs[q] += __shfl_xor(rowabs[q], o, 64);
      }
      if ((lane & 15) == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) red[wave * 16 + 4 * (lane >> 4) + q] = rowabs[q];
      }
      __syncthreads();
      if (tid < 16 && i0 + tid < g.M)
        GW(g.norm_out)[(size_t)jt * g.norm_ld + i0 + tid] =
            (red[tid] + red[16 + tid]) + (red[32 + tid] + red[48 + tid]);
    }
  } else if (g.epi == EPI_MSE) {  // td7.py:256 encoder loss, grad wrt zsa
    float d2 = 0.f;
    if (jok) {
      const float4 tv = mat_ld4(g.tgt, ib, j);
      const float tq[4] = {tv.x, tv.y, tv.z, tv.w};
      float gr[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float tn = tq[q] * norm_inv(g.tgt_norm, ib + q);
        const float d = (acc[q] + pre_b) - tn;
        gr[q] = (2.f * d) * g.mse_scale;  // mse_scale = 1/n
        d2 += d * d;
      }
      mat_st4(g.out, ib, j, make_float4(gr[0], gr[1], gr[2], gr[3]));
    }
    d2 = wg_sum(d2, red);
    if (tid == 0) GW(g.loss_part)[t] = d2;
  } else {  // EPI_ADAM (torch.optim.Adam single-tensor law, see oracle/agents.py)
    const CAS AdamArgs& ad = g.adam;
    const double tt = (double)(*G(ad.t) + 1);
    const double bc1 = 1.0 - pow((double)ad.beta1, tt);
    const double bc2 = 1.0 - pow((double)ad.beta2, tt);
    const float step_size = (float)((double)ad.lr / bc1);
    const float bc2s = (float)sqrt(bc2);
    float gg = 0.f;
    if (active && jok) {
      const float p4[4] = {pp.x, pp.y, pp.z, pp.w}, m4[4] = {mm.x, mm.y, mm.z, mm.w}, v4[4] = {vv.x, vv.y, vv.z, vv.w};
      float po[4], mo[4], vo[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float gv = acc[q];
        float m = m4[q], v2 = v4[q];
        m = m + (1.f - ad.beta1) * (gv - m);
        v2 = v2 * ad.beta2 + ((1.f - ad.beta2) * gv) * gv;
        const float denom = sqrtf(v2) / bc2s + ad.eps;
        const bool ok = ib + q < g.M;  // weight rows past out stay untouched (zero)
        po[q] = ok ? p4[q] + (-step_size * m) / denom : p4[q];
        mo[q] = ok ? m : m4[q];
        vo[q] = ok ? v2 : v4[q];
        gg += ok ? gv * gv : 0.f;
      }
      const float4 P = make_float4(po[0], po[1], po[2], po[3]);
      if (bias_tile) {
        st4g(GW(ad.b) + ib, P);
        st4g(GW(ad.b) + ib + ad.mo, make_float4(mo[0], mo[1], mo[2], mo[3]));
        st4g(GW(ad.b) + ib + ad.vo, make_float4(vo[0], vo[1], vo[2], vo[3]));
      } else {
        st4g(GW(ad.w.t) + wt, P);
        st4g(GW(ad.w.t) + wt + ad.mo, make_float4(mo[0], mo[1], mo[2], mo[3]));
        st4g(GW(ad.w.t) + wt + ad.vo, make_float4(vo[0], vo[1], vo[2], vo[3]));
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
        else GW(ad.gsq)[it * (g.tiles_n - 1) + jt] = gg;
      }
    }
  }
}

// ---------------------------------------------------------------- AvgL1Norm backward

// 16 rows per workgroup, 4 per wave: lane k reads a float4 (4 rows) of column k
// from the T images; the per-row dot products are wave reductions.
__device__ __forceinline__ void op_normbwd(const CAS NormBwdArgs& a, int t) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = t * 16 + wave * 4;
  if (r0 >= a.rows) return;
  float inv[4], gmv[4];
  bool clamped[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float s = 0.f;  // m recomputed from the same partials the forward consumers used
    for (int p = 0; p < a.norm.nparts; ++p) s += G(a.norm.part)[(size_t)p * a.norm.ld + r0 + q + a.norm.row0];
    const float mean = s / (float)a.width;
    clamped[q] = mean < 1e-8f;
    inv[q] = 1.f / (clamped[q] ? 1e-8f : mean);
  }
  float4 xv[8], gv[8];
  float dot[4] = {0.f, 0.f, 0.f, 0.f};
  const int per = (a.width + 63) / 64;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int k = lane + 64 * u;
    const bool in = u < per && k < a.width;
    xv[u] = in ? mat_ld4(a.x, r0, k) : make_float4(0.f, 0.f, 0.f, 0.f);
    gv[u] = in ? mat_ld4(a.g, r0, k) : make_float4(0.f, 0.f, 0.f, 0.f);
    dot[0] += gv[u].x * xv[u].x;
    dot[1] += gv[u].y * xv[u].y;
    dot[2] += gv[u].z * xv[u].z;
    dot[3] += gv[u].w * xv[u].w;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    dot[q] = wave_sum(dot[q]);
    // y = x / m: dy/dx path g/m ; dm path -(sum g x)/m^2 * sign(x)/n (unless clamped)
    gmv[q] = clamped[q] ? 0.f : (-dot[q] * inv[q] * inv[q]) / (float)a.width;
  }
  auto sgn = [](float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); };
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int k = lane + 64 * u;
    if (u < per && k < a.width) {
      const float4 o = make_float4(gv[u].x * inv[0] + sgn(xv[u].x) * gmv[0], gv[u].y * inv[1] + sgn(xv[u].y) * gmv[1],
                                   gv[u].z * inv[2] + sgn(xv[u].z) * gmv[2], gv[u].w * inv[3] + sgn(xv[u].w) * gmv[3]);
      mat_st4(a.dx, r0, k, o);
    }
  }
}

// ---------------------------------------------------------------- critic heads

// Last critic layer (H -> 1) as a dot product fused with the TD target / loss /
// priority / policy objective and the gradient into the last hidden layer.
// 16 rows per workgroup, 4 per wave (lane k: float4 of 4 rows from T images).
__device__ __forceinline__ void op_head(const CAS HeadArgs& h, int t, float* smem) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = t * 16 + wave * 4;
  float acc0 = 0.f, acc1 = 0.f;  // per-wave loss terms (sum over its rows)
  int kmax = (int)0x80000000, kmin = 0x7FFFFFFF;
  if (r0 < h.rows) {
    float q[2][4];
    float wv[2][8];
    const int per = (h.H + 63) / 64;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = lane + 64 * u;
        const bool in = u < per && k < h.H;
        wv[n][u] = in ? G(h.w[n])[tidx(h.w_rbs, 0, k)] : 0.f;
        const float4 hv = in ? mat_ld4(h.h[n], r0, k) : make_float4(0.f, 0.f, 0.f, 0.f);
        s[0] += hv.x * wv[n][u];
        s[1] += hv.y * wv[n][u];
        s[2] += hv.z * wv[n][u];
        s[3] += hv.w * wv[n][u];
      }
      const float bb = G(h.b[n])[0];
#pragma unroll
      for (int r = 0; r < 4; ++r) q[n][r] = wave_sum(s[r]) + bb;
    }
    float dq[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    bool want_dz = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = r0 + r;
      switch (h.mode) {
        case HEAD_TD7_TARGET: {  // td7.py:211-218
          float v = fminf(q[0][r], q[1][r]);
          v = fminf(fmaxf(v, G(h.vt)[1]), G(h.vt)[0]);
          const float y = G(h.reward)[b] + (h.gamma * v) * G(h.notdone)[b];
          if (lane == 0) GW(h.y)[b] = y;
          kmax = max(kmax, fkey(y));
          kmin = min(kmin, fkey(y));
          break;
        }
        case HEAD_MLP_TARGET: {  // td3.py:160-164, sac.py:188-193
          float v = fminf(q[0][r], q[1][r]);
          if (h.sac) v = v - expf(G(h.log_alpha)[0]) * G(h.logpi)[b];
          const float y = G(h.reward)[b] + (h.gamma * v) * G(h.notdone)[b];
          if (lane == 0) GW(h.y)[b] = y;
          break;
        }
        case HEAD_TD7_LOSS:
        case HEAD_MLP_LOSS: {  // td7.py:231-244, td3.py:169-182
          const float y = G(h.y)[b];
          float dmax = 0.f;
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            const float diff = q[n][r] - y;
            if (h.lap) {
              const float d = fabsf(diff);
              const float hub = d < 1.f ? 0.5f * (d * d) : d;
              if (n == 0) acc0 += hub; else acc1 += hub;
              const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
              dq[n][r] = (d < 1.f ? d : 1.f) * sg * h.inv_b;
              dmax = fmaxf(dmax, d);
            } else {
              const float e = y - q[n][r];
              if (n == 0) acc0 += e * e; else acc1 += e * e;
              dq[n][r] = -e * h.inv_b;
            }
          }
          if (h.lap && lane == 0) GW(h.prio)[b] = (float)pow((double)fmaxf(dmax, 1.f), 0.4);
          want_dz = true;
          break;
        }
        case HEAD_TD7_POLICY: {  // td7.py:274-275
          acc0 += q[0][r] + q[1][r];
          dq[0][r] = dq[1][r] = -0.5f * h.inv_b;
          want_dz = true;
          break;
        }
        case HEAD_MLP_POLICY: {  // td3.py:191, sac.py:227-229
          const float mn = fminf(q[0][r], q[1][r]);
          // torch.minimum backward: ties split the gradient
          const float gq = -h.inv_b;
          dq[0][r] = q[0][r] < q[1][r] ? gq : (q[0][r] == q[1][r] ? 0.5f * gq : 0.f);
          dq[1][r] = q[1][r] < q[0][r] ? gq : (q[0][r] == q[1][r] ? 0.5f * gq : 0.f);
          if (h.sac) {
            const float lp = G(h.logpi)[b];
            acc0 += -mn + lp * expf(G(h.log_alpha)[0]);
            acc1 += lp;
          } else {
            acc0 += mn;
          }
          want_dz = true;
          break;
        }
      }
    }
    if (want_dz) {
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        if (lane == 0 && h.dq[n].t) mat_st4(h.dq[n], r0, 0, make_float4(dq[n][0], dq[n][1], dq[n][2], dq[n][3]));
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = lane + 64 * u;
          if (u < per && k < h.H) {
            const float4 d = mat_ld4(h.dsrc[n], r0, k);
            const float w = wv[n][u];
            mat_st4(h.dz[n], r0, k,
                    make_float4((dq[n][0] * w) * act_bwd(h.dact, d.x), (dq[n][1] * w) * act_bwd(h.dact, d.y),
                                (dq[n][2] * w) * act_bwd(h.dact, d.z), (dq[n][3] * w) * act_bwd(h.dact, d.w)));
          }
        }
      }
    }
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
  if (threadIdx.x == 0) {
    if (h.loss_part) {
      GAS float* lp = GW(h.loss_part);
      lp[t * 4 + 0] = (red[0] + red[2]) + (red[4] + red[6]);
      lp[t * 4 + 1] = (red[1] + red[3]) + (red[5] + red[7]);
      lp[t * 4 + 2] = 0.f;
      lp[t * 4 + 3] = 0.f;
    }
    if (h.mode == HEAD_TD7_TARGET) {  // value_max / value_min tracking (td7.py:217-218)
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

// ---------------------------------------------------------------- replay sampling

constexpr int kBlk = 4096;  // priorities per block-sum

// Exact fp64 block sums of the priorities (lap.py:47; Q8: any-order fp64 is exact).
__device__ __forceinline__ void op_sample_reduce(const CAS SampleArgs& s, int t, float* smem) {
  const long long size = *G(s.size);
  const long long base = (long long)t * kBlk;
  double acc = 0.0;
#pragma unroll
  for (int u = 0; u < kBlk / (4 * kThreads); ++u) {
    const long long k = base + (long long)(u * kThreads + threadIdx.x) * 4;
    if (k + 3 < size) {
      const float4 v = ld4g(G(s.priority) + k);
      acc += ((double)v.x + (double)v.y) + ((double)v.z + (double)v.w);
    } else {
      for (int e = 0; e < 4; ++e)
        if (k + e < size) acc += (double)G(s.priority)[k + e];
    }
  }
  acc = wave_sum_d(acc);
  double* dred = reinterpret_cast<double*>(smem);
  if ((threadIdx.x & 63) == 0) dred[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) GW(s.bsum)[t] = (dred[0] + dred[1]) + (dred[2] + dred[3]);
}

// Exclusive scan of 256 per-thread doubles held in LDS, by one wave, fixed order.
__device__ __forceinline__ void scan256(double* tsum) {
  const int tid = threadIdx.x;
  if (tid < 64) {
    const double v0 = tsum[4 * tid], v1 = tsum[4 * tid + 1], v2 = tsum[4 * tid + 2], v3 = tsum[4 * tid + 3];
    const double s4 = ((v0 + v1) + v2) + v3;
    double inc = s4;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double nv = __shfl_up(inc, o, 64);
      if (tid >= o) inc += nv;
    }
    const double ex = inc - s4;
    tsum[4 * tid] = ex;
    tsum[4 * tid + 1] = ex + v0;
    tsum[4 * tid + 2] = (ex + v0) + v1;
    tsum[4 * tid + 3] = ((ex + v0) + v1) + v2;
  }
}

// One workgroup per query: uniform / LAP index search (searchsorted left over the
// fp32-rounded exact prefix), noise for this row, then the coalesced row gather.
__device__ __forceinline__ void op_sample_gather(const CAS SampleArgs& s, int b, float* smem) {
  const int tid = threadIdx.x;
  const long long size = *G(s.size);
  const int tape = *G(s.tape_mode);
  const long long pos = *G(s.tape_pos);
  const uint2 key = make_uint2((unsigned)s.seed, (unsigned)(s.seed >> 32));
  const unsigned long long step = (unsigned long long)*G(s.ctrl_rng);
  // noise tensors for this row (T images)
  for (int j = tid; j < s.A; j += kThreads) {
    float e, e2 = 0.f;
    if (tape) {
      e = G(s.tape_eps)[((size_t)pos * s.B + b) * s.A + j];
      if (s.eps2.t) e2 = G(s.tape_eps2)[((size_t)pos * s.B + b) * s.A + j];
    } else {
      const uint4 r = philox(key, make_uint4((unsigned)(b * s.A + j), 1u, (unsigned)step, (unsigned)(step >> 32)));
      e = normal_from(r.x, r.y);
      e2 = normal_from(r.z, r.w);
    }
    mat_st(s.eps, b, j, e);
    if (s.eps2.t) mat_st(s.eps2, b, j, e2);
  }
  long long* found = reinterpret_cast<long long*>(smem);  // [1]
  double* tsum = reinterpret_cast<double*>(smem) + 2;     // [256]
  double* pref = tsum + kThreads;                         // [nb <= 2048]
  long long ind;
  if (tape == 2) {
    ind = G(s.tape_ind)[(size_t)pos * s.B + b];
  } else {
    float u;
    if (tape) u = G(s.tape_u)[(size_t)pos * s.B + b];
    else u = u01(philox(key, make_uint4((unsigned)b, 0u, (unsigned)step, (unsigned)(step >> 32))).x);
    if (tid == 0) GW(s.u_out)[b] = u;
    if (!s.lap) {
      // searchsorted(cumsum(ones(size)), u*size): first j in 1..size with j >= v
      const float v = u * (float)size;
      const long long k = (long long)ceilf(v) - 1;
      ind = k < 0 ? 0 : (k > size - 1 ? size - 1 : k);
    } else {
      // exact fp64 prefix over block sums, rounded to fp32 per element (Q8)
      const int nb = (int)((size + kBlk - 1) / kBlk);
      const int per = (nb + kThreads - 1) / kThreads;
      double loc = 0.0;
      for (int q = 0; q < per; ++q) {
        const int k = tid * per + q;
        if (k < nb) {
          loc += G(s.bsum)[k];
          pref[k] = loc;
        }
      }
      tsum[tid] = loc;
      __syncthreads();
      scan256(tsum);
      __syncthreads();
      const double off = tsum[tid];
      for (int q = 0; q < per; ++q) {
        const int k = tid * per + q;
        if (k < nb) pref[k] += off;
      }
      __syncthreads();
      const float total = (float)pref[nb - 1];
      const float v = u * total;
      // first block whose rounded inclusive prefix >= v (monotone)
      int lo = 0, hi = nb - 1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((float)pref[mid] >= v) hi = mid;
        else lo = mid + 1;
      }
      const double base = lo ? pref[lo - 1] : 0.0;
      const long long e0 = (long long)lo * kBlk + (long long)tid * 16;
      // each thread owns 16 consecutive priorities of the block
      float pv[16];
      double tl = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        pv[q] = (e0 + q < size) ? G(s.priority)[e0 + q] : 0.f;
        tl += (double)pv[q];
      }
      __syncthreads();
      tsum[tid] = tl;
      if (tid == 0) *found = 0x7FFFFFFFFFFFFFFFll;
      __syncthreads();
      scan256(tsum);
      __syncthreads();
      double run = base + tsum[tid];
      long long mine = 0x7FFFFFFFFFFFFFFFll;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        run += (double)pv[q];
        if (mine == 0x7FFFFFFFFFFFFFFFll && e0 + q < size && (float)run >= v) mine = e0 + q;
      }
      if (mine != 0x7FFFFFFFFFFFFFFFll) atomicMin((unsigned long long*)found, (unsigned long long)mine);
      __syncthreads();
      ind = *found;
      if (ind >= size) ind = size - 1;
    }
  }
  // gather the transition into the batch images (rows b and B + b of ss)
  const GAS float* st = G(s.state) + (size_t)ind * s.Sp;
  const GAS float* nst = G(s.next_state) + (size_t)ind * s.Sp;
  for (int k = tid; k < s.Sp; k += kThreads) {
    mat_st(s.ss, b, k, st[k]);
    mat_st(s.ss, s.B + b, k, nst[k]);
  }
  const GAS float* ac = G(s.action) + (size_t)ind * s.Ap;
  for (int k = tid; k < s.Ap; k += kThreads) mat_st(s.a, b, k, ac[k]);
  if (tid == 0) {
    GW(s.r)[b] = G(s.reward)[ind];
    GW(s.nd)[b] = G(s.notdone)[ind];
    GW(s.ind)[b] = ind;
  }
}

// LAPReplayMemory.update_priority (lap.py:66-69): last duplicate wins (Q9).
__device__ __forceinline__ void op_priority(const CAS PriorityArgs& a, float* smem) {
  long long* sind = reinterpret_cast<long long*>(smem);
  float* red = smem + 2 * 1024;
  for (int b = threadIdx.x; b < a.B; b += kThreads) sind[b] = G(a.ind)[b];
  __syncthreads();
  float mx = -INFINITY;
  for (int b = threadIdx.x; b < a.B; b += kThreads) {
    const long long me = sind[b];
    bool last = true;
    for (int c = b + 1; c < a.B; ++c)
      if (sind[c] == me) {
        last = false;
        break;
      }
    const float pv = G(a.p)[b];
    if (last) GW(a.priority)[me] = pv;
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
  const float w = expf(G(s.log_alpha)[0]) * s.inv_b;  // d obj / d logpi_b
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

// Deterministic workgroup sum of p[i*stride], i < n (fixed strided + tree order).
__device__ float block_sum(const float* p, int n, int stride, float* red) {
  const GAS float* q = G(p);
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += kThreads) s += q[(size_t)i * stride];
  return wg_sum(s, red);
}

__device__ __forceinline__ void op_step_end(const CAS StepEndArgs& a, float* smem) {
  float* red = smem;
  float* vals = smem + 8;
  const float nanv = __int_as_float(0x7FC00000);
  const float slp = a.logpi_part ? block_sum(a.logpi_part + 1, a.nlogpi, 4, red) : 0.f;
  for (int k = 0; k < a.ninfo; ++k) {
    float v = 0.f;
    if (a.kind[k] == INFO_SUM || a.kind[k] == INFO_SAC_POL) {
      v = block_sum(a.part[k], a.npart[k], a.stride[k], red);
    } else if (a.kind[k] == INFO_GNORM) {
      // per-tensor sum of squares -> sqrt -> sum (rl/nn/utils.py:13-19)
      for (int q = 0; q < a.ngsq_t; ++q) {
        const float ss = block_sum(a.gsq + a.gsq_off[q], a.gsq_off[q + 1] - a.gsq_off[q], 1, red);
        v += sqrtf(ss);
      }
    }
    if (threadIdx.x == 0) vals[k] = v;
  }
  if (threadIdx.x != 0) return;
  const float la = a.log_alpha ? G(a.log_alpha)[0] : 0.f;
  const float alpha = expf(la);
  // mean_b(-lp_b - target_entropy); d/dla mean(exp(la) * c) = exp(la) * mean(c)
  const float gmean = (-slp) * a.inv_b - a.target_entropy;
  const float tmp_obj = alpha * gmean;
  for (int k = 0; k < a.ninfo; ++k) {
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
    vals[k] = v;
  }
  if (a.log_alpha && a.la_lr > 0.f) {  // optim_tmp.step (sac.py:283)
    const float g = tmp_obj;
    const double tt = (double)(G(a.la_t)[0] + 1);
    const double bc1 = 1.0 - pow(0.9, tt), bc2 = 1.0 - pow(0.999, tt);
    float m = G(a.la_m)[0], v2 = G(a.la_v)[0];
    m = m + (1.f - 0.9f) * (g - m);
    v2 = v2 * 0.999f + ((1.f - 0.999f) * g) * g;
    const float denom = sqrtf(v2) / (float)sqrt(bc2) + 1e-8f;
    GW(a.la_m)[0] = m;
    GW(a.la_v)[0] = v2;
    GW(a.log_alpha)[0] = la + (-(float)(a.la_lr / bc1) * m) / denom;
    GW(a.la_t)[0] += 1;
  }
  if (a.info_slot) {
    int slot = G(a.info_slot)[0];
    if (slot >= a.info_cap) slot = a.info_cap - 1;
    for (int k = 0; k < a.ninfo; ++k) GW(a.info)[(size_t)slot * kInfoMax + k] = vals[k];
    GW(a.info_slot)[0] = slot + 1;
  }
  for (int c = 0; c < 16; ++c)
    if (a.cmask & (1 << c)) GW(a.counters)[c] += 1;
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

__device__ __forceinline__ void op_ctrl(const CAS CtrlArgs& c) {
  if (threadIdx.x == 0) {
    GW(c.vt)[0] = unkey(G(c.vmax_key)[0]);
    GW(c.vt)[1] = unkey(G(c.vmin_key)[0]);
  }
}

// ---------------------------------------------------------------- dispatch

__global__ __launch_bounds__(kThreads) void rle_level(const LevelArgs la) {
  __shared__ __attribute__((aligned(16))) float smem[6144];  // 24 KB
  const CAS Op* ops = (const CAS Op*)la.ops;
  const int wg = blockIdx.x;
  // op of this workgroup: from the kernel-argument table (SGPRs, no dependent
  // descriptor loads), or by scanning descriptors for an oversized level
  int k = 0, kind;
  if (la.nops <= kLevelOps) {
#pragma unroll
    for (int q = 1; q < kLevelOps; ++q) k = (q < la.nops && la.wg_begin[q] <= wg) ? q : k;
    kind = la.kind[k];
  } else {
    while (k + 1 < la.nops && ops[k + 1].wg_begin <= wg) ++k;
    kind = ops[k].kind;
  }
  const CAS Op& op = ops[k];
  const int t = wg - (la.nops <= kLevelOps ? la.wg_begin[k] : op.wg_begin);
  switch (kind) {
    case OP_GEMM: op_gemm(op.gemm, t, smem); break;
    case OP_NORMBWD: op_normbwd(op.nb, t); break;
    case OP_SAMPLE_REDUCE: op_sample_reduce(op.sample, t, smem); break;
    case OP_SAMPLE_GATHER: op_sample_gather(op.sample, t, smem); break;
    case OP_HEAD: op_head(op.head, t, smem); break;
    case OP_PRIORITY: op_priority(op.prio, smem); break;
    case OP_SAC_ACTOR: op_sac_actor(op.sac, t); break;
    case OP_SAC_ACTOR_BWD: op_sac_actor_bwd(op.sac, t); break;
    case OP_STEP_END: op_step_end(op.end, smem); break;
    case OP_POLYAK: op_polyak(op.flat, t); break;
    case OP_COPY: op_copy(op.flat, t); break;
    case OP_MAXRED: op_maxred(op.flat, t, smem); break;
    case OP_CTRL: op_ctrl(op.ctrl); break;
    default: break;
  }
}

// ---------------------------------------------------------------- standalone kernels

// Scatter `count` staged transitions into the ring at ptr (wrapping).
__global__ void rle_append_kernel(float* state, float* next_state, float* action, float* reward, float* notdone,
                                  float* priority, const float* st_s, const float* st_ns, const float* st_a,
                                  const float* st_r, const float* st_d, long long ptr, long long cap, int count,
                                  int Sp, int Ap, const float* max_priority, int lap) {
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
    if (lap) priority[row] = *max_priority;
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

hipError_t launch_level(const Op* d_ops, const Op* h_ops, int nops, int nwg, hipStream_t st) {
  LevelArgs la{};
  la.ops = d_ops;
  la.nops = nops;
  for (int q = 0; q < nops && q < kLevelOps; ++q) {
    la.wg_begin[q] = h_ops[q].wg_begin;
    la.kind[q] = (unsigned char)h_ops[q].kind;
  }
  hipLaunchKernelGGL(rle_level, dim3(nwg), dim3(kThreads), 0, st, la);
  return hipGetLastError();
}
hipError_t launch_append(float* state, float* next_state, float* action, float* reward, float* notdone,
                         float* priority, const float* st_s, const float* st_ns, const float* st_a,
                         const float* st_r, const float* st_d, long long ptr, long long cap, int count, int Sp,
                         int Ap, const float* max_priority, int lap, hipStream_t st) {
  hipLaunchKernelGGL(rle_append_kernel, dim3(count), dim3(256), 0, st, state, next_state, action, reward, notdone,
                     priority, st_s, st_ns, st_a, st_r, st_d, ptr, cap, count, Sp, Ap, max_priority, lap);
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
