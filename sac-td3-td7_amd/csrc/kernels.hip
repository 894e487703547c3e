// Device side of the MI355X off-policy update engine (gfx950 / CDNA4).
//
// A gradient step is a DAG of ops scheduled into dependency levels on the
// host (engine.cpp).  Each level is ONE launch of `rle_level`, whose
// workgroups are partitioned over that level's ops (Op::wg_begin); every
// workgroup is 256 threads (4 waves of 64).  The whole step is captured into
// a hipGraph, so one gradient step = one graph launch, no host sync.
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

namespace rle {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- utilities

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

// Ordered-int key of a float: monotone under signed int comparison.
__device__ __forceinline__ int fkey(float f) {
  int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float unkey(int k) {
  return __int_as_float(k >= 0 ? k : k ^ 0x7FFFFFFF);
}

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
  float s = 0.f;
  for (int p = 0; p < nparts; ++p) s += part[(size_t)p * ld + row];
  float m = s / (float)width;
  return m < 1e-8f ? 1e-8f : m;
}

// ---------------------------------------------------------------- GEMM

struct OpTables {
  float inv_lane[kMaxSeg];      // contiguous+normed segs: 1/m for this lane's x
  int tab_off[kMaxSeg];         // strided+normed segs: LDS table offset (or -1)
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ float4 load_operand(const Operand& op, int x, int r, const OpTables& tb,
                                               const float* tabs) {
  for (int s = 0; s < op.nseg; ++s) {
    const Seg& sg = op.seg[s];
    if (x >= sg.x0 && x < sg.x1 && r >= sg.r0 && r < sg.r1) {
      float4 v;
      if (!sg.strided) {
        v = ld4(sg.p + (size_t)(x - sg.x0) * sg.ld + (r - sg.r0));
        if (sg.norm) {
          float iv = tb.inv_lane[s];
          v.x *= iv; v.y *= iv; v.z *= iv; v.w *= iv;
        }
      } else {
        const float* q = sg.p + (size_t)(r - sg.r0) * sg.ld + (x - sg.x0);
        const int nr = sg.r1 - r;  // rows past r1 (reduction padding) read as zero
        v.x = q[0];
        v.y = nr > 1 ? q[sg.ld] : 0.f;
        v.z = nr > 2 ? q[2 * sg.ld] : 0.f;
        v.w = nr > 3 ? q[3 * sg.ld] : 0.f;
        if (sg.norm) {
          const float* t = tabs + tb.tab_off[s] + (r - sg.r0);
          v.x *= t[0];
          if (nr > 1) v.y *= t[1];
          if (nr > 2) v.z *= t[2];
          if (nr > 3) v.w *= t[3];
        }
      }
      return v;
    }
  }
  return make_float4(0.f, 0.f, 0.f, 0.f);
}

// Builds per-lane inverse norms and LDS tables for normed segments.
__device__ void prep_tables(const Operand& op, int x, OpTables& tb, float* tabs, int& tab_used) {
  for (int s = 0; s < kMaxSeg; ++s) {
    tb.inv_lane[s] = 1.f;
    tb.tab_off[s] = -1;
  }
  for (int s = 0; s < op.nseg; ++s) {
    const Seg& sg = op.seg[s];
    if (!sg.norm) continue;
    if (!sg.strided) {
      if (x >= sg.x0 && x < sg.x1)
        tb.inv_lane[s] = 1.f / norm_m(sg.norm, sg.norm_ld, x - sg.x0 + sg.norm_row0, sg.norm_nparts,
                                      sg.norm_width);
    } else {
      int n = sg.r1 - sg.r0;
      tb.tab_off[s] = tab_used;
      for (int i = threadIdx.x; i < n; i += kThreads)
        tabs[tab_used + i] =
            1.f / norm_m(sg.norm, sg.norm_ld, i + sg.norm_row0, sg.norm_nparts, sg.norm_width);
      tab_used += (n + 3) & ~3;
    }
  }
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

__device__ void op_gemm(const GemmArgs& g, int t, float* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int it = t / g.tiles_n, jt = t - it * g.tiles_n;
  const int i0 = it * kTile, j0 = jt * kTile;
  const bool bias_tile = (g.epi == EPI_ADAM) && (j0 >= g.adam.bias_col);
  float* red = smem;             // [4][256]
  float* tabs = smem + 4 * 256;  // normalisation tables
  const int xa = i0 + (lane & 15), xb = j0 + (lane & 15), rl = 4 * (lane >> 4);

  OpTables ta, tbb;
  int used = 0;
  prep_tables(g.A, xa, ta, tabs, used);
  if (!bias_tile) prep_tables(g.B, xb, tbb, tabs, used);
  if (used) __syncthreads();

  const int nch = (g.R + 15) >> 4;
  const int c0 = (nch * wave) >> 2, c1 = (nch * (wave + 1)) >> 2;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const float bone = (xb == g.adam.bias_col) ? 1.f : 0.f;
  for (int c = c0; c < c1; ++c) {
    const int r = c * 16 + rl;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (xa < g.M && r < g.R) a = load_operand(g.A, xa, r, ta, tabs);
    if (bias_tile) {
      if (r < g.R) b = make_float4(bone, bone, bone, bone);
    } else if (xb < g.N && r < g.R) {
      b = load_operand(g.B, xb, r, tbb, tabs);
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
  }
  // C layout (16x16x4): lane l holds rows 4*(l>>4)+q, col l&15.
#pragma unroll
  for (int q = 0; q < 4; ++q) red[wave * 256 + (4 * (lane >> 4) + q) * 16 + (lane & 15)] = acc[q];
  __syncthreads();
  float v = red[tid] + red[256 + tid] + red[512 + tid] + red[768 + tid];
  const int row = tid >> 4, col = tid & 15;
  const int i = i0 + row, j = j0 + col;

  if (g.epi == EPI_STORE) {
    float y = 0.f;
    const bool ok = (i < g.M) && (j < g.N);
    if (ok) {
      if (g.bias) v += g.bias[j];
      if (g.pre) g.pre[(size_t)i * g.ldpre + j] = v;
      y = act_fwd(g.act, v);
      if (g.noise && i >= g.noise_row0) {
        float e = g.noise[(size_t)(i - g.noise_row0) * g.ldnoise + j] * g.noise_sigma;
        e = fminf(fmaxf(e, -g.noise_clip), g.noise_clip);
        y = fminf(fmaxf(y + e, -1.f), 1.f);
      }
      if (g.dsrc) y *= act_bwd(g.dact, g.dsrc[(size_t)i * g.lddact + j]);
      g.out[(size_t)i * g.ldo + j] = y;
    }
    if (g.norm_out) {
      float s = ok ? fabsf(y) : 0.f;
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (col == 0 && i < g.M) g.norm_out[(size_t)jt * g.norm_ld + i] = s;
    }
  } else if (g.epi == EPI_MSE) {
    float d2 = 0.f;
    if (i < g.M && j < g.N) {
      if (g.bias) v += g.bias[j];
      const Seg& sg = g.tgt;
      float tv = sg.p[(size_t)(i - sg.x0) * sg.ld + j];
      if (sg.norm)
        tv *= 1.f / norm_m(sg.norm, sg.norm_ld, i - sg.x0 + sg.norm_row0, sg.norm_nparts, sg.norm_width);
      float d = v - tv;
      g.out[(size_t)i * g.ldo + j] = (2.f * d) * g.mse_scale;  // mse_scale = 1/n
      d2 = d * d;
    }
    d2 = wave_sum(d2);
    __syncthreads();
    if (lane == 0) red[wave] = d2;
    __syncthreads();
    if (tid == 0) g.loss_part[t] = red[0] + red[1] + red[2] + red[3];
  } else {  // EPI_ADAM (torch.optim.Adam single-tensor law, see oracle/agents.py)
    const AdamArgs& ad = g.adam;
    float* p = nullptr;
    if (bias_tile) {
      if (j == ad.bias_col && i < g.M) p = ad.b + i;
    } else if (i < g.M && j < g.N) {
      p = ad.w + (size_t)i * ad.ldw + j;
    }
    float gg = 0.f;
    if (p) {
      const double tt = (double)(*ad.t + 1);
      const double bc1 = 1.0 - pow((double)ad.beta1, tt);
      const double bc2 = 1.0 - pow((double)ad.beta2, tt);
      const float step_size = (float)((double)ad.lr / bc1);
      const float bc2s = (float)sqrt(bc2);
      float* m = p + ad.mo;
      float* vv = p + ad.vo;
      float mm = *m, v2 = *vv;
      mm = mm + (1.f - ad.beta1) * (v - mm);
      v2 = v2 * ad.beta2 + ((1.f - ad.beta2) * v) * v;
      const float denom = sqrtf(v2) / bc2s + ad.eps;
      *m = mm;
      *vv = v2;
      *p = *p + (-step_size * mm) / denom;
      gg = v * v;
    }
    if (ad.gsq) {
      gg = wave_sum(gg);
      __syncthreads();
      if (lane == 0) red[wave] = gg;
      __syncthreads();
      if (tid == 0) {
        float s = red[0] + red[1] + red[2] + red[3];
        if (bias_tile) ad.gsq_b[it] = s;
        else ad.gsq[it * (g.tiles_n - 1) + jt] = s;
      }
    }
  }
}

// ---------------------------------------------------------------- AvgL1Norm backward

__device__ void op_normbwd(const NormBwdArgs& a, int t) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = t * 4 + wave;
  if (row >= a.rows) return;
  const float* x = a.x + (size_t)row * a.ldx;
  const float* g = a.g + (size_t)row * a.ldg;
  // m recomputed from the same partials the forward consumers used
  float s = 0.f;
  for (int p = 0; p < a.norm_nparts; ++p) s += a.norm[(size_t)p * a.norm_ld + row + a.norm_row0];
  const float mean = s / (float)a.width;
  const bool clamped = mean < 1e-8f;
  const float m = clamped ? 1e-8f : mean;
  const float inv = 1.f / m;
  float dot = 0.f;
  for (int k = lane; k < a.width; k += 64) dot += g[k] * x[k];
  dot = wave_sum(dot);
  // y = x / m: dy/dx path g/m ; dm path -(sum g x)/m^2 * sign(x)/n (unless clamped)
  const float gm = clamped ? 0.f : (-dot * inv * inv) / (float)a.width;
  float* dx = a.dx + (size_t)row * a.lddx;
  for (int k = lane; k < a.width; k += 64) {
    const float xv = x[k];
    const float sg = xv > 0.f ? 1.f : (xv < 0.f ? -1.f : 0.f);
    dx[k] = g[k] * inv + sg * gm;
  }
}

// ---------------------------------------------------------------- critic heads

__device__ void op_head(const HeadArgs& h, int t, float* smem) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = t * 4 + wave;
  float acc0 = 0.f, acc1 = 0.f;  // per-row loss terms
  float ykey = 0.f;
  bool valid = b < h.rows;
  if (valid) {
    float q[2];
    for (int n = 0; n < 2; ++n) {
      const float* hr = h.h[n] + (size_t)b * h.ldh;
      float s = 0.f;
      for (int k = lane; k < h.H; k += 64) s += hr[k] * h.w[n][k];
      q[n] = wave_sum(s) + h.b[n][0];
    }
    float dq[2] = {0.f, 0.f};
    bool want_dz = false;
    switch (h.mode) {
      case HEAD_TD7_TARGET: {
        float v = fminf(q[0], q[1]);
        v = fminf(fmaxf(v, h.vt[1]), h.vt[0]);
        float y = h.reward[b] + (h.gamma * v) * h.notdone[b];
        if (lane == 0) h.y[b] = y;
        ykey = y;
        break;
      }
      case HEAD_MLP_TARGET: {
        float v = fminf(q[0], q[1]);
        if (h.sac) v = v - expf(h.log_alpha[0]) * h.logpi[b];
        float y = h.reward[b] + (h.gamma * v) * h.notdone[b];
        if (lane == 0) h.y[b] = y;
        break;
      }
      case HEAD_TD7_LOSS:
      case HEAD_MLP_LOSS: {
        const float y = h.y[b];
        float dmax = 0.f;
        for (int n = 0; n < 2; ++n) {
          const float diff = q[n] - y;
          if (h.lap) {
            const float d = fabsf(diff);
            const float hub = d < 1.f ? 0.5f * (d * d) : d;
            if (n == 0) acc0 += hub; else acc1 += hub;
            const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
            dq[n] = (d < 1.f ? d : 1.f) * sg * h.inv_b;
            dmax = fmaxf(dmax, d);
          } else {
            const float e = y - q[n];
            if (n == 0) acc0 += e * e; else acc1 += e * e;
            dq[n] = -e * h.inv_b;
          }
        }
        if (h.lap && lane == 0) h.prio[b] = (float)pow((double)fmaxf(dmax, 1.f), 0.4);
        want_dz = true;
        break;
      }
      case HEAD_TD7_POLICY: {
        acc0 = q[0] + q[1];
        dq[0] = dq[1] = -0.5f * h.inv_b;
        want_dz = true;
        break;
      }
      case HEAD_MLP_POLICY: {
        const float mn = fminf(q[0], q[1]);
        // torch.minimum backward: ties split the gradient
        const float g = -h.inv_b;
        dq[0] = q[0] < q[1] ? g : (q[0] == q[1] ? 0.5f * g : 0.f);
        dq[1] = q[1] < q[0] ? g : (q[0] == q[1] ? 0.5f * g : 0.f);
        if (h.sac) {
          const float lp = h.logpi[b];
          acc0 = -mn + lp * expf(h.log_alpha[0]);
          acc1 = lp;
        } else {
          acc0 = mn;
        }
        want_dz = true;
        break;
      }
    }
    if (want_dz) {
      for (int n = 0; n < 2; ++n) {
        if (lane == 0 && h.dq[n]) h.dq[n][b] = dq[n];
        const float* ds = h.dsrc[n] + (size_t)b * h.ldd;
        float* dz = h.dz[n] + (size_t)b * h.lddz;
        for (int k = lane; k < h.H; k += 64) dz[k] = (dq[n] * h.w[n][k]) * act_bwd(h.dact, ds[k]);
      }
    }
  }
  // workgroup partials (fixed order) + value tracking
  float* red = smem;
  int* ired = reinterpret_cast<int*>(smem + 16);
  if (lane == 0) {
    red[wave * 2 + 0] = valid ? acc0 : 0.f;
    red[wave * 2 + 1] = valid ? acc1 : 0.f;
    ired[wave * 2 + 0] = valid ? fkey(ykey) : (int)0x80000000;
    ired[wave * 2 + 1] = valid ? fkey(ykey) : (int)0x7FFFFFFF;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (h.loss_part) {
      h.loss_part[t * 4 + 0] = red[0] + red[2] + red[4] + red[6];
      h.loss_part[t * 4 + 1] = red[1] + red[3] + red[5] + red[7];
    }
    if (h.mode == HEAD_TD7_TARGET) {
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

__device__ void op_sample_reduce(const SampleArgs& s, int t, float* smem) {
  const long long size = *s.size;
  const long long base = (long long)t * kBlk;
  double acc = 0.0;
  for (int k = threadIdx.x; k < kBlk; k += kThreads) {
    long long i = base + k;
    if (i < size) acc += (double)s.priority[i];
  }
  acc = wave_sum_d(acc);
  double* dred = reinterpret_cast<double*>(smem);
  if ((threadIdx.x & 63) == 0) dred[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) s.bsum[t] = dred[0] + dred[1] + dred[2] + dred[3];
}

__device__ void op_sample_gather(const SampleArgs& s, int b, float* smem) {
  const int tid = threadIdx.x;
  const long long size = *s.size;
  const int tape = *s.tape_mode;
  const long long pos = *s.tape_pos;
  const uint2 key = make_uint2((unsigned)s.seed, (unsigned)(s.seed >> 32));
  const unsigned long long step = (unsigned long long)*s.ctrl_rng;
  // noise tensors for this row
  for (int j = tid; j < s.A; j += kThreads) {
    float e, e2 = 0.f;
    if (tape) {
      e = s.tape_eps[((size_t)pos * s.B + b) * s.A + j];
      if (s.eps2) e2 = s.tape_eps2[((size_t)pos * s.B + b) * s.A + j];
    } else {
      uint4 r = philox(key, make_uint4((unsigned)(b * s.A + j), 1u, (unsigned)step, (unsigned)(step >> 32)));
      e = normal_from(r.x, r.y);
      e2 = normal_from(r.z, r.w);
    }
    s.eps[(size_t)b * s.ldeps + j] = e;
    if (s.eps2) s.eps2[(size_t)b * s.ldeps + j] = e2;
  }
  __shared__ long long found_s;
  long long ind;
  if (tape == 2) {
    ind = s.tape_ind[(size_t)pos * s.B + b];
  } else {
    float u;
    if (tape) u = s.tape_u[(size_t)pos * s.B + b];
    else u = u01(philox(key, make_uint4((unsigned)b, 0u, (unsigned)step, (unsigned)(step >> 32))).x);
    if (tid == 0) s.u_out[b] = u;
    if (!s.lap) {
      // searchsorted(cumsum(ones(size)), u*size): first j in 1..size with j >= v
      const float v = u * (float)size;
      long long k = (long long)ceilf(v) - 1;
      ind = k < 0 ? 0 : (k > size - 1 ? size - 1 : k);
    } else {
      // exact fp64 prefix over block sums, rounded to fp32 per element (Q8)
      double* pref = reinterpret_cast<double*>(smem);          // [nb]
      double* wsum = pref + 2048;                              // [4]
      const int nb = (int)((size + kBlk - 1) / kBlk);
      const int per = (nb + kThreads - 1) / kThreads;
      double loc = 0.0;
      for (int q = 0; q < per; ++q) {
        int k = tid * per + q;
        if (k < nb) { loc += s.bsum[k]; pref[k] = loc; }
      }
      // exclusive scan of thread totals
      double* tsum = wsum + 8;                                  // [256]
      tsum[tid] = loc;
      __syncthreads();
      if (tid == 0) {
        double run = 0.0;
        for (int q = 0; q < kThreads; ++q) { double x = tsum[q]; tsum[q] = run; run += x; }
      }
      __syncthreads();
      const double off = tsum[tid];
      for (int q = 0; q < per; ++q) {
        int k = tid * per + q;
        if (k < nb) pref[k] += off;
      }
      __syncthreads();
      const float total = (float)pref[nb - 1];
      const float v = u * total;
      // first block whose rounded inclusive prefix >= v (monotone)
      int lo = 0, hi = nb - 1;
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if ((float)pref[mid] >= v) hi = mid; else lo = mid + 1;
      }
      const int blk = lo;
      const double base = blk ? pref[blk - 1] : 0.0;
      const long long e0 = (long long)blk * kBlk;
      // each thread owns 16 consecutive priorities of the block
      double tl = 0.0;
      float pv[16];
      for (int q = 0; q < 16; ++q) {
        long long i = e0 + tid * 16 + q;
        pv[q] = (i < size) ? s.priority[i] : 0.f;
        tl += (double)pv[q];
      }
      __syncthreads();
      tsum[tid] = tl;
      if (tid == 0) found_s = 0x7FFFFFFFFFFFFFFFll;
      __syncthreads();
      if (tid == 0) {
        double run = 0.0;
        for (int q = 0; q < kThreads; ++q) { double x = tsum[q]; tsum[q] = run; run += x; }
      }
      __syncthreads();
      double run = base + tsum[tid];
      long long mine = 0x7FFFFFFFFFFFFFFFll;
      for (int q = 0; q < 16; ++q) {
        long long i = e0 + tid * 16 + q;
        run += (double)pv[q];
        if (i < size && (float)run >= v) { mine = i; break; }
      }
      if (mine != 0x7FFFFFFFFFFFFFFFll) atomicMin((unsigned long long*)&found_s, (unsigned long long)mine);
      __syncthreads();
      ind = found_s;
      if (ind >= size) ind = size - 1;
    }
  }
  // gather the transition (coalesced float4 copies)
  const float4* st = reinterpret_cast<const float4*>(s.state + (size_t)ind * s.Sp);
  const float4* nst = reinterpret_cast<const float4*>(s.next_state + (size_t)ind * s.Sp);
  float4* d0 = reinterpret_cast<float4*>(s.ss + (size_t)b * s.ldss);
  float4* d1 = reinterpret_cast<float4*>(s.ss + (size_t)(s.B + b) * s.ldss);
  for (int k = tid; k < s.Sp / 4; k += kThreads) {
    d0[k] = st[k];
    d1[k] = nst[k];
  }
  const float4* ac = reinterpret_cast<const float4*>(s.action + (size_t)ind * s.Ap);
  float4* da = reinterpret_cast<float4*>(s.a + (size_t)b * s.lda);
  for (int k = tid; k < s.Ap / 4; k += kThreads) da[k] = ac[k];
  if (tid == 0) {
    s.r[b] = s.reward[ind];
    s.nd[b] = s.notdone[ind];
    s.ind[b] = ind;
  }
}

// LAPReplayMemory.update_priority (lap.py:66-69): last duplicate wins (Q9).
__device__ void op_priority(const PriorityArgs& a, float* smem) {
  long long* sind = reinterpret_cast<long long*>(smem);
  float* red = smem + 2 * 1024;
  for (int b = threadIdx.x; b < a.B; b += kThreads) sind[b] = a.ind[b];
  __syncthreads();
  float mx = -INFINITY;
  for (int b = threadIdx.x; b < a.B; b += kThreads) {
    const long long me = sind[b];
    bool last = true;
    for (int c = b + 1; c < a.B; ++c)
      if (sind[c] == me) { last = false; break; }
    const float pv = a.p[b];
    if (last) a.priority[me] = pv;
    mx = fmaxf(mx, pv);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    *a.max_priority = fmaxf(m, *a.max_priority);
  }
}

// ---------------------------------------------------------------- SAC Gaussian-tanh

__device__ void op_sac_actor(const SacActorArgs& s, int t) {
  const int b = t * kThreads + threadIdx.x;
  if (b >= s.rows) return;
  const float* o = s.out + (size_t)b * s.ldo;
  const float* e = (b < s.eps_row_split) ? s.eps2 + (size_t)b * s.ldeps
                                         : s.eps + (size_t)(b - s.eps_row_split) * s.ldeps;
  const float c = (float)0.9189385332046727;  // log(sqrt(2*pi))
  float lp = 0.f, corr = 0.f;
  for (int j = 0; j < s.A; ++j) {
    const float mu = o[s.mean_off + j];
    const float ls = fminf(fmaxf(o[s.ls_off + j], s.min_log_std), s.max_log_std);
    const float sd = expf(ls);
    const float u = mu + e[j] * sd;
    const float a = tanhf(u);
    const float var = sd * sd;
    const float d = u - mu;
    lp += -(d * d) / (2.f * var) - logf(sd) - c;
    corr += logf((1.f - a * a) + 1e-6f);
    s.act[(size_t)b * s.ldact + j] = a;
  }
  s.logpi[b] = lp - corr;
}

__device__ void op_sac_actor_bwd(const SacActorArgs& s, int t) {
  const int b = t * kThreads + threadIdx.x;
  if (b >= s.rows) return;
  const float* o = s.out + (size_t)b * s.ldo;
  const float* e = s.eps2 + (size_t)b * s.ldeps;
  const float w = expf(s.log_alpha[0]) * s.inv_b;   // d obj / d logpi_b
  for (int j = 0; j < s.A; ++j) {
    const float mu = o[s.mean_off + j];
    const float lsr = o[s.ls_off + j];
    const float ls = fminf(fmaxf(lsr, s.min_log_std), s.max_log_std);
    const float sd = expf(ls);
    const float u = mu + e[j] * sd;
    const float a = tanhf(u);
    const float var = sd * sd;
    const float d = u - mu;
    // logpi = sum(-d^2/(2 var) - log sd - c) - sum log(1 - a^2 + 1e-6)
    float ga = s.da[(size_t)b * s.ldda + j] + (w / ((1.f - a * a) + 1e-6f)) * (2.f * a);
    float gu = ga * (1.f - a * a);
    gu += -(w / (2.f * var)) * (2.f * d);           // d(-d^2/(2var))/du
    float gmu = (w / (2.f * var)) * (2.f * d);      // via d = u - mu
    float gvar = (w * (d * d)) / ((2.f * var) * (2.f * var)) * 2.f;
    float gsd = gvar * (2.f * sd) - w / sd;
    gmu += gu;
    gsd += gu * e[j];
    float gls = gsd * sd;
    if (!(lsr >= s.min_log_std && lsr <= s.max_log_std)) gls = 0.f;
    s.dout[(size_t)b * s.lddout + s.mean_off + j] = gmu;
    s.dout[(size_t)b * s.lddout + s.ls_off + j] = gls;
  }
}

// ---------------------------------------------------------------- step end

__device__ void op_step_end(const StepEndArgs& a) {
  if (threadIdx.x != 0) return;
  float vals[kInfoMax];
  const float nanv = __int_as_float(0x7FC00000);
  float la = a.log_alpha ? *a.log_alpha : 0.f;
  const float alpha = expf(la);
  float slp = 0.f;
  if (a.logpi_part)
    for (int i = 0; i < a.nlogpi; ++i) slp += a.logpi_part[i * 4 + 1];
  // mean_b(-lp_b - target_entropy); d/dla mean(exp(la) * c) = exp(la) * mean(c)
  const float gmean = (-slp) * a.inv_b - a.target_entropy;
  const float tmp_obj = alpha * gmean;
  for (int k = 0; k < a.ninfo; ++k) {
    float v = 0.f;
    switch (a.kind[k]) {
      case INFO_SUM:
        for (int i = 0; i < a.npart[k]; ++i) v += a.part[k][i * a.stride[k]];
        v *= a.scale[k];
        break;
      case INFO_NAN: v = nanv; break;
      case INFO_GNORM: {
        // per-tensor sum of squares -> sqrt -> sum (rl/nn/utils.py:13-19)
        float tot = 0.f, cur = 0.f;
        int tcur = a.gsq_tensor[0];
        for (int i = 0; i < a.ngsq; ++i) {
          if (a.gsq_tensor[i] != tcur) { tot += sqrtf(cur); cur = 0.f; tcur = a.gsq_tensor[i]; }
          cur += a.gsq[i];
        }
        v = tot + sqrtf(cur);
        break;
      }
      case INFO_SAC_TMP: v = alpha; break;
      case INFO_SAC_NTMP: v = tmp_obj; break;  // d/dla mean(exp(la)*c) = exp(la)*mean(c)
      case INFO_SAC_POL: {
        float s = 0.f;
        for (int i = 0; i < a.npart[k]; ++i) s += a.part[k][i * a.stride[k]];
        v = s * a.scale[k] + tmp_obj;
        break;
      }
      case INFO_SAC_TMPL: v = tmp_obj; break;
      case INFO_SAC_ENT: v = -slp * a.inv_b; break;
    }
    vals[k] = v;
  }
  if (a.log_alpha && a.la_lr > 0.f) {
    const float g = tmp_obj;
    const double tt = (double)(*a.la_t + 1);
    const double bc1 = 1.0 - pow(0.9, tt), bc2 = 1.0 - pow(0.999, tt);
    float m = *a.la_m, v2 = *a.la_v;
    m = m + (1.f - 0.9f) * (g - m);
    v2 = v2 * 0.999f + ((1.f - 0.999f) * g) * g;
    const float denom = sqrtf(v2) / (float)sqrt(bc2) + 1e-8f;
    *a.la_m = m;
    *a.la_v = v2;
    *a.log_alpha = la + (-(float)(a.la_lr / bc1) * m) / denom;
    *a.la_t += 1;
  }
  int slot = *a.info_slot;
  if (slot >= a.info_cap) slot = a.info_cap - 1;
  for (int k = 0; k < a.ninfo; ++k) a.info[(size_t)slot * kInfoMax + k] = vals[k];
  *a.info_slot = slot + 1;
  for (int c = 0; c < 16; ++c)
    if (a.cmask & (1 << c)) a.counters[c] += 1;
}

// ---------------------------------------------------------------- flat ops

__device__ void op_polyak(const FlatArgs& f, int t) {
  const long long i0 = ((long long)t * kThreads + threadIdx.x) * 4;
  for (long long i = i0; i < i0 + 4 && i < f.n; ++i) {
    const float s = f.self_alias ? f.dst[i] : f.src[i];
    // tau*src + dst*(1-tau), each product rounded separately (Q2, no FMA)
    f.dst[i] = __fadd_rn(__fmul_rn(f.tau, s), __fmul_rn(f.dst[i], f.omt));
  }
}

__device__ void op_copy(const FlatArgs& f, int t) {
  const long long i0 = ((long long)t * kThreads + threadIdx.x) * 4;
  for (long long i = i0; i < i0 + 4 && i < f.n; ++i) f.dst[i] = f.src[i];
}

__device__ void op_maxred(const FlatArgs& f, int t, float* smem) {
  float mx = -INFINITY;
  if (f.stage == 0) {
    const long long size = *f.size;
    const long long per = (size + f.nwg - 1) / f.nwg;
    const long long b0 = (long long)t * per, b1 = min(size, b0 + per);
    for (long long i = b0 + threadIdx.x; i < b1; i += kThreads) mx = fmaxf(mx, f.src[i]);
  } else {
    for (int i = threadIdx.x; i < f.nwg; i += kThreads) mx = fmaxf(mx, f.partial[i]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) smem[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(smem[0], smem[1]), fmaxf(smem[2], smem[3]));
    if (f.stage == 0) f.partial[t] = m; else *f.out = m;
  }
}

__device__ void op_ctrl(const CtrlArgs& c) {
  if (threadIdx.x == 0) {
    c.vt[0] = unkey(*c.vmax_key);
    c.vt[1] = unkey(*c.vmin_key);
  }
}

// ---------------------------------------------------------------- dispatch

__global__ __launch_bounds__(kThreads) void rle_level(const Op* __restrict__ ops, int nops) {
  __shared__ __attribute__((aligned(16))) float smem[8192];  // 32 KB
  const int wg = blockIdx.x;
  int k = 0;
  while (k + 1 < nops && ops[k + 1].wg_begin <= wg) ++k;
  const Op& op = ops[k];
  const int t = wg - op.wg_begin;
  switch (op.kind) {
    case OP_GEMM: op_gemm(op.gemm, t, smem); break;
    case OP_NORMBWD: op_normbwd(op.nb, t); break;
    case OP_SAMPLE_REDUCE: op_sample_reduce(op.sample, t, smem); break;
    case OP_SAMPLE_GATHER: op_sample_gather(op.sample, t, smem); break;
    case OP_HEAD: op_head(op.head, t, smem); break;
    case OP_PRIORITY: op_priority(op.prio, smem); break;
    case OP_SAC_ACTOR: op_sac_actor(op.sac, t); break;
    case OP_SAC_ACTOR_BWD: op_sac_actor_bwd(op.sac, t); break;
    case OP_STEP_END: op_step_end(op.end); break;
    case OP_POLYAK: op_polyak(op.flat, t); break;
    case OP_COPY: op_copy(op.flat, t); break;
    case OP_MAXRED: op_maxred(op.flat, t, smem); break;
    case OP_CTRL: op_ctrl(op.ctrl); break;
    default: break;
  }
}

// ---------------------------------------------------------------- standalone kernels

// Scatter `count` staged transitions into the ring at ptr (wrapping).
__global__ void rle_append_kernel(float* state, float* next_state, float* action, float* reward,
                                  float* notdone, float* priority, const float* st_s, const float* st_ns,
                                  const float* st_a, const float* st_r, const float* st_d, long long ptr,
                                  long long cap, int count, int Sp, int Ap, const float* max_priority,
                                  int lap) {
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
__global__ void rle_fill_kernel(float* state, float* next_state, float* action, float* reward,
                                float* notdone, float* priority, long long n, int S, int Sp, int A, int Ap,
                                unsigned long long seed) {
  const long long row = blockIdx.x;
  if (row >= n) return;
  const uint2 key = make_uint2((unsigned)seed, (unsigned)(seed >> 32));
  for (int k = threadIdx.x; k < Sp; k += blockDim.x) {
    uint4 r = philox(key, make_uint4((unsigned)row, (unsigned)k, 7u, (unsigned)(row >> 32)));
    state[row * Sp + k] = k < S ? normal_from(r.x, r.y) : 0.f;
    next_state[row * Sp + k] = k < S ? normal_from(r.z, r.w) : 0.f;
  }
  for (int k = threadIdx.x; k < Ap; k += blockDim.x) {
    uint4 r = philox(key, make_uint4((unsigned)row, (unsigned)k, 8u, (unsigned)(row >> 32)));
    action[row * Ap + k] = k < A ? 2.f * u01(r.x) - 1.f : 0.f;
  }
  if (threadIdx.x == 0) {
    uint4 r = philox(key, make_uint4((unsigned)row, 0u, 9u, (unsigned)(row >> 32)));
    reward[row] = normal_from(r.x, r.y);
    notdone[row] = u01(r.z) < 0.99f ? 1.f : 0.f;
    priority[row] = 1.f;
  }
}

}  // namespace rle

// ---------------------------------------------------------------- host launchers

extern "C++" {
namespace rle {
hipError_t launch_level(const Op* d_ops, int nops, int nwg, hipStream_t st) {
  hipLaunchKernelGGL(rle_level, dim3(nwg), dim3(kThreads), 0, st, d_ops, nops);
  return hipGetLastError();
}
hipError_t launch_append(float* state, float* next_state, float* action, float* reward, float* notdone,
                         float* priority, const float* st_s, const float* st_ns, const float* st_a,
                         const float* st_r, const float* st_d, long long ptr, long long cap, int count,
                         int Sp, int Ap, const float* max_priority, int lap, hipStream_t st) {
  hipLaunchKernelGGL(rle_append_kernel, dim3(count), dim3(256), 0, st, state, next_state, action, reward,
                     notdone, priority, st_s, st_ns, st_a, st_r, st_d, ptr, cap, count, Sp, Ap, max_priority,
                     lap);
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
}
