// Op descriptors shared by the host program builder (engine.cpp) and the
// device dispatch kernel (kernels.hip).  Plain POD; one level of a step graph
// is an array of Op, launched as ONE kernel whose workgroups are partitioned
// over the ops by Op::wg_begin.
#pragma once
#include <stdint.h>

namespace rle {

constexpr int kThreads = 256;   // 4 waves per workgroup, every op kind
constexpr int kTileM = 16;      // GEMM output tile rows (v_mfma_f32_16x16x4_f32)
constexpr int kTileN = 64;      // widest GEMM output tile (GemmArgs::tn in {16, 32, 64})
constexpr int kMaxSeg = 4;
constexpr int kInfoMax = 8;     // floats per step in the info ring
constexpr int kMaxHidden = 6;   // hidden layers of a TD3 / SAC MLP (rle.h RLE_MAX_HIDDEN)
constexpr int kGsqT = 2 * (kMaxHidden + 1);  // TD3 actor tensors (weight, bias per layer) in norm/policy

enum OpKind : int {
  OP_GEMM = 1,
  OP_NORMBWD = 2,
  OP_SAMPLE_REDUCE = 3,
  OP_SAMPLE_GATHER = 4,
  OP_HEAD = 5,
  OP_PRIORITY = 6,
  OP_SAC_ACTOR = 7,
  OP_SAC_ACTOR_BWD = 8,
  OP_STEP_END = 9,
  OP_POLYAK = 10,
  OP_COPY = 11,
  OP_MAXRED = 12,
  OP_CTRL = 13,
  OP_NOISE = 14,        // target-smoothing / rsample noise of the batch (SampleArgs)
  OP_FOLDBIAS = 15,     // bias of a folded weight block (FoldBiasArgs)
};

// ---------------------------------------------------------------- tensor images
//
// Every 2D tensor that feeds a GEMM lives in 16x16 "fragment blocks" of 1 KB
// (rows and columns padded to 16), in one or both of two images:
//   N image (row fragments):    block (rb, cb) at n + (rb * cbn + cb) * 256,
//                               element (r, c) inside at ((c%16)/4)*64 + (r%16)*4 + c%4
//   T image (column fragments): block (rb, cb) at t + (cb * rbs + rb) * 256,
//                               element (r, c) inside at ((r%16)/4)*64 + (c%16)*4 + r%4
// Lane l of a wave reads float l*4..l*4+3 of a block: in the N image that is row
// l%16, columns 4(l/16)..+3 -- exactly the v_mfma_f32_16x16x4_f32 A/B fragment
// when the reduction runs along columns; the T image gives the fragment when
// it runs along rows.  So every GEMM operand load is one lane-linear 16-byte
// load per lane per 16-wide reduction chunk (a whole 1 KB block per wave).
struct Mat {
  float* n;   // N image (nullptr: not kept)
  float* t;   // T image (nullptr: not kept)
  int cbn;    // column blocks per row-block in the N image
  int rbs;    // row blocks per column-block in the T image (the allocation's, for sub-views)
};

// Deferred AvgL1Norm of a producer output (rl/nn/sale.py:11-13): the consumer
// value is x / m(row), m = max(sum_p part[p*ld + row0 + row] / width, 1e-8).
struct NormRef {
  const float* part;
  int ld, row0, nparts, width;
};

// One rectangle of a GEMM operand in (x, r) space: x = output row (operand A)
// or output column (operand B); r = reduction index.  The operand is an image
// (N or T, whichever makes r the fragment's reduction direction) starting at p:
//   block of (x, r) = p + ((x - x0) / 16 * xs + (r - r0) / 16) * 256
// Reduction segments are 16-aligned and back to back (r0 of one == padded r1 of
// the previous); x-split segments (GEMM_DW B only) are 16-aligned in x.
struct Seg {
  const float* p;
  int xs;          // blocks per x-block step
  int x0, x1, r0, r1;
  int pad_;
  NormRef norm;    // norm.part == nullptr: plain operand
};

struct Operand {
  Seg seg[kMaxSeg];
  int nseg;
  int pad_[3];
};

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_ELU = 2, ACT_TANH = 3 };

enum Epi : int {
  EPI_STORE = 0,   // out = act(acc + bias); optional pre-act store, |y| partials, derivative mask, tanh-noise
  EPI_ADAM = 1,    // acc is dL/dW (or dL/db on the bias tile column): Adam in place
  EPI_MSE = 2,     // acc (+bias) = zsa; grad = 2 (zsa - tgt) / n ; loss partial sum of squares
  EPI_QHEAD = 3,   // critic's last hidden layer with its H -> 1 head and a constant dL/dq fused:
                   // out = qscale * w3 * act'(z) (= dZ), loss partial sum of act(z) * w3 (+ M b3)
  EPI_NBDOT = 4,   // DX whose output g feeds an AvgL1Norm backward deferred into its consumer:
                   // out = g, per-tile row partials of sum_j g x (x: nbx) into norm_out
  EPI_ACT = 5,     // act graph (TD7 / TD3 actor's tanh layer): environment action, ActArgs
  EPI_QDOT = 6,    // EPI_STORE (forward) + per-tile row partials of sum_j act(z)_j w_j (w: qw, a
                   // critic's H -> 1 head row) into norm_out: the loss head's q without a row load
  EPI_SACBWD = 7,  // DX of the SAC actor objective's action gradient da: the squashed-Gaussian
                   // backward (as OP_SAC_ACTOR_BWD) per element in the epilogue -> d / d(mean | log_std)
  EPI_SACFWD = 8,  // the SAC actor's raw head (tile = whole rows, tn 64 >= 2A): raw stored, then the
                   // rsample, tanh action and log pi of the tile's rows (as OP_SAC_ACTOR)
};

// Environment action of an act graph (td7.py:141-156, td3.py:114-129, sac.py:132-152), written
// as compact [n][A] rows straight into host-mapped memory:
//   TD7 / TD3 (EPI_ACT):     a = clip(tanh(z) + sigma * eps, -1, 1)   (eps = 0: deterministic)
//   SAC (OP_SAC_ACTOR):      a = tanh(mean + exp(clamp(log_std)) * eps)
//   out = a * scale + bias   (fp32, unfused, as numpy's float32 ops)
// eps: ctl[0] = 0 none (deterministic), 1 Philox normal at counter (ctl[1], ctl[2]) keyed by seed,
// 2 the host tape eps[n][A] (parity).
struct ActArgs {
  float* out;
  const int* ctl;
  const float* eps;
  const float* scale;     // [A]   (rle_set_action_map)
  const float* bias;      // [A]
  const float* sigma;     // [1]   TD7 / TD3 exploration_noise
  int n, A;
  unsigned long long seed;
};
// GEMM_DW variant whose A operand (dZ) is an AvgL1Norm backward applied on load:
// a = g / m + sign(x) * gm, gm = -(sum_j g x) / (n m^2) (0 when m is clamped), rows by LDS table
constexpr int kDwNb = 1;  // (in the act slot of a DW variant id)

struct AdamArgs {
  Mat w;                 // weight images [N out rows][K cols] (both kept: FWD reads N, DX reads T)
  float* b;              // bias [16 * row blocks] (bias tile column j0 == bias_col)
  long long mo, vo;      // element offsets of m / v arrays relative to params (m, v kept at T-image offsets)
  const float* step;     // lr / (1 - beta1^t) of this optimizer's next step (Ctrl::adam_step, STEP_END)
  const float* bc2s;     // sqrt(1 - beta2^t) (Ctrl::adam_bc2s)
  float lr, beta1, beta2, eps;
  float omb1, omb2;      // (float)(1 - beta1), (float)(1 - beta2) as torch casts the Python scalars
  int bias_col;          // first column of the bias tile = K rounded up to the tile width tn
  float ptau;            // != 0: the self-aliased Polyak p <- tau p + p (1 - tau) applied to the updated
                         // value (TD3's target policy is the policy, td3.py:200-204)
  float* gsq;            // optional: per-tile sum of squared grads (weights), [tiles]
  float* gsq_b;          // optional: per-tile sum of squared grads (bias), [tiles_m]
};

// Variant id of a GEMM op = pre * 512 + mode * 128 + epi * 8 + act * 2 + norm (pre: one A
// segment is the actor's tanh output layer recomputed in the workgroup, PreArgs; act: the forward
// activation for GEMM_FWD, the derivative mask for GEMM_DX, kDwNb or 0 for GEMM_DW; norm: some operand
// segment carries a deferred AvgL1Norm).
constexpr int gemm_vid(int mode, int epi, int act, int norm, int pre = 0) {
  return pre * 512 + mode * 128 + epi * 8 + act * 2 + norm;
}
// (the level-launch entry keeps it in bits 20-30: bit 31 of entry 0 is the descriptor-prefetch flag)
static_assert(gemm_vid(2, 8, 15, 1, 3) < 2048, "GEMM variant ids fit 11 bits");

// The compiled GEMM variants: X(mode, epilogue, activation, norm, pre, PK, sets) -- the variant id's fields
// (gemm_vid), gemm_v's path (PK: 0 plain, 1 pre-GEMM, 2 fused loss head, 3 pre-layer, 4 pre-layer behind a
// pre-GEMM, 5 SAC raw head pre-GEMM) and the kernel sets that hold it (bit 0: TD7, bit 1: TD3 / SAC; the
// extended instance holds all).  kernels.hip op_gemm dispatches exactly these, and the engine refuses a
// program with an op whose id is not in its kernel set.  (sets 0: the extended instance only -- the TD7 policy
// pass's q-head under a non-default critic activation, rle_config act_critic)
#define RLE_GEMM_VARIANTS(X)                        \
  X(GEMM_FWD, EPI_STORE, ACT_NONE, 0, 0, 0, 3)      \
  X(GEMM_FWD, EPI_STORE, ACT_NONE, 1, 0, 0, 1)      \
  X(GEMM_FWD, EPI_STORE, ACT_RELU, 0, 0, 0, 3)      \
  X(GEMM_FWD, EPI_STORE, ACT_RELU, 1, 0, 0, 1)      \
  X(GEMM_FWD, EPI_STORE, ACT_ELU, 0, 0, 0, 3)       \
  X(GEMM_FWD, EPI_STORE, ACT_ELU, 1, 0, 0, 1)       \
  X(GEMM_FWD, EPI_STORE, ACT_TANH, 0, 0, 0, 3)      \
  X(GEMM_FWD, EPI_STORE, ACT_TANH, 1, 0, 0, 1)      \
  X(GEMM_FWD, EPI_QHEAD, ACT_ELU, 0, 0, 0, 1)       \
  X(GEMM_FWD, EPI_QHEAD, ACT_RELU, 0, 0, 0, 0)      \
  X(GEMM_FWD, EPI_QHEAD, ACT_NONE, 0, 0, 0, 0)      \
  X(GEMM_FWD, EPI_MSE, ACT_NONE, 0, 0, 0, 1)        \
  X(GEMM_FWD, EPI_MSE, ACT_NONE, 1, 0, 0, 1)        \
  X(GEMM_FWD, EPI_ACT, ACT_TANH, 0, 0, 0, 3)        \
  X(GEMM_FWD, EPI_QDOT, ACT_ELU, 0, 0, 0, 1)        \
  X(GEMM_FWD, EPI_QDOT, ACT_RELU, 0, 0, 0, 2)       \
  X(GEMM_DX, EPI_STORE, ACT_NONE, 0, 0, 0, 3)       \
  X(GEMM_DX, EPI_STORE, ACT_RELU, 0, 0, 0, 3)       \
  X(GEMM_DX, EPI_STORE, ACT_ELU, 0, 0, 0, 3)        \
  X(GEMM_DX, EPI_STORE, ACT_TANH, 0, 0, 0, 3)       \
  X(GEMM_DX, EPI_NBDOT, ACT_NONE, 0, 0, 0, 1)       \
  X(GEMM_DW, EPI_ADAM, ACT_NONE, 0, 0, 0, 3)        \
  X(GEMM_DW, EPI_ADAM, ACT_NONE, 1, 0, 0, 1)        \
  X(GEMM_DW, EPI_ADAM, kDwNb, 0, 0, 0, 1)           \
  X(GEMM_FWD, EPI_STORE, ACT_NONE, 0, 1, 1, 1)      \
  X(GEMM_FWD, EPI_STORE, ACT_RELU, 0, 1, 1, 3)      \
  X(GEMM_FWD, EPI_STORE, ACT_ELU, 1, 1, 1, 1)       \
  X(GEMM_DX, EPI_STORE, ACT_RELU, 0, 1, 1, 3)       \
  X(GEMM_DX, EPI_SACBWD, ACT_NONE, 0, 0, 0, 2)      \
  X(GEMM_FWD, EPI_SACFWD, ACT_NONE, 0, 0, 0, 2)     \
  X(GEMM_DX, EPI_STORE, ACT_ELU, 0, 2, 2, 1)        \
  X(GEMM_DX, EPI_STORE, ACT_RELU, 0, 2, 2, 2)       \
  X(GEMM_FWD, EPI_STORE, ACT_RELU, 0, 3, 3, 2)      \
  X(GEMM_FWD, EPI_QDOT, ACT_RELU, 0, 3, 3, 2)       \
  X(GEMM_DX, EPI_STORE, ACT_RELU, 0, 3, 3, 2)       \
  X(GEMM_FWD, EPI_QDOT, ACT_RELU, 1, 3, 4, 2)       \
  X(GEMM_FWD, EPI_STORE, ACT_RELU, 1, 1, 5, 2)
// the variants kernels.hip gemm_wide implements (64-row LDS-staged tiles, GemmHot::wide): forward and input-gradient
// GEMMs with a plain, q-dot, MSE, q-head or AvgL1Norm-dot epilogue and no in-tile prologue
constexpr bool wide_variant(int mode, int epi, int pk) {
  return pk == 0 && mode != 2 /* GEMM_DW */ &&
         (epi == EPI_STORE || epi == EPI_QDOT || epi == EPI_MSE || epi == EPI_QHEAD || epi == EPI_NBDOT);
}
// kernel sets (rle_level's KS): TD7, TD3 / SAC, and the extended instance (every variant, plus the opt-in
// register-blocked weight-gradient tiles and the fused priority sampler)
// KS_TD7W: the TD7 set with the 64-row LDS-staged tiles (GemmHot::wide) and a larger LDS allocation, for
// batches >= 512 (rle_plan wide)
enum KernelSet : int { KS_TD7 = 0, KS_MLP = 1, KS_EXT = 2, KS_TD7W = 3, KS_COUNT = 4 };
// the agent family whose variants (RLE_GEMM_VARIANTS sets bit) and ops an instance compiles
constexpr int ks_family(int ks) { return ks == KS_TD7W ? KS_TD7 : ks; }

enum GemmMode : int {
  GEMM_FWD = 0,   // A contiguous (activations), B contiguous (W rows):  Y = X W^T
  GEMM_DX = 1,    // A contiguous (dZ), B strided (W columns):            dX = dZ W
  GEMM_DW = 2,    // A strided (dZ^T), B strided (X):                     dW = dZ^T X
};

// Copies of every field the GEMM prologue and the first operand segment need, packed
// at the start of GemmArgs so the kernel reads them in ONE scalar-load batch
// (filled by the host from the fields below; kernels.hip gemm_v).
struct GemmHot {
  int ks_log, tiles_n, tn, N, R;
  float inv_tiles_n;
  int bias_col, nseg_a, nseg_b;
  int a0xs, a0r0, a0r1, b0xs, tiles;  // tiles = tiles_m * tiles_n
  const float* a0p;
  const float* b0p;
  const float* bias;
  // XCD-aware tile order (xb > 0): workgroups t with equal t % 8 run on one XCD (round-robin
  // dispatch); each such residue class takes a contiguous run of tiles in a banded order
  // (bands of xb tile columns, rows inside a band, columns inside a row), i.e. a compact
  // rectangle, so an XCD reads few distinct A row-blocks and B column-blocks.
  int xb, tmb;                    // band width in tiles, tiles per full band (tiles_m * xb)
  float inv_tmb, inv_xb, inv_blast;
  int nfull;                      // full bands; the last band is tiles_n - nfull * xb wide
  // register-blocked wide weight-gradient tile (tn 32 / 64): the 4 waves split the reduction in
  // quarters and each accumulates every column block of the tile (kernels.hip rb_run); 0: column
  // groups x splits
  int rb;
  // 64-row LDS-staged tile (rle_plan wide; the TD7 instance at B >= 512, kernels.hip gemm_wide): the
  // workgroup's 4 waves own 16 rows each of a 64 x wide output tile (wide = tn: 64 or 32), every W chunk staged
  // once in LDS for all four; tiles counts 64-row tiles, GemmArgs::tiles_m 16-row blocks; 0: 16-row tiles
  int wide;
  int pad_[4];
};
static_assert(sizeof(GemmHot) == 128, "GemmHot is loaded as 2 x 16 dwords");

// Tile (it, jt) of workgroup t of a GEMM under the XCD-aware order (GemmHot::xb > 0); the same
// code runs in the kernel (scalar registers) and in the host planner, which checks that it
// is a bijection before enabling it.
__host__ __device__ inline void xcd_tile(int t, int T, int tiles_n, int xb, int tmb, int nfull, float inv_tmb,
                                         float inv_xb, float inv_blast, int& it, int& jt) {
  const int q = T >> 3, m = T & 7, r0 = t & 7;
  const int p = r0 * q + (r0 < m ? r0 : m) + (t >> 3);
  const int band = (int)(((float)p + 0.5f) * inv_tmb);
  const int rem = p - band * tmb;
  const bool full = band < nfull;
  const int bw = full ? xb : tiles_n - nfull * xb;
  it = (int)(((float)rem + 0.5f) * (full ? inv_xb : inv_blast));
  jt = band * xb + rem - it * bw;
}

// The actor's output layer (rl/nn/sale.py:77-83 / mlp.py:55-68, N = act_dim <= 32) recomputed
// by a consuming GEMM for its own 16 rows into an LDS fragment block, so the consumer does not
// wait a level for it ("pre-GEMM"):
//   FWD: a = clamp(tanh(X W^T + b) + clamp(sigma * eps, +-c), +-1)   (target policy smoothing)
//   DX:  a = (sum_t dZ_t W_t) * (1 - act^2)                           (grad wrt the tanh input)
// The result replaces the consumer's A segment `seg` (reduction width <= 32).
struct PreArgs {
  Operand A, B;        // operands in the conventions of GemmArgs A / B for `mode`
  int mode;            // GEMM_FWD or GEMM_DX
  int N, R;            // output columns (<= 32), reduction length
  int seg;             // consumer A segment produced
  int act;             // (pre-layer, has_pre 3) the layer's activation
  int sac_a;           // (has_pre 5) action dims A: the output is SAC's raw head [mean | log_std], 2A wide
  const float* bias;   // FWD
  // FWD: smoothing noise (T image, consumer rows), sigma, clip; has_pre 5: the rsample noise and the
  // log-std clamp (noise_sigma = min, noise_clip = max)
  Mat noise; float noise_sigma, noise_clip;
  Mat dsrc;            // DX: saved tanh output (T image, consumer rows)
};

enum HeadMode : int {
  HEAD_TD7_TARGET = 0,   // tq_i, y = r + g*clamp(min, vt_min, vt_max)*nd, vmax/vmin
  HEAD_TD7_LOSS = 1,     // q_i, LAP huber (or MSE), priority, dq, dZ
  HEAD_TD7_POLICY = 2,   // q_i, loss = -mean(cat), dZ
  HEAD_MLP_TARGET = 3,   // TD3 / SAC target: y = r + g*(min - alpha*logpi)*nd
  HEAD_MLP_LOSS = 4,     // MSE (or TD3 LAP per-critic mean), priority
  HEAD_MLP_POLICY = 5,   // TD3: -mean(min);  SAC: mean(-min + alpha*logpi)
};

struct HeadArgs {                   // 4 rows per workgroup (1 per wave)
  int mode, rows, H, lap;
  Mat h[2];                          // last hidden (post-activation) of each twin, N image
  Mat dsrc[2];                       // derivative source (Z for ELU, H for ReLU), N image
  int dact;
  int nvalid;                        // batch rows: rows past it (the batch padded to 16) add nothing (fused heads)
  const float* w[2];                 // last-layer weight row: N image of a [1][H] matrix
  int w_cbn;                         // its column blocks
  const float* b[2];                 // last-layer bias [1]
  const float* reward; const float* notdone;
  float* y;                          // target (written by *_TARGET, read by *_LOSS)
  Mat dz[2];                         // grad wrt last hidden pre-activation (N + T)
  Mat dq[2];                         // grad wrt q, T image of [rows][1] (dW of last layer)
  float* loss_part;                  // per-workgroup partial sums [wg][4]
  float* prio;                       // LAP priority out [rows]
  float gamma;
  int sac;                           // SAC: alpha term
  int alpha_lin;                     // SAC fixed temperature: *log_alpha holds alpha itself (sac.py:55-60)
  const float* logpi;                // SAC logpi [rows] (target rows / policy rows)
  const float* log_alpha;            // SAC log alpha scalar
  int* vmax_key; int* vmin_key;      // TD7 value tracking (ordered-int keys)
  const float* vt;                   // TD7 [vt_max, vt_min]
  float inv_b;                       // 1/B (policy loss scale)
  // *_LOSS with the target head fused in (one level fewer): tgt_mode is HEAD_TD7_TARGET or
  // HEAD_MLP_TARGET and y is computed per row from the target twins' last hidden layer
  // (th / tw / tb, as h / w / b), reward, notdone, vt (TD7) or alpha * logpi (SAC);
  // -1: y is read from the `y` vector written by a separate *_TARGET head.
  int tgt_mode;
  Mat th[2];
  const float* tw[2];
  const float* tb[2];
  // EPI_QDOT partials of the twins' q (qp) and of the target twins' q (tp): [n][ld], summed over
  // the n column tiles (null: q is the dot product of the h / th row with w / tw)
  const float* qp[2];
  const float* tp[2];
  int qp_n[2], tp_n[2];  // column tiles of each twin's producer (their tile plans may differ)
  int qp_ld, tp_ld;
};

// EPI_SACBWD operands (the policy rows of the actor's raw head and their rsample draws)
struct SacBwdArgs {
  Mat raw;                           // raw head output [2B][2A(p)]: mean | log_std (T image)
  Mat eps2;                          // policy rsample noise [B][Ap] (T image)
  Mat dout;                          // grad wrt the raw output [B][2A(p)]
  const float* log_alpha;            // log alpha, or alpha itself (alpha_lin)
  float inv_b, min_log_std, max_log_std;
  int alpha_lin, mean_off, ls_off;
  int nvalid;                        // batch rows (rows past it: no gradient)
};

// EPI_SACFWD operands (sac.py:132-152 rsample of both row halves: policy rows < eps_row_split)
struct SacFwdArgs {
  Mat eps, eps2;                     // target / policy rsample noise (T images)
  Mat act;                           // tanh action [2B][Ap]
  float* logpi;                      // [2B]
  float min_log_std, max_log_std;
  int A, mean_off, ls_off, eps_row_split;
};

struct GemmArgs {
  GemmHot hot;           // (first: two s_load_dwordx16)
  int mode;              // GemmMode (operand layouts; every segment of an operand shares it)
  int M, N, R;           // output rows, output cols (x-extent of B), reduction length
  int tn;                // tile width: 16 x tn output tile; the 4 waves are tn/16 column groups
                         // x 64/tn reduction splits (partials summed through LDS, fixed order)
  int tiles_m, tiles_n;  // tiles_n = cdiv(N, tn), + 1 bias tile column for EPI_ADAM
  int vid;               // compiled variant (host: gemm_variant): mode, epilogue, activation, norm
  int ks_log;            // log2(64 / tn): reduction splits per tile
  float inv_tiles_n;     // 1 / tiles_n (tile row = floor((t + 0.5) * inv_tiles_n))
  int epi;
  int act;               // forward activation (EPI_STORE)
  Operand A, B;
  Mat out;                         // output images (EPI_STORE, EPI_MSE)
  const float* bias;
  Mat pre;                         // pre-activation store, T image (optional)
  float* norm_out; int norm_ld;    // |y| partials: norm_out[jt * norm_ld + i] (optional)
  int dact;                        // derivative mask: out *= act'(dsrc(i, j))
  Mat dsrc;                        // T image
  Mat noise; int noise_row0; float noise_sigma, noise_clip;  // tanh-noise (T image)
  Mat tgt; NormRef tgt_norm;       // EPI_MSE target (T image of a normed view)
  float* loss_part;                // EPI_MSE / EPI_QHEAD per-tile partial sums
  float mse_scale;                 // 1/n
  const float* qw; const float* qb; int qw_cbn;  // EPI_QHEAD: head weight row (N image of [1][N]), bias
  float qscale;                    // EPI_QHEAD: dL/dq
  Mat nbx; int nbx_xs;             // EPI_NBDOT / kDwNb: x of the AvgL1Norm (T image; DW: its x-block step)
  NormRef nbm;                     // kDwNb: m of x's rows (producer |x| partials)
  const float* nbdot; int nbdot_ld, nbdot_n;  // kDwNb: the EPI_NBDOT producer's row partials of sum g x
  int has_pre;                     // 1: pre-GEMM (prea) in use; 2: loss head fused into this DX (hd);
                                   // 3: pre-layer (prea); 4: pre-layer behind a pre-GEMM (prea, prea2;
                                   // variant id: pre 3 with the norm bit, which a pre-layer never sets);
                                   // 5: SAC's raw head + rsample as the pre-GEMM (prea; variant id: pre 1
                                   // with the norm bit on a ReLU forward, which no pre-GEMM consumer has)
  union {
    PreArgs prea;
    // has_pre 2 (TD7 critic backward, engine.cpp build_td7): the HEAD_TD7_LOSS head (target
    // twins fused) of this tile's rows runs in the workgroup, and the DX's A operand dZ of critic
    // head_n's last hidden layer = dq * w3 * act'(z) is formed on load from z (segment 0); the
    // tile-column-0 workgroups store what the standalone head stored (dz / dq of critic head_n;
    // head_n 0 also the priorities, loss partials and value bounds)
    HeadArgs hd;
    SacBwdArgs sb;  // EPI_SACBWD (has_pre 0)
    SacFwdArgs sf;  // EPI_SACFWD (has_pre 0)
  };
  union {
    int head_n;    // has_pre 2: the critic whose DX this is
    int mvalid;    // EPI_QHEAD / EPI_MSE: batch rows of M (rows past it, the batch padded to 16, add nothing)
    int nb_width;  // kDwNb with nbm finalized (nparts 1, width 1; engine.cpp norm_fin): x's width for the sign term
  };
  AdamArgs adam;
  ActArgs ao;                      // EPI_ACT
  // has_pre 4 (TD3 target critics, engine.cpp mlp_critic_fwd): the pre-layer prea's input segment
  // prea2.seg is itself computed in-tile first, by the pre-GEMM prea2 (the target action), so the
  // first layer behind the target action costs no level of its own
  PreArgs prea2;
  int pad_tail_[2];                // (Op: whole 64-byte lines)
};

// AvgL1Norm backward: dx = (g - sign(x) * (sum g*y)/n) / m, y = x/m (row-wise);
// 4 rows per workgroup (1 per wave), N images in, N + T images out.
// fwd = 1: the forward itself, dx = x / m (g = x; diagnostics: rle_eval's zs output).
// fwd = 2 (finalize): mout[row] = mean |x| of the row (norm_mean of its partials, before the 1e-8 clamp), one
// thread per row -- read by the weight gradients as a one-partial NormRef of width 1, the same floats
struct NormBwdArgs {
  Mat g, x, dx;
  int rows, width;
  NormRef norm;  // partials for m (x rows)
  int fwd, pad_;
  float* mout;
};


enum { kTapeU = 1, kTapeInd = 2, kTapeEps = 4 };

struct SampleArgs {
  // replay
  const float* state; const float* next_state; const float* action;
  const float* reward; const float* notdone;
  float* priority;
  int S, Sp, A, Ap;
  const long long* size;             // device replay size
  long long cap;                     // replay capacity (priority array length)
  int lap, B;                        // B: the padded batch (ss row offset of next_state)
  int nq;                            // queries = batch rows (<= B; rows past it stay zero)
  double* bsum; int nblk;            // LAP block sums (fp64), 4096 priorities per block
  double* ssum;                      // LAP sub-block sums (fp64), 64 priorities each (64 per block)
  // outputs
  Mat ss;                            // [2B][Sp] rows 0..B-1 state, B..2B-1 next_state (N + T)
  Mat a;                             // [B][Ap] (N + T)
  float* r; float* nd;               // [B]
  long long* ind;                    // [B]
  float* u_out;                      // [B] uniform used (debug)
  Mat eps;                           // [B][Ap] target smoothing / SAC next noise (T)
  Mat eps2;                          // [B][Ap] SAC policy noise (optional, T)
  // randomness
  const long long* ctrl_rng;         // step counter for Philox
  unsigned long long seed;
  const int* tape_mode;              // kTape* bits: which draws come from tapes (others: Philox)
  const long long* tape_pos;
  const float* tape_u; const float* tape_eps; const float* tape_eps2; const long long* tape_ind;
  int ahead;                         // 1: draws of the NEXT step (prefetch at the end of a step)
  // LAP: the previous step's priority update not yet applied to priority / bsum / ssum (its
  // OP_PRIORITY runs after this op): pend_p[b] for row pend_ind[b], b < pend_n, last duplicate
  // wins (lap.py:66-69); the search reads the sums and priorities as that update leaves them
  const long long* pend_ind; const float* pend_p; int pend_n;
};

struct PriorityArgs {
  float* priority; const long long* ind; const float* p; int B;
  float* max_priority;
  double* bsum;          // LAP block sums kept in step with the scatter (nullptr: none)
  double* ssum;          // ... and the sub-block sums
};

struct SacActorArgs {
  ActArgs ao;                        // act graph: ao.out != nullptr -> environment actions only
  Mat out;                           // raw head output [rows][2A(p)]: mean | log_std (T)
  int A, rows;                       // rows = 2B
  Mat eps; int eps_row_split; Mat eps2;  // rows < split use eps2 (policy), else eps (target) (T)
  Mat act;                           // tanh action (N + T)
  float* logpi;                      // [rows]
  float min_log_std, max_log_std;
  int mean_off, ls_off;              // column offsets of mean / log_std blocks
  // backward
  Mat da;                            // grad wrt action from critics [B][Ap] (T)
  Mat dout;                          // grad wrt raw output [B][2A(p)] (N + T)
  const float* log_alpha; float inv_b;
  int alpha_lin;                     // as HeadArgs::alpha_lin
};

// Step end: info ring row + counter increments + SAC temperature Adam.
struct StepEndArgs {
  long long* counters; int cmask;            // counters[i] += 1 for every bit i of cmask
  int* info_slot; float* info; int info_cap;
  // up to kInfoMax info values, each = scale * sum(parts[0..n)) (or special)
  const float* part[kInfoMax]; int npart[kInfoMax]; int stride[kInfoMax]; float scale[kInfoMax];
  int kind[kInfoMax]; int ninfo;
  // SAC temperature
  float* log_alpha; float* la_m; float* la_v; long long* la_t; float la_lr; float target_entropy;
  float* adam_step; float* adam_bc2s; float adam_lr[4];  // (SAC autotune) slot 3: the temperature optimizer's bias corrections from this step's control op
  const float* logpi_part; int nlogpi; float inv_b;
  const float* gsq; int gsq_off[kGsqT + 1]; int ngsq_t;  // TD3 grad norm: tensor t = tiles [off[t], off[t+1])
  // 0: the whole step end; 1: counters (+ the SAC temperature update, which needs the logpi sum)
  // -- what the next step depends on; 2: the info row -- what only the host reads, scheduled
  // wherever it is not the longest op.  sac_scratch: {alpha before the update, logpi sum},
  // written by mode 1 for mode 2 (autotuned SAC temperature)
  int mode;
  float* sac_scratch;
};

enum InfoKind : int {
  INFO_SUM = 0,       // scale * sum
  INFO_NAN = 1,       // NaN (policy loss on a non-policy step)
  INFO_GNORM = 2,     // sum_t sqrt(sum of tiles of tensor t)
  INFO_SAC_TMP = 3,   // exp(log_alpha) before update
  INFO_SAC_NTMP = 4,  // d obj / d log_alpha
  INFO_SAC_POL = 5,   // policy_obj + tmp_obj
  INFO_SAC_TMPL = 6,  // tmp_obj
  INFO_SAC_ENT = 7,   // -mean(logpi)
};

// Bias of a layer whose input block [col0, col0 + H) is fed by a linear layer folded
// into it (y = W[:, blk] (V x + c) = (W[:, blk] V) x + W[:, blk] c):
// bout[o] = bbase[o] + sum_z W[o][col0 + z] * bin[z], o < H.  One workgroup.
struct FoldBiasArgs {
  const float* wn; int cbn; int col0;  // W: N image, column blocks per row block
  int H;                               // outputs (rows of W) = width of the block
  const float* bin;                    // bias of the folded-in layer [H]
  const float* bbase;                  // bias of the consuming layer [H]
  float* bout;                         // [H]
};

struct FlatArgs {   // POLYAK / COPY / MAXRED
  float* dst; const float* src; long long n;
  float tau, omt; int self_alias;     // self_alias: p <- tau*p + p*(1-tau) (TD3 quirk Q2)
  const long long* size; float* partial; int nwg; float* out;   // MAXRED
  int stage;
};

struct CtrlArgs {   // small control-plane writes
  int mode;          // 0: value bounds copy at the hard update; 1: Adam scalars from the counters
  const int* vmax_key; const int* vmin_key; float* vt;
  const long long* counters; float* adam_step; float* adam_bc2s; float adam_lr[4];
  // (mode 1, SAC with an autotuned temperature: the temperature optimizer's bias corrections from its step
  // count into adam_step[3] / adam_bc2s[3], so the step end does not compute them on the chain)
  const long long* la_t; float la_lr;
};

struct Op {
  int kind;
  int wg_begin;     // first workgroup of this op within its level launch
  int wg_count;
  int seq;          // host: GEMM creation index (tile-width plan), unused on the device
  union {
    GemmArgs gemm;
    NormBwdArgs nb;
    HeadArgs head;
    SampleArgs sample;
    PriorityArgs prio;
    SacActorArgs sac;
    StepEndArgs end;
    FlatArgs flat;
    CtrlArgs ctrl;
    FoldBiasArgs fb;
  };
};
// kernels.hip gemm_v touches the descriptor's 64-byte lines by fixed offsets from &gemm (its
// TL_* lists): ops are 64-byte aligned in their tables and the GEMM fields sit at these offsets.
static_assert(sizeof(HeadArgs) <= sizeof(PreArgs), "GemmArgs: the fused head shares the pre-GEMM's fields");
static_assert(sizeof(Op) % 64 == 0 && offsetof(Op, gemm) == 16, "Op layout (descriptor line touches)");
static_assert(16 + sizeof(HeadArgs) <= 8 * 64 && 16 + sizeof(StepEndArgs) <= 8 * 64 && 16 + sizeof(SampleArgs) <= 8 * 64,
              "rle_level touches 8 descriptor lines of a non-GEMM op");
static_assert(offsetof(GemmArgs, A) == 0xb0 && offsetof(GemmArgs, B) == 0x1a0 && offsetof(GemmArgs, out) == 0x290 &&
                  offsetof(GemmArgs, noise) == 0x2f0 && offsetof(GemmArgs, nbx) == 0x370 &&
                  offsetof(GemmArgs, prea) == 0x3c0 && offsetof(GemmArgs, adam) == 0x600 &&
                  offsetof(GemmArgs, ao) == 0x670 && offsetof(GemmArgs, prea2) == 0x6b0,
              "GemmArgs layout (descriptor line touches)");

// ---- B = 1 act chain (rle_act_sample, one observation): ONE launch of nwg workgroups
// (kernels.hip rle_act_chain).  Workgroup w owns row block w of every hidden layer, its next
// layer's weights loaded into registers while the current one is handed off; after each layer
// the workgroups exchange the layer output as 8-byte {value, call tag} granules (sc1 stores /
// loads: a stale granule is re-read until its tag is this call's), so a layer costs one
// hand-off instead of one kernel launch.  The head runs with the act epilogue (ActArgs):
// TD7 / TD3 row block w in workgroup w, SAC whole in workgroup 0; each head workgroup then
// stores the call tag into its pinned `done` slot with a system-scope release; the host polls.
constexpr int kActMaxL = 7;
constexpr int kActVec = 512;   // floats per LDS vector slot
struct ActLayer {
  const float* wn;     // weights, N image [out][K] (fragment blocks)
  const float* bias;   // [16 * row blocks]
  int cbn, rbs, out;   // column blocks (K / 16), row blocks, rows
  int act;             // ACT_*
  int in0, in1;        // input vector slots (in1 < 0: one segment); in1 starts at column k0
  int k0;              // padded width of segment 0
  int norm;            // output AvgL1Norm'd (sale.py:11-13) before its consumers read it
  int dst;             // output vector slot
  int sync;            // exchange after this layer (0: the next layer does not read it)
  int pad_[2];
};
struct ActChainArgs {
  ActLayer L[kActMaxL];
  int nl, nwg;
  int sac;             // last layer: SAC raw head (mean | log_std) + rsample law, else tanh + EPI_ACT law
  int Sp;              // observation slot width
  unsigned long long* xbuf;  // [nl][kActVec] granules {float bits, tag}
  unsigned tag;        // this call's tag (never 0)
  int heads;           // head workgroups (0 .. heads-1) that set their `done` slot per call
  int* err;            // 1: a hand-off timed out (pinned)
  unsigned* done;      // [64] per head workgroup: tag of the last call it finished (pinned)
  unsigned long long* stamps;  // optional [nwg][16] s_memrealtime phase stamps (RLE_ACT_PROF)
  int mode;            // ActArgs::ctl[0] semantics, carried here (no host-memory read in the kernel)
  int fail_wg;         // tests (RLE_ACT_FAIL_WG, one call): this workgroup withholds its layer-0 granules
  unsigned ctr_lo, ctr_hi;  // Philox counter of this call
  float eps[32];       // mode 2: the draw [A] (A <= 32)
  ActArgs ao;
  float min_log_std, max_log_std;
  float obs[384];      // the observation (padded, zeros)
};

// Kernel argument of one level launch: the workgroup -> op table travels in the
// kernarg segment (one scalar load burst) instead of being searched in memory.
constexpr int kLevelOps = 12;  // ops per launch: the op table is 12 preloaded kernel arguments
struct LevelArgs {
  const Op* ops;
  unsigned long long* trace;  // optional phase timestamps [wg][4] (s_memrealtime, 100 MHz)
  // op q: first workgroup (bits 0-15; 0xffff past the last op) | kind << 16 (4 bits) | GEMM
  // variant id << 20 (GemmArgs::vid: the variant is chosen before any descriptor load)
  unsigned entry[kLevelOps];
};
constexpr int kMaxLevelWG = 0xfffe;  // workgroups per launch (16-bit entry field)

// One rle_level dispatch as an AQL packet needs it (engine.cpp direct dispatch, rle_plan.dispatch 1): the
// kernel-argument bytes (rle_level<false>'s 76-byte segment: no hidden arguments) and the
// workgroup count.  launch_level appends one per dispatch while g_level_rec is set.
struct LevelLaunch {
  unsigned char ka[80];
  unsigned grid;  // workgroups
  int ks;         // the rle_level instance (KernelSet)
};

// Device control block.
struct Ctrl {
  long long counters[16];   // [0..3] adam steps per optimizer, [4] rng step, [5] tape pos
  long long size;           // replay size (mirrors host)
  int info_slot;
  int tape_mode;
  int vmax_key, vmin_key;   // ordered-int keys of value_max / value_min
  float vt[2];              // value_target_max, value_target_min
  float max_priority;
  float log_alpha, la_m, la_v;
  long long la_t;
  float adam_step[4];       // per optimizer counter 0..2: lr / (1 - 0.9^(t+1)), t = counters[c]
  float adam_bc2s[4];       // sqrt(1 - 0.999^(t+1))
};

enum Counter : int { CNT_ADAM_Q = 0, CNT_ADAM_PI = 1, CNT_ADAM_ENC = 2, CNT_RNG = 4, CNT_TAPE = 5 };

}  // namespace rle
