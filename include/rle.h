/*
 * rle.h — C ABI of the MI355X off-policy update engine (librle.so).
 *
 * The reference (seungju-k1m/sac-td3-td7) has no FFI: its hot path is the
 * Python method Agent.train_ops(batch, replay_buffer) (rl/agent/abc.py:23-28)
 * driven by run_train_ops (rl/runner/run.py:87-96).  This ABI sits UNDER the
 * Python classes that mirror that interface (sac-td3-td7_amd/rl); each entry
 * point below names the reference interface it replaces.
 *
 * Conventions: every function returns 0 on success or a negative error code;
 * rle_last_error() returns a thread-local message for the last failure.  All
 * pointers are host pointers borrowed for the duration of the call; the
 * engine owns all device memory.  A handle is bound to one device and one
 * HIP stream and is not thread-safe.  Plain C types only (no torch types).
 */
#ifndef RLE_H
#define RLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define RLE_TD7 0
#define RLE_TD3 1
#define RLE_SAC 2

#define RLE_INFO_MAX 8

#define RLE_OK 0
#define RLE_EINVAL (-1)
#define RLE_EHIP (-2)
#define RLE_ESTATE (-3)

typedef struct rle_replay rle_replay;
typedef struct rle_engine rle_engine;

typedef struct rle_config {
  int algo;                 /* RLE_TD7 / RLE_TD3 / RLE_SAC */
  int state_dim, action_dim;
  int hidden;               /* hidden width (TD7: hdim; TD3/SAC: every hidden layer unless n_hidden is set) */
  int batch;                /* B, 1..1024 (padded to 16 rows inside; the padded rows count in nothing) */
  int use_lap;              /* TD7/TD3: LAP Huber + priority update */
  float discount;           /* td7.py:37 / td3.py:36 / sac.py:30 */
  float policy_lr, critic_lr;
  float tau;                /* TD3/SAC Polyak */
  float target_policy_noise, noise_clip;
  int policy_freq;          /* TD7/TD3 */
  int target_update_rate;   /* TD7 hard update period */
  float min_log_std, max_log_std;  /* SAC */
  float tmp;                /* SAC: < 0 => auto temperature (sac.py:36,55) */
  unsigned long long seed;  /* Philox stream for sampling / noise */
  int device;
  /* Net shapes beyond the defaults (make_nn, td7.py:46-61 / td3.py:44-58 / sac.py:40-52): */
  int zs_dim;               /* TD7: SALE embedding width (sale.py:23 zs_dim); 0 = hidden.  `hidden` is hdim */
  int n_hidden;             /* TD3/SAC: hidden layers of make_mlp (mlp.py:10-35), 2..RLE_MAX_HIDDEN; 0 = two
                               layers of `hidden` (mlp.py:45-47) */
  int hidden_sizes[8];      /* TD3/SAC: their widths, input side first (each a multiple of 4, <= 512) */
  /* Hidden-layer activations (RLE_ACT_*; 0 = the reference default of that net).  TD7: SALEActor / SALECritic /
     SALEEncoder `activ` (sale.py:25,67,97: ReLU / ELU / ELU); TD3/SAC: make_mlp's action_fn of the policy and of the
     critics (mlp.py:13, default ReLU; act_encoder must be 0).  A non-default activation runs its programs on the
     extended kernel instance without RLE_FUSE_PRELAYER, PRE, TWOSTAGE and SACPRE (and, for identity critics, without
     QDOT and HEADDX). */
  int act_actor, act_critic, act_encoder;
} rle_config;
#define RLE_MAX_HIDDEN 6
#define RLE_ACT_DEFAULT 0
#define RLE_ACT_RELU 1
#define RLE_ACT_ELU 2       /* alpha = 1 (F.elu / nn.ELU defaults) */
#define RLE_ACT_IDENTITY 3  /* action_fn "Identity" / nn.Identity(): no activation between the Linear layers */

/* Step-program plan: the schedule and tile-plan choices that decide how the step's reductions are
 * split (so its fp32 summation order) and how its ops are fused.  Every engine starts from the
 * defaults (rle_plan_default); rle_set_plan changes them before the engine's first step, and
 * rle_get_plan reports the values in effect.  No environment variable changes a plan. */
#define RLE_FUSE_PRELAYER (1u << 0)  /* small-K first layers recomputed in-tile by the next layer   */
#define RLE_FUSE_PRE      (1u << 1)  /* actor output layer recomputed in-tile by its consumers      */
#define RLE_FUSE_QDOT     (1u << 2)  /* TD7 q from per-tile row partials of the last hidden layers  */
#define RLE_FUSE_HEADDX   (1u << 3)  /* critic loss heads fused into the DX of the last hidden layer */
#define RLE_FUSE_NBDEFER  (1u << 4)  /* TD7 AvgL1Norm backward deferred into the weight gradient    */
#define RLE_FUSE_SACFWD   (1u << 5)  /* SAC rsample in the actor raw head's epilogue                */
#define RLE_FUSE_SACBWD   (1u << 6)  /* SAC squashed-Gaussian backward in the da DX's epilogue      */
#define RLE_FUSE_FOLD     (1u << 7)  /* TD7 fixed target encoder's zsa3 folded into target critics  */
#define RLE_FUSE_PIPOLYAK (1u << 8)  /* TD3 aliased target-policy Polyak in the actor's Adam         */
#define RLE_FUSE_ENDSPLIT (1u << 9)  /* step end split into counters and info row                  */
#define RLE_FUSE_PRIOSAMPLE (1u << 10) /* LAP priority update applied by the next batch's sampler (opt-in,
                                        fuse_on): one level fewer per step pair, but the heavy critic
                                        weight-gradient ops then share a level with the next batch's
                                        first layers (TD7 Humanoid A/B: -4.5%)                        */
#define RLE_FUSE_TWOSTAGE (1u << 11) /* TD3 target critics' first layer (behind the pre-GEMM target
                                        action) recomputed in-tile by their second layer             */
#define RLE_FUSE_SACPRE   (1u << 12) /* SAC raw head + target rsample recomputed in-tile by the target
                                        critics' first layer                                         */
#define RLE_FUSE_NORMFIN  (1u << 13) /* TD7: the AvgL1Norm row means finalized once (a small op the level after
                                        their producer) for the weight gradients' per-row tables      */
#define RLE_FUSE_OPT_IN RLE_FUSE_PRIOSAMPLE  /* fusions off unless set in fuse_on                      */
typedef struct rle_plan {
  int level_cap;        /* workgroups per level the tile planner targets (0: resident capacity; TD7 at B >= 1024 5/4
                           (3/2 when lpt is 0); TD3 7/8 when lpt is 0) */
  int steps_per_graph;  /* steps per multi-step graph (-1: TD7 6, SAC 8, TD3 16; 0: single-step only)  */
  int pre_tn;           /* tile width of pre-GEMM consumers (0: TD3 64, else 32)                         */
  int pl_tn;            /* tile width of pre-layer consumers (0: SAC 32, else 64)                        */
  int tn_min;           /* narrowest GEMM tile (0: 16)                                                   */
  int flat_div;         /* Polyak / copy workgroups count 1 / flat_div in the planner (0: 4)            */
  int balance;          /* rebalance pass: 0 off, 1 any item, 2 no Adam items, 3 no Adam items and only under a
                           twice-longer op (-1: TD7 3, SAC 2, TD3 1)                                        */
  int tiny_w, uni_w, tiny_wg;  /* rebalance weights: step end, uniform sampler, tiny-op bound (-1: 30,
                                  SAC 30 / TD3 8 / TD7 60, 2) */
  int sched_cap;        /* 1: the scheduler defers ops past level_cap workgroups to a later level       */
  unsigned fuse_off;    /* RLE_FUSE_* bits switched off (A/B, tests); 0 = every default fusion on       */
  unsigned fuse_on;     /* RLE_FUSE_OPT_IN bits switched on                                             */
  int rb;               /* 1: 32 / 64-wide weight-gradient tiles register-blocked (the 4 waves split the batch
                           rows, each accumulates every column block; -1: default)                       */
  int pl_w;             /* rebalance weight added to GEMMs with an in-tile prologue (pre-layer, two-stage,
                           SAC raw head; -1: default, SAC 24, else 0)                                     */
  int lap_w, head_w, adam_w; /* rebalance weights: LAP sampler, loss head, added to Adam-epilogue GEMMs
                                (-1: 60, 60, SAC 16 / else 8)                                             */
  int wide;             /* 64 / 32: forward / input-gradient GEMMs over >= 64 rows as 64 x 64 / 64 x 32 tiles with
                           every W chunk staged once in LDS for the tile's four 16-row blocks (kernels.hip
                           gemm_wide; 1 = 64; 0 off; -1: default = off, slower than the 16-row tiles as
                           measured)                                                     */
  int lpt;              /* 1: each level's ops in its launch ordered longest first (estimated workgroup time),
                           so a level with more workgroups than the device holds dispatches its long tiles in
                           the first round and its long workgroups start first; 0: program order; -1: default = 1) */
  /* Launch choices (they change no result: the same ops, tiles and summation order either way) */
  int dispatch;         /* how the step programs' level launches reach the device: 1 direct AQL kernel-dispatch
                           packets in the engine's own HSA queue; 0 hipGraph replays on the engine's HIP stream;
                           2 level launches on the stream without a graph (A/B); -1: default = 1            */
  int dpf;              /* 1: each launch leads with one workgroup per XCD that loads the next launch's op
                           descriptors into that XCD's L2; 0 off (A/B); -1: default = 1                     */
  int xcd;              /* 1: XCD-aware tile order (each XCD a compact band of a GEMM's tiles); 0 row-major
                           (A/B); -1: default = 1                                                          */
} rle_plan;

/* ---- replay memory: rl/replay_memory/{lap,simple}.py ---------------------- */

/* LAPReplayMemory.__init__ (lap.py:15-29) / SimpleReplayMemory.__init__ (simple.py:15-27). */
int rle_replay_create(int device, long long capacity, int state_dim, int action_dim, int lap,
                      rle_replay** out);
int rle_replay_destroy(rle_replay* r);
/* append (lap.py:31-43): rows of fp32 state[S], action[A] (already a/scale - bias), reward,
 * next_state[S], notdone (1 - terminated).  count rows, host pointers. */
int rle_replay_append(rle_replay* r, const float* state, const float* action, const float* reward,
                      const float* next_state, const float* notdone, long long count);
/* ptr / size / max_priority (lap.py:18-29, len = ptr Q6). */
int rle_replay_state(rle_replay* r, long long* ptr, long long* size, float* max_priority);
/* Test / bench hooks. */
int rle_replay_fill_random(rle_replay* r, long long count, unsigned long long seed);
int rle_replay_get_priority(rle_replay* r, float* out, long long n);
int rle_replay_set_priority(rle_replay* r, const float* p, long long n, float max_priority);
/* Device LAP/uniform index search with given uniforms (lap.py:47-54, simple.py:45-54). */
int rle_replay_sample_indices(rle_replay* r, int n, const float* u, long long* ind_out);
/* LAPReplayMemory.update_priority (lap.py:66-69) with explicit indices (any values; with a
 * priority below 1 the block sums are recomputed instead of updated in place).  Every replay
 * operation waits for the steps already enqueued by engines bound to the replay. */
int rle_replay_update_priority(rle_replay* r, int n, const long long* ind, const float* p);
/* LAPReplayMemory.reset_max_priority (lap.py:71-73). */
int rle_replay_reset_max_priority(rle_replay* r);
/* Gather rows (state, action, reward, next_state, notdone) for indices (lap.py:55-60). */
int rle_replay_gather(rle_replay* r, int n, const long long* ind, float* state, float* action,
                      float* reward, float* next_state, float* notdone);

/* ---- agent: rl/agent/{td7,td3,sac}.py ------------------------------------- */

/* TD7.__init__ (td7.py:34-87) / TD3.__init__ (td3.py:33-74) / SAC.__init__ (sac.py:27-77). */
int rle_create(const rle_config* cfg, rle_engine** out);
int rle_destroy(rle_engine* e);
/* The default plan (every field "default"); the engine's plan before its first step; the plan in
 * effect (defaults resolved for this engine's algorithm and device). */
int rle_plan_default(rle_plan* out);
int rle_set_plan(rle_engine* e, const rle_plan* plan);
int rle_get_plan(rle_engine* e, rle_plan* out);
/* Bind the replay the step samples from (the replay_buffer arg of train_ops). */
int rle_bind_replay(rle_engine* e, rle_replay* r);
/* Parameter import/export in the reference's state_dict layout (Agent.load_state_dict,
 * td7.py:114-125; deepcopy / pickle, abc.py:38-55).  net: "policy", "q1", "q2", "target_q1",
 * "target_q2", "encoder", "fixed_encoder", "fixed_encoder_target"; name: e.g. "q01.weight",
 * "mlp.2.bias"; SAC temperature: net "tmp", name "log_alpha". */
int rle_param_numel(rle_engine* e, const char* net, const char* name, long long* numel);
int rle_get_param(rle_engine* e, const char* net, const char* name, float* out, long long n);
int rle_set_param(rle_engine* e, const char* net, const char* name, const float* in, long long n);
/* Optimizer state: which = 0 (m) / 1 (v) of the param's Adam; step counter per optimizer. */
int rle_get_adam(rle_engine* e, const char* net, const char* name, int which, float* out, long long n);
int rle_set_adam(rle_engine* e, const char* net, const char* name, int which, const float* in,
                 long long n);
/* Device counters: [0] critic Adam t, [1] policy Adam t, [2] encoder Adam t, [3] n_runs,
 * [4] rng step, [5] SAC temperature Adam t. */
int rle_get_counters(rle_engine* e, long long* out6);
int rle_set_counters(rle_engine* e, const long long* in6);
// Philox counter of the act path's exploration draws (rle_act_sample mode 1): carried across
// engine rebuilds and pickling so a rebuilt agent does not repeat earlier draws (the reference's
// torch.randn stream, td7.py:153, never restarts either).
int rle_get_act_counter(rle_engine* e, unsigned long long* out);
int rle_set_act_counter(rle_engine* e, unsigned long long v);
/* TD7 value clipping state [value_max, value_min, value_target_max, value_target_min]. */
int rle_get_value_bounds(rle_engine* e, float* out4);
int rle_set_value_bounds(rle_engine* e, const float* in4);

/* n_steps x Agent.train_ops(replay.sample(B), replay) (run_train_ops, run.py:87-96), fully on
 * device incl. sampling and LAP priority update.  info_out: [n_steps][RLE_INFO_MAX] (per-agent
 * key order; NaN = None).  One host sync per call. */
int rle_step(rle_engine* e, int n_steps, float* info_out);
/* Benchmark form of rle_step: n_steps without info readback; *gpu_ms = the engine's elapsed time.
 * Under the default direct AQL dispatch (rle_plan.dispatch 1; the levels go to the engine's own HSA
 * queue, opened at its first step) that is HOST WALL time from the first doorbell to the last
 * packet's completion signal; with dispatch 0 / 2 (hipGraph replays / launches on the stream) it is
 * HIP event time on the engine's stream.  The host thread sleeps while the expected remainder of the burst exceeds 150 us
 * and spins only for the tail (rle_aql_wait_plan); a burst that does not complete within 60 s closes
 * the engine's queue (every later step fails).  Syncs once at the end. */
int rle_step_timed(rle_engine* e, int n_steps, float* gpu_ms);
/* Enqueue n_steps as rle_step does, without any host sync or info readback (the device info
 * ring keeps the last rows); rle_synchronize waits.  Lets one host thread drive several
 * independent seeds (engines, each on its own stream) on one GPU concurrently -- SURVEY
 * §8(f) rank 4, beyond the reference's one agent per process (scripts/td7_exp.sh:1-4). */
int rle_step_async(rle_engine* e, int n_steps);
/* Parity / explicit-batch mode: replace draws of the next n_steps with tapes; each tape
 * is optional and a NULL one keeps its Philox stream.  u [n][B] (torch.rand in sample),
 * eps [n][B][A] (randn_like target noise, or SAC next-state rsample noise), eps_pi [n][B][A]
 * (SAC policy rsample noise; SAC takes eps and eps_pi together), ind [n][B] (explicit
 * indices, e.g. the batch a replay's sample() drew; overrides u).  At least one of u / ind.
 * Pass n_steps = 0 to return to Philox; stepping past the tape's end is an error. */
int rle_set_tapes(rle_engine* e, int n_steps, const float* u, const float* eps, const float* eps_pi,
                  const long long* ind);
/* Last sampled indices (LAPReplayMemory.ind) [B]. */
int rle_last_indices(rle_engine* e, long long* ind_out);
/* Agent.sample / _inference_action forward (td7.py:158-162, td3.py:131-135, sac.py:154-159):
 * obs [n][S] (n <= 1024) -> out [n][W]: TD7 tanh actor output (W = A); TD3 actor MLP output
 * before tanh (W = A); SAC raw (mean | log_std) head (W = 2A).  Raw network outputs (evaluation and
 * diagnostics); rle_act_sample returns the environment action. */
int rle_act(rle_engine* e, const float* obs, int n, float* out);
/* Agent.sample (td7.py:141-156, td3.py:114-129, sac.py:132-152) as ONE device program: the B = n
 * actor (TD7: + fixed encoder) forward, exploration noise, clip and the action map, written by the
 * last kernel straight into pinned host memory.  obs [n][S] -> out [n][A] environment actions:
 *   TD7 / TD3: clip(tanh(pi(s)) + exploration_noise * eps, -1, 1) * scale + bias
 *   SAC:       tanh(mean + exp(clamp(log_std)) * eps) * scale + bias
 * mode 0: deterministic (eps = 0); 1: eps from the engine's own Philox stream (counter advanced
 * per call; the reference draws torch.randn_like from torch's global generator instead);
 * 2: eps given as eps [n][A] (parity tape).  Syncs. */
int rle_act_sample(rle_engine* e, const float* obs, int n, int mode, const float* eps, float* out);
/* The environment action map of rle_act_sample: scale [A], bias [A] (get_action_bias_scale,
 * rl/utils/miscellaneous.py:59-66) and TD7 / TD3 exploration_noise (td7.py:41, td3.py:40).
 * Default: identity, 0.1. */
int rle_set_action_map(rle_engine* e, const float* scale, const float* bias, float exploration_noise);
/* Forward diagnostics on a given batch (host rows s [n][S], a [n][A], n <= 1024), for parity
 * checks of the nets the step trains:
 *   RLE_EVAL_Q:   critic `net`'s estimate_q_value -> out [n].  TD7 (SALECritic, sale.py:106-121)
 *                 on zs = encode_state(s), zsa = encode_state_action(zs, a) of encoder `enc`
 *                 (online critics use "fixed_encoder", target critics "fixed_encoder_target",
 *                 td7.py:175-230); TD3/SAC (MLPCritic, mlp.py:98-101) ignore `enc`.
 *   RLE_EVAL_ZS:  encoder `net`'s encode_state(s) (sale.py:41-46) -> out [n][zs_dim] (a unused).
 *   RLE_EVAL_ZSA: encoder `net`'s encode_state_action(encode_state(s), a) (sale.py:48-55)
 *                 -> out [n][zs_dim].
 * Runs on the engine's stream after any enqueued step; syncs. */
#define RLE_EVAL_Q 0
#define RLE_EVAL_ZS 1
#define RLE_EVAL_ZSA 2
int rle_eval(rle_engine* e, int what, const char* net, const char* enc, const float* s, const float* a, int n,
             float* out);
/* SAC._rsample (sac.py:164-172) on given distribution parameters through the step's own
 * squashed-Gaussian op: log_std clamped to [min_log_std, max_log_std] (sac.py:154-159),
 * u = mean + eps * exp(log_std), action = tanh(u), log_pi [n] (annotation.py:12 EPS). */
int rle_sac_rsample(rle_engine* e, const float* mean, const float* log_std, const float* eps, int n, float* action,
                    float* log_pi);
/* Info rows [n][RLE_INFO_MAX] of the last rle_step / rle_step_async call (its first n steps;
 * n <= 4096).  Syncs the engine stream. */
int rle_get_info(rle_engine* e, int n, float* out);
/* rle_level dispatches enqueued so far by rle_step* (every step graph replay: single-step,
 * multi-step, batch prime, hard update, fold refresh); differences over a timed burst give
 * the exact launches per gradient step (roofline accounting).  Engine-side, no sync. */
int rle_launch_count(rle_engine* e, long long* n);
/* Launches per gradient step of each captured graph kind (for roofline accounting). */
int rle_graph_stats(rle_engine* e, int* levels_policy_step, int* levels_plain_step);
/* Human-readable description of a captured graph (which: 0 policy step, 1 plain step,
 * 2 hard update): one line per level with workgroups and ops.  Writes at most len bytes. */
int rle_graph_describe(rle_engine* e, int which, char* buf, int len);
/* Diagnostics: phase timestamps of the last replay of a captured graph (graphs are
 * traced only when RLE_TRACE=1 is set in the environment before the first step).
 * out[4*w .. 4*w+3] = s_memrealtime (100 MHz) at entry, main-loop start, main-loop
 * end (GEMM ops) and exit of workgroup w, levels concatenated in order; *n_out = number
 * of workgroups written (0 when tracing is off). */
int rle_graph_trace(rle_engine* e, int which, unsigned long long* out, long long cap, long long* n_out);
/* Timestamps per workgroup in rle_graph_trace rows: 4, or 16 in diagnostics builds
 * (-DRLE_TRACE_FINE: slots 4.. are finer in-op stamps). */
int rle_trace_stride(void);
/* The AQL wait policy of rle_step / rle_step_timed (no GPU): given the expected duration of what is
 * outstanding and the time waited so far, returns 0 spin on the completion signal, 1 sleep *sleep_us
 * then check again, 2 time out (the engine's queue is then closed). */
int rle_aql_wait_plan(double expected_us, double elapsed_us, double timeout_s, double* sleep_us);
/* Self-test of the AQL queue's failure handling (no GPU, no HSA call): a queue closed by a timed-out
 * burst refuses new bursts and completes at once, also for other engines sharing its hardware queue,
 * and no doorbell publishes a run of packets that straddles the ring's end.  0 when every check holds. */
int rle_aql_selftest(void);
/* Copy all weights/optimizer state/counters of src into dst (checkpoint agent,
 * ckpt_agent.load_state_dict(agent), run_w_checkpoint.py:140). Same config required. */
int rle_copy_state(rle_engine* dst, rle_engine* src);
int rle_synchronize(rle_engine* e);

const char* rle_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* RLE_H */
