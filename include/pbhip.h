/*
 * pbhip.h -- C-ABI of libpbhip.so, the MI355X (gfx950) batched
 * Metropolis-Hastings / CondCov-Gibbs engine behind probayes_amd.
 *
 * The reference (probayes 0.0.8) has no C/FFI layer: its boundary is the pure
 * Python SP API.  Each entry point below replaces one piece of the per-chain
 * Python call stack of SP.next (sp.py:221-258) for N chains at once; the
 * reference interface it stands in for is cited beside it.  Bindings: the
 * ctypes stub in probayes_amd/_lib.py (and INTEGRATION.md).
 *
 * Conventions
 *  - Every function returns int status: 0 = PBH_OK, < 0 = error; the message
 *    is in pbh_last_error() (thread-local).  No function throws or aborts.
 *  - Host buffers are caller-allocated; the engine owns every device buffer.
 *  - One engine per device, calls on one engine must not be concurrent.
 *    Multi-GPU = one process (or thread) per device + pbh_rccl_*.
 *  - Chain-major arrays on the host are [chain][dim]; device and trace arrays
 *    are dim-major with the chain index fastest ([step][dim][chain]).
 *  - All arithmetic is IEEE fp64 (constants.py:7 DEFAULT_FP_PRECISION = 64).
 */
#ifndef PBHIP_H
#define PBHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBH_ABI_VERSION 6
#define PBH_MAX_DIM 32

#define PBH_OK 0
#define PBH_ERR_ARG (-1)
#define PBH_ERR_HIP (-2)
#define PBH_ERR_STATE (-3)
#define PBH_ERR_UNSUPPORTED (-4)
#define PBH_ERR_RCCL (-5)

/* Joint density forms the engine lowers. */
enum pbh_target_kind {
  PBH_TARGET_DIAG_GAUSS = 1,  /* sum_i norm.logpdf(x_i, mu_i, sigma_i)        */
  PBH_TARGET_NORM_IID = 2,    /* np.sum(norm.logpdf(obs, x[loc], x[scale]))   */
  PBH_TARGET_GMM = 3,         /* logsumexp_k(logw_k + sum_i logpdf(x_i,mu_ki,sd_k)) */
  PBH_TARGET_NORM_PDF = 4,    /* prod_i norm.pdf(x_i, loc_i, scale_i)          */
  PBH_TARGET_UNIFORM_PDF = 5, /* prod_i uniform.pdf(x_i, lo_i, scale_i)        */
  PBH_TARGET_MVN = 6          /* multivariate_normal.pdf at the permuted x     */
};
enum pbh_pscale { PBH_PSCALE_LOG = 0, PBH_PSCALE_LIN = 1 };
enum pbh_scores {
  PBH_SCORES_HASTINGS = 1, PBH_SCORES_METROPOLIS = 2, PBH_SCORES_GIBBS = 3
};
enum pbh_tran_kind { PBH_TRAN_CONST = 1, PBH_TRAN_GAUSS_PDF = 2 };
enum pbh_proposal_kind {
  PBH_PROP_GAUSS = 1,   /* callable Delta(norm.rvs(loc, scale)) per dim        */
  PBH_PROP_SPHERE = 2,  /* tuple delta, field.py:509-531                      */
  PBH_PROP_UNIFORM = 3, /* list delta, variable.py:625-633                    */
  PBH_PROP_GIBBS = 4,   /* CondCov conditional draw, cond_cov.py:42-65        */
  PBH_PROP_VARDELTA = 5 /* per-variable deltas (a Delta of containers, or a
                           bare scalar Field delta): field.py:266-306,
                           variable.py:600-640                                */
};
/* Per-variable delta modes of PBH_PROP_VARDELTA (Variable.eval_delta,
 * variable.py:618-633).  Replay streams hold, per variable, the raw uniform
 * (POLARITY, UNIFORM), the randint value (RANDINT) or nothing (FIXED).     */
enum pbh_var_delta {
  PBH_VAR_FIXED = 0,     /* bare scalar: x + delta                             */
  PBH_VAR_POLARITY = 1,  /* (delta,): +delta if uniform() > 0.5 else -delta    */
  PBH_VAR_UNIFORM = 2,   /* [delta]: uniform(-delta, delta)                    */
  PBH_VAR_RANDINT = 3    /* [delta] of an int variable: randint(-delta, delta),
                            bounds truncated toward zero as NumPy does         */
};
enum pbh_rng_mode {
  PBH_RNG_REPLAY = 0,    /* randoms read from a caller-supplied [T][R][N]
                            stream; reference arithmetic (parity mode)        */
  PBH_RNG_PHILOX = 1,    /* production: Philox-4x32-10 keyed by (seed, global
                            chain id); fp64 Box-Muller normals on 52-bit
                            uniforms (table-driven log / sqrt / sincos, a few
                            ulp from libm), fp64 chain arithmetic in the
                            production (FMA) forms                            */
  PBH_RNG_PHILOX_F64 = 2, /* Philox-4x32-10 with libm fp64 Box-Muller normals
                            and the reference arithmetic of REPLAY             */
  PBH_RNG_XOSHIRO = 3,   /* production: one xoshiro128** stream per chain (per
                            lane half), seeded by SplitMix64 of (seed, global
                            chain id); otherwise as PHILOX                    */
  PBH_RNG_PHILOX_FP32 = 4 /* comparison only (the round-1 production form):
                            as PHILOX but fp32 hardware Box-Muller normals on
                            24-bit uniforms (|z| <= 5.77) with exact sign
                            symmetry; lane-pair diagonal-Gauss kernel only   */
};
/* What pbh_run accumulates besides the trace (pbh_set_collect). */
enum pbh_collect {
  PBH_COLLECT_MOMENTS = 1   /* per-chain sum / sumsq / n_acc (pbh_get_moments) */
};

/* Joint density + acceptance (replaces RF.set_prob/set_tran + SP.set_scores:
 * rf.py:91,169; sp.py:57-100; prob.py:331-380; rf_utils.py:10-42).
 * All pointers are host pointers, copied into device memory by the call.   */
typedef struct pbh_model {
  int32_t dim;          /* d, 1..PBH_MAX_DIM                                  */
  int32_t target_kind;  /* enum pbh_target_kind                               */
  int32_t pscale;       /* enum pbh_pscale of the density (pscales.py:21-41)   */
  int32_t scores;       /* enum pbh_scores (sp_utils.py:87-91)                */
  /* target parameters (meaning per kind):
   *   DIAG_GAUSS : a = mu[d], b = sigma[d], c = log(sigma)[d], e = 1/sigma[d]
   *   NORM_IID   : a = obs[n], n = n_obs, i0 = loc dim, i1 = scale dim
   *   GMM        : a = logw[K], b = mu[K*d], c = sd[K], e = log(sd)[K], n = K
   *   NORM_PDF   : a = loc[d], b = scale[d]
   *   UNIFORM_PDF: a = lo[d], b = scale[d]
   *   MVN        : a = mean[d], b = whitening U[d*d] row-major (scipy
   *                CovViaPSD._LP), c = {rank*log(2pi) + log_pdet}; the density
   *                is taken at x[perm] with prob.py:354-357's fixed perm     */
  const double *a, *b, *c, *e;
  const int32_t *perm;
  int64_t n;
  int32_t i0, i1;
  /* joint=True uniform root prior (rv_utils.py:8-47); has_prior = 0/1 */
  int32_t has_prior;
  const double *prior_lo, *prior_hi;
  const int32_t *prior_lo_incl, *prior_hi_incl;
  double prior_logp;
  /* per-dim change of variable: 1 = (log, exp) ufun (variable.py:693-697) */
  const int32_t *ufun;
  /* transition q(x'|x) (rf.py:169-239, 490-538) */
  int32_t tran_kind;    /* enum pbh_tran_kind                                 */
  int32_t tran_sym;     /* 1 = symmetric (r = None), 0 = tuple tran           */
  double tran_value;    /* CONST: value of q                                  */
  double tran_scale;    /* GAUSS_PDF: sigma                                   */
  const double *tran_offset;  /* GAUSS_PDF: loc offset per dim               */
  const int32_t *tran_order;  /* GAUSS_PDF: multiplication order of dims     */
} pbh_model;

/* Proposal (replaces RF.set_delta / Field.eval_delta / apply_delta:
 * field.py:220-317, 469-552; variable.py:600-739).                         */
typedef struct pbh_proposal {
  int32_t kind;             /* enum pbh_proposal_kind (not GIBBS)            */
  const double *loc;        /* GAUSS: loc[d]                                  */
  const double *scale;      /* GAUSS: scale[d]                                */
  const int32_t *order;     /* GAUSS: dim receiving the j-th draw             */
  double delta;             /* SPHERE: delta (already * rss if scale=True)    */
  const double *lengths;    /* SPHERE: per-dim multiplier (lengths or 1)      */
  const double *delta_vec;  /* UNIFORM: delta[d]                              */
  /* Optional covariance-matrix random walk (any kind): the base delta is
   * multiplied by tfun[d*d] (row-major), i.e. delta' = tfun . delta, as
   * RF.eval_delta does with the Cholesky factor that RF.set_tran(ndarray)
   * installs (rf.py:210-220, 340-354).  NULL = no tfun.                    */
  const double *tfun;
  /* VARDELTA: var_mode[d] (enum pbh_var_delta); the steps are delta_vec[d] */
  const int32_t *var_mode;
  /* Optional, any MH kind.  var_int[d] = 1: an int variable, whose proposed
   * value is truncated toward zero (revtype, variable.py:697).  NULL = none. */
  const int32_t *var_int;
  /* Optional, any MH kind: bound=True (variable.py:700-739), per dim
   * bound_on[d]; limits bound_lo[d] <= bound_hi[d] (the vset limits) and
   * which are exclusive (bound_xlo[d], bound_xhi[d]).  With both limits
   * closed the proposal is clamped; an exclusive side it crosses returns the
   * predecessor value (both exclusive: anything outside (lo, hi); one
   * exclusive: strictly beyond it), the other side is clamped.  NULL = none. */
  const int32_t *bound_on;
  const double *bound_lo, *bound_hi;
  const int32_t *bound_xlo, *bound_xhi;
} pbh_proposal;

/* CondCov Gibbs tables (replaces CondCov.__init__ + RF.eval_tfun cycling:
 * cond_cov.py:22-39, rf.py:446-458).  Precomputed on the host like the
 * reference does (np.linalg.inv, norm.cdf).                                  */
typedef struct pbh_gibbs {
  const double *mean;   /* mu[d]                                             */
  const double *coef;   /* coef[d*(d-1)]: row i = Sigma_{i,-i} Sigma_{-i,-i}^-1 */
  const double *stdv;   /* conditional sd[d]                                 */
  const double *cdf;    /* cdf limits [d*2] (lo, hi)                         */
  int32_t tsteps;       /* coordinates per SP step (rf.py:446-452)            */
} pbh_gibbs;

typedef struct pbh_engine pbh_engine;

/* ---- engine lifetime ---------------------------------------------------- */
const char *pbh_last_error(void);
int pbh_abi_version(void);
int pbh_device_count(int *count);
int pbh_create(int device, pbh_engine **out);
/* Destroys the engine.  Its device buffers, stream and events (drained) stay
 * in a process-wide cache for the next engine of the same device (one
 * engine per SP.sampler call); PBH_CACHE_MB bounds the cached buffers
 * (default 32 768, 0: no cache).                                            */
int pbh_destroy(pbh_engine *eng);
/* Frees every cached buffer and stream (an allocation that fails does this
 * itself and retries).                                                       */
int pbh_cache_release(void);
/* Cached (idle) bytes, and allocations served from / missed in the cache.  */
int pbh_cache_info(int64_t *idle_bytes, int64_t *hits, int64_t *misses);

/* ---- model ------------------------------------------------------------- */
int pbh_set_model(pbh_engine *eng, const pbh_model *model);
int pbh_set_proposal(pbh_engine *eng, const pbh_proposal *prop);
int pbh_set_gibbs(pbh_engine *eng, const pbh_gibbs *gibbs);

/* ---- chains and randomness (SP.sampler(init, ...): sp.py:261-278) ------- */
/* Allocates chain state for chains [chain_offset, chain_offset + n) and copies
 * init [n][d]; the first pbh_run step proposes from init and auto-accepts
 * (sp_utils.py:24-25, App. A-3).                                            */
int pbh_init_chains(pbh_engine *eng, int64_t n_chains, int64_t chain_offset,
                    const double *init);
/* Global step index of the first pbh_run step (default 0): the phase of the
 * CondCov coordinate cycle, which the reference keeps per RF across samplers
 * (RF.__cond_mod, rf.py:446-452), and the Philox step counter.  Only right
 * after pbh_init_chains.                                                     */
int pbh_set_step(pbh_engine *eng, int64_t step);
int pbh_set_rng(pbh_engine *eng, int32_t mode, uint64_t seed);
/* Checkpoint / resume: everything a chain needs to continue
 * exactly -- state x [N][d] and its prob lp [N], the global step index
 * (Philox counter, CondCov cycle phase), whether step 1 is behind (the
 * auto-accept, sp.py:231-232), and for XOSHIRO the per-chain generator
 * state [8][N] (NULL otherwise).  pbh_restore goes after pbh_init_chains
 * (same N) and pbh_set_rng; it detaches a trace buffer and replay rows
 * (pbh_alloc_trace again); a run from the restored engine continues the
 * checkpointed one step for step.  The production Gibbs
 * kernel's persisted g, Q are recomputed from x (v.prob then agrees to its
 * refresh tolerance, 1e-9).                                                 */
int pbh_get_checkpoint(pbh_engine *eng, double *x, double *lp, int64_t *step,
                       int32_t *has_pred, uint32_t *xo);
int pbh_restore(pbh_engine *eng, const double *x, const double *lp,
                int64_t step, int32_t has_pred, const uint32_t *xo);
/* The device legacy streams' state for a checkpoint (pbh_legacy_seed):
 * key [words][N] with words per chain from pbh_legacy_state_words (624 in
 * place, 1248 double-buffered, 640 for the default chunked layout: the
 * current block, moved into buffer 0 by the get; the words are the device
 * layout, opaque to the caller and valid only for an engine seeded with the
 * same layout), the read position pos [N]
 * (packed with the layout's buffer indices), the cached-gauss flag
 * has [N] and value gauss [N] (NumPy's RandomState has_gauss / gauss).
 * After pbh_restore on an engine with legacy streams, pbh_legacy_replay
 * refuses until pbh_set_legacy_state restores the checkpoint's state.       */
int pbh_legacy_state_words(pbh_engine *eng, int64_t *words_per_chain);
int pbh_get_legacy_state(pbh_engine *eng, uint32_t *key, int32_t *pos,
                         int32_t *has, double *gauss);
int pbh_set_legacy_state(pbh_engine *eng, const uint32_t *key,
                         const int32_t *pos, const int32_t *has,
                         const double *gauss);
/* Replaces the chains' state (x [N][d], lp [N]), the global step and the
 * step-1 flag at any point; every generator state (xoshiro, legacy streams)
 * continues where it is.  The trace buffer and the replay rows are
 * detached: pbh_alloc_trace / pbh_upload_replay / pbh_legacy_replay again
 * before pbh_run.  Used by the SP facade's incremental samplers (SP.reset,
 * sp.py:113-128) to restart chains at init or to rewind to the last step
 * handed out.                                                               */
int pbh_set_chains(pbh_engine *eng, const double *x, const double *lp,
                   int64_t step, int32_t has_pred);
/* The carried logs of the ufun dims (production modes: the log of a ufun
 * dim is chain state, the accepted proposal's log x + delta, variable.py:
 * 693-697 without the round trip through exp): lx [N][d] row-major (the
 * non-ufun columns unused); valid = 0 when they are not maintained (another
 * RNG mode, or a fresh / restored state: then ln x at the next launch).  A
 * checkpoint of a production ufun model carries them so that a restored
 * engine continues the run bit for bit.                                    */
int pbh_get_chain_logs(pbh_engine *eng, double *lx, int32_t *valid);
int pbh_set_chain_logs(pbh_engine *eng, const double *lx);
/* Replay stream [n_steps][R][n_chains] (R = d + 1 for MH, 1 for Gibbs),
 * consumed from the next pbh_run step on.                                   */
int pbh_upload_replay(pbh_engine *eng, int64_t n_steps, const double *rand);
int pbh_stream_width(pbh_engine *eng, int32_t *r);
/* The same streams generated on the device: one NumPy legacy RandomState per
 * chain (MT19937 seeded as RandomState(seeds[c]), random_sample, polar
 * legacy gauss with its cached deviate), drawn in the reference's per-step
 * order.  pbh_legacy_seed seeds the engine's chains;
 * each pbh_legacy_replay fills the replay stream with the next n_steps rows
 * of every chain's generator (continuing where the last call stopped) for
 * the runs from the current step on.  pbh_get_replay copies steps [first,
 * first + n_steps) of the current stream back: draw < 0 gives every draw in
 * the pbh_upload_replay layout [n][R][N], draw = j only draw j, [n][N].   */
int pbh_legacy_seed(pbh_engine *eng, const uint32_t *seeds);
int pbh_legacy_replay(pbh_engine *eng, int64_t n_steps);
/* Sizes the replay stream buffer for n_steps rows without drawing (the
 * buffer only grows; a later generation or upload of at most that many rows
 * allocates nothing).  Rows already in the buffer are dropped when it grows:
 * reserve before filling it.                                               */
int pbh_reserve_replay(pbh_engine *eng, int64_t n_steps);
int pbh_get_replay(pbh_engine *eng, int64_t first, int64_t n_steps,
                   int32_t draw, double *out);
/* pbh_legacy_replay(n) followed by pbh_run(n), in one kernel per launch:
 * each step's draws are generated into the step's registers and never
 * written to HBM.  The chains, trace, moments and legacy generator state are
 * those of generation + run chunk by chunk (steps_per_launch as pbh_run);
 * forms the fused kernel does not cover (Gibbs, per-variable deltas, a
 * permuted draw order, a d without an instantiation) run that way.  REPLAY
 * RNG, after pbh_legacy_seed.  No replay rows are held afterwards.  Replaces
 * the reference's per-step np.random draws + SP.next (sp.py:221-258).      */
int pbh_legacy_run(pbh_engine *eng, int64_t n_steps, int32_t steps_per_launch);
/* on != 0: pbh_legacy_run also keeps each step's MH threshold t (the
 * reference's metropolis_thresh draw, sp_utils.py:30-31, which SP.next
 * returns as opqrstuv.t, sp.py:249-258) on the device; pbh_get_thresholds
 * copies steps [first, first + n_steps) of the last pbh_legacy_run as
 * [n_steps][n_chains].  (The fused kernel stores them as it draws them.)   */
int pbh_set_record_threshold(pbh_engine *eng, int32_t on);
int pbh_get_thresholds(pbh_engine *eng, int64_t first, int64_t n_steps, double *out);
/* The next n_steps draws of every chain's device RandomState (after
 * pbh_legacy_seed) into out [n_steps][n_chains], the chain's generator
 * continuing: kind PBH_DRAWS_LINREG draws what the gibbs_linreg example's
 * cond_reg consumes at global step step0 + t (examples/mcmc/gibbs_linreg.py:
 * 38-47): standard_gamma(param) when (step0 + t) % 3 == 2, else the legacy
 * gauss (NumPy's legacy_standard_gamma: Marsaglia-Tsang over the polar gauss
 * and random_sample, the shape < 1 and shape == 1 branches included);
 * PBH_DRAWS_GAUSS the legacy gauss every step.                             */
enum pbh_draws { PBH_DRAWS_GAUSS = 0, PBH_DRAWS_LINREG = 1 };
int pbh_legacy_draws(pbh_engine *eng, int64_t n_steps, int64_t step0, int32_t kind,
                     double param, double *out);

/* ---- running (SP.walk / sample_generator: sp.py:281-295, sp_utils.py:8-16) */
/* Device trace ring for the next runs: every thin-th step is recorded.
 * debug = 1 also records proposals p_x, p_p and the score s; OR-ed with
 * PBH_TRACE_NOFILL the records are not zero-filled (the caller's next run
 * writes every one of them).                                                */
enum { PBH_TRACE_NOFILL = 0x100 };
int pbh_alloc_trace(pbh_engine *eng, int64_t capacity, int32_t thin,
                    int32_t debug);
/* Launches n_steps chain-steps on the engine stream (asynchronous);
 * steps_per_launch bounds one kernel's fused step loop (0 = all).          */
int pbh_run(pbh_engine *eng, int64_t n_steps, int32_t steps_per_launch);
int pbh_sync(pbh_engine *eng);
/* pbh_run + pbh_sync in one call (one host-to-library crossing: the
 * synchronous walk of sp.py:281-295 for a batch of steps).                  */
int pbh_run_wait(pbh_engine *eng, int64_t n_steps, int32_t steps_per_launch);
/* flags = OR of enum pbh_collect; default PBH_COLLECT_MOMENTS.  With 0 the
 * kernels keep no running moments (no per-launch read-modify-write of them);
 * pbh_trace_stats then reduces the recorded trace on the device instead.   */
int pbh_set_collect(pbh_engine *eng, int32_t flags);
/* Kernel-only time of the last pbh_run (HIP events on the engine stream;
 * for a resident-server command, its first workgroup's sight of the command
 * to its last workgroup's completion on the device's 100 MHz clock).       */
int pbh_last_run_ms(pbh_engine *eng, double *ms, int64_t *launches);
/* Resident sampling server (opt-in, PBH_SERVER=1 at pbh_create; the
 * walk/next loop of sp.py:221-295 kept resident on the device): a run that is
 * one steady-state lane-pair launch (the cfg2 form, production Philox, thin
 * 1, past step 1, every record inside the trace) becomes a command to a
 * kernel that stays resident with the chain state in registers; the kernel
 * leaves after PBH_SERVER_IDLE_MS (default 1000) without a command.  Every
 * other entry point stops it first; pbh_server_stop stops it explicitly
 * (chain state stored, stream idle); pbh_destroy stops it.  active = the
 * server kernel is running; commands / launches: totals of this engine.    */
int pbh_server_stop(pbh_engine *eng);
int pbh_server_info(pbh_engine *eng, int32_t *active, int64_t *commands,
                    int64_t *launches);
/* Diagnostic: the server's per-workgroup completion words of the last
 * command (seq, the 100 MHz stamps of its sight and completion); n = the
 * workgroup count, at most cap entries copied.                             */
int pbh_server_stamps(pbh_engine *eng, int32_t cap, uint32_t *seq, uint64_t *t0,
                      uint64_t *t1, int32_t *n);

/* ---- results (SP.__call__(samples) summary: sp.py:131-198) -------------- */
int pbh_get_state(pbh_engine *eng, double *x, double *logp);
int pbh_trace_len(pbh_engine *eng, int64_t *n_recorded);
/* Copies recorded steps [first, first + n) of the trace:
 * x [n][d][N], logp [n][N], acc [n][ceil(N/64)] accept bitmask words
 * (bit j of word w = chain 64 w + j).  Optional debug buffers may be NULL. */
int pbh_get_trace(pbh_engine *eng, int64_t first, int64_t n, double *x,
                  double *logp, uint64_t *acc, double *p_x, double *p_p,
                  double *s);
/* Per-chain running moments over every step since the last reset:
 * sum[d][N], sumsq[d][N] of the accepted state, n_acc[N] accepts.          */
int pbh_get_moments(pbh_engine *eng, double *sum, double *sumsq,
                    int64_t *n_acc, int64_t *n_steps);
int pbh_reset_moments(pbh_engine *eng);
/* Per-(chain, dim) effective sample size of trace records [first, first +
 * count) on the device: Geyer's initial positive sequence over the
 * autocorrelations of each centred series (the estimator behind cfg5's
 * ESS/s); the autocorrelations by FFT (two series per
 * 4 096-point transform, count <= 2 048; direct sums above that or with
 * PBH_ESS_FFT=0); ess [d][N] on the host (may be NULL).  The result also
 * stays in the engine for pbh_rccl_allgather_stats.                         */
int pbh_trace_ess(pbh_engine *eng, int64_t first, int64_t count, double *ess);
/* The sum over chains of pbh_trace_ess's per-chain ESS, per dim: total[d]
 * (cfg5's ESS is the min over dims of the summed per-chain
 * ESS), reduced on the device -- d doubles cross to the host, not d N.      */
int pbh_trace_ess_total(pbh_engine *eng, int64_t first, int64_t count, double *total);
/* The same per-chain statistics reduced on the device from trace records
 * [first, first + count) (PD summate + expectation over a recorded trace,
 * pd_utils.py:332-411, pd.py:373-407, without copying the trace to the
 * host).  The result replaces the engine's moment buffers (what
 * pbh_rccl_allgather_stats sends, n_steps = count); host pointers may be
 * NULL.                                                                     */
int pbh_trace_stats(pbh_engine *eng, int64_t first, int64_t count, double *sum,
                    double *sumsq, int64_t *n_acc);
/* PD.expectation of a summary over trace records [first, first + count) on
 * the device (pd.py:373-405): per chain and dim sum_t p_t v_t^e /
 * max(tiny, sum_t p_t), p_t = v.prob rescaled to linear (exp_logp of the
 * recorded log-prob under a log pscale), v^e = v when exponent is 0 (the
 * reference's `val ** exponent if exponent else val`), sums in record
 * order.  out [d][N] on the host.                                           */
int pbh_trace_expectation(pbh_engine *eng, int64_t first, int64_t count,
                          double exponent, double *out);

/* ---- multi-GPU: one RCCL all-gather over xGMI --------- */
int pbh_rccl_unique_id(uint8_t id[128]);
int pbh_rccl_init(pbh_engine *eng, int32_t rank, int32_t world,
                  const uint8_t id[128]);
/* The largest N_local over the ranks (a collective: every rank calls it).  */
int pbh_rccl_max_chains(pbh_engine *eng, int64_t *n_max);
/* The one collective of the data path: gathers every
 * rank's per-chain statistics into out[world][3d+1][n_max] on the host,
 * rows sum[d], sumsq[d], n_acc, ess[d] (the moment buffers: in-kernel
 * moments or pbh_trace_stats; ess: pbh_trace_ess, NaN before), and every
 * rank's N_local into counts[world].  Ranks may hold different N_local (the
 * ragged contiguous blocks of dist.shard): rank r's columns >= counts[r] are
 * padding.  Every rank enters every collective whatever fails locally, and
 * all ranks then return the same error.                                     */
int pbh_rccl_allgather_stats(pbh_engine *eng, double *out, int64_t *counts);
/* Max-reduces one double over ranks (bench timing).                         */
int pbh_rccl_allreduce_max(pbh_engine *eng, double *value);
int pbh_rccl_destroy(pbh_engine *eng);

/* ---- likelihoods (likelihoods.py) --------------------------------------- */
/* bool_perm_freq (likelihoods.py:45-101): counts[2^cols] (C order: the first
 * column is the most significant index bit, each dimension ordered [False,
 * True]) of the boolean row patterns of bool2d [rows][cols] (one byte per
 * element, non-zero = True).  1 <= cols <= 26; rows = 0 gives zero counts.
 * Host buffers.  The kernel runs `reps` >= 1 times on device-resident input
 * after one untimed warm-up launch (counts of the last run are returned);
 * *kernel_ms (may be NULL) receives
 * the average kernel time from HIP events.                                  */
int pbh_bool_perm_freq(int device, int64_t rows, int32_t cols,
                       const uint8_t *bool2d, int64_t *counts, int32_t reps,
                       double *kernel_ms);

/* ---- user-conditional Gibbs: conjugate linear regression ---------------- */
/* Replaces the per-chain loop of SP.next -> RF.eval_tfun (rf.py:413-462)
 * over the user conditional cond_reg of examples/mcmc/gibbs_linreg.py:34-62
 * (paras = beta_0 & beta_1 & y_sigma, tsteps = 1, gibbs scores), with
 * v.prob = sum_j norm.logpdf(y_j, b0 + b1 x_j, y_sigma) + the joint uniform
 * root priors (rf.py:541-562, rv_utils.py:30-38).
 * hyper[6] = beta_0_mu, beta_0_sigma, beta_1_mu, beta_1_sigma,
 *            y_sigma_alpha, y_sigma_beta (cond_reg's keyword defaults);
 * vsets[6] = closed (lo, hi) of beta_0, beta_1, y_sigma (joint=True: each
 * adds -log(hi - lo) inside, NEARLY_NEGATIVE_INF outside); NULL = no prior
 * terms (joint=False).  Step k of the chain
 * (absolute k = step0 + t) updates parameter k mod 3 (the RF's __cond_mod).
 * init/final_x [3][n_chains]; rand [n_steps][n_chains] (REPLAY: the standard
 * gauss, or standard_gamma(alpha + n_obs/2) on y_sigma steps, in NumPy's
 * legacy order); trace_x [n_steps][3][n_chains], trace_lp [n_steps][n_chains]
 * (either may be NULL: then no device trace is kept).  rng_mode REPLAY /
 * PHILOX_F64 use the reference's arithmetic; PHILOX uses centred sufficient
 * statistics.  Host buffers; the chain runs `reps` >= 1 times from init on
 * device-resident inputs (reps > 1: after one untimed warm-up), *kernel_ms
 * (may be NULL) = the average kernel time.                                  */
int pbh_linreg_gibbs(int device, int64_t n_obs, const double *x_obs,
                     const double *y_obs, const double *hyper,
                     const double *vsets, int64_t n_chains,
                     int64_t chain_offset, int64_t n_steps, int64_t step0,
                     const double *init, int32_t rng_mode, uint64_t seed,
                     const double *rand, double *trace_x, double *trace_lp,
                     double *final_x, double *final_lp, int32_t reps,
                     double *kernel_ms);

/* ---- diagnostics -------------------------------------------------------- */
/* Evaluates the production-mode acceptance filter and the exact ratio form
 * (sp_utils.py:40-64) on device for n triples (lp, lp', t = u01(t0, t1)).
 * out[i]: bit 0 = exact decision s >= t, bit 1 = the filter decided without
 * the exact fallback, bit 2 = the filter's decision.                        */
int pbh_check_accept(int device, int64_t n, const double *lp,
                     const double *lpp, const uint32_t *t0, const uint32_t *t1,
                     int32_t lin, uint8_t *out);

/* Evaluates the production Gibbs kernel's fp64 Box-Muller (box_muller_fast:
 * the cheap log / sin / cos) and the libm form on n Philox-like blocks
 * words[n][4]; fast[n][2], ref[n][2] receive (z0, z1) of each.             */
int pbh_check_normals(int device, int64_t n, const uint32_t *words,
                      double *fast, double *ref);

/* The production fp64 normals (bm96_pair, PBH_RNG_PHILOX / XOSHIRO) on n
 * word triples words[n][3]: fast[n][2] = bm96_pair, ref[n][2] = the same u1
 * and angle through libm log / sqrt / sincos.  pbh_bm64_tables fills
 * out[4162] with the engine's tables ({-2 ln c_j, 1/c_j} x 1025, {sin, cos}
 * x 1024 over the full turn, 2^(i/64) x 64).                                */
int pbh_check_normals64(int device, int64_t n, const uint32_t *words,
                        double *fast, double *ref);
int pbh_bm64_tables(double *out);

#ifdef __cplusplus
}
#endif
#endif /* PBHIP_H */
