// pbh_kernels.h -- kernel argument block shared by the engine (host) and the
// gfx950 kernels.  Passed by value as the kernarg segment; every pointer in it
// is a device pointer and every array read through it is read with a
// wave-uniform address (scalar loads).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

namespace pbh {

// Dispatch timing of pbh_run's timed region: the start / stop events ride on
// the first / last kernel dispatch packet itself (hipExtLaunchKernel), so the
// queue carries no extra event-marker packets between the host's launch and
// the kernel.  pbh_run sets them; every MH / Gibbs launch goes through
// pbh_launch, which consumes the start event on the first dispatch.
struct LaunchEvents {
  hipEvent_t start = nullptr, stop = nullptr;
};
LaunchEvents &launch_events();   // thread-local (pbh_dispatch.cpp)
bool module_launch();            // not PBH_MODULE_LAUNCH=0 (pbh_dispatch.cpp)
hipFunction_t kernel_function(const void *kernel);   // cached hipGetFuncBySymbol

template <typename F, typename... Args>
inline void pbh_launch(F kernel, const dim3 &grid, const dim3 &block,
                       size_t shm, hipStream_t st, Args... args) {
  LaunchEvents &ev = launch_events();
  if (ev.start || ev.stop) {   // events on the dispatch packet (PBH_EVENT_MARKERS=0)
    (void)hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)shm, st, ev.start,
                                ev.stop, 0u, args...);
  } else if (const hipFunction_t fn = module_launch()
                 ? kernel_function(reinterpret_cast<const void *>(kernel)) : nullptr) {
    // hipModuleLaunchKernel on the kernel's hipFunction_t, cached per kernel:
    // no per-launch symbol lookup (≈ 0.5 us less host enqueue per launch,
    // profiles/r03o_s20probe.jsonl); PBH_MODULE_LAUNCH=0 keeps
    // hipLaunchKernelGGL
    void *params[] = {reinterpret_cast<void *>(&args)...};
    (void)hipModuleLaunchKernel(fn, grid.x, grid.y, grid.z, block.x, block.y, block.z,
                                (unsigned)shm, st, params, nullptr);
  } else {
    hipLaunchKernelGGL(kernel, grid, block, shm, st, args...);
  }
  ev.start = nullptr;
}


struct KArgs {
  // ---- model (pbh_model) ----
  int32_t d, target, pscale, scores;
  const double *ta, *tb, *tc, *te;  // target parameter arrays (see pbhip.h)
  int64_t tn;                       // n_obs (NORM_IID) or K (GMM)
  int32_t i0, i1;                   // NORM_IID loc / scale dims
  int32_t has_prior;
  const double *plo, *phi;
  uint32_t plo_incl, phi_incl;      // bitmasks over dims
  double prior_logp;
  uint32_t ufun;                    // bitmask: dim uses the (log, exp) ufun
  int32_t tran_kind, tran_sym, tran_rev;  // tran_rev: product order reversed
  double tran_value, tran_scale;
  const double *tran_off;
  // ---- proposal ----
  int32_t prop;
  const double *ploc, *pscl, *plen, *pdel;
  int32_t ploc_zero;  // GAUSS: every loc is 0 (the production lane-pair
                      // kernel then forms x + z scale as one fma)
  double sdelta;
  const double *ptf;  // covariance RW: delta' = ptf[d][d] . delta (rf.py:340-354)
  int32_t has_tfun;
  uint64_t vmode;     // VARDELTA: enum pbh_var_delta, 2 bits per dim
  uint32_t vint;      // bitmask: int variable (proposal truncated)
  uint32_t bnd_on, bnd_xlo, bnd_xhi;  // bound=True: on / exclusive lo / hi
  const double *blo, *bhi;            // bound limits [d]
  // ---- gibbs ----
  const double *gmean, *gcoef, *gstdv, *gcdf;
  int32_t tsteps;
  // ---- host-evaluated constants (bit-identical to the reference's) ----
  const double *tw;  // DIAG_GAUSS production path: sqrt(0.5) / sigma
  double ksum;       // DIAG_GAUSS production path: sum(logC + log sigma)
  double log_npi;    // np.log(NEARLY_POSITIVE_INF)
  double norm_logC;  // np.log(np.sqrt(2*np.pi))
  double norm_C;     // np.sqrt(2*np.pi)
  // ---- run ----
  int64_t n;         // chains on this engine
  int64_t off;       // global id of chain 0 (Philox key input)
  int32_t n_steps;   // steps in this launch
  int64_t g0;        // global step index of the launch's first step
  int32_t has_pred;  // chains already hold an accepted pred (step > 1)
  double *x;         // state [d][n]
  double *lp;        // log/lin prob of the state [n]
  int32_t rng;       // PBH_RNG_*
  uint32_t seed_lo, seed_hi;
  const double *rep; // replay stream [T][R][n]
  uint32_t *xo;      // xoshiro128** states [4][2][n] (word, lane half, chain)
  int64_t rep_row0;  // replay step index of g0
  int32_t R;         // replay draws per step
  // ---- trace ----
  double *tx, *tlp, *tpx, *tpp, *ts;
  uint64_t *tacc;
  int32_t thin;
  int64_t rec_base;  // records made before the trace buffer was allocated
  int64_t rec_cap;
  int32_t debug;
  int64_t W;         // accept-mask words per recorded step = ceil(n / 64)
  int32_t pair_ok;   // engine allows the lane-pair kernel (see launch_mh_d)
  int32_t simple_acc;  // acceptance is the ratio form of beta lp', beta lp
                       // (metropolis, or hastings with a constant tran, q~ > 0)
  double acc_beta;     // 1, or q~ for a constant tuple tran (App. A-1)
  int32_t gibbs_mfma;  // Gibbs density quadratic form on MFMA (d <= 16)
  // ---- production CondCov Gibbs (gibbs_fast_kernel) ----
  int32_t gibbs_fast;  // engine allows the production Gibbs kernel
  const double *gpp;   // precision of the permuted density in x order [d][d]
  const double *gmup;  // mean of the permuted density in x order [d]
  const double *gzlo, *gzhi;  // ndtri(cdf limits): truncation of z per dim
  const double *gak;   // a_k = mean_k - coef_k . mean_-k
  double gconst;       // rank * log(2 pi) + log_pdet
  double *gq;          // persisted g = P'(x - mu') [d][n] and Q [n]
  int32_t gq_init;     // 1: recompute g, Q from x at entry
  // production modes (PHILOX, XOSHIRO) with ufun dims: the log of each ufun
  // dim of the state is chain state, [d][N], carried from the accepted
  // proposal's log (x' = exp(lx + delta), lx' = lx + delta) instead of the
  // log of the exp'd value at every step; lx_init = 1: ln x at entry
  double *lx;
  int32_t lx_init;
  int32_t gibbs_lanes; // lanes per chain (1, 2, 4; 0 = default for d)
  int32_t gmm_lanes;   // lanes per chain of the GMM kernel (2 or 4)
  int32_t gmm_full;    // the quad kernel's steady-state form is allowed
  int32_t pair_full;   // the lane-pair kernel's steady-state form is allowed
  int32_t iid_full;    // cfg1's steady-state iid-Normal form is allowed
  int32_t iid_pair;    // ... on lane pairs (mh_iid_pair_kernel)
  int32_t fair;        // alternate the SIMD's wave priorities every 2^fair real-time ticks (0: off)
  int32_t pair_wg;     // FULL pair kernel's workgroup size (256 or 512)
  int32_t fair_rel;    // FULL pair kernel: the alternation clock starts at the wave's loop entry
  // resident sampling server (FULL pair kernel, SRV): the host command block
  // and the per-workgroup completion words (pinned, fine-grained host
  // memory, SrvCmd / SrvDone), and the idle exit in 10 ns ticks
  void *srv_cmd;
  void *srv_done;
  void *srv_mail;     // the device mailbox of the command (SrvCmd)
  int64_t srv_idle;
  // srv_mode bit 0 (direct, the default): the host writes each command
  // straight into srv_mail (fine-grained device memory through the host's
  // mapping of it) and every workgroup polls it; 0 (relay): workgroup 0
  // polls srv_cmd and copies each command into srv_mail for the others
  int32_t srv_mode;
  // ---- moments ----
  int32_t moments;     // 1: accumulate sum / sumsq / n_acc (pbh_set_collect)
  double *msum, *msq;
  int64_t *nacc;
  // ---- production fp64 normals: bm64 tables (pbh_device.h), global copy
  const double *bm64;
};
// The resident server's host command block and completion words (engine:
// pbh_server_*, kernel: mh_pair_kernel<..., SRV>).  The host writes the
// fields, then seq (release).  Workgroup 0's first wave alone polls the host
// block (one PCIe read in flight: 256 workgroups polling host memory at once
// took ~45 us per read) and relays each command to a device-memory mailbox
// of the same layout, which every other workgroup's first wave polls; each
// workgroup runs the command and writes its SrvDone (seq last) to host
// memory.  op: 0 run, 1 exit.
// One 16-byte record, read and relayed whole (one PCIe read, one mailbox
// store): seq, n, then arg = g0 (bits 0-47) | fair (48-52) | fair_rel (53)
// | op (54) | seq & 0xFF (56-63).  The check byte rejects a torn read (new
// seq, old fields): the host writes n and arg, then seq.
struct alignas(16) SrvCmd {
  uint32_t seq, n;
  uint64_t arg;
};
__host__ __device__ inline uint64_t srv_arg(int64_t g0, uint32_t fair, uint32_t fair_rel,
                                            uint32_t op, uint32_t seq) {
  return ((uint64_t)g0 & 0xFFFFFFFFFFFFull) | ((uint64_t)(fair & 31u) << 48) |
         ((uint64_t)(fair_rel & 1u) << 53) | ((uint64_t)(op & 1u) << 54) |
         ((uint64_t)(seq & 0xFFu) << 56);
}
struct SrvDone {
  uint32_t seq, pad;
  uint64_t t0, t1;   // s_memrealtime (100 MHz) when the command was seen / done
  uint64_t pad2;
};
constexpr uint32_t kSrvRun = 0, kSrvExit = 1;


// The production Gibbs kernel runs for the Philox RNG without debug records,
// d <= 16 (its per-lane constant block grows as d^2).
inline bool gibbs_fast_form(const KArgs &a) {
  return a.gibbs_fast && a.rng == 1 /* PBH_RNG_PHILOX */ && !a.debug && a.d <= 16;
}

// Host launchers (pbh_kernels.hip).
hipError_t launch_mh(const KArgs &a, hipStream_t s, size_t lds_bytes);
hipError_t launch_gibbs(const KArgs &a, hipStream_t s);
// the resident server (FULL lane-pair kernel, SRV): check = only report
// whether `a` qualifies and the grid is resident at once (wgs: workgroups)
hipError_t launch_mh_server(const KArgs &a, hipStream_t s, int32_t *wgs, bool check);
hipError_t launch_xo_seed(uint32_t *xo, int64_t n, int64_t off, uint64_t seed,
                          hipStream_t s);
bool mh_dim_supported(int d);
hipError_t launch_check_normals(int64_t n, const uint32_t *words, double *fast,
                                double *ref);
// bm96_pair (the production fp64 normals) and its libm form on n word triples.
hipError_t launch_check_normals64(int64_t n, const uint32_t *words,
                                  const double *tab, double *fast, double *ref);
// per-chain sums / sums of squares / accept counts of trace records
hipError_t launch_trace_stats(const double *tx, const uint64_t *tacc, int64_t n,
                              int32_t d, int64_t W, int64_t first,
                              int64_t count, double *sum, double *sumsq,
                              int64_t *nacc, hipStream_t s);
// per-(chain, dim) initial-positive-sequence ESS of trace records
hipError_t launch_trace_expectation(const double *tx, const double *tlp,
                                    int64_t n, int32_t d, int64_t first,
                                    int64_t count, double exponent, int32_t lin,
                                    double log_npi, double *out, hipStream_t s);
// fft: 2 = the 2 048-point FFT form for count <= 1 536 records with the
// 4 096-point form for the pairs it cannot decide (list: (d n + 1) / 2 + 1
// int32 of device scratch), 1 = the 4 096-point form for count <= 2 048
// records, 0 (or a longer trace) = the direct-sum kernel
hipError_t launch_trace_ess(const double *tx, int64_t n, int32_t d,
                            int64_t first, int64_t count, double *ess,
                            hipStream_t st, int fft, int32_t *list);
// total[k] = sum over chains of ess[k][c] (one workgroup per dim, a fixed
// summation order)
hipError_t launch_ess_total(const double *ess, int64_t n, int32_t d, double *total,
                            hipStream_t st);
// Host: the bm64 LDS tables (kBm64Doubles doubles, long-double accurate).
void bm64_tables(double *out);
// the legacy generator's log table (pbh_legacy.hip log_leg): 129 rows of
// {ln c_j rounded to a multiple of 2^-32, the remainder}, then 1 / c_j, for
// c_j = 1/2 + j/256; kLegLogDoubles doubles (a multiple of two)
constexpr int kLegLogN = 129, kLegLogInv = 2 * kLegLogN, kLegLogDoubles = 3 * kLegLogN + 1;
void legacy_log_table(double *out);
// Legacy (NumPy RandomState) stream generation (pbh_legacy.hip).
struct LegacyArgs {
  uint32_t *key;        // MT19937 words [624][n]
  int32_t *pos;         // next word per chain [n]
  double *gauss;        // cached polar deviate [n]
  int32_t *has_gauss;   // [n]
  const int32_t *order; // draw j -> replay row order[j] (MH)
  double *out;          // replay rows [n_steps][R][n]
  int64_t n, n_steps, step0;
  int32_t d, R, gibbs, normal;
  int32_t db;           // 1: double-buffered state [2][624][n] (legacy_gen_db);
                        // 2: four chunked blocks [4][20][n][32 words] (Mt4)
  int32_t win;          // with db: consume through the LDS window (Mt3)
  int32_t vardelta;     // VARDELTA: per-dim modes vmode, steps vdelta [d]
  uint64_t vmode;
  const double *vdelta;
  const double *lgtab;  // legacy_log_table (Mt4's polar log)
  int32_t wp;           // with db == 2: the word-parallel generator for MH
                        // streams of doubles (every position even)
  double *thr;          // the fused kernel: each step's threshold [n_steps][n]
                        // (nullptr: not kept)
};
// pbh_legacy_draws: per chain, n_steps draws of kind (pbh_draws) into a.out
// [n_steps][n] (Mt4 state)
hipError_t launch_legacy_draws(const LegacyArgs &a, int32_t kind, double param,
                               hipStream_t s);
hipError_t launch_legacy_seed(uint32_t *key, int32_t *pos, double *gauss,
                              int32_t *has_gauss, const uint32_t *seeds,
                              int64_t n, int32_t db, hipStream_t s);
hipError_t launch_legacy_gen(const LegacyArgs &a, hipStream_t s);
// Mt4 state: twist every chain's buffers ahead until `want` (<= 15) blocks
// follow its current one (legacy_ahead_kernel)
hipError_t launch_legacy_ahead(uint32_t *key, int32_t *pos, int64_t n, int32_t want,
                               hipStream_t s);
// Mt4 state: each chain's current block into buffer 0, buffer / ready fields
// of pos cleared (the checkpoint form: the first 20 x 32 words per chain)
hipError_t launch_legacy_normalize(uint32_t *key, int32_t *pos, int64_t n, hipStream_t s);
// The fused REPLAY kernel: generation and the REPLAY chain-step in one
// launch (la: the generator's state, a: the run's kernel arguments, a.n_steps
// = la.n_steps).  hipErrorNotSupported: the form is not covered (the caller
// runs launch_legacy_gen + launch_mh); check: report only.
hipError_t launch_legacy_mh(const LegacyArgs &la, const KArgs &a, hipStream_t s, bool check);

// bool_perm_freq histogram (pbh_likelihoods.hip); counts must be zeroed,
// scratch holds bool_perm_scratch_words(n_cu) u64 partials.
int bool_perm_max_cols();
int64_t bool_perm_scratch_words(int n_cu);
hipError_t launch_bool_perm_freq(const uint8_t *in, int64_t rows, int cols,
                                 unsigned long long *counts,
                                 unsigned long long *scratch, int n_cu,
                                 hipStream_t s);
hipError_t launch_check_accept(int64_t n, const double *lp, const double *lpp,
                               const uint32_t *t0, const uint32_t *t1,
                               int32_t lin, double log_npi, uint8_t *out);

// user-conditional Gibbs of the gibbs_linreg model (pbh_linreg.hip).
// hyper: p0, m0, p1, m1, alpha_post, beta, sxx, prior[3], logC;
// stats: xbar, ybar, Cxx, Cxy, Cyy (centred; PHILOX's fast form).
struct LinregArgs {
  const double *x_obs, *y_obs;
  int64_t n_obs;
  double hyper[11], stats[5], bounds[6];  // bounds: (lo, hi) per parameter
  double *state, *lp_state;
  const double *rand;
  double *tx, *tp;
  int64_t n, chain_offset, n_steps, step0;
  uint64_t seed;
  int32_t mode;
  int32_t pair;   // PHILOX: one chain per lane pair (linreg_pair_kernel)
};
int64_t linreg_max_obs();
hipError_t launch_linreg_gibbs(const LinregArgs &a, hipStream_t s);

}  // namespace pbh
