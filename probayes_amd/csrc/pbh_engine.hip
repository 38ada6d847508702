// pbh_engine.hip -- the C-ABI of include/pbhip.h: engine state, device
// memory, launches, HIP-event timing and the RCCL trace all-gather.
//
// The engine owns every device buffer; the caller passes host pointers.
// Nothing here throws across the C boundary: errors become status codes with
// a thread-local message (pbh_last_error).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/pbhip.h"
#include "pbh_kernels.h"
#include "pbh_device.h"

using pbh::KArgs;

struct pbh_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  unsigned ev_flags = 0;   // the events' hipEventCreateWithFlags flags
  // model / proposal / gibbs (device constant blocks)
  bool has_model = false, has_prop = false, has_gibbs = false;
  int d = 0;
  KArgs k{};
  double *dmodel = nullptr, *dprop = nullptr, *dgibbs = nullptr;
  std::vector<int32_t> draw_order;  // GAUSS: dim receiving the j-th draw
  // chains
  int64_t n = 0, off = 0;
  double *x = nullptr, *lp = nullptr;
  bool has_pred = false;
  int64_t g = 0;  // chain-steps done since pbh_init_chains
  // randomness
  int32_t rng = PBH_RNG_PHILOX;
  uint64_t seed = 0;
  double *rep = nullptr;
  int64_t rep_steps = 0, rep_g0 = 0;
  size_t rep_alloc = 0;          // doubles allocated at rep (device streams reuse it)
  uint32_t *xo = nullptr;      // xoshiro128** states [4][2][n]
  bool xo_seeded = false;
  // legacy NumPy RandomState per chain (pbh_legacy_seed)
  uint32_t *mt_key = nullptr;
  int mt_mode = 0;             // mt_key layout: 0 [624][n], 1 [2][624][n], 2 Mt4's
                               // [4][20][n][32] (four chunked blocks)
  bool legacy_db = true;       // PBH_LEGACY_DB=0: the in-place state
  bool legacy_k4 = true;       // PBH_LEGACY_K4=0: the round-3 double-buffered state
  bool legacy_win = true;      // PBH_LEGACY_WIN=0: HBM-direct consumption (Mt2)
  bool legacy_fused = true;    // PBH_LEGACY_FUSED=0: pbh_legacy_run as generation + run
  bool legacy_wp = true;       // PBH_LEGACY_WP=0: the chain-per-lane generator for MH streams
  bool legacy_ahead = true;    // PBH_LEGACY_AHEAD=0: no twist-ahead pass before fused launches
  bool mt_odd = false;         // a stream may sit at an odd word (randint drew single words)
  bool rec_thr = false;        // pbh_set_record_threshold: keep pbh_legacy_run's thresholds
  double *thr = nullptr;       // [thr_steps][n] thresholds of the last pbh_legacy_run
  double *ess_tot = nullptr;   // pbh_trace_ess_total's per-dim sums (PBH_MAX_DIM)
  size_t thr_alloc = 0;
  int64_t thr_steps = 0;
  int32_t *mt_pos = nullptr, *mt_has = nullptr, *mt_order = nullptr;
  double *mt_gauss = nullptr;
  bool mt_stale = false;       // pbh_restore ran: the streams wait for
                               // pbh_set_legacy_state (the checkpoint's)
  // trace
  int64_t cap = 0;
  int32_t thin = 1, debug = 0;
  int64_t rec_base = 0;
  double *tx = nullptr, *tlp = nullptr, *tpx = nullptr, *tpp = nullptr,
         *ts = nullptr;
  uint64_t *tacc = nullptr;
  // moments (pbh_set_collect)
  int32_t collect = PBH_COLLECT_MOMENTS;
  double *msum = nullptr, *msq = nullptr;
  int64_t *nacc = nullptr;
  int64_t mom_steps = 0;
  // production fp64 normal tables (bm64, pbh_device.h), read into LDS
  double *bm64 = nullptr;
  double *lgtab = nullptr;     // legacy_log_table (device legacy streams)
  double *ess = nullptr;     // [d][n] per-chain ESS (pbh_trace_ess), NaN before
  int32_t *ess_list = nullptr;   // the 2 048-point ESS form's fallback list
  int64_t ess_list_len = 0;
  double *ess_host = nullptr;    // pinned staging of the ESS copy-out
  int64_t ess_host_len = 0;
  bool spin_sync = true;     // poll <= 2 ms, then block; PBH_SYNC=block: block
  bool sync_event = false;   // PBH_SYNC=event: poll the last run's end event
  // timing events as marker packets around the launches (default), or
  // PBH_EVENT_MARKERS=0: on the first / last dispatch packet
  // (hipExtLaunchKernel: 2 us less GPU time, 3-4 us more host enqueue and
  // ~7 us more wall per short launch, measured: profiles/r02j_events.jsonl)
  bool gmm_full = true;      // PBH_GMM_FULL=0: no steady-state quad kernel
  bool pair_full = true;     // PBH_PAIR_FULL=0: no steady-state pair kernel
  int ess_fft = 2;           // PBH_ESS_FFT=1: the 4 096-point form only, 0: direct sums
  bool iid_full = true;      // PBH_IID_FULL=0: no steady-state iid kernel
  bool iid_pair = false;     // PBH_IID_PAIR=1: the steady-state iid kernel on lane pairs (measured slower)
  int fair = 11;             // PBH_FAIR=k: wave priorities alternate every 2^k x 10 ns (0: off)
  int pair_wg = 512;         // PBH_PAIR_WG=256: FULL pair kernel in 4-wave workgroups
                             // (512: one table copy per CU, 20-step launches ~5 % faster)
  // Launches of <= 64 steps (the driver's 20-step shape): the alternation
  // clock starts at each wave's loop entry and hands over once, half-way
  // (2^10 ticks = 10.24 us for 20 steps) -- the
  // free-running clock put the one hand-over anywhere in the launch or nowhere
  // (profiles/r04f_phase.jsonl: the last wave ends 26.4-29.2 us into a k11
  // launch, 26.5-26.6 us with the launch-relative clock)
  int fair_short = 10;       // PBH_FAIR_SHORT=k
  int fair_rel = 0;          // PBH_FAIR_REL=1: long launches use the relative clock too
  bool event_markers = true;
  bool pair_enabled = true;  // PBH_NO_PAIR=1 disables the lane-pair kernel
  bool gibbs_mfma = true;    // PBH_GIBBS_MFMA=0 keeps the VALU quadratic form
  bool gibbs_fast = true;    // PBH_GIBBS_FAST=0 keeps the ndtri kernel for Philox
  int gibbs_lanes = 0;       // PBH_GIBBS_LANES: lanes per chain of that kernel
  int gmm_lanes = 4;         // PBH_GMM_LANES: lanes per chain of the GMM kernel
  // MVN target on the host (for the production Gibbs tables)
  std::vector<double> mvn_mean, mvn_U;
  double mvn_const = 0.;
  // production Gibbs: persisted g = P'(x - mu'), Q per chain
  double *gq = nullptr;
  // production ufun logs carried as chain state ([d][n], KArgs.lx)
  double *lx = nullptr;
  bool lx_valid = false;
  bool gq_valid = false;
  // timing of the last pbh_run
  bool timed = false;
  int64_t last_launches = 0;
  // resident sampling server (PBH_SERVER=1; pbh_server_*): the FULL pair
  // kernel launched once, each eligible pbh_run a command in pinned host
  // memory; srv_timed: the last run was a command (timed by its stamps)
  bool srv_enabled = false;
  bool srv_active = false;
  bool srv_timed = false;
  uint32_t srv_seq = 0, srv_pending = 0;
  int32_t srv_wgs = 0;
  int64_t srv_idle_ms = 1000;      // PBH_SERVER_IDLE_MS: the kernel's idle exit
  pbh::SrvCmd *srv_cmd = nullptr;  // pinned, fine-grained
  pbh::SrvDone *srv_done = nullptr;
  pbh::SrvCmd *srv_mail = nullptr;   // the device mailbox the workgroups poll
  int32_t srv_done_len = 0;
  // the command protocol (KArgs.srv_mode): 1 direct (the default) --
  // srv_mail is fine-grained device memory the host writes through srv_wmail
  // (its host mapping) and every workgroup polls; 0 relay -- workgroup 0
  // polls the pinned host block srv_cmd and copies each command into
  // srv_mail.  Direct needs a host mapping whose stores the device sees: the
  // first launch probes it (srv_probed) and falls back to the relay.
  int32_t srv_mode = 1;
  bool srv_probed = false;
  bool srv_mail_fine = false;        // srv_mail came from the fine-grained pool
  pbh::SrvCmd *srv_wmail = nullptr;
  // srv_last: the last submit (or launch) -- never moved forward at a wait:
  // a command completes after its submit, and each workgroup's idle timer
  // starts at its completion, so idle measured from the submit is an upper
  // bound on the kernel's own
  std::chrono::steady_clock::time_point srv_last{};
  // a server command was lost (the kernel ended or hung before completing
  // it): the chain state may be partly advanced, so runs refuse until
  // pbh_init_chains / pbh_restore / pbh_set_chains replace it
  bool state_lost = false;
  int64_t srv_commands = 0, srv_launches = 0;
  // RCCL
  ncclComm_t comm = nullptr;
  int32_t rank = 0, world = 1;
  double *gather_send = nullptr, *gather_recv = nullptr, *scalar = nullptr;
};

namespace {

// words of legacy state per chain in each layout (pbh_engine.mt_mode)
constexpr double pbh_mt_block_words() { return 624.0; }
// (mode 2: pbh_mt.h kK4 = 16 buffers of 20 chunks of 32 words)
int64_t mt_words(int mode) { return mode == 2 ? 16 * 20 * 32 : mode == 1 ? 2 * 624 : 624; }
// words per chain of the checkpoint form (pbh_get/set_legacy_state): Mt4's
// current block alone, moved into buffer 0 (launch_legacy_normalize)
int64_t mt_state_words(int mode) { return mode == 2 ? 20 * 32 : mt_words(mode); }

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                        \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess)                                                    \
      return fail(PBH_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

#define RCCL_TRY(expr)                                                       \
  do {                                                                       \
    ncclResult_t _r = (expr);                                                \
    if (_r != ncclSuccess)                                                   \
      return fail(PBH_ERR_RCCL, "%s failed: %s", #expr, ncclGetErrorString(_r)); \
  } while (0)

// ---------------------------------------------------------------------------
// Engine resource cache.  The device buffers, stream and events of a
// destroyed engine are kept (its stream drained first) for the next engine on
// the same device: a seeded SP.sampler builds one engine per call, and at
// 65 536 chains the hipMalloc / hipFree of its state and trace buffers and
// the stream setup were ~7 ms around an 11.6 ms run
// (profiles/r06_facade/setup_probe.jsonl).  Only buffers of destroyed
// engines enter the cache, so nothing in it has work in flight; a live
// engine's reallocations free as before.  Buffers are reused at exactly
// their size (engines of one shape ask for the same sizes).  Bounded by
// PBH_CACHE_MB (default 32 768 of the 288 GB; 0 disables it); an allocation
// that fails empties the cache and retries; pbh_cache_release empties it.
// ---------------------------------------------------------------------------
struct ResCache {
  std::mutex mu;
  std::unordered_map<void *, size_t> live;              // dalloc'd buffers: bytes
  std::multimap<std::pair<int, size_t>, void *> idle;   // (device, bytes) -> buffer
  size_t idle_bytes = 0, cap = 0;
  struct Strm { int device; unsigned flags; hipStream_t s; hipEvent_t e0, e1; };
  std::vector<Strm> streams;
  int64_t hits = 0, misses = 0;
};
ResCache &res_cache() {
  static ResCache *c = [] {   // never destroyed: engines may outlive statics
    ResCache *r = new ResCache();
    size_t mb = 32768;
    if (const char *m = std::getenv("PBH_CACHE_MB")) mb = std::strtoull(m, nullptr, 10);
    r->cap = mb << 20;
    return r;
  }();
  return *c;
}

int cur_device() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  return dev;
}

// frees every idle buffer and cached stream; returns how many buffers
int cache_release_all() {
  ResCache &c = res_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  int freed = 0;
  const int dev0 = cur_device();
  for (auto &kv : c.idle) {
    (void)hipSetDevice(kv.first.first);
    (void)hipFree(kv.second);
    ++freed;
  }
  c.idle.clear();
  c.idle_bytes = 0;
  for (auto &st : c.streams) {
    (void)hipSetDevice(st.device);
    (void)hipEventDestroy(st.e0);
    (void)hipEventDestroy(st.e1);
    (void)hipStreamDestroy(st.s);
  }
  c.streams.clear();
  (void)hipSetDevice(dev0);
  return freed;
}

template <class T>
void dfree(T *&p) {
  if (p) {
    ResCache &c = res_cache();
    {
      std::lock_guard<std::mutex> lk(c.mu);
      c.live.erase(static_cast<void *>(p));
    }
    (void)hipFree(p);
  }
  p = nullptr;
}

// a buffer of a destroyed engine (its stream drained): into the cache while
// it fits, else freed
template <class T>
void dretire(T *&p) {
  if (!p) return;
  ResCache &c = res_cache();
  void *v = static_cast<void *>(p);
  p = nullptr;
  {
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.live.find(v);
    if (it != c.live.end() && c.idle_bytes + it->second <= c.cap) {
      c.idle.emplace(std::make_pair(cur_device(), it->second), v);
      c.idle_bytes += it->second;
      c.live.erase(it);
      return;
    }
    if (it != c.live.end()) c.live.erase(it);
  }
  (void)hipFree(v);
}

template <class T>
int dalloc(T *&p, size_t count) {
  dfree(p);
  if (count == 0) return PBH_OK;
  const size_t bytes = count * sizeof(T);
  ResCache &c = res_cache();
  {
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.idle.find(std::make_pair(cur_device(), bytes));
    if (it != c.idle.end()) {
      p = static_cast<T *>(it->second);
      c.idle.erase(it);
      c.idle_bytes -= bytes;
      c.live.emplace(static_cast<void *>(p), bytes);
      ++c.hits;
      return PBH_OK;
    }
    ++c.misses;
  }
  hipError_t err = hipMalloc((void **)&p, bytes);
  if (err == hipErrorOutOfMemory && cache_release_all() > 0) {
    (void)hipGetLastError();
    err = hipMalloc((void **)&p, bytes);
  }
  if (err != hipSuccess) {
    p = nullptr;
    return fail(PBH_ERR_HIP, "hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(err));
  }
  std::lock_guard<std::mutex> lk(c.mu);
  c.live.emplace(static_cast<void *>(p), bytes);
  return PBH_OK;
}

int upload(double *&dst, const std::vector<double> &h, hipStream_t s) {
  int rc = dalloc(dst, h.size() ? h.size() : 1);
  if (rc) return rc;
  if (h.size())
    HIP_TRY(hipMemcpyAsync(dst, h.data(), h.size() * sizeof(double),
                           hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  return PBH_OK;
}

// Appends host array a[0:n] to a packed block; returns its offset.
size_t pack(std::vector<double> &blk, const double *a, int64_t n) {
  const size_t o = blk.size();
  for (int64_t i = 0; i < n; ++i) blk.push_back(a[i]);
  return o;
}

int check_ptr(const void *p, const char *name) {
  return p ? PBH_OK : fail(PBH_ERR_ARG, "%s must not be NULL", name);
}

// init [n][d] (the caller's row-major chains) -> x [d][n]
__global__ void chains_to_dim_major(const double *init, double *x, int64_t n, int32_t d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n * d) {
    const int64_t c = i / d, k = i - c * d;
    x[k * n + c] = init[i];
  }
}

__global__ void nacc_to_f64(const int64_t *nacc, double *out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (double)nacc[i];
}

void free_trace(pbh_engine *e) {
  dfree(e->tx); dfree(e->tlp); dfree(e->tpx); dfree(e->tpp); dfree(e->ts);
  dfree(e->tacc);
  e->cap = 0;
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------------------
// Resident sampling server (PBH_SERVER=1, bench.py's default): the FULL pair
// kernel launched once per series of eligible runs (mh_pair_kernel<..., SRV>)
// keeps the chain state in registers and the tables in LDS; each pbh_run is a
// command in pinned host memory, each workgroup reports (seq, stamps).
// Invariants: one command in flight; a command is written only when the
// previous one completed and the host has been idle for less than half the
// kernel's idle exit (so no workgroup can have left on its own); every entry
// point that touches the device state, the trace or the stream stops the
// server first (SRV_STOP); pbh_sync never syncs the stream while it runs;
// pbh_destroy stops it.
// ---------------------------------------------------------------------------
namespace {
using srv_clk = std::chrono::steady_clock;

bool srv_kernel_ended(pbh_engine *e) { return hipStreamQuery(e->stream) == hipSuccess; }

// the first workgroup from `from` on that has not reported `seq` (srv_wgs:
// all have)
int32_t srv_first_pending(const pbh_engine *e, uint32_t seq, int32_t from) {
  for (int32_t w = from; w < e->srv_wgs; ++w)
    if (__atomic_load_n(&e->srv_done[w].seq, __ATOMIC_ACQUIRE) != seq) return w;
  return e->srv_wgs;
}
bool srv_all_done(const pbh_engine *e, uint32_t seq) {
  return srv_first_pending(e, seq, 0) == e->srv_wgs;
}

// every workgroup reported `seq`; ok_if_ended: an ended kernel is no error
// (the exit command: workgroups that left idle do not acknowledge it).  The
// scan resumes at the first workgroup not yet seen done; the stream is
// queried (a runtime call with a lock) only after a millisecond of waiting.
int srv_wait(pbh_engine *e, uint32_t seq, bool ok_if_ended) {
  const auto t0 = srv_clk::now();
  int32_t w = 0;
  for (uint64_t it = 1;; ++it) {
    w = srv_first_pending(e, seq, w);
    if (w == e->srv_wgs) return PBH_OK;
    if ((it & 4095) == 0) {
      const auto el = srv_clk::now() - t0;
      if (el > std::chrono::milliseconds(1) && srv_kernel_ended(e)) {
        if (srv_all_done(e, seq) || ok_if_ended) return PBH_OK;
        // the kernel left without the command (some workgroups may have run
        // it): the server is gone -- the next eligible run relaunches -- and
        // the chain state is unusable until replaced
        e->srv_active = false;
        e->srv_pending = 0;
        (void)hipStreamSynchronize(e->stream);   // ended: returns at once
        (void)hipGetLastError();
        e->state_lost = true;
        return fail(PBH_ERR_HIP, "sampling server ended before command %u completed "
                    "(chain state lost: restore a checkpoint or init the chains)", seq);
      }
      if (el > std::chrono::seconds(120)) {
        e->state_lost = true;
        return fail(PBH_ERR_HIP, "sampling server: command %u not completed in 120 s", seq);
      }
    }
  }
}

// a command where the server polls it: the host block (relay) or the device
// mailbox through its host mapping (direct: stored through to the device)
void srv_write(pbh_engine *e, uint32_t n, uint64_t arg, uint32_t q) {
  pbh::SrvCmd *cmd = (e->srv_mode & 1) ? e->srv_wmail : e->srv_cmd;
  cmd->n = n;
  cmd->arg = arg;
  __atomic_store_n(&cmd->seq, q, __ATOMIC_RELEASE);
  if (e->srv_mode & 1) __builtin_ia32_sfence();   // out of any write-combining buffer
}

int srv_stop(pbh_engine *e) {
  if (!e->srv_active) return PBH_OK;
  HIP_TRY(hipSetDevice(e->device));
  int rc = PBH_OK;
  if (e->srv_pending) {
    rc = srv_wait(e, e->srv_pending, false);
    e->srv_pending = 0;
  }
  if (!srv_kernel_ended(e)) {
    const uint32_t q = ++e->srv_seq;
    srv_write(e, 0u, pbh::srv_arg(0, 0u, 0u, pbh::kSrvExit, q), q);
    const int rc2 = srv_wait(e, q, true);
    if (!rc) rc = rc2;
  }
  const hipError_t err = hipStreamSynchronize(e->stream);
  e->srv_active = false;
  if (!rc && err != hipSuccess)
    rc = fail(PBH_ERR_HIP, "sampling server exit: %s", hipGetErrorString(err));
  return rc;
}

// the fine-grained device mailbox and the host's mapping of it (direct)
int srv_alloc_fine(pbh_engine *e) {
  hipError_t err = hipExtMallocWithFlags((void **)&e->srv_mail, sizeof(pbh::SrvCmd),
                                         hipDeviceMallocFinegrained);
  if (err != hipSuccess) {
    e->srv_mail = nullptr;
    return fail(PBH_ERR_HIP, "server mailbox: %s", hipGetErrorString(err));
  }
  e->srv_mail_fine = true;
  hipPointerAttribute_t at{};
  err = hipPointerGetAttributes(&at, e->srv_mail);
  e->srv_wmail = static_cast<pbh::SrvCmd *>(err == hipSuccess ? at.hostPointer : nullptr);
  if (!e->srv_wmail) {
    dfree(e->srv_mail);
    return fail(PBH_ERR_UNSUPPORTED, "server mailbox: no host mapping");
  }
  return PBH_OK;
}

// direct commands work here: the mailbox has a host mapping, and a pattern
// stored through it reads back from the device (a copy engine read of the
// device memory); otherwise the relay form serves
int srv_probe_direct(pbh_engine *e) {
  dfree(e->srv_mail);
  if (const int rc = srv_alloc_fine(e)) return rc;
  const uint32_t pat[4] = {0x5eed1234u, 0x0badf00du, 0x600df00du, 0xfeedfaceu};
  volatile uint32_t *w = reinterpret_cast<volatile uint32_t *>(e->srv_wmail);
  for (int i = 0; i < 4; ++i) w[i] = pat[i];
  __builtin_ia32_sfence();
  uint32_t back[4] = {0, 0, 0, 0};
  const hipError_t err = hipMemcpy(back, e->srv_mail, sizeof back, hipMemcpyDeviceToHost);
  if (err != hipSuccess || std::memcmp(back, pat, sizeof back) != 0) {
    (void)hipGetLastError();
    dfree(e->srv_mail);
    e->srv_wmail = nullptr;
    return fail(PBH_ERR_UNSUPPORTED, "server mailbox: host stores not seen by the device");
  }
  return PBH_OK;
}

int srv_launch(pbh_engine *e, pbh::KArgs k) {
  int32_t wgs = 0;
  hipError_t err = pbh::launch_mh_server(k, e->stream, &wgs, true);
  if (err != hipSuccess) return fail(PBH_ERR_UNSUPPORTED, "no resident server form");
  if (!e->srv_cmd) {
    err = hipHostMalloc((void **)&e->srv_cmd, sizeof(pbh::SrvCmd), hipHostMallocCoherent);
    if (err != hipSuccess) {
      e->srv_cmd = nullptr;
      return fail(PBH_ERR_HIP, "server command block: %s", hipGetErrorString(err));
    }
  }
  if (e->srv_done_len < wgs) {
    if (e->srv_done) (void)hipHostFree(e->srv_done);
    e->srv_done = nullptr;
    e->srv_done_len = 0;
    err = hipHostMalloc((void **)&e->srv_done, (size_t)wgs * sizeof(pbh::SrvDone),
                        hipHostMallocCoherent);
    if (err != hipSuccess) {
      e->srv_done = nullptr;
      return fail(PBH_ERR_HIP, "server completion words: %s", hipGetErrorString(err));
    }
    e->srv_done_len = wgs;
  }
  if (!e->srv_probed) {   // direct: a host mapping whose stores the device sees
    e->srv_probed = true;
    if ((e->srv_mode & 1) && srv_probe_direct(e) != PBH_OK) e->srv_mode &= ~1;
  }
  const bool direct = (e->srv_mode & 1) != 0;
  if (e->srv_mail && direct != e->srv_mail_fine) dfree(e->srv_mail);
  if (!e->srv_mail) {
    if (direct) {
      if (const int rc = srv_alloc_fine(e)) return rc;
    } else {
      err = hipMalloc((void **)&e->srv_mail, sizeof(pbh::SrvCmd));
      if (err != hipSuccess) {
        e->srv_mail = nullptr;
        return fail(PBH_ERR_HIP, "server mailbox: %s", hipGetErrorString(err));
      }
      e->srv_mail_fine = false;
      e->srv_wmail = nullptr;
    }
  }
  // the previous server (if any) has ended: sequence numbers restart
  HIP_TRY(hipMemsetAsync(e->srv_mail, 0, sizeof(pbh::SrvCmd), e->stream));
  // direct: the host writes the mailbox from the first command on, outside
  // the stream's order -- the zeroing above must have run by then
  if (direct) HIP_TRY(hipStreamSynchronize(e->stream));
  std::memset(e->srv_done, 0, (size_t)wgs * sizeof(pbh::SrvDone));
  std::memset(e->srv_cmd, 0, sizeof(pbh::SrvCmd));
  std::atomic_thread_fence(std::memory_order_seq_cst);
  e->srv_seq = 0;
  void *dcmd = nullptr, *ddone = nullptr;
  HIP_TRY(hipHostGetDevicePointer(&dcmd, e->srv_cmd, 0));
  HIP_TRY(hipHostGetDevicePointer(&ddone, e->srv_done, 0));
  k.srv_cmd = dcmd;
  k.srv_done = ddone;
  k.srv_mail = e->srv_mail;
  k.srv_mode = e->srv_mode;
  k.srv_idle = e->srv_idle_ms * 100000;   // 10 ns ticks
  err = pbh::launch_mh_server(k, e->stream, &wgs, false);
  if (err != hipSuccess) return fail(PBH_ERR_HIP, "server launch: %s", hipGetErrorString(err));
  e->srv_wgs = wgs;
  e->srv_active = true;
  e->srv_last = srv_clk::now();
  ++e->srv_launches;
  return PBH_OK;
}
// a run command (the previous one completed): n and arg, then seq
void srv_submit(pbh_engine *e, int64_t n_steps, int32_t fair, int32_t fair_rel) {
  const uint32_t q = ++e->srv_seq;
  srv_write(e, (uint32_t)n_steps,
            pbh::srv_arg(e->g, (uint32_t)fair, (uint32_t)fair_rel, pbh::kSrvRun, q), q);
  e->srv_pending = q;
  e->srv_last = srv_clk::now();
  e->g += n_steps;
  e->has_pred = true;
  e->mom_steps += n_steps;
  e->timed = true;
  e->srv_timed = true;
  e->last_launches = 1;
  ++e->srv_commands;
}
}  // namespace

#define SRV_STOP(e)                        \
  do {                                     \
    if ((e)->srv_active) {                 \
      const int srv_rc_ = srv_stop(e);     \
      if (srv_rc_) return srv_rc_;         \
    }                                      \
  } while (0)


const char *pbh_last_error(void) { return g_err.c_str(); }

int pbh_abi_version(void) { return PBH_ABI_VERSION; }

int pbh_device_count(int *count) {
  if (check_ptr(count, "count")) return PBH_ERR_ARG;
  HIP_TRY(hipGetDeviceCount(count));
  return PBH_OK;
}

int pbh_create(int device, pbh_engine **out) {
  if (check_ptr(out, "out")) return PBH_ERR_ARG;
  *out = nullptr;
  int nd = 0;
  HIP_TRY(hipGetDeviceCount(&nd));
  if (device < 0 || device >= nd)
    return fail(PBH_ERR_ARG, "device %d out of range (%d devices)", device, nd);
  HIP_TRY(hipSetDevice(device));
  // The runtime spins on completion signals instead of yielding / sleeping
  // on them (hipDeviceScheduleSpin): the host sees a short launch end ~2 us
  // sooner (tools/ubench/launch_lat.hip, profiles/r04d_launch_lat.jsonl).
  // The flag is process-wide for the device, so it is the host
  // application's choice: opt-in with PBH_SPIN_FLAG=1 (bench.py sets it).  A
  // device already in use keeps its flags (the call then fails, harmlessly);
  // only that call's own error is cleared, never one the application had
  // pending before it.
  {
    const char *sf = std::getenv("PBH_SPIN_FLAG");
    if (sf && sf[0] == '1') {
      const hipError_t before = hipPeekAtLastError();
      if (hipSetDeviceFlags(hipDeviceScheduleSpin) != hipSuccess && before == hipSuccess)
        (void)hipGetLastError();
    }
  }
  pbh_engine *e = new pbh_engine();
  e->device = device;
  if (const char *np = std::getenv("PBH_NO_PAIR")) e->pair_enabled = np[0] != '1';
  if (const char *gm = std::getenv("PBH_GIBBS_MFMA")) e->gibbs_mfma = gm[0] != '0';
  if (const char *gf = std::getenv("PBH_GIBBS_FAST")) e->gibbs_fast = gf[0] != '0';
  if (const char *gl = std::getenv("PBH_GIBBS_LANES")) e->gibbs_lanes = std::atoi(gl);
  if (const char *ml = std::getenv("PBH_GMM_LANES")) e->gmm_lanes = std::atoi(ml);
  if (const char *sy = std::getenv("PBH_SYNC")) {
    e->spin_sync = std::strcmp(sy, "block") != 0;
    e->sync_event = std::strcmp(sy, "event") == 0;
  }
  if (const char *em = std::getenv("PBH_EVENT_MARKERS")) e->event_markers = std::atoi(em) != 0;
  if (const char *gf = std::getenv("PBH_GMM_FULL")) e->gmm_full = std::atoi(gf) != 0;
  if (const char *pf = std::getenv("PBH_PAIR_FULL")) e->pair_full = std::atoi(pf) != 0;
  if (const char *sv = std::getenv("PBH_SERVER")) e->srv_enabled = sv[0] == '1';
  // PBH_SERVER_DIRECT=0: the relay form (workgroup 0 polls the host block);
  // the default writes commands straight into device memory
  if (const char *sd = std::getenv("PBH_SERVER_DIRECT")) e->srv_mode = sd[0] == '1' ? 1 : 0;
  if (const char *si = std::getenv("PBH_SERVER_IDLE_MS"))
    e->srv_idle_ms = std::max<int64_t>(1, std::min<int64_t>(10000, std::atoll(si)));
  if (const char *ef = std::getenv("PBH_ESS_FFT")) e->ess_fft = std::atoi(ef);
  if (const char *fi = std::getenv("PBH_IID_FULL")) e->iid_full = std::atoi(fi) != 0;
  if (const char *fp = std::getenv("PBH_IID_PAIR")) e->iid_pair = std::atoi(fp) != 0;
  if (const char *fa = std::getenv("PBH_FAIR")) e->fair = std::min(20, std::max(0, std::atoi(fa)));
  if (const char *wg = std::getenv("PBH_PAIR_WG")) e->pair_wg = std::atoi(wg);
  if (const char *fs = std::getenv("PBH_FAIR_SHORT"))
    e->fair_short = std::min(20, std::max(0, std::atoi(fs)));
  if (const char *fr = std::getenv("PBH_FAIR_REL")) e->fair_rel = std::atoi(fr) != 0;
  if (const char *ld = std::getenv("PBH_LEGACY_DB")) e->legacy_db = std::atoi(ld) != 0;
  if (const char *lw = std::getenv("PBH_LEGACY_WIN")) e->legacy_win = std::atoi(lw) != 0;
  if (const char *lk = std::getenv("PBH_LEGACY_K4")) e->legacy_k4 = std::atoi(lk) != 0;
  if (const char *lf = std::getenv("PBH_LEGACY_FUSED")) e->legacy_fused = std::atoi(lf) != 0;
  if (const char *lp = std::getenv("PBH_LEGACY_WP")) e->legacy_wp = std::atoi(lp) != 0;
  if (const char *la = std::getenv("PBH_LEGACY_AHEAD")) e->legacy_ahead = std::atoi(la) != 0;
  // PBH_EVENT_FLAGS: hipEventCreateWithFlags flags of the timing events (an
  // A/B switch for the markers' fences; default 0 = hipEventDefault)
  unsigned ev_flags = 0;
  if (const char *ef = std::getenv("PBH_EVENT_FLAGS")) ev_flags = (unsigned)std::strtoul(ef, nullptr, 0);
  e->ev_flags = ev_flags;
  hipError_t err = hipSuccess;
  {   // a destroyed engine's stream and events (drained), else new ones
    ResCache &c = res_cache();
    std::lock_guard<std::mutex> lk(c.mu);
    for (size_t i = 0; i < c.streams.size(); ++i)
      if (c.streams[i].device == device && c.streams[i].flags == ev_flags) {
        e->stream = c.streams[i].s;
        e->ev0 = c.streams[i].e0;
        e->ev1 = c.streams[i].e1;
        c.streams.erase(c.streams.begin() + (ptrdiff_t)i);
        break;
      }
  }
  if (!e->stream) {
    err = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (err == hipSuccess) err = hipEventCreateWithFlags(&e->ev0, ev_flags);
    if (err == hipSuccess) err = hipEventCreateWithFlags(&e->ev1, ev_flags);
  }
  if (err == hipSuccess) {
    static const std::vector<double> tab = [] {   // computed once per process
      std::vector<double> t(pbh::kBm64Doubles);
      pbh::bm64_tables(t.data());
      return t;
    }();
    if (dalloc(e->bm64, tab.size()) != PBH_OK) err = hipErrorOutOfMemory;
    if (err == hipSuccess)
      err = hipMemcpy(e->bm64, tab.data(), tab.size() * sizeof(double),
                      hipMemcpyHostToDevice);
  }
  if (err != hipSuccess) {
    pbh_destroy(e);
    return fail(PBH_ERR_HIP, "stream/event/table setup failed: %s",
                hipGetErrorString(err));
  }
  *out = e;
  return PBH_OK;
}

int pbh_destroy(pbh_engine *e) {
  if (!e) return PBH_OK;
  (void)hipSetDevice(e->device);
  if (e->srv_active) (void)srv_stop(e);   // never leave the server running
  bool drained = true;
  if (e->stream) drained = hipStreamSynchronize(e->stream) == hipSuccess;
  (void)hipGetLastError();
  if (e->comm) ncclCommDestroy(e->comm);
  // the device buffers into the resource cache (nothing in flight: the
  // stream drained), or freed after a failed stream
  auto put = [&](auto *&p) {
    if (drained) dretire(p);
    else dfree(p);
  };
  put(e->dmodel); put(e->dprop); put(e->dgibbs);
  put(e->x); put(e->lp); put(e->rep); put(e->xo); put(e->gq); put(e->lx);
  put(e->thr);
  put(e->mt_key); put(e->mt_pos); put(e->mt_has); put(e->mt_order);
  put(e->mt_gauss);
  put(e->tx); put(e->tlp); put(e->tpx); put(e->tpp); put(e->ts); put(e->tacc);
  e->cap = 0;
  put(e->msum); put(e->msq); put(e->nacc);
  put(e->gather_send); put(e->gather_recv); put(e->scalar);
  put(e->bm64); put(e->ess); put(e->lgtab); dfree(e->ess_list); put(e->ess_tot);
  if (e->ess_host) (void)hipHostFree(e->ess_host);
  if (e->srv_cmd) (void)hipHostFree(e->srv_cmd);
  if (e->srv_done) (void)hipHostFree(e->srv_done);
  dfree(e->srv_mail);
  bool kept = false;
  if (drained && e->stream && e->ev0 && e->ev1) {
    ResCache &c = res_cache();
    std::lock_guard<std::mutex> lk(c.mu);
    if (c.cap > 0 && c.streams.size() < 8) {
      c.streams.push_back({e->device, e->ev_flags, e->stream, e->ev0, e->ev1});
      kept = true;
    }
  }
  if (!kept) {
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    if (e->stream) (void)hipStreamDestroy(e->stream);
  }
  delete e;
  return PBH_OK;
}

int pbh_cache_release(void) {
  (void)cache_release_all();
  return PBH_OK;
}

int pbh_cache_info(int64_t *idle_bytes, int64_t *hits, int64_t *misses) {
  ResCache &c = res_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  if (idle_bytes) *idle_bytes = (int64_t)c.idle_bytes;
  if (hits) *hits = c.hits;
  if (misses) *misses = c.misses;
  return PBH_OK;
}

// ---------------------------------------------------------------------------
// model
// ---------------------------------------------------------------------------
int pbh_set_model(pbh_engine *e, const pbh_model *m) {
  if (check_ptr(e, "engine") || check_ptr(m, "model")) return PBH_ERR_ARG;
  SRV_STOP(e);
  const int d = m->dim;
  if (d < 1 || d > PBH_MAX_DIM)
    return fail(PBH_ERR_ARG, "dim %d outside 1..%d", d, PBH_MAX_DIM);
  if (!pbh::mh_dim_supported(d))
    return fail(PBH_ERR_UNSUPPORTED,
                "dim %d has no compiled kernel (1-12, 16, 20, 24, 32)", d);
  if (m->pscale != PBH_PSCALE_LOG && m->pscale != PBH_PSCALE_LIN)
    return fail(PBH_ERR_ARG, "bad pscale %d", m->pscale);
  if (m->scores < PBH_SCORES_HASTINGS || m->scores > PBH_SCORES_GIBBS)
    return fail(PBH_ERR_ARG, "bad scores %d", m->scores);
  if (e->x && d != e->d)
    return fail(PBH_ERR_STATE, "dim %d differs from initialised chains (%d)",
                d, e->d);
  std::vector<double> blk;
  size_t oa = 0, ob = 0, oc = 0, oe = 0, oplo = 0, ophi = 0, otoff = 0;
  const double *A = m->a, *B = m->b, *C = m->c, *E = m->e;
  int64_t na = 0, nb = 0, nc = 0, ne = 0;
  switch (m->target_kind) {
    case PBH_TARGET_DIAG_GAUSS: na = nb = nc = ne = d; break;
    case PBH_TARGET_NORM_IID:
      if (m->n < 1) return fail(PBH_ERR_ARG, "NORM_IID needs n_obs >= 1");
      if (m->i0 < 0 || m->i0 >= d || m->i1 < 0 || m->i1 >= d)
        return fail(PBH_ERR_ARG, "NORM_IID loc/scale dims out of range");
      na = m->n;
      break;
    case PBH_TARGET_GMM:
      if (m->n < 1) return fail(PBH_ERR_ARG, "GMM needs K >= 1");
      na = m->n; nb = m->n * d; nc = ne = m->n;
      break;
    case PBH_TARGET_NORM_PDF:
    case PBH_TARGET_UNIFORM_PDF: na = nb = d; break;
    case PBH_TARGET_MVN: na = d; nb = (int64_t)d * d; nc = 1; break;
    default: return fail(PBH_ERR_ARG, "bad target kind %d", m->target_kind);
  }
  if ((na && !A) || (nb && !B) || (nc && !C) || (ne && !E))
    return fail(PBH_ERR_ARG, "target arrays missing for kind %d",
                m->target_kind);
  oa = pack(blk, A, na); ob = pack(blk, B, nb); oc = pack(blk, C, nc);
  oe = pack(blk, E, ne);
  // Production-path (PBH_RNG_PHILOX) diagonal-Gauss constants: w = sqrt(.5)
  // / sigma and ksum = sum(logC + log sigma), so the density is
  // -sum (w (x - mu))^2 - ksum: three fp64 ops per dim.  Parity modes use
  // the reference's expression instead.
  size_t ow = 0;
  double ksum = 0.;
  if (m->target_kind == PBH_TARGET_DIAG_GAUSS) {
    std::vector<double> w(d);
    const double logC = std::log(std::sqrt(2 * M_PI));
    for (int i = 0; i < d; ++i) {
      w[i] = std::sqrt(0.5) / B[i];
      ksum += logC + C[i];
    }
    ow = pack(blk, w.data(), d);
  }
  if (m->target_kind == PBH_TARGET_GMM) {
    // Production path: w_k = sqrt(0.5) / sd_k, c_k = logw_k - d (logC +
    // log sd_k), so a_k = c_k - sum_i ((x_i - mu_ki) w_k)^2.
    const double logC = std::log(std::sqrt(2 * M_PI));
    std::vector<double> wc(2 * m->n);
    for (int64_t k = 0; k < m->n; ++k) {
      wc[k] = std::sqrt(0.5) / C[k];
      wc[m->n + k] = A[k] - d * (logC + E[k]);
    }
    ow = pack(blk, wc.data(), 2 * m->n);
  }
  if (m->target_kind == PBH_TARGET_NORM_IID) {
    // Production path: centred sufficient statistics of the observations,
    // sum_j (obs_j - mu)^2 = S2 + n (obar - mu)^2 -> O(1) per chain-step.
    double mean = 0., s2 = 0.;
    for (int64_t j = 0; j < m->n; ++j) mean += A[j];
    mean /= (double)m->n;
    for (int64_t j = 0; j < m->n; ++j) s2 += (A[j] - mean) * (A[j] - mean);
    const double st[2] = {mean, s2};
    ow = pack(blk, st, 2);
  }
  uint32_t lo_incl = 0, hi_incl = 0, ufun = 0;
  if (m->has_prior) {
    if (!m->prior_lo || !m->prior_hi || !m->prior_lo_incl || !m->prior_hi_incl)
      return fail(PBH_ERR_ARG, "prior arrays missing");
    oplo = pack(blk, m->prior_lo, d);
    ophi = pack(blk, m->prior_hi, d);
    for (int i = 0; i < d; ++i) {
      if (m->prior_lo_incl[i]) lo_incl |= 1u << i;
      if (m->prior_hi_incl[i]) hi_incl |= 1u << i;
    }
  }
  if (m->ufun)
    for (int i = 0; i < d; ++i)
      if (m->ufun[i]) ufun |= 1u << i;
  int tran_rev = 0;
  if (m->tran_kind == PBH_TRAN_GAUSS_PDF) {
    if (!m->tran_offset) return fail(PBH_ERR_ARG, "tran_offset missing");
    otoff = pack(blk, m->tran_offset, d);
    if (m->tran_order) {
      bool ident = true, rev = true;
      for (int i = 0; i < d; ++i) {
        ident = ident && m->tran_order[i] == i;
        rev = rev && m->tran_order[i] == d - 1 - i;
      }
      if (!ident && !rev)
        return fail(PBH_ERR_UNSUPPORTED,
                    "tran_order must be the identity or reversed");
      tran_rev = ident ? 0 : 1;
    }
  } else if (m->tran_kind != PBH_TRAN_CONST) {
    return fail(PBH_ERR_ARG, "bad tran kind %d", m->tran_kind);
  }
  if (blk.empty()) blk.push_back(0.);
  HIP_TRY(hipSetDevice(e->device));
  int rc = upload(e->dmodel, blk, e->stream);
  if (rc) return rc;
  KArgs &k = e->k;
  const double *base = e->dmodel;
  k.d = d; k.target = m->target_kind; k.pscale = m->pscale; k.scores = m->scores;
  k.ta = base + oa; k.tb = base + ob; k.tc = base + oc; k.te = base + oe;
  k.tw = base + ow; k.ksum = ksum;
  k.tn = (m->target_kind == PBH_TARGET_NORM_IID || m->target_kind == PBH_TARGET_GMM) ? m->n : 0;
  k.i0 = m->i0; k.i1 = m->i1;
  k.has_prior = m->has_prior ? 1 : 0;
  k.plo = base + oplo; k.phi = base + ophi;
  k.plo_incl = lo_incl; k.phi_incl = hi_incl;
  k.prior_logp = m->prior_logp;
  k.ufun = ufun;
  k.tran_kind = m->tran_kind; k.tran_sym = m->tran_sym ? 1 : 0; k.tran_rev = tran_rev;
  k.tran_value = m->tran_value; k.tran_scale = m->tran_scale;
  k.tran_off = base + otoff;
  // Constants the reference evaluates with NumPy on the host; the IEEE
  // results of these host libm calls are what the kernels compare against.
  k.log_npi = std::log(1.7976931348623158e+308);
  k.norm_C = std::sqrt(2 * M_PI);
  k.norm_logC = std::log(k.norm_C);
  if (m->target_kind == PBH_TARGET_MVN) {
    e->mvn_mean.assign(A, A + d);
    e->mvn_U.assign(B, B + (size_t)d * d);
    e->mvn_const = C[0];
  } else {
    e->mvn_mean.clear();
    e->mvn_U.clear();
  }
  e->d = d;
  e->has_model = true;
  e->lx_valid = false;   // the ufun mask may differ
  return PBH_OK;
}

int pbh_set_proposal(pbh_engine *e, const pbh_proposal *p) {
  if (check_ptr(e, "engine") || check_ptr(p, "proposal")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->has_model) return fail(PBH_ERR_STATE, "pbh_set_model first");
  const int d = e->d;
  std::vector<double> blk;
  size_t oloc = 0, oscl = 0, olen = 0, odel = 0;
  uint64_t vmode = 0;
  int32_t ploc_zero = 0;
  e->draw_order.assign(d, 0);
  for (int i = 0; i < d; ++i) e->draw_order[i] = i;
  switch (p->kind) {
    case PBH_PROP_GAUSS: {
      if (!p->loc || !p->scale) return fail(PBH_ERR_ARG, "GAUSS needs loc, scale");
      ploc_zero = 1;
      for (int i = 0; i < d; ++i) ploc_zero &= p->loc[i] == 0.0 ? 1 : 0;
      oloc = pack(blk, p->loc, d);
      oscl = pack(blk, p->scale, d);
      if (p->order) {
        std::vector<int> seen(d, 0);
        for (int j = 0; j < d; ++j) {
          const int k = p->order[j];
          if (k < 0 || k >= d || seen[k]++)
            return fail(PBH_ERR_ARG, "order must be a permutation of 0..%d", d - 1);
          e->draw_order[j] = k;
        }
      }
      break;
    }
    case PBH_PROP_SPHERE:
      if (!p->lengths) return fail(PBH_ERR_ARG, "SPHERE needs lengths");
      olen = pack(blk, p->lengths, d);
      break;
    case PBH_PROP_UNIFORM:
      if (!p->delta_vec) return fail(PBH_ERR_ARG, "UNIFORM needs delta_vec");
      odel = pack(blk, p->delta_vec, d);
      break;
    case PBH_PROP_VARDELTA:
      if (!p->delta_vec || !p->var_mode)
        return fail(PBH_ERR_ARG, "VARDELTA needs delta_vec and var_mode");
      for (int i = 0; i < d; ++i) {
        const int md = p->var_mode[i];
        if (md < PBH_VAR_FIXED || md > PBH_VAR_RANDINT)
          return fail(PBH_ERR_ARG, "var_mode[%d] = %d is not a pbh_var_delta", i, md);
        if (!std::isfinite(p->delta_vec[i]))
          return fail(PBH_ERR_ARG, "delta_vec[%d] must be finite", i);
        if (md == PBH_VAR_RANDINT &&
            !(std::trunc(p->delta_vec[i]) >= 1. && p->delta_vec[i] < 2147483648.))
          return fail(PBH_ERR_ARG, "randint(-%g, %g): low >= high or range "
                      "beyond 32 bits", p->delta_vec[i], p->delta_vec[i]);
        vmode |= (uint64_t)md << (2 * i);
      }
      odel = pack(blk, p->delta_vec, d);
      break;
    default:
      return fail(PBH_ERR_ARG, "bad proposal kind %d (GIBBS: pbh_set_gibbs)", p->kind);
  }
  size_t otf = 0;
  if (p->tfun) {
    for (int i = 0; i < d * d; ++i)
      if (!std::isfinite(p->tfun[i])) return fail(PBH_ERR_ARG, "tfun must be finite");
    otf = pack(blk, p->tfun, (size_t)d * d);
  }
  uint32_t vint = 0, bnd_on = 0, bxlo = 0, bxhi = 0;
  size_t oblo = 0, obhi = 0;
  if (p->var_int)
    for (int i = 0; i < d; ++i) vint |= (p->var_int[i] ? 1u : 0u) << i;
  if (p->bound_on) {
    if (!p->bound_lo || !p->bound_hi || !p->bound_xlo || !p->bound_xhi)
      return fail(PBH_ERR_ARG, "bound_on needs bound_lo/hi and bound_xlo/xhi");
    for (int i = 0; i < d; ++i) {
      if (!p->bound_on[i]) continue;
      if (!(p->bound_lo[i] <= p->bound_hi[i]))
        return fail(PBH_ERR_ARG, "bound[%d]: lo > hi", i);
      bnd_on |= 1u << i;
      bxlo |= (p->bound_xlo[i] ? 1u : 0u) << i;
      bxhi |= (p->bound_xhi[i] ? 1u : 0u) << i;
    }
    oblo = pack(blk, p->bound_lo, d);
    obhi = pack(blk, p->bound_hi, d);
  }
  HIP_TRY(hipSetDevice(e->device));
  int rc = upload(e->dprop, blk, e->stream);
  if (rc) return rc;
  KArgs &k = e->k;
  k.prop = p->kind;
  k.vmode = vmode;
  k.vint = vint;
  k.bnd_on = bnd_on; k.bnd_xlo = bxlo; k.bnd_xhi = bxhi;
  k.blo = e->dprop + oblo; k.bhi = e->dprop + obhi;
  k.ploc = e->dprop + oloc; k.pscl = e->dprop + oscl;
  k.ploc_zero = ploc_zero;
  k.plen = e->dprop + olen; k.pdel = e->dprop + odel;
  k.sdelta = p->delta;
  k.ptf = p->tfun ? e->dprop + otf : nullptr;
  k.has_tfun = p->tfun ? 1 : 0;
  e->has_prop = true;
  e->has_gibbs = false;
  return PBH_OK;
}

int pbh_set_gibbs(pbh_engine *e, const pbh_gibbs *gb) {
  if (check_ptr(e, "engine") || check_ptr(gb, "gibbs")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->has_model) return fail(PBH_ERR_STATE, "pbh_set_model first");
  if (e->k.target != PBH_TARGET_MVN || e->k.scores != PBH_SCORES_GIBBS)
    return fail(PBH_ERR_UNSUPPORTED,
                "CondCov Gibbs needs an MVN target and gibbs scores");
  const int d = e->d;
  if (!gb->mean || !gb->stdv || !gb->cdf || (d > 1 && !gb->coef))
    return fail(PBH_ERR_ARG, "gibbs tables missing");
  if (gb->tsteps < 1 || gb->tsteps > d)
    return fail(PBH_ERR_ARG, "tsteps %d outside 1..%d", gb->tsteps, d);
  std::vector<double> blk;
  const size_t om = pack(blk, gb->mean, d);
  const size_t oc = pack(blk, gb->coef ? gb->coef : gb->mean, d > 1 ? (int64_t)d * (d - 1) : 0);
  const size_t os = pack(blk, gb->stdv, d);
  const size_t ocdf = pack(blk, gb->cdf, 2 * d);
  // Production-kernel tables (gibbs_fast_kernel).  The density is taken at
  // y = x[perm] (prob.py:354-357): P = U U^T in y order; re-indexed to x
  // order P'[j][j'] = P[inv(j)][inv(j')], mu'[j] = mean[inv(j)].  z limits
  // are ndtri of the cdf limits (the truncation cond_cov.py:57-62 applies).
  std::vector<int> inv(d);
  for (int i = 0; i < d; ++i) {
    const int pi = d <= 1 ? 0 : (d == 2 ? 1 - i : (i < d - 1 ? d - 2 - i : d - 1));
    inv[pi] = i;
  }
  std::vector<double> pp((size_t)d * d), mup(d), zlo(d), zhi(d);
  for (int j = 0; j < d; ++j) {
    mup[j] = e->mvn_mean[inv[j]];
    for (int jj = 0; jj < d; ++jj) {
      double acc = 0.;
      for (int o = 0; o < d; ++o)
        acc += e->mvn_U[(size_t)inv[j] * d + o] * e->mvn_U[(size_t)inv[jj] * d + o];
      pp[(size_t)j * d + jj] = acc;
    }
  }
  for (int j = 0; j < d; ++j) {
    zlo[j] = pbh::ndtri(gb->cdf[2 * j]);
    zhi[j] = pbh::ndtri(gb->cdf[2 * j + 1]);
  }
  std::vector<double> ak(d);
  for (int k = 0; k < d; ++k) {
    double acc = 0.;
    for (int i = 0, jj = 0; i < d; ++i) {
      if (i == k) continue;
      acc += gb->coef[(size_t)k * (d - 1) + jj++] * gb->mean[i];
    }
    ak[k] = gb->mean[k] - acc;
  }
  const size_t oak = pack(blk, ak.data(), d);
  const size_t opp = pack(blk, pp.data(), (int64_t)d * d);
  const size_t omup = pack(blk, mup.data(), d);
  const size_t ozlo = pack(blk, zlo.data(), d);
  const size_t ozhi = pack(blk, zhi.data(), d);
  HIP_TRY(hipSetDevice(e->device));
  int rc = upload(e->dgibbs, blk, e->stream);
  if (rc) return rc;
  KArgs &k = e->k;
  k.gmean = e->dgibbs + om; k.gcoef = e->dgibbs + oc;
  k.gstdv = e->dgibbs + os; k.gcdf = e->dgibbs + ocdf;
  k.gpp = e->dgibbs + opp; k.gmup = e->dgibbs + omup;
  k.gzlo = e->dgibbs + ozlo; k.gzhi = e->dgibbs + ozhi;
  k.gak = e->dgibbs + oak;
  k.gconst = e->mvn_const;
  k.tsteps = gb->tsteps;
  e->gq_valid = false;
  k.prop = PBH_PROP_GIBBS;
  e->draw_order.assign(gb->tsteps, 0);
  for (int i = 0; i < gb->tsteps; ++i) e->draw_order[i] = i;
  e->has_gibbs = true;
  e->has_prop = false;
  return PBH_OK;
}

// ---------------------------------------------------------------------------
// chains, randomness
// ---------------------------------------------------------------------------
int pbh_init_chains(pbh_engine *e, int64_t n, int64_t off, const double *init) {
  if (check_ptr(e, "engine") || check_ptr(init, "init")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->has_model) return fail(PBH_ERR_STATE, "pbh_set_model first");
  if (n < 1 || off < 0) return fail(PBH_ERR_ARG, "bad n_chains/offset");
  // kernels address a chain's trace word through a 32-bit buffer offset
  // (chain * 8 bytes; per-GPU shards of 2^28 chains are far above the 288 GB)
  if (n > ((int64_t)1 << 28)) return fail(PBH_ERR_ARG, "n_chains > 2^28 per engine");
  const int d = e->d;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (n != e->n) {
    free_trace(e);
    int rc = dalloc(e->x, (size_t)n * d);
    if (!rc) rc = dalloc(e->lp, n);
    if (!rc) rc = dalloc(e->msum, (size_t)n * d);
    if (!rc) rc = dalloc(e->msq, (size_t)n * d);
    if (!rc) rc = dalloc(e->nacc, n);
    if (!rc) rc = dalloc(e->xo, (size_t)8 * n);
    if (!rc) rc = dalloc(e->gq, (size_t)(d + 1) * n);
    if (!rc) rc = dalloc(e->lx, (size_t)d * n);
    if (!rc) rc = dalloc(e->ess, (size_t)d * n);
    if (rc) return rc;
  }
  // no ESS computed yet: every byte 0xFF is a NaN (all-ones exponent and
  // mantissa), set on the device instead of copying a host array of NaNs
  e->gq_valid = false;
  e->lx_valid = false;
  hipStream_t st = e->stream;
  const size_t nd = (size_t)n * d;
  HIP_TRY(hipMemsetAsync(e->ess, 0xFF, nd * sizeof(double), st));
  // the caller's [n][d] rows go up as they are (msum is the staging buffer,
  // zeroed after) and are transposed to x's [d][n] on the device
  HIP_TRY(hipMemcpyAsync(e->msum, init, nd * sizeof(double), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(chains_to_dim_major, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, st,
                     e->msum, e->x, n, (int32_t)d);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemsetAsync(e->lp, 0, n * sizeof(double), st));
  HIP_TRY(hipMemsetAsync(e->msum, 0, nd * sizeof(double), st));
  HIP_TRY(hipMemsetAsync(e->msq, 0, nd * sizeof(double), st));
  HIP_TRY(hipMemsetAsync(e->nacc, 0, n * sizeof(int64_t), st));
  HIP_TRY(hipStreamSynchronize(st));
  e->n = n;
  e->off = off;
  e->xo_seeded = false;
  e->state_lost = false;
  e->has_pred = false;
  e->g = 0;
  e->mom_steps = 0;
  e->rec_base = 0;
  dfree(e->rep);
  e->rep_alloc = 0;
  e->rep_steps = 0;
  e->rep_g0 = 0;
  return PBH_OK;
}

int pbh_set_step(pbh_engine *e, int64_t g) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->x) return fail(PBH_ERR_STATE, "pbh_init_chains first");
  if (e->has_pred || e->cap > 0 || e->rep)
    return fail(PBH_ERR_STATE, "pbh_set_step goes right after pbh_init_chains");
  if (g < 0) return fail(PBH_ERR_ARG, "step index must be >= 0");
  e->g = g;
  return PBH_OK;
}

int pbh_set_rng(pbh_engine *e, int32_t mode, uint64_t seed) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (mode != PBH_RNG_REPLAY && mode != PBH_RNG_PHILOX &&
      mode != PBH_RNG_PHILOX_F64 && mode != PBH_RNG_XOSHIRO &&
      mode != PBH_RNG_PHILOX_FP32)
    return fail(PBH_ERR_ARG, "bad rng mode %d", mode);
  e->rng = mode;
  e->seed = seed;
  e->xo_seeded = false;   // (re)seeded from (seed, chain id) at the next run
  return PBH_OK;
}

int pbh_stream_width(pbh_engine *e, int32_t *r) {
  if (check_ptr(e, "engine") || check_ptr(r, "r")) return PBH_ERR_ARG;
  if (e->has_gibbs) *r = e->k.tsteps;
  else if (e->has_prop) *r = e->d + 1;
  else return fail(PBH_ERR_STATE, "no proposal or gibbs tables set");
  return PBH_OK;
}

int pbh_upload_replay(pbh_engine *e, int64_t n_steps, const double *rand) {
  if (check_ptr(e, "engine") || check_ptr(rand, "rand")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->x) return fail(PBH_ERR_STATE, "pbh_init_chains first");
  int32_t R = 0;
  int rc = pbh_stream_width(e, &R);
  if (rc) return rc;
  if (n_steps < 1) return fail(PBH_ERR_ARG, "n_steps must be >= 1");
  const int64_t n = e->n;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  rc = dalloc(e->rep, (size_t)n_steps * R * n);
  e->rep_alloc = rc ? 0 : (size_t)n_steps * R * n;
  if (rc) return rc;
  // Reorder draws so that device row k feeds dim k (GAUSS Delta keyword
  // order); the threshold row (index d for MH) stays last.
  std::vector<double> row((size_t)R * n);
  for (int64_t t = 0; t < n_steps; ++t) {
    const double *src = rand + (size_t)t * R * n;
    for (int j = 0; j < R; ++j) {
      const int dst = j < (int)e->draw_order.size() ? e->draw_order[j] : j;
      std::memcpy(&row[(size_t)dst * n], src + (size_t)j * n, n * sizeof(double));
    }
    HIP_TRY(hipMemcpy(e->rep + (size_t)t * R * n, row.data(),
                      row.size() * sizeof(double), hipMemcpyHostToDevice));
  }
  e->k.R = R;
  e->rep_steps = n_steps;
  e->rep_g0 = e->g;
  return PBH_OK;
}

int pbh_legacy_seed(pbh_engine *e, const uint32_t *seeds) {
  if (check_ptr(e, "engine") || check_ptr(seeds, "seeds")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->x) return fail(PBH_ERR_STATE, "pbh_init_chains first");
  const int64_t n = e->n;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  // the state layout is fixed at seeding
  // (Mt4's resources take 32-bit byte offsets: its state must span < 2^32 B)
  e->mt_mode = !e->legacy_db ? 0
               : (e->legacy_k4 && e->legacy_win && mt_words(2) * 4 * n < (int64_t(1) << 32)) ? 2
                                                                                          : 1;
  e->mt_stale = false;
  e->mt_odd = false;
  int rc = dalloc(e->mt_key, (size_t)mt_words(e->mt_mode) * n);
  if (!rc) rc = dalloc(e->mt_pos, n);
  if (!rc) rc = dalloc(e->mt_has, n);
  if (!rc) rc = dalloc(e->mt_gauss, n);
  if (rc) return rc;
  uint32_t *dseeds = nullptr;
  rc = dalloc(dseeds, n);
  if (rc) return rc;
  hipError_t err = hipMemcpy(dseeds, seeds, n * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (err == hipSuccess)
    err = pbh::launch_legacy_seed(e->mt_key, e->mt_pos, e->mt_gauss, e->mt_has,
                                  dseeds, n, e->mt_mode, e->stream);
  if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
  dfree(dseeds);
  if (err != hipSuccess)
    return fail(PBH_ERR_HIP, "pbh_legacy_seed: %s", hipGetErrorString(err));
  return PBH_OK;
}

int pbh_reserve_replay(pbh_engine *e, int64_t n_steps) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  int32_t R = 0;
  int rc = pbh_stream_width(e, &R);
  if (rc) return rc;
  if (n_steps < 1) return fail(PBH_ERR_ARG, "n_steps must be >= 1");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  const size_t need = (size_t)n_steps * R * e->n;
  if (!e->rep || e->rep_alloc < need) {
    // the stream rows in use (if any) are not kept: reserve before the
    // generation or upload that fills them
    rc = dalloc(e->rep, need);
    e->rep_alloc = rc ? 0 : need;
    e->rep_steps = 0;
  }
  return rc;
}

int pbh_legacy_replay(pbh_engine *e, int64_t n_steps) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->mt_key) return fail(PBH_ERR_STATE, "pbh_legacy_seed first");
  if (e->mt_stale)
    return fail(PBH_ERR_STATE, "pbh_restore ran after pbh_legacy_seed: set the "
                "checkpoint's legacy state (pbh_set_legacy_state) first");
  int32_t R = 0;
  int rc = pbh_stream_width(e, &R);
  if (rc) return rc;
  if (n_steps < 1) return fail(PBH_ERR_ARG, "n_steps must be >= 1");
  const int64_t n = e->n;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  // consecutive stream generations of the same (or a smaller) size reuse the
  // buffer: a 250-step cfg2-width stream is 1.4 GB, and a free + malloc of it
  // per call was 0.3-0.5 ms of the call
  const size_t need = (size_t)n_steps * R * n;
  if (!e->rep || e->rep_alloc < need) {
    rc = dalloc(e->rep, need);
    e->rep_alloc = rc ? 0 : need;
  }
  if (!rc && !e->has_gibbs) {
    rc = dalloc(e->mt_order, e->d);
    if (!rc) HIP_TRY(hipMemcpy(e->mt_order, e->draw_order.data(),
                               e->d * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  if (rc) return rc;
  pbh::LegacyArgs a{};
  a.key = e->mt_key; a.pos = e->mt_pos; a.gauss = e->mt_gauss;
  a.has_gauss = e->mt_has; a.order = e->mt_order; a.out = e->rep;
  a.n = n; a.n_steps = n_steps; a.step0 = e->g;
  a.d = e->d; a.R = R; a.gibbs = e->has_gibbs ? 1 : 0;
  a.normal = (!e->has_gibbs && e->k.prop == PBH_PROP_GAUSS) ? 1 : 0;
  a.vardelta = (!e->has_gibbs && e->k.prop == PBH_PROP_VARDELTA) ? 1 : 0;
  a.db = e->mt_mode;
  a.win = e->legacy_win ? 1 : 0;
  a.vmode = e->k.vmode;
  a.vdelta = e->k.pdel;
  a.wp = (e->legacy_wp && !e->mt_odd) ? 1 : 0;
  if (a.vardelta) e->mt_odd = true;   // randint may leave odd positions
  if (!e->lgtab) {
    std::vector<double> lt(pbh::kLegLogDoubles);
    pbh::legacy_log_table(lt.data());
    rc = dalloc(e->lgtab, lt.size());
    if (rc) return rc;
    HIP_TRY(hipMemcpy(e->lgtab, lt.data(), lt.size() * sizeof(double), hipMemcpyHostToDevice));
  }
  a.lgtab = e->lgtab;
  // Launches of at most kLegacyLaunchSteps steps: the generator counts a
  // launch's stream quads per chain in 32-bit ints (Mt4's head index), and a
  // step takes a bounded-in-expectation but unbounded number of words (polar
  // rejections, randint masks), so the launch length is what is bounded:
  // 2^20 steps x R <= 33 draws x ~3 words per draw is ~2^27 quads << 2^31.
  // The state (position, block, pending gauss) persists between launches, so
  // the split is invisible in the stream.
  constexpr int64_t kLegacyLaunchSteps = int64_t(1) << 20;
  // the twist-ahead pass (as pbh_legacy_run) for the chain-per-lane Mt4
  // generator -- Gibbs rows, per-variable deltas, raw draws, odd positions;
  // the word-parallel generator twists in its own LDS.  Words per step: Gibbs
  // at most 2R, per-variable at least 2 per draw (randint's masked
  // rejections beyond that twist in the generator), raw 2(d + 1), normal the
  // polar method's mean + 8 sigma
  const bool wp_path = a.wp && !a.gibbs && !a.vardelta;
  const bool ahead = e->legacy_ahead && e->mt_mode == 2 && !wp_path;
  const double dd = (double)e->d;
  auto ahead_words = [&](int64_t m) {
    const double mm = (double)m;
    if (a.gibbs) return 2.0 * (mm * R + 2.0);
    if (a.vardelta || !a.normal) return 2.0 * (mm * (dd + 1.0) + 2.0);
    return 2.0 * (mm * (4.0 * dd / 3.14159265358979 + 1.0) +
                  8.0 * std::sqrt(mm * 4.0 * 0.3480 * dd / 2.0) + 2.0);
  };
  int64_t k_fit = kLegacyLaunchSteps;
  if (ahead) {
    k_fit = std::min<int64_t>(n_steps, kLegacyLaunchSteps);
    while (k_fit > 1 && ahead_words(k_fit) > 14.0 * pbh_mt_block_words()) k_fit = k_fit * 7 / 8;
  }
  hipError_t err = hipSuccess;
  for (int64_t done = 0; done < n_steps && err == hipSuccess;) {
    const int64_t k = std::min(std::min(n_steps - done, kLegacyLaunchSteps), k_fit);
    if (ahead) {
      const int32_t want = std::min<int32_t>(
          15, 1 + (int32_t)std::ceil(ahead_words(k) / pbh_mt_block_words()));
      err = pbh::launch_legacy_ahead(e->mt_key, e->mt_pos, n, want, e->stream);
      if (err != hipSuccess) break;
    }
    a.out = e->rep + (size_t)done * R * n;
    a.n_steps = k;
    a.step0 = e->g + done;
    err = pbh::launch_legacy_gen(a, e->stream);
    done += k;
  }
  if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
  if (err != hipSuccess)
    return fail(PBH_ERR_HIP, "pbh_legacy_replay: %s", hipGetErrorString(err));
  e->k.R = R;
  e->rep_steps = n_steps;
  e->rep_g0 = e->g;
  return PBH_OK;
}

int pbh_get_replay(pbh_engine *e, int64_t first, int64_t n_steps, int32_t draw,
                   double *out) {
  if (check_ptr(e, "engine") || check_ptr(out, "out")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->rep) return fail(PBH_ERR_STATE, "no replay stream");
  if (first < 0 || n_steps < 0 || first + n_steps > e->rep_steps)
    return fail(PBH_ERR_ARG, "rows [%lld, %lld) outside the %lld-row stream",
                (long long)first, (long long)(first + n_steps),
                (long long)e->rep_steps);
  const int R = e->k.R;
  const int64_t n = e->n;
  if (draw >= R) return fail(PBH_ERR_ARG, "draw %d >= R = %d", draw, R);
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (draw >= 0) {
    const int src = draw < (int)e->draw_order.size() ? e->draw_order[draw] : draw;
    HIP_TRY(hipMemcpy2D(out, n * sizeof(double),
                        e->rep + (size_t)first * R * n + (size_t)src * n,
                        (size_t)R * n * sizeof(double), n * sizeof(double),
                        n_steps, hipMemcpyDeviceToHost));
    return PBH_OK;
  }
  std::vector<double> row((size_t)R * n);
  for (int64_t t = 0; t < n_steps; ++t) {
    HIP_TRY(hipMemcpy(row.data(), e->rep + (size_t)(first + t) * R * n,
                      row.size() * sizeof(double), hipMemcpyDeviceToHost));
    double *dst = out + (size_t)t * R * n;
    // undo pbh_upload_replay's reordering: draw j sits in row draw_order[j]
    for (int j = 0; j < R; ++j) {
      const int src = j < (int)e->draw_order.size() ? e->draw_order[j] : j;
      std::memcpy(dst + (size_t)j * n, &row[(size_t)src * n], n * sizeof(double));
    }
  }
  return PBH_OK;
}

// ---------------------------------------------------------------------------
// running
// ---------------------------------------------------------------------------
int pbh_alloc_trace(pbh_engine *e, int64_t capacity, int32_t thin, int32_t debug) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  // PBH_TRACE_NOFILL: the caller's next run writes every record (no zero fill)
  const bool nofill = (debug & PBH_TRACE_NOFILL) != 0;
  debug &= ~PBH_TRACE_NOFILL;
  SRV_STOP(e);
  if (!e->x) return fail(PBH_ERR_STATE, "pbh_init_chains first");
  if (capacity < 0 || thin < 1) return fail(PBH_ERR_ARG, "bad capacity/thin");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  free_trace(e);
  const int64_t n = e->n, d = e->d, W = (n + 63) / 64;
  int rc = PBH_OK;
  if (capacity > 0) {
    rc = dalloc(e->tx, (size_t)capacity * d * n);
    if (!rc) rc = dalloc(e->tlp, (size_t)capacity * n);
    if (!rc) rc = dalloc(e->tacc, (size_t)capacity * W);
    if (!rc && debug) {
      rc = dalloc(e->tpx, (size_t)capacity * d * n);
      if (!rc) rc = dalloc(e->tpp, (size_t)capacity * n);
      if (!rc) rc = dalloc(e->ts, (size_t)capacity * n);
    }
  }
  if (rc) {
    free_trace(e);
    return rc;
  }
  if (capacity > 0 && !nofill) {
    // zero-fill: unwritten records read as zeros, and every page of the
    // trace is mapped and touched before the first run writes it (the
    // first writes of a short run otherwise pay the translation misses)
    const size_t dn = (size_t)capacity * d * n;
    HIP_TRY(hipMemsetAsync(e->tx, 0, dn * sizeof(double), e->stream));
    HIP_TRY(hipMemsetAsync(e->tlp, 0, (size_t)capacity * n * sizeof(double), e->stream));
    HIP_TRY(hipMemsetAsync(e->tacc, 0, (size_t)capacity * W * sizeof(uint64_t), e->stream));
    if (debug) {
      HIP_TRY(hipMemsetAsync(e->tpx, 0, dn * sizeof(double), e->stream));
      HIP_TRY(hipMemsetAsync(e->tpp, 0, (size_t)capacity * n * sizeof(double), e->stream));
      HIP_TRY(hipMemsetAsync(e->ts, 0, (size_t)capacity * n * sizeof(double), e->stream));
    }
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  e->cap = capacity;
  e->thin = thin;
  e->debug = debug ? 1 : 0;
  e->rec_base = e->g / thin;
  return PBH_OK;
}

#ifdef PBH_PHASES
// Probe build only: per-wave phase stamps of the last FULL pair launch
// (8 words per wave; pbh_kernels_impl.h PBH_PHASE).
static double *phase_buffer() {
  static double *buf = nullptr;
  if (!buf && hipMalloc(&buf, 4 << 20) == hipSuccess) hipMemset(buf, 0, 4 << 20);
  return buf;
}
extern "C" int pbh_phase_dump(uint64_t *dst, int64_t words) {
  if (words > (4 << 20) / 8) return PBH_ERR_ARG;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(dst, phase_buffer(), words * 8, hipMemcpyDeviceToHost));
  return PBH_OK;
}
#endif

// pbh_run's (and pbh_legacy_run's) argument checks
static int run_checks(pbh_engine *e, int64_t n_steps) {
  if (!e->has_model || (!e->has_prop && !e->has_gibbs))
    return fail(PBH_ERR_STATE, "model and proposal/gibbs tables must be set");
  if (!e->x) return fail(PBH_ERR_STATE, "pbh_init_chains first");
  if (e->state_lost)
    return fail(PBH_ERR_STATE, "chain state lost by an incomplete sampling-server command: "
                "pbh_restore, pbh_set_chains or pbh_init_chains first");
  if (e->has_gibbs != (e->k.scores == PBH_SCORES_GIBBS))
    return fail(PBH_ERR_STATE, "gibbs scores need gibbs tables and vice versa");
  if (n_steps < 0) return fail(PBH_ERR_ARG, "n_steps < 0");
  if (e->rng == PBH_RNG_PHILOX_FP32 && e->has_gibbs)
    return fail(PBH_ERR_UNSUPPORTED, "PHILOX_FP32 is a lane-pair MH comparison mode");
  if (e->cap > 0) {
    const int64_t recs = (e->g + n_steps) / e->thin - e->rec_base;
    if (recs > e->cap)
      return fail(PBH_ERR_STATE, "trace capacity %lld < %lld records",
                  (long long)e->cap, (long long)recs);
  }
  return PBH_OK;
}

// a run's kernel arguments (the per-launch fields g0, n_steps, has_pred,
// rep_row0, gq_init, lx, lx_init, fair, fair_rel are set per launch) and the
// dynamic LDS of the NORM_IID observation stage
static void run_args(pbh_engine *e, KArgs &k, size_t &lds) {
  k = e->k;
  k.n = e->n;
  k.off = e->off;
  k.x = e->x;
  k.lp = e->lp;
  k.rng = e->rng;
  k.seed_lo = (uint32_t)e->seed;
  k.seed_hi = (uint32_t)(e->seed >> 32);
  k.rep = e->rep;
#ifdef PBH_PHASES
  if (!k.rep) k.rep = phase_buffer();   // probe build: the FULL kernel's stamps
#endif
  k.xo = e->xo;
  k.tx = e->tx; k.tlp = e->tlp; k.tpx = e->tpx; k.tpp = e->tpp; k.ts = e->ts;
  k.tacc = e->tacc;
  k.thin = e->cap > 0 ? e->thin : 1;
  k.rec_base = e->rec_base;
  k.rec_cap = e->cap;
  k.debug = e->debug;
  k.W = (e->n + 63) / 64;
  {
    // The lane-pair kernel drops the per-step tran evaluation: allowed when
    // the constant tran's rescaled value q~ > 0 (sp_utils.py:52-54 never
    // returns None); see pair_form in pbh_kernels_impl.h.
    const double v = k.tran_value;
    const double qt = k.pscale == PBH_PSCALE_LIN
                          ? v : (v <= k.log_npi ? std::exp(v) : 1.7976931348623158e+308);
    k.pair_ok = (e->pair_enabled && (k.scores == PBH_SCORES_METROPOLIS || qt > 0.0)) ? 1 : 0;
    // metropolis_scores / hastings_scores with a constant tran are the ratio
    // form of (lp', lp) -- or, for a tuple tran, of (lp' q~, lp q~): the
    // reverse value equals the forward one (rf.py:536), sp_utils.py:59-64.
    k.simple_acc = (k.scores == PBH_SCORES_METROPOLIS ||
                    (k.scores == PBH_SCORES_HASTINGS &&
                     k.tran_kind == PBH_TRAN_CONST && qt > 0.0)) ? 1 : 0;
    k.acc_beta = (k.scores == PBH_SCORES_HASTINGS && !k.tran_sym) ? qt : 1.0;
  }
  k.gibbs_mfma = e->gibbs_mfma ? 1 : 0;
  k.gibbs_fast = e->gibbs_fast ? 1 : 0;
  k.gibbs_lanes = e->gibbs_lanes;
  k.gmm_lanes = e->gmm_lanes;
  k.gmm_full = e->gmm_full ? 1 : 0;
  k.pair_full = e->pair_full ? 1 : 0;
  k.iid_full = e->iid_full ? 1 : 0;
  k.iid_pair = e->iid_pair ? 1 : 0;
  k.fair = e->fair;
  k.pair_wg = e->pair_wg;
  k.gq = e->gq;
  k.moments = (e->collect & PBH_COLLECT_MOMENTS) ? 1 : 0;
  k.msum = e->msum; k.msq = e->msq; k.nacc = e->nacc;
  k.bm64 = e->bm64;
  lds = (k.target == PBH_TARGET_NORM_IID && k.tn <= 16384 &&
                      k.rng != PBH_RNG_PHILOX)   // production: O(1) statistics
                         ? (size_t)k.tn * sizeof(double) : 0;
}

int pbh_run(pbh_engine *e, int64_t n_steps, int32_t steps_per_launch) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  // PBH_TRACE_ENQUEUE=1: the host time of each enqueue phase to stderr
  // (diagnostic of short-launch latency)
  static const bool trace_enq = [] {
    const char *t = std::getenv("PBH_TRACE_ENQUEUE");
    return t && t[0] == '1';
  }();
  using clk = std::chrono::steady_clock;
  const auto tq0 = clk::now();
  auto tq = [&](const char *what) {
    if (trace_enq)
      std::fprintf(stderr, "pbh_run %s %.2f us\n", what,
                   std::chrono::duration<double, std::micro>(clk::now() - tq0).count());
  };
  if (const int rc = run_checks(e, n_steps)) return rc;
  if (n_steps == 0) {
    e->timed = false;
    e->last_launches = 0;
    return PBH_OK;
  }
  if (e->rng == PBH_RNG_REPLAY &&
      (!e->rep || e->g < e->rep_g0 || e->g + n_steps > e->rep_g0 + e->rep_steps))
    return fail(PBH_ERR_STATE,
                "replay stream covers steps [%lld, %lld), run needs [%lld, %lld)",
                (long long)e->rep_g0, (long long)(e->rep_g0 + e->rep_steps),
                (long long)e->g, (long long)(e->g + n_steps));
  // a running server and a run of its form: the command straight away (no
  // kernel-argument block, no device call; the server's form was checked at
  // its launch and every entry point that could change it stops it)
  if (e->srv_active && (steps_per_launch <= 0 || steps_per_launch >= n_steps) &&
      n_steps <= (1 << 30) && e->g + n_steps < (int64_t(1) << 47) &&
      !(e->collect & PBH_COLLECT_MOMENTS) && e->has_pred && e->cap > 0 && e->thin == 1 &&
      e->g - e->rec_base >= 0 && e->g + n_steps - e->rec_base <= e->cap) {
    if (e->srv_pending) {
      const int rc = srv_wait(e, e->srv_pending, false);
      e->srv_pending = 0;
      if (rc) return rc;
    }
    if (srv_clk::now() - e->srv_last <= std::chrono::milliseconds(e->srv_idle_ms / 2)) {
      const bool short_run = n_steps <= 64;
      srv_submit(e, n_steps, short_run ? e->fair_short : e->fair,
                 short_run ? 1 : e->fair_rel);
      tq("server command (fast path)");
      return PBH_OK;
    }
  }
  HIP_TRY(hipSetDevice(e->device));
  if (e->rng == PBH_RNG_XOSHIRO && !e->xo_seeded) {
    HIP_TRY(pbh::launch_xo_seed(e->xo, e->n, e->off, e->seed, e->stream));
    e->xo_seeded = true;
  }
  const int64_t spl = steps_per_launch > 0 ? steps_per_launch : n_steps;
  KArgs k;
  size_t lds = 0;
  run_args(e, k, lds);
  const bool gfast = e->has_gibbs && pbh::gibbs_fast_form(k);
  // the resident server: one command for the whole run when the run is one
  // steady-state lane-pair launch (launch_mh_server's check); anything else
  // stops a running server and launches normally
  if (e->srv_enabled && !e->has_gibbs && spl >= n_steps && n_steps <= (1 << 30)) {
    pbh::KArgs kc = k;
    kc.g0 = e->g;
    kc.n_steps = (int32_t)n_steps;
    kc.has_pred = e->has_pred ? 1 : 0;
    const bool short_run = n_steps <= 64;
    kc.fair = short_run ? e->fair_short : e->fair;
    kc.fair_rel = short_run ? 1 : e->fair_rel;
    kc.srv_cmd = kc.srv_done = kc.srv_mail = reinterpret_cast<void *>(1);   // the check only
    int32_t wgs = 0;
    // a running server's form (model, proposal, RNG, trace) was checked at
    // its launch -- every entry point that changes them stops it -- so only
    // this run's own shape is checked (no occupancy query per command)
    const bool form = e->g + n_steps < (int64_t(1) << 47) &&   // srv_arg's 48-bit step
        (e->srv_active
             ? (!k.moments && e->has_pred && e->cap > 0 && e->thin == 1 &&
                e->g - e->rec_base >= 0 && e->g + n_steps - e->rec_base <= e->cap)
             : pbh::launch_mh_server(kc, e->stream, &wgs, true) == hipSuccess);
    if (form) {
      if (e->srv_active) {
        if (e->srv_pending) {   // one command in flight
          const int rc = srv_wait(e, e->srv_pending, false);
          e->srv_pending = 0;
          if (rc) return rc;
        }
        // a server that has ended, or whose idle exit could be near, is
        // replaced: a command never races the kernel's own exit
        const auto idle = srv_clk::now() - e->srv_last;
        // (the stream query only after a pause: back-to-back commands cannot
        // have seen the kernel leave, and srv_wait notices a faulted one)
        if (idle > std::chrono::milliseconds(e->srv_idle_ms / 2) ||
            (idle > std::chrono::milliseconds(1) && srv_kernel_ended(e))) {
          const int rc = srv_stop(e);
          if (rc) return rc;
        }
      }
      if (!e->srv_active) {
        const int rc = srv_launch(e, kc);
        if (rc) return rc;
      }
      srv_submit(e, n_steps, kc.fair, kc.fair_rel);
      tq("server command");
      return PBH_OK;
    }
    (void)hipGetLastError();
  }
  SRV_STOP(e);
  e->srv_timed = false;
  // the timed region: events on the first / last dispatch packet, or (with
  // PBH_EVENT_MARKERS=1) separate marker packets around the launches
  pbh::LaunchEvents &lev = pbh::launch_events();
  tq("args");
  if (e->event_markers) {
    HIP_TRY(hipEventRecord(e->ev0, e->stream));
    tq("event0");
    lev = {};
  } else {
    lev.start = e->ev0;
    lev.stop = nullptr;
  }
  int64_t launches = 0;
  for (int64_t done = 0; done < n_steps;) {
    const int64_t m = std::min(spl, n_steps - done);
    if (!e->event_markers && done + m >= n_steps) lev.stop = e->ev1;
    k.n_steps = (int32_t)m;
    const bool short_launch = m <= 64;
    k.fair = short_launch ? e->fair_short : e->fair;
    k.fair_rel = short_launch ? 1 : e->fair_rel;
    k.g0 = e->g;
    k.has_pred = e->has_pred ? 1 : 0;
    k.rep_row0 = e->g - e->rep_g0;
    k.gq_init = e->gq_valid ? 0 : 1;
    k.lx = e->lx;
    k.lx_init = e->lx_valid ? 0 : 1;
    hipError_t err = e->has_gibbs ? pbh::launch_gibbs(k, e->stream)
                                  : pbh::launch_mh(k, e->stream, lds);
    if (err != hipSuccess) {
      lev = {};
      return fail(PBH_ERR_HIP, "kernel launch failed: %s", hipGetErrorString(err));
    }
    e->g += m;
    e->has_pred = true;
    e->gq_valid = gfast;   // only the production Gibbs kernel maintains g, Q
    // the production MH kernels maintain the carried ufun logs
    e->lx_valid = !e->has_gibbs && k.ufun != 0 &&
                  (e->rng == PBH_RNG_PHILOX || e->rng == PBH_RNG_XOSHIRO);
    done += m;
    ++launches;
  }
  lev = {};
  tq("launches");
  if (e->event_markers) HIP_TRY(hipEventRecord(e->ev1, e->stream));
  tq("event1");
  e->mom_steps += n_steps;
  e->timed = true;
  e->last_launches = launches;
  return PBH_OK;
}

// Generation and the REPLAY chain-step in one kernel per launch (pbh_legacy.hip
// legacy_mh_kernel): the draws never pass through HBM.  Same chains, trace
// and legacy state as pbh_legacy_replay + pbh_run chunk by chunk, which is
// what runs for the forms the fused kernel does not cover (Gibbs, per-
// variable deltas, a permuted draw order, the pre-Mt4 state layouts, a d
// without an instantiation) and with PBH_LEGACY_FUSED=0.  The stream buffer
// is not written: afterwards no replay rows are held (pbh_get_replay).
int pbh_legacy_run(pbh_engine *e, int64_t n_steps, int32_t steps_per_launch) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (e->rng != PBH_RNG_REPLAY)
    return fail(PBH_ERR_STATE, "pbh_legacy_run runs the REPLAY RNG (pbh_set_rng)");
  if (!e->mt_key) return fail(PBH_ERR_STATE, "pbh_legacy_seed first");
  if (e->mt_stale)
    return fail(PBH_ERR_STATE, "pbh_restore ran after pbh_legacy_seed: set the "
                "checkpoint's legacy state (pbh_set_legacy_state) first");
  if (const int rc = run_checks(e, n_steps)) return rc;
  if (n_steps == 0) {
    e->timed = false;
    e->last_launches = 0;
    return PBH_OK;
  }
  const int64_t spl = steps_per_launch > 0 ? steps_per_launch : n_steps;
  int32_t R = 0;
  if (const int rc = pbh_stream_width(e, &R)) return rc;
  HIP_TRY(hipSetDevice(e->device));
  KArgs k;
  size_t lds = 0;
  run_args(e, k, lds);
  if (!e->lgtab) {
    std::vector<double> lt(pbh::kLegLogDoubles);
    pbh::legacy_log_table(lt.data());
    if (const int rc = dalloc(e->lgtab, lt.size())) return rc;
    HIP_TRY(hipMemcpy(e->lgtab, lt.data(), lt.size() * sizeof(double), hipMemcpyHostToDevice));
  }
  pbh::LegacyArgs la{};
  la.key = e->mt_key; la.pos = e->mt_pos; la.gauss = e->mt_gauss;
  la.has_gauss = e->mt_has; la.order = nullptr; la.out = nullptr;
  la.n = e->n; la.d = e->d; la.R = R; la.gibbs = e->has_gibbs ? 1 : 0;
  la.normal = (!e->has_gibbs && e->k.prop == PBH_PROP_GAUSS) ? 1 : 0;
  la.vardelta = (!e->has_gibbs && e->k.prop == PBH_PROP_VARDELTA) ? 1 : 0;
  la.db = e->mt_mode;
  la.win = e->legacy_win ? 1 : 0;
  la.lgtab = e->lgtab;
  bool ident = true;
  for (int j = 0; j < (int)e->draw_order.size(); ++j) ident = ident && e->draw_order[j] == j;
  const bool fused = e->legacy_fused && ident &&
                     pbh::launch_legacy_mh(la, k, e->stream, true) == hipSuccess;
  // the thresholds (pbh_set_record_threshold): MH only (Gibbs draws none)
  const bool keep_thr = e->rec_thr && !e->has_gibbs;
  e->thr_steps = 0;
  if (keep_thr && e->thr_alloc < (size_t)n_steps * e->n) {
    if (const int rc = dalloc(e->thr, (size_t)n_steps * e->n)) {
      e->thr_alloc = 0;
      return rc;
    }
    e->thr_alloc = (size_t)n_steps * e->n;
  }
  if (!fused) {
    for (int64_t done = 0; done < n_steps;) {
      const int64_t m = std::min(spl, n_steps - done);
      int rc = pbh_legacy_replay(e, m);
      if (!rc && keep_thr)   // the stream's threshold row, [m][n]
        HIP_TRY(hipMemcpy2DAsync(e->thr + (size_t)done * e->n, e->n * sizeof(double),
                                 e->rep + (size_t)e->d * e->n, (size_t)R * e->n * sizeof(double),
                                 e->n * sizeof(double), m, hipMemcpyDeviceToDevice, e->stream));
      if (!rc) rc = pbh_run(e, m, 0);
      if (rc) return rc;
      done += m;
    }
    e->thr_steps = keep_thr ? n_steps : 0;
    return PBH_OK;
  }
  e->srv_timed = false;
  pbh::LaunchEvents &lev = pbh::launch_events();
  if (e->event_markers) {
    HIP_TRY(hipEventRecord(e->ev0, e->stream));
    lev = {};
  } else {
    lev.start = e->ev0;
    lev.stop = nullptr;
  }
  // launches of at most 2^20 steps, as pbh_legacy_replay (Mt4's 32-bit head)
  constexpr int64_t kLegacyLaunchSteps = int64_t(1) << 20;
  // twist-ahead (legacy_ahead_kernel, PBH_LEGACY_AHEAD=0 off): each launch's
  // blocks are twisted before it by one wavefront per chain, so the fused
  // kernel only consumes; a launch is at most what 15 blocks ahead hold with
  // an 8-sigma margin on the polar method's attempts (a chain that needs more
  // twists in the fused kernel, as without the pre-pass)
  const bool ahead = e->legacy_ahead && e->mt_mode == 2 && !e->mt_odd;
  const double dd = (double)e->d;
  // doubles per step (mean, variance): normal -- d/2 pairs at 4/pi attempts
  // of two doubles (attempt-count variance 0.348 per pair) + the threshold;
  // raw -- d + 1
  const double dmean = la.normal ? 4.0 * dd / 3.14159265358979 + 1.0 : dd + 1.0;
  const double dvar = la.normal ? 4.0 * 0.3480 * dd / 2.0 : 0.0;
  auto ahead_words = [&](int64_t m) {   // words of m steps, 8 sigma
    return 2.0 * ((double)m * dmean + 8.0 * std::sqrt((double)m * dvar) + 2.0);
  };
  int64_t m_fit = spl;
  if (ahead) {   // 14 whole blocks after the current one's (up to 624) words
    while (m_fit > 1 && ahead_words(m_fit) > 14.0 * pbh_mt_block_words()) m_fit = m_fit * 7 / 8;
  }
  int64_t launches = 0;
  for (int64_t done = 0; done < n_steps;) {
    int64_t m = std::min(std::min(spl, kLegacyLaunchSteps), n_steps - done);
    if (ahead) {
      m = std::min(m, m_fit);
      const int32_t want = std::min<int32_t>(
          15, 1 + (int32_t)std::ceil(ahead_words(m) / pbh_mt_block_words()));
      const hipError_t ea = pbh::launch_legacy_ahead(e->mt_key, e->mt_pos, e->n, want,
                                                     e->stream);
      if (ea != hipSuccess) {
        lev = {};
        return fail(PBH_ERR_HIP, "pbh_legacy_run (twist-ahead): %s", hipGetErrorString(ea));
      }
    }
    if (!e->event_markers && done + m >= n_steps) lev.stop = e->ev1;
    k.n_steps = (int32_t)m;
    k.g0 = e->g;
    k.has_pred = e->has_pred ? 1 : 0;
    k.rep_row0 = 0;
    k.lx = e->lx;
    k.lx_init = 1;
    la.n_steps = m;
    la.step0 = e->g;
    la.thr = keep_thr ? e->thr + (size_t)done * e->n : nullptr;
    const hipError_t err = pbh::launch_legacy_mh(la, k, e->stream, false);
    if (err != hipSuccess) {
      lev = {};
      return fail(PBH_ERR_HIP, "pbh_legacy_run: %s", hipGetErrorString(err));
    }
    e->g += m;
    e->has_pred = true;
    done += m;
    ++launches;
  }
  lev = {};
  if (e->event_markers) HIP_TRY(hipEventRecord(e->ev1, e->stream));
  e->gq_valid = false;
  e->lx_valid = false;
  e->thr_steps = keep_thr ? n_steps : 0;
  // the stream rows are not written: none are held from here on
  e->k.R = R;
  e->rep_steps = 0;
  e->rep_g0 = e->g;
  e->mom_steps += n_steps;
  e->timed = true;
  e->last_launches = launches;
  return PBH_OK;
}

int pbh_run_wait(pbh_engine *e, int64_t n_steps, int32_t steps_per_launch) {
  const int rc = pbh_run(e, n_steps, steps_per_launch);
  if (rc) return rc;
  return pbh_sync(e);
}

int pbh_set_record_threshold(pbh_engine *e, int32_t on) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  e->rec_thr = on != 0;
  return PBH_OK;
}

int pbh_get_thresholds(pbh_engine *e, int64_t first, int64_t n_steps, double *out) {
  if (check_ptr(e, "engine") || check_ptr(out, "out")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (first < 0 || n_steps < 0 || first + n_steps > e->thr_steps)
    return fail(PBH_ERR_ARG, "thresholds [%lld, %lld) not held (%lld kept by the last "
                "pbh_legacy_run; pbh_set_record_threshold first)", (long long)first,
                (long long)(first + n_steps), (long long)e->thr_steps);
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  HIP_TRY(hipMemcpy(out, e->thr + (size_t)first * e->n, (size_t)n_steps * e->n * sizeof(double),
                    hipMemcpyDeviceToHost));
  return PBH_OK;
}

int pbh_legacy_draws(pbh_engine *e, int64_t n_steps, int64_t step0, int32_t kind,
                     double param, double *out) {
  if (check_ptr(e, "engine") || check_ptr(out, "out")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->mt_key) return fail(PBH_ERR_STATE, "pbh_legacy_seed first");
  if (e->mt_stale)
    return fail(PBH_ERR_STATE, "pbh_restore ran after pbh_legacy_seed: set the "
                "checkpoint's legacy state (pbh_set_legacy_state) first");
  if (e->mt_mode != 2) return fail(PBH_ERR_UNSUPPORTED, "pbh_legacy_draws needs the Mt4 state");
  if (kind != PBH_DRAWS_GAUSS && kind != PBH_DRAWS_LINREG)
    return fail(PBH_ERR_ARG, "bad draws kind %d", kind);
  if (n_steps < 0 || step0 < 0) return fail(PBH_ERR_ARG, "n_steps, step0 must be >= 0");
  if (!(param >= 0.0)) return fail(PBH_ERR_ARG, "gamma shape must be >= 0");
  if (n_steps == 0) return PBH_OK;
  const int64_t n = e->n;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  double *dout = nullptr;
  if (const int rc = dalloc(dout, (size_t)n_steps * n)) return rc;
  pbh::LegacyArgs a{};
  a.key = e->mt_key; a.pos = e->mt_pos; a.gauss = e->mt_gauss; a.has_gauss = e->mt_has;
  a.out = dout; a.n = n; a.n_steps = n_steps; a.step0 = step0; a.d = 1; a.R = 1;
  a.db = e->mt_mode;
  hipError_t err = pbh::launch_legacy_draws(a, kind, param, e->stream);
  if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
  if (err == hipSuccess)
    err = hipMemcpy(out, dout, (size_t)n_steps * n * sizeof(double), hipMemcpyDeviceToHost);
  dfree(dout);
  if (err != hipSuccess) return fail(PBH_ERR_HIP, "pbh_legacy_draws: %s", hipGetErrorString(err));
  return PBH_OK;
}

// The engine stream's completion, as pbh_sync waits for it: polled for up to
// 2 ms (PBH_SYNC, spin_sync), then a blocking wait.  A blocking
// hipStreamSynchronize wakes ~10-50 us after a short kernel ends.
static hipError_t stream_wait(pbh_engine *e) {
  if (!e->spin_sync) return hipStreamSynchronize(e->stream);
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t q;
  while ((q = hipStreamQuery(e->stream)) == hipErrorNotReady) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(2000))
      return hipStreamSynchronize(e->stream);
  }
  return q;
}

int pbh_sync(pbh_engine *e) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  if (e->srv_active) {   // never the stream: the server kernel is on it
    if (e->srv_pending) {
      const int rc = srv_wait(e, e->srv_pending, false);
      e->srv_pending = 0;
      return rc;
    }
    return PBH_OK;
  }
  HIP_TRY(hipSetDevice(e->device));
  if (e->spin_sync) {
    // poll the stream for up to 2 ms: a short launch's completion is seen
    // within a microsecond or so (a blocking wait sleeps on the completion
    // signal and wakes ~10 us late); longer waits block, so that a long run
    // does not hold a host core at 100 %
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t q;
    // PBH_SYNC=event: the end event of the last run first (the stream's
    // last packet when nothing was enqueued after it), then the stream
    if (e->sync_event && e->timed) {
      while ((q = hipEventQuery(e->ev1)) == hipErrorNotReady) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(2000)) break;
      }
    }
    while ((q = hipStreamQuery(e->stream)) == hipErrorNotReady) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(2000)) {
        q = hipStreamSynchronize(e->stream);
        break;
      }
    }
    HIP_TRY(q);
  } else {
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  return PBH_OK;
}

int pbh_set_collect(pbh_engine *e, int32_t flags) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  if (flags & ~PBH_COLLECT_MOMENTS) return fail(PBH_ERR_ARG, "bad collect flags %d", flags);
  e->collect = flags;
  return PBH_OK;
}

int pbh_last_run_ms(pbh_engine *e, double *ms, int64_t *launches) {
  if (check_ptr(e, "engine") || check_ptr(ms, "ms")) return PBH_ERR_ARG;
  if (!e->timed) {
    *ms = 0.;
    if (launches) *launches = 0;
    return PBH_OK;
  }
  if (e->srv_timed) {
    // the last run was a server command: the first workgroup's sight of it
    // to the last workgroup's completion, on the 100 MHz real-time clock
    if (e->srv_active && e->srv_pending) {
      const int rc = pbh_sync(e);
      if (rc) return rc;
    }
    uint64_t t0 = ~0ull, t1 = 0;
    for (int32_t w = 0; w < e->srv_wgs; ++w) {
      t0 = std::min<uint64_t>(t0, __atomic_load_n(&e->srv_done[w].t0, __ATOMIC_ACQUIRE));
      t1 = std::max<uint64_t>(t1, __atomic_load_n(&e->srv_done[w].t1, __ATOMIC_ACQUIRE));
    }
    *ms = t1 > t0 ? (double)(t1 - t0) * 1e-5 : 0.;
    if (launches) *launches = e->last_launches;
    return PBH_OK;
  }
  HIP_TRY(hipEventSynchronize(e->ev1));
  float f = 0.f;
  HIP_TRY(hipEventElapsedTime(&f, e->ev0, e->ev1));
  *ms = f;
  if (launches) *launches = e->last_launches;
  return PBH_OK;
}

int pbh_server_stop(pbh_engine *e) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  return PBH_OK;
}

int pbh_server_info(pbh_engine *e, int32_t *active, int64_t *commands, int64_t *launches) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  if (active) *active = e->srv_active && !srv_kernel_ended(e) ? 1 : 0;
  if (commands) *commands = e->srv_commands;
  if (launches) *launches = e->srv_launches;
  return PBH_OK;
}

int pbh_server_stamps(pbh_engine *e, int32_t cap, uint32_t *seq, uint64_t *t0,
                      uint64_t *t1, int32_t *n) {
  if (check_ptr(e, "engine") || check_ptr(n, "n")) return PBH_ERR_ARG;
  *n = e->srv_done ? e->srv_wgs : 0;
  for (int32_t w = 0; w < *n && w < cap; ++w) {
    if (seq) seq[w] = __atomic_load_n(&e->srv_done[w].seq, __ATOMIC_ACQUIRE);
    if (t0) t0[w] = __atomic_load_n(&e->srv_done[w].t0, __ATOMIC_ACQUIRE);
    if (t1) t1[w] = __atomic_load_n(&e->srv_done[w].t1, __ATOMIC_ACQUIRE);
  }
  return PBH_OK;
}

// ---------------------------------------------------------------------------
// results
// ---------------------------------------------------------------------------
int pbh_get_state(pbh_engine *e, double *x, double *logp) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->x) return fail(PBH_ERR_STATE, "pbh_init_chains first");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  const int64_t n = e->n;
  const int d = e->d;
  if (x) {
    std::vector<double> xt((size_t)n * d);
    HIP_TRY(hipMemcpy(xt.data(), e->x, xt.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (int64_t c = 0; c < n; ++c)
      for (int k = 0; k < d; ++k) x[(size_t)c * d + k] = xt[(size_t)k * n + c];
  }
  if (logp) HIP_TRY(hipMemcpy(logp, e->lp, n * sizeof(double), hipMemcpyDeviceToHost));
  return PBH_OK;
}

int pbh_get_checkpoint(pbh_engine *e, double *x, double *lp, int64_t *step,
                       int32_t *has_pred, uint32_t *xo) {
  int rc = pbh_get_state(e, x, lp);
  if (rc) return rc;
  if (step) *step = e->g;
  if (has_pred) *has_pred = e->has_pred ? 1 : 0;
  if (xo) {
    if (e->rng != PBH_RNG_XOSHIRO)
      return fail(PBH_ERR_STATE, "no xoshiro state (rng is not XOSHIRO)");
    HIP_TRY(hipSetDevice(e->device));
    if (!e->xo_seeded) {   // before the first run: the state pbh_run would seed
      HIP_TRY(pbh::launch_xo_seed(e->xo, e->n, e->off, e->seed, e->stream));
      e->xo_seeded = true;
    }
    HIP_TRY(hipStreamSynchronize(e->stream));
    HIP_TRY(hipMemcpy(xo, e->xo, (size_t)8 * e->n * sizeof(uint32_t),
                      hipMemcpyDeviceToHost));
  }
  return PBH_OK;
}

int pbh_restore(pbh_engine *e, const double *x, const double *lp, int64_t step,
                int32_t has_pred, const uint32_t *xo) {
  if (check_ptr(e, "engine") || check_ptr(x, "x") || check_ptr(lp, "lp"))
    return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->x) return fail(PBH_ERR_STATE, "pbh_init_chains first");
  if (step < 0) return fail(PBH_ERR_ARG, "step index must be >= 0");
  if (e->rng == PBH_RNG_XOSHIRO && !xo)
    return fail(PBH_ERR_ARG, "XOSHIRO needs the generator state xo");
  const int64_t n = e->n;
  const int d = e->d;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  std::vector<double> xt((size_t)n * d);
  for (int64_t c = 0; c < n; ++c)
    for (int k = 0; k < d; ++k) xt[(size_t)k * n + c] = x[(size_t)c * d + k];
  HIP_TRY(hipMemcpy(e->x, xt.data(), xt.size() * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->lp, lp, n * sizeof(double), hipMemcpyHostToDevice));
  if (xo) {
    if (e->rng != PBH_RNG_XOSHIRO)
      return fail(PBH_ERR_ARG, "xo given but the rng is not XOSHIRO");
    HIP_TRY(hipMemcpy(e->xo, xo, (size_t)8 * n * sizeof(uint32_t), hipMemcpyHostToDevice));
    e->xo_seeded = true;
  }
  e->g = step;
  e->has_pred = has_pred != 0;
  e->gq_valid = false;   // the production Gibbs kernel recomputes g, Q from x
  e->state_lost = false;
  e->lx_valid = false;   // ... and the ufun logs (pbh_set_chain_logs restores them)
  e->cap = 0;            // a trace / replay rows of the engine are detached
  e->rep_steps = 0;
  e->rep_g0 = step;
  // device legacy streams: their state is not in x / lp / step; until the
  // checkpoint's is set (pbh_set_legacy_state) the streams refuse to draw
  e->mt_stale = e->mt_key != nullptr;
  return PBH_OK;
}

int pbh_set_chains(pbh_engine *e, const double *x, const double *lp,
                   int64_t step, int32_t has_pred) {
  if (check_ptr(e, "engine") || check_ptr(x, "x") || check_ptr(lp, "lp"))
    return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->x) return fail(PBH_ERR_STATE, "pbh_init_chains first");
  if (step < 0) return fail(PBH_ERR_ARG, "step index must be >= 0");
  const int64_t n = e->n;
  const int d = e->d;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  std::vector<double> xt((size_t)n * d);
  for (int64_t c = 0; c < n; ++c)
    for (int k = 0; k < d; ++k) xt[(size_t)k * n + c] = x[(size_t)c * d + k];
  HIP_TRY(hipMemcpy(e->x, xt.data(), xt.size() * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->lp, lp, n * sizeof(double), hipMemcpyHostToDevice));
  e->g = step;
  e->has_pred = has_pred != 0;
  e->gq_valid = false;
  e->lx_valid = false;
  e->cap = 0;            // the trace and the replay rows are detached
  e->state_lost = false;
  e->rep_steps = 0;
  e->rep_g0 = step;
  return PBH_OK;
}

int pbh_get_chain_logs(pbh_engine *e, double *lx, int32_t *valid) {
  if (check_ptr(e, "engine") || check_ptr(valid, "valid")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->x) return fail(PBH_ERR_STATE, "pbh_init_chains first");
  *valid = e->lx_valid ? 1 : 0;
  if (!e->lx_valid || !lx) return PBH_OK;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  const int64_t n = e->n, d = e->d;
  std::vector<double> t((size_t)n * d);
  HIP_TRY(hipMemcpy(t.data(), e->lx, t.size() * sizeof(double), hipMemcpyDeviceToHost));
  for (int64_t c = 0; c < n; ++c)
    for (int64_t k = 0; k < d; ++k) lx[(size_t)c * d + k] = t[(size_t)k * n + c];
  return PBH_OK;
}

int pbh_set_chain_logs(pbh_engine *e, const double *lx) {
  if (check_ptr(e, "engine") || check_ptr(lx, "lx")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->x) return fail(PBH_ERR_STATE, "pbh_init_chains first");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  const int64_t n = e->n, d = e->d;
  std::vector<double> t((size_t)n * d);
  for (int64_t c = 0; c < n; ++c)
    for (int64_t k = 0; k < d; ++k) t[(size_t)k * n + c] = lx[(size_t)c * d + k];
  HIP_TRY(hipMemcpy(e->lx, t.data(), t.size() * sizeof(double), hipMemcpyHostToDevice));
  e->lx_valid = true;
  return PBH_OK;
}

int pbh_legacy_state_words(pbh_engine *e, int64_t *words) {
  if (check_ptr(e, "engine") || check_ptr(words, "words")) return PBH_ERR_ARG;
  *words = e->mt_key ? mt_state_words(e->mt_mode) : 0;
  return PBH_OK;
}

int pbh_get_legacy_state(pbh_engine *e, uint32_t *key, int32_t *pos,
                         int32_t *has, double *gauss) {
  if (check_ptr(e, "engine") || check_ptr(key, "key") || check_ptr(pos, "pos") ||
      check_ptr(has, "has") || check_ptr(gauss, "gauss"))
    return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->mt_key) return fail(PBH_ERR_STATE, "no legacy streams (pbh_legacy_seed)");
  if (e->mt_stale) return fail(PBH_ERR_STATE, "legacy state stale after pbh_restore");
  const int64_t n = e->n;
  const size_t kw = (size_t)mt_state_words(e->mt_mode) * n;
  HIP_TRY(hipSetDevice(e->device));
  if (e->mt_mode == 2)   // the current blocks into buffer 0: the key's prefix
    HIP_TRY(pbh::launch_legacy_normalize(e->mt_key, e->mt_pos, n, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  HIP_TRY(hipMemcpy(key, e->mt_key, kw * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(pos, e->mt_pos, n * sizeof(int32_t), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(has, e->mt_has, n * sizeof(int32_t), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(gauss, e->mt_gauss, n * sizeof(double), hipMemcpyDeviceToHost));
  return PBH_OK;
}

int pbh_set_legacy_state(pbh_engine *e, const uint32_t *key, const int32_t *pos,
                         const int32_t *has, const double *gauss) {
  if (check_ptr(e, "engine") || check_ptr(key, "key") || check_ptr(pos, "pos") ||
      check_ptr(has, "has") || check_ptr(gauss, "gauss"))
    return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->mt_key) return fail(PBH_ERR_STATE, "pbh_legacy_seed first (the layout)");
  const int64_t n = e->n;
  const size_t kw = (size_t)mt_state_words(e->mt_mode) * n;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  HIP_TRY(hipMemcpy(e->mt_key, key, kw * sizeof(uint32_t), hipMemcpyHostToDevice));
  if (e->mt_mode == 2) {   // the checkpoint form: the block in buffer 0
    std::vector<int32_t> p0(pos, pos + n);
    for (auto &v : p0) v &= 0xFFFF;
    HIP_TRY(hipMemcpy(e->mt_pos, p0.data(), n * sizeof(int32_t), hipMemcpyHostToDevice));
  } else {
    HIP_TRY(hipMemcpy(e->mt_pos, pos, n * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  HIP_TRY(hipMemcpy(e->mt_has, has, n * sizeof(int32_t), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->mt_gauss, gauss, n * sizeof(double), hipMemcpyHostToDevice));
  e->mt_stale = false;
  e->mt_odd = false;
  for (int64_t c = 0; c < n && !e->mt_odd; ++c) e->mt_odd = (pos[c] & 1) != 0;
  return PBH_OK;
}

int pbh_trace_len(pbh_engine *e, int64_t *n_recorded) {
  if (check_ptr(e, "engine") || check_ptr(n_recorded, "n_recorded")) return PBH_ERR_ARG;
  const int64_t r = e->cap > 0 ? e->g / e->thin - e->rec_base : 0;
  *n_recorded = std::max<int64_t>(0, std::min(r, e->cap));
  return PBH_OK;
}

int pbh_get_trace(pbh_engine *e, int64_t first, int64_t cnt, double *x,
                  double *logp, uint64_t *acc, double *p_x, double *p_p,
                  double *s) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  int64_t rec = 0;
  pbh_trace_len(e, &rec);
  if (first < 0 || cnt < 0 || first + cnt > rec)
    return fail(PBH_ERR_ARG, "trace range [%lld, %lld) outside [0, %lld)",
                (long long)first, (long long)(first + cnt), (long long)rec);
  if ((p_x || p_p || s) && !e->debug)
    return fail(PBH_ERR_STATE, "debug trace not allocated");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  const size_t n = e->n, d = e->d, W = (e->n + 63) / 64;
  if (cnt == 0) return PBH_OK;
  if (x) HIP_TRY(hipMemcpy(x, e->tx + first * d * n, cnt * d * n * sizeof(double), hipMemcpyDeviceToHost));
  if (logp) HIP_TRY(hipMemcpy(logp, e->tlp + first * n, cnt * n * sizeof(double), hipMemcpyDeviceToHost));
  if (acc) HIP_TRY(hipMemcpy(acc, e->tacc + first * W, cnt * W * sizeof(uint64_t), hipMemcpyDeviceToHost));
  if (p_x) HIP_TRY(hipMemcpy(p_x, e->tpx + first * d * n, cnt * d * n * sizeof(double), hipMemcpyDeviceToHost));
  if (p_p) HIP_TRY(hipMemcpy(p_p, e->tpp + first * n, cnt * n * sizeof(double), hipMemcpyDeviceToHost));
  if (s) HIP_TRY(hipMemcpy(s, e->ts + first * n, cnt * n * sizeof(double), hipMemcpyDeviceToHost));
  return PBH_OK;
}

int pbh_get_moments(pbh_engine *e, double *sum, double *sumsq, int64_t *n_acc,
                    int64_t *n_steps) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->x) return fail(PBH_ERR_STATE, "pbh_init_chains first");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  const size_t dn = (size_t)e->d * e->n;
  if (sum) HIP_TRY(hipMemcpy(sum, e->msum, dn * sizeof(double), hipMemcpyDeviceToHost));
  if (sumsq) HIP_TRY(hipMemcpy(sumsq, e->msq, dn * sizeof(double), hipMemcpyDeviceToHost));
  if (n_acc) HIP_TRY(hipMemcpy(n_acc, e->nacc, e->n * sizeof(int64_t), hipMemcpyDeviceToHost));
  if (n_steps) *n_steps = e->mom_steps;
  return PBH_OK;
}

int pbh_trace_stats(pbh_engine *e, int64_t first, int64_t count, double *sum,
                    double *sumsq, int64_t *n_acc) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  int64_t rec = 0;
  pbh_trace_len(e, &rec);
  if (first < 0 || count < 0 || first + count > rec)
    return fail(PBH_ERR_ARG, "trace range [%lld, %lld) outside [0, %lld)",
                (long long)first, (long long)(first + count), (long long)rec);
  HIP_TRY(hipSetDevice(e->device));
  const int64_t n = e->n, W = (n + 63) / 64;
  HIP_TRY(pbh::launch_trace_stats(e->tx, e->tacc, n, e->d, W, first, count,
                                  e->msum, e->msq, e->nacc, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->mom_steps = count;
  const size_t dn = (size_t)e->d * n;
  if (sum) HIP_TRY(hipMemcpy(sum, e->msum, dn * sizeof(double), hipMemcpyDeviceToHost));
  if (sumsq) HIP_TRY(hipMemcpy(sumsq, e->msq, dn * sizeof(double), hipMemcpyDeviceToHost));
  if (n_acc) HIP_TRY(hipMemcpy(n_acc, e->nacc, n * sizeof(int64_t), hipMemcpyDeviceToHost));
  return PBH_OK;
}

int pbh_trace_expectation(pbh_engine *e, int64_t first, int64_t count,
                          double exponent, double *out) {
  if (check_ptr(e, "engine") || check_ptr(out, "out")) return PBH_ERR_ARG;
  SRV_STOP(e);
  int64_t rec = 0;
  pbh_trace_len(e, &rec);
  if (first < 0 || count < 1 || first + count > rec)
    return fail(PBH_ERR_ARG, "trace range [%lld, %lld) outside [0, %lld)",
                (long long)first, (long long)(first + count), (long long)rec);
  if (!std::isfinite(exponent)) return fail(PBH_ERR_ARG, "exponent must be finite");
  HIP_TRY(hipSetDevice(e->device));
  const size_t dn = (size_t)e->d * e->n;
  double *dout = nullptr;
  HIP_TRY(hipMalloc(&dout, dn * sizeof(double)));
  hipError_t err = pbh::launch_trace_expectation(
      e->tx, e->tlp, e->n, e->d, first, count, exponent,
      e->k.pscale == PBH_PSCALE_LIN ? 1 : 0, e->k.log_npi, dout, e->stream);
  if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
  if (err == hipSuccess)
    err = hipMemcpy(out, dout, dn * sizeof(double), hipMemcpyDeviceToHost);
  (void)hipFree(dout);
  if (err != hipSuccess)
    return fail(PBH_ERR_HIP, "pbh_trace_expectation: %s", hipGetErrorString(err));
  return PBH_OK;
}

int pbh_trace_ess(pbh_engine *e, int64_t first, int64_t count, double *ess) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  int64_t rec = 0;
  pbh_trace_len(e, &rec);
  if (first < 0 || count < 2 || first + count > rec)
    return fail(PBH_ERR_ARG, "ESS needs >= 2 records inside [0, %lld), got [%lld, %lld)",
                (long long)rec, (long long)first, (long long)(first + count));
  HIP_TRY(hipSetDevice(e->device));
  const int64_t dn = (int64_t)e->d * e->n;
  if (e->ess_fft >= 2 && e->ess_list_len < (dn + 1) / 2 + 1) {
    dfree(e->ess_list);
    e->ess_list_len = 0;
    HIP_TRY(hipMalloc(&e->ess_list, ((dn + 1) / 2 + 1) * sizeof(int32_t)));
    e->ess_list_len = (dn + 1) / 2 + 1;
  }
  HIP_TRY(pbh::launch_trace_ess(e->tx, e->n, e->d, first, count, e->ess, e->stream,
                                e->ess_fft, e->ess_list));
  if (ess) {
    // through a pinned staging buffer: a pageable copy of the 512 KB cfg5
    // result was ~0.1 ms of the call
    if (e->ess_host_len < dn) {
      if (e->ess_host) (void)hipHostFree(e->ess_host);
      e->ess_host = nullptr;
      e->ess_host_len = 0;
      HIP_TRY(hipHostMalloc(&e->ess_host, dn * sizeof(double), hipHostMallocDefault));
      e->ess_host_len = dn;
    }
    HIP_TRY(hipMemcpyAsync(e->ess_host, e->ess, dn * sizeof(double), hipMemcpyDeviceToHost,
                           e->stream));
    HIP_TRY(stream_wait(e));
    std::memcpy(ess, e->ess_host, dn * sizeof(double));
  }
  return PBH_OK;
}

int pbh_trace_ess_total(pbh_engine *e, int64_t first, int64_t count, double *total) {
  if (check_ptr(e, "engine") || check_ptr(total, "total")) return PBH_ERR_ARG;
  // the per-chain ESS on the device (no copy), then the per-dim sums
  if (const int rc = pbh_trace_ess(e, first, count, nullptr)) return rc;
  const int d = e->d;
  if (!e->ess_host || e->ess_host_len < d) {
    if (e->ess_host) (void)hipHostFree(e->ess_host);
    e->ess_host = nullptr;
    e->ess_host_len = 0;
    HIP_TRY(hipHostMalloc(&e->ess_host, d * sizeof(double), hipHostMallocDefault));
    e->ess_host_len = d;
  }
  // the totals land in the scalar scratch (d doubles, allocated lazily)
  if (!e->ess_tot) {
    if (const int rc = dalloc(e->ess_tot, PBH_MAX_DIM)) return rc;
  }
  HIP_TRY(pbh::launch_ess_total(e->ess, e->n, d, e->ess_tot, e->stream));
  HIP_TRY(hipMemcpyAsync(e->ess_host, e->ess_tot, d * sizeof(double), hipMemcpyDeviceToHost,
                         e->stream));
  HIP_TRY(stream_wait(e));
  std::memcpy(total, e->ess_host, d * sizeof(double));
  return PBH_OK;
}

int pbh_reset_moments(pbh_engine *e) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->x) return fail(PBH_ERR_STATE, "pbh_init_chains first");
  HIP_TRY(hipSetDevice(e->device));
  const size_t dn = (size_t)e->d * e->n;
  HIP_TRY(hipMemsetAsync(e->msum, 0, dn * sizeof(double), e->stream));
  HIP_TRY(hipMemsetAsync(e->msq, 0, dn * sizeof(double), e->stream));
  HIP_TRY(hipMemsetAsync(e->nacc, 0, e->n * sizeof(int64_t), e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->mom_steps = 0;
  return PBH_OK;
}

// ---------------------------------------------------------------------------
// RCCL
// ---------------------------------------------------------------------------
int pbh_rccl_unique_id(uint8_t id[128]) {
  if (check_ptr(id, "id")) return PBH_ERR_ARG;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId uid;
  RCCL_TRY(ncclGetUniqueId(&uid));
  std::memcpy(id, &uid, 128);
  return PBH_OK;
}

int pbh_rccl_init(pbh_engine *e, int32_t rank, int32_t world, const uint8_t id[128]) {
  if (check_ptr(e, "engine") || check_ptr(id, "id")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (world < 1 || rank < 0 || rank >= world) return fail(PBH_ERR_ARG, "bad rank/world");
  HIP_TRY(hipSetDevice(e->device));
  if (e->comm) {
    ncclCommDestroy(e->comm);
    e->comm = nullptr;
  }
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  if (!e->scalar) {
    int rc = dalloc(e->scalar, 4);   // the agreement / max-reduce scratch
    if (rc) return rc;
  }
  RCCL_TRY(ncclCommInitRank(&e->comm, world, uid, rank));
  e->rank = rank;
  e->world = world;
  return PBH_OK;
}

namespace {

// Every rank enters every collective of a gather, whatever failed locally: a
// rank that cannot proceed votes a positive status in an all-reduce of
// (status, count, -count) under ncclMax -- 0 = ok, rank + 1 = this rank
// failed -- and every rank then returns the same error: no rank is left
// waiting inside RCCL (a collective only some ranks enter never completes).
// The vote is a finite number on purpose: a float max may drop a NaN operand
// depending on the operand order (fmax, compare-select), so a NaN vote could
// vanish at world >= 2; a positive status survives any max.  When the vote
// cannot be copied to the device, the fallback fills the whole vote with
// 0x3F bytes (4.8e-4 per double: still positive, so still "failed").  Local
// HIP failures between two agreements are not returned on the spot: they
// become the rank's vote at the next agreement, which every rank enters.
constexpr unsigned char kFailFill = 0x3F;   // 0x3F3F...3F = 4.8e-4 > 0

int vote_failure(const char *what, double status) {
  if (status >= 1.)
    return fail(PBH_ERR_STATE, "%s: rank %d could not take part (the highest failing "
                "rank; see its own error)", what, (int)status - 1);
  return fail(PBH_ERR_STATE, "%s: a rank could not take part (see its own error)", what);
}

int rccl_agree(pbh_engine *e, bool ok, int64_t n, int64_t *n_max, const char *what) {
  double v[3] = {ok ? 0. : (double)(e->rank + 1), (double)n, -(double)n};
  hipError_t h = hipMemcpy(e->scalar, v, sizeof v, hipMemcpyHostToDevice);
  if (h != hipSuccess) (void)hipMemset(e->scalar, kFailFill, sizeof v);
  // the collective is entered whatever happened above
  const ncclResult_t r = ncclAllReduce(e->scalar, e->scalar, 3, ncclFloat64, ncclMax,
                                       e->comm, e->stream);
  hipError_t s = hipStreamSynchronize(e->stream);
  if (s == hipSuccess) s = hipMemcpy(v, e->scalar, sizeof v, hipMemcpyDeviceToHost);
  if (r != ncclSuccess)
    return fail(PBH_ERR_RCCL, "%s: %s", what, ncclGetErrorString(r));
  if (h != hipSuccess || s != hipSuccess)
    return fail(PBH_ERR_HIP, "%s: %s", what, hipGetErrorString(h != hipSuccess ? h : s));
  if (!(v[0] == 0.)) return vote_failure(what, v[0]);
  if (n_max) *n_max = (int64_t)v[1];
  return PBH_OK;
}

// Fault injection for the tests (PBH_FAULT_GATHER="rank[:step]", step 1 =
// no chains, 2 = the buffers, 3 = packing; default 3): this rank fails that
// step of pbh_rccl_allgather_stats locally.
bool fault_at(const pbh_engine *e, int step) {
  const char *f = std::getenv("PBH_FAULT_GATHER");
  if (!f || !*f) return false;
  int rank = -1, st = 3;
  if (std::sscanf(f, "%d:%d", &rank, &st) < 1) return false;
  return rank == e->rank && st == step;
}

hipError_t keep(hipError_t acc, hipError_t e) { return acc != hipSuccess ? acc : e; }

}  // namespace

int pbh_rccl_max_chains(pbh_engine *e, int64_t *n_max) {
  if (check_ptr(e, "engine") || check_ptr(n_max, "n_max")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->comm) return fail(PBH_ERR_STATE, "pbh_rccl_init first");
  const bool ok = hipSetDevice(e->device) == hipSuccess;
  return rccl_agree(e, ok && e->x != nullptr, e->n, n_max, "pbh_rccl_max_chains");
}

int pbh_rccl_allgather_stats(pbh_engine *e, double *out, int64_t *counts) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->comm) return fail(PBH_ERR_STATE, "pbh_rccl_init first");
  // a bad argument is this rank's failure: it still takes part
  bool ok = out != nullptr && counts != nullptr;
  ok = hipSetDevice(e->device) == hipSuccess && ok;
  // 1. agree on the padded width; a rank without chains stops everyone
  int64_t nm = 0;
  int rc = rccl_agree(e, ok && e->x != nullptr && !fault_at(e, 1), e->n, &nm,
                      "pbh_rccl_allgather_stats");
  if (rc) return rc;
  const int64_t n = e->n, d = e->d, rows = 3 * d + 2;   // + the count row
  // 2. buffers
  ok = !dalloc(e->gather_send, (size_t)rows * nm) &&
       !dalloc(e->gather_recv, (size_t)rows * nm * e->world) && !fault_at(e, 2);
  rc = rccl_agree(e, ok, n, nullptr, "pbh_rccl_allgather_stats (buffers)");
  if (rc) return rc;
  // 3. pack [rows][nm]: sum, sumsq, n_acc, ess, then the rank's count; a
  // failure here is this rank's vote at the third agreement
  hipError_t err = hipMemsetAsync(e->gather_send, 0, (size_t)rows * nm * sizeof(double),
                                  e->stream);
  const size_t pitch = (size_t)nm * sizeof(double);
  err = keep(err, hipMemcpy2DAsync(e->gather_send, pitch, e->msum, n * sizeof(double),
                                   n * sizeof(double), d, hipMemcpyDeviceToDevice, e->stream));
  err = keep(err, hipMemcpy2DAsync(e->gather_send + d * nm, pitch, e->msq, n * sizeof(double),
                                   n * sizeof(double), d, hipMemcpyDeviceToDevice, e->stream));
  if (err == hipSuccess) {
    hipLaunchKernelGGL(nacc_to_f64, dim3((unsigned)((n + 255) / 256)), dim3(256),
                       0, e->stream, e->nacc, e->gather_send + 2 * d * nm, n);
    err = hipGetLastError();
  }
  err = keep(err, hipMemcpy2DAsync(e->gather_send + (2 * d + 1) * nm, pitch, e->ess,
                                   n * sizeof(double), n * sizeof(double), d,
                                   hipMemcpyDeviceToDevice, e->stream));
  const double cnt = (double)n;
  err = keep(err, hipMemcpyAsync(e->gather_send + (3 * d + 1) * nm, &cnt, sizeof cnt,
                                 hipMemcpyHostToDevice, e->stream));
  err = keep(err, hipStreamSynchronize(e->stream));
  rc = rccl_agree(e, err == hipSuccess && !fault_at(e, 3), n, nullptr,
                  "pbh_rccl_allgather_stats (packing)");
  if (rc) {
    if (err != hipSuccess)
      return fail(PBH_ERR_HIP, "pbh_rccl_allgather_stats: %s", hipGetErrorString(err));
    return rc;
  }
  // 4. the one all-gather over xGMI (every rank is here)
  RCCL_TRY(ncclAllGather(e->gather_send, e->gather_recv, (size_t)rows * nm,
                         ncclFloat64, e->comm, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  std::vector<double> all((size_t)rows * nm * e->world);
  HIP_TRY(hipMemcpy(all.data(), e->gather_recv, all.size() * sizeof(double),
                    hipMemcpyDeviceToHost));
  for (int r = 0; r < e->world; ++r) {
    const double *src = all.data() + (size_t)r * rows * nm;
    std::memcpy(out + (size_t)r * (rows - 1) * nm, src, (size_t)(rows - 1) * nm * sizeof(double));
    counts[r] = (int64_t)src[(size_t)(rows - 1) * nm];
  }
  return PBH_OK;
}

int pbh_rccl_allreduce_max(pbh_engine *e, double *value) {
  if (check_ptr(e, "engine") || check_ptr(value, "value")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (!e->comm) return fail(PBH_ERR_STATE, "pbh_rccl_init first");
  // (value, status): the status is rccl_agree's finite vote
  double v[2] = {*value, 0.};
  hipError_t h = hipSetDevice(e->device);
  if (h != hipSuccess) v[1] = (double)(e->rank + 1);
  h = keep(h, hipMemcpy(e->scalar, v, sizeof v, hipMemcpyHostToDevice));
  if (h != hipSuccess) (void)hipMemset(e->scalar, kFailFill, sizeof v);
  // entered whatever happened above (a positive status tells every rank)
  const ncclResult_t r = ncclAllReduce(e->scalar, e->scalar, 2, ncclFloat64, ncclMax,
                                       e->comm, e->stream);
  hipError_t s = hipStreamSynchronize(e->stream);
  if (s == hipSuccess) s = hipMemcpy(v, e->scalar, sizeof v, hipMemcpyDeviceToHost);
  if (r != ncclSuccess) return fail(PBH_ERR_RCCL, "pbh_rccl_allreduce_max: %s",
                                    ncclGetErrorString(r));
  if (h != hipSuccess || s != hipSuccess)
    return fail(PBH_ERR_HIP, "pbh_rccl_allreduce_max: %s",
                hipGetErrorString(h != hipSuccess ? h : s));
  if (!(v[1] == 0.)) return vote_failure("pbh_rccl_allreduce_max", v[1]);
  *value = v[0];
  return PBH_OK;
}

int pbh_rccl_destroy(pbh_engine *e) {
  if (check_ptr(e, "engine")) return PBH_ERR_ARG;
  SRV_STOP(e);
  if (e->comm) {
    HIP_TRY(hipSetDevice(e->device));
    RCCL_TRY(ncclCommDestroy(e->comm));
    e->comm = nullptr;
  }
  return PBH_OK;
}

int pbh_check_accept(int device, int64_t n, const double *lp,
                     const double *lpp, const uint32_t *t0, const uint32_t *t1,
                     int32_t lin, uint8_t *out) {
  if (check_ptr(lp, "lp") || check_ptr(lpp, "lpp") || check_ptr(t0, "t0") ||
      check_ptr(t1, "t1") || check_ptr(out, "out"))
    return PBH_ERR_ARG;
  if (n <= 0) return fail(PBH_ERR_ARG, "n must be positive");
  HIP_TRY(hipSetDevice(device));
  double *dlp = nullptr, *dlpp = nullptr;
  uint32_t *d0 = nullptr, *d1 = nullptr;
  uint8_t *dout = nullptr;
  int rc = dalloc(dlp, n);
  if (!rc) rc = dalloc(dlpp, n);
  if (!rc) rc = dalloc(d0, n);
  if (!rc) rc = dalloc(d1, n);
  if (!rc) rc = dalloc(dout, n);
  hipError_t err = hipSuccess;
  if (!rc) {
    err = hipMemcpy(dlp, lp, n * sizeof(double), hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipMemcpy(dlpp, lpp, n * sizeof(double), hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipMemcpy(d0, t0, n * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipMemcpy(d1, t1, n * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (err == hipSuccess)
      err = pbh::launch_check_accept(n, dlp, dlpp, d0, d1, lin,
                                     std::log(1.7976931348623158e+308), dout);
    if (err == hipSuccess) err = hipMemcpy(out, dout, n, hipMemcpyDeviceToHost);
  }
  dfree(dlp); dfree(dlpp); dfree(d0); dfree(d1); dfree(dout);
  if (rc) return rc;
  if (err != hipSuccess)
    return fail(PBH_ERR_HIP, "pbh_check_accept: %s", hipGetErrorString(err));
  return PBH_OK;
}

int pbh_bool_perm_freq(int device, int64_t rows, int32_t cols,
                       const uint8_t *bool2d, int64_t *counts, int32_t reps,
                       double *kernel_ms) {
  if (check_ptr(counts, "counts")) return PBH_ERR_ARG;
  if (cols < 1 || cols > pbh::bool_perm_max_cols())
    return fail(PBH_ERR_ARG, "cols must be in 1..%d, got %d",
                pbh::bool_perm_max_cols(), cols);
  if (rows < 0) return fail(PBH_ERR_ARG, "rows must be >= 0");
  if (rows > 0 && !bool2d) return fail(PBH_ERR_ARG, "bool2d must not be NULL");
  if (reps < 1) return fail(PBH_ERR_ARG, "reps must be >= 1");
  const int64_t nbins = (int64_t)1 << cols;
  if (kernel_ms) *kernel_ms = 0.;
  if (rows == 0) {
    std::memset(counts, 0, nbins * sizeof(int64_t));
    return PBH_OK;
  }
  HIP_TRY(hipSetDevice(device));
  int n_cu = 0;
  HIP_TRY(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device));
  uint8_t *din = nullptr;
  unsigned long long *dcnt = nullptr, *dscr = nullptr;
  int rc = dalloc(din, rows * cols);
  if (!rc) rc = dalloc(dcnt, nbins);
  if (!rc) rc = dalloc(dscr, pbh::bool_perm_scratch_words(n_cu));
  hipError_t err = hipSuccess;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  double total = 0.;
  if (!rc) {
    err = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (err == hipSuccess) err = hipEventCreate(&e0);
    if (err == hipSuccess) err = hipEventCreate(&e1);
    if (err == hipSuccess)
      err = hipMemcpy(din, bool2d, (size_t)(rows * cols), hipMemcpyHostToDevice);
    // r = 0 is an untimed warm-up launch (the code object loads lazily on
    // the first launch); the average is over the `reps` timed launches
    for (int r = 0; r <= reps && err == hipSuccess; ++r) {
      err = hipMemsetAsync(dcnt, 0, nbins * sizeof(unsigned long long), st);
      if (err == hipSuccess) err = hipEventRecord(e0, st);
      if (err == hipSuccess) err = pbh::launch_bool_perm_freq(din, rows, cols, dcnt, dscr, n_cu, st);
      if (err == hipSuccess) err = hipEventRecord(e1, st);
      if (err == hipSuccess) err = hipEventSynchronize(e1);
      float ms = 0.f;
      if (err == hipSuccess) err = hipEventElapsedTime(&ms, e0, e1);
      if (r > 0) total += ms;
    }
    if (err == hipSuccess)
      err = hipMemcpy(counts, dcnt, nbins * sizeof(int64_t), hipMemcpyDeviceToHost);
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  dfree(din); dfree(dcnt); dfree(dscr);
  if (rc) return rc;
  if (err != hipSuccess)
    return fail(PBH_ERR_HIP, "pbh_bool_perm_freq: %s", hipGetErrorString(err));
  if (kernel_ms) *kernel_ms = total / reps;
  return PBH_OK;
}

int pbh_check_normals64(int device, int64_t n, const uint32_t *words,
                        double *fast, double *ref) {
  if (check_ptr(words, "words") || check_ptr(fast, "fast") || check_ptr(ref, "ref"))
    return PBH_ERR_ARG;
  if (n <= 0) return fail(PBH_ERR_ARG, "n must be positive");
  HIP_TRY(hipSetDevice(device));
  std::vector<double> tab(pbh::kBm64Doubles);
  pbh::bm64_tables(tab.data());
  uint32_t *dw = nullptr;
  double *df = nullptr, *dr = nullptr, *dt = nullptr;
  int rc = dalloc(dw, 3 * n);
  if (!rc) rc = dalloc(df, 2 * n);
  if (!rc) rc = dalloc(dr, 2 * n);
  if (!rc) rc = dalloc(dt, tab.size());
  hipError_t err = hipSuccess;
  if (!rc) {
    err = hipMemcpy(dw, words, 3 * n * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (err == hipSuccess)
      err = hipMemcpy(dt, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice);
    if (err == hipSuccess) err = pbh::launch_check_normals64(n, dw, dt, df, dr);
    if (err == hipSuccess) err = hipMemcpy(fast, df, 2 * n * sizeof(double), hipMemcpyDeviceToHost);
    if (err == hipSuccess) err = hipMemcpy(ref, dr, 2 * n * sizeof(double), hipMemcpyDeviceToHost);
  }
  dfree(dw); dfree(df); dfree(dr); dfree(dt);
  if (rc) return rc;
  if (err != hipSuccess)
    return fail(PBH_ERR_HIP, "pbh_check_normals64: %s", hipGetErrorString(err));
  return PBH_OK;
}

int pbh_bm64_tables(double *out) {
  if (check_ptr(out, "out")) return PBH_ERR_ARG;
  pbh::bm64_tables(out);
  return PBH_OK;
}

int pbh_check_normals(int device, int64_t n, const uint32_t *words,
                      double *fast, double *ref) {
  if (check_ptr(words, "words") || check_ptr(fast, "fast") || check_ptr(ref, "ref"))
    return PBH_ERR_ARG;
  if (n <= 0) return fail(PBH_ERR_ARG, "n must be positive");
  HIP_TRY(hipSetDevice(device));
  uint32_t *dw = nullptr;
  double *df = nullptr, *dr = nullptr;
  int rc = dalloc(dw, 4 * n);
  if (!rc) rc = dalloc(df, 2 * n);
  if (!rc) rc = dalloc(dr, 2 * n);
  hipError_t err = hipSuccess;
  if (!rc) {
    err = hipMemcpy(dw, words, 4 * n * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (err == hipSuccess) err = pbh::launch_check_normals(n, dw, df, dr);
    if (err == hipSuccess) err = hipMemcpy(fast, df, 2 * n * sizeof(double), hipMemcpyDeviceToHost);
    if (err == hipSuccess) err = hipMemcpy(ref, dr, 2 * n * sizeof(double), hipMemcpyDeviceToHost);
  }
  dfree(dw); dfree(df); dfree(dr);
  if (rc) return rc;
  if (err != hipSuccess)
    return fail(PBH_ERR_HIP, "pbh_check_normals: %s", hipGetErrorString(err));
  return PBH_OK;
}


// numpy's pairwise sum of a contiguous float64 array (the 8-accumulator
// leaf of <= 128 terms, split at n/2 rounded down to a multiple of 8).
static double np_pairwise_host(const double *a, int64_t n) {
  if (n < 8) {
    double r = 0.;
    for (int64_t i = 0; i < n; ++i) r += a[i];
    return r;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return np_pairwise_host(a, n2) + np_pairwise_host(a + n2, n - n2);
}

int pbh_linreg_gibbs(int device, int64_t n_obs, const double *x_obs,
                     const double *y_obs, const double *hyper,
                     const double *vsets, int64_t n_chains,
                     int64_t chain_offset, int64_t n_steps, int64_t step0,
                     const double *init, int32_t rng_mode, uint64_t seed,
                     const double *rand, double *trace_x, double *trace_lp,
                     double *final_x, double *final_lp, int32_t reps,
                     double *kernel_ms) {
  if (check_ptr(x_obs, "x_obs") || check_ptr(y_obs, "y_obs") ||
      check_ptr(hyper, "hyper") || check_ptr(init, "init"))
    return PBH_ERR_ARG;
  if (n_obs < 1 || n_obs > pbh::linreg_max_obs())
    return fail(PBH_ERR_ARG, "n_obs must be in 1..%lld, got %lld",
                (long long)pbh::linreg_max_obs(), (long long)n_obs);
  if (n_chains < 1 || n_steps < 0 || step0 < 0 || chain_offset < 0)
    return fail(PBH_ERR_ARG, "n_chains must be >= 1 and n_steps, step0, "
                "chain_offset >= 0");
  if (rng_mode != PBH_RNG_REPLAY && rng_mode != PBH_RNG_PHILOX &&
      rng_mode != PBH_RNG_PHILOX_F64)
    return fail(PBH_ERR_UNSUPPORTED, "pbh_linreg_gibbs: rng_mode %d", rng_mode);
  if (rng_mode == PBH_RNG_REPLAY && n_steps > 0 && !rand)
    return fail(PBH_ERR_ARG, "REPLAY needs rand [n_steps][n_chains]");
  if (reps < 1) return fail(PBH_ERR_ARG, "reps must be >= 1");
  if (hyper[1] == 0. || hyper[3] == 0.)
    return fail(PBH_ERR_ARG, "prior sigmas must be non-zero");
  const double alpha_post = hyper[4] + 0.5 * (double)n_obs;
  if (!(alpha_post >= 1.))
    return fail(PBH_ERR_ARG, "y_sigma_alpha + n_obs/2 must be >= 1");
  pbh::LinregArgs h{};
  std::vector<double> sq(n_obs);
  // centred statistics for the FAST form, two passes in long double
  long double mx = 0.L, my = 0.L;
  for (int64_t j = 0; j < n_obs; ++j) {
    sq[j] = x_obs[j] * x_obs[j];
    mx += x_obs[j];
    my += y_obs[j];
  }
  mx /= (long double)n_obs;
  my /= (long double)n_obs;
  long double cxx = 0.L, cxy = 0.L, cyy = 0.L;
  for (int64_t j = 0; j < n_obs; ++j) {
    const long double dx = x_obs[j] - mx, dy = y_obs[j] - my;
    cxx += dx * dx;
    cxy += dx * dy;
    cyy += dy * dy;
  }
  h.hyper[0] = 1. / (hyper[1] * hyper[1]); h.hyper[1] = hyper[0];
  h.hyper[2] = 1. / (hyper[3] * hyper[3]); h.hyper[3] = hyper[2];
  h.hyper[4] = alpha_post; h.hyper[5] = hyper[5];
  h.hyper[6] = np_pairwise_host(sq.data(), n_obs);
  for (int k = 0; k < 3; ++k) {
    if (vsets) {
      if (!(vsets[2 * k] < vsets[2 * k + 1]))
        return fail(PBH_ERR_ARG, "vsets[%d] must have lo < hi", k);
      h.hyper[7 + k] = -std::log(vsets[2 * k + 1] - vsets[2 * k]);
      h.bounds[2 * k] = vsets[2 * k];
      h.bounds[2 * k + 1] = vsets[2 * k + 1];
    } else {            // joint=False: no prior terms (lp + 0.0 == lp)
      h.hyper[7 + k] = 0.;
      h.bounds[2 * k] = -HUGE_VAL;
      h.bounds[2 * k + 1] = HUGE_VAL;
    }
  }
  h.hyper[10] = std::log(std::sqrt(2. * M_PI));
  h.stats[0] = (double)mx; h.stats[1] = (double)my; h.stats[2] = (double)cxx;
  h.stats[3] = (double)cxy; h.stats[4] = (double)cyy;
  h.n_obs = n_obs; h.n = n_chains; h.chain_offset = chain_offset;
  h.n_steps = n_steps; h.step0 = step0; h.seed = seed; h.mode = rng_mode;
  {
    // the lane-pair kernel is measured slower (1.60 vs 1.22 ms at 65 536
    // chains x 1 000 steps); PBH_LINREG_PAIR=1 selects it for A/B runs
    const char *p_env = std::getenv("PBH_LINREG_PAIR");
    h.pair = p_env && p_env[0] == '1';
  }
  if (kernel_ms) *kernel_ms = 0.;
  HIP_TRY(hipSetDevice(device));
  const int64_t T = n_steps, N = n_chains;
  double *dxo = nullptr, *dyo = nullptr, *dinit = nullptr, *dstate = nullptr,
         *dlp = nullptr, *drand = nullptr, *dtx = nullptr, *dtp = nullptr;
  int rc = dalloc(dxo, n_obs);
  if (!rc) rc = dalloc(dyo, n_obs);
  if (!rc) rc = dalloc(dinit, 3 * N);
  if (!rc) rc = dalloc(dstate, 3 * N);
  if (!rc) rc = dalloc(dlp, N);
  if (!rc && rng_mode == PBH_RNG_REPLAY && T > 0) rc = dalloc(drand, T * N);
  if (!rc && T > 0 && trace_x) rc = dalloc(dtx, T * 3 * N);
  if (!rc && T > 0 && trace_lp) rc = dalloc(dtp, T * N);
  hipError_t err = hipSuccess;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  double total = 0.;
  if (!rc) {
    err = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (err == hipSuccess) err = hipEventCreate(&e0);
    if (err == hipSuccess) err = hipEventCreate(&e1);
    if (err == hipSuccess) err = hipMemcpy(dxo, x_obs, n_obs * 8, hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipMemcpy(dyo, y_obs, n_obs * 8, hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipMemcpy(dinit, init, 3 * N * 8, hipMemcpyHostToDevice);
    if (err == hipSuccess && drand)
      err = hipMemcpy(drand, rand, T * N * 8, hipMemcpyHostToDevice);
    h.x_obs = dxo; h.y_obs = dyo; h.state = dstate; h.lp_state = dlp;
    h.rand = drand; h.tx = dtx; h.tp = dtp;
    // r = 0 is an untimed warm-up launch, made only when timing several
    // repetitions (a single run is the sampler's own)
    for (int r = reps > 1 ? 0 : 1; r <= reps && err == hipSuccess && T > 0; ++r) {
      err = hipMemcpyAsync(dstate, dinit, 3 * N * 8, hipMemcpyDeviceToDevice, st);
      if (err == hipSuccess) err = hipEventRecord(e0, st);
      if (err == hipSuccess) err = pbh::launch_linreg_gibbs(h, st);
      if (err == hipSuccess) err = hipEventRecord(e1, st);
      if (err == hipSuccess) err = hipEventSynchronize(e1);
      float ms = 0.f;
      if (err == hipSuccess) err = hipEventElapsedTime(&ms, e0, e1);
      if (r > 0) total += ms;
    }
    if (err == hipSuccess && trace_x && T > 0)
      err = hipMemcpy(trace_x, dtx, T * 3 * N * 8, hipMemcpyDeviceToHost);
    if (err == hipSuccess && trace_lp && T > 0)
      err = hipMemcpy(trace_lp, dtp, T * N * 8, hipMemcpyDeviceToHost);
    if (err == hipSuccess && final_x)
      err = hipMemcpy(final_x, T > 0 ? dstate : dinit, 3 * N * 8, hipMemcpyDeviceToHost);
    if (err == hipSuccess && final_lp && T > 0)
      err = hipMemcpy(final_lp, dlp, N * 8, hipMemcpyDeviceToHost);
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  dfree(dxo); dfree(dyo); dfree(dinit); dfree(dstate); dfree(dlp);
  dfree(drand); dfree(dtx); dfree(dtp);
  if (rc) return rc;
  if (err != hipSuccess)
    return fail(PBH_ERR_HIP, "pbh_linreg_gibbs: %s", hipGetErrorString(err));
  if (kernel_ms) *kernel_ms = total / reps;
  return PBH_OK;
}

}  // extern "C"
