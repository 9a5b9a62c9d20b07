// art_capi.cpp -- the extern "C" boundary of libart.so (declared in include/art.h).
//
// Host-pointer entry points (what a Julia ccall passes) stage through pooled device
// buffers on the library's own HIP stream; device-pointer entry points run
// asynchronously on the caller's stream. No torch types cross this boundary.
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/art.h"
#include "art_core.h"
#include "art_internal.h"


namespace {

// g_mu: every entry point (the calls of one process are serialised); g_ring_mu: the launch ring
// and the latched statistics, which the asynchronous host calls' worker threads also touch
// (they never take g_mu, so a caller holding it may wait for them)
std::mutex g_mu, g_ring_mu;
thread_local std::string g_err;
double g_last_ms = 0.0;
unsigned long long g_last_stats[art::N_STATS] = {0};
int g_last_grid = 0;
// What the art_propagate_host* calls ran as (art_host_path_counters): calls, streamed
// pipeline completions, streamed give-ups (each batch then ran again as one launch), chunked
// pipeline calls, single-launch calls
enum { HC_CALLS, HC_STREAMED, HC_GIVEUPS, HC_CHUNKED, HC_SINGLE, HC_N };
std::atomic<uint64_t> g_host_cnt[HC_N] = {};

// One propagate launch's bookkeeping: the HIP events around the integrator kernel, an event
// after its statistics were copied to pinned host memory, and that memory. A ring of them per
// device lets launches on different streams be in flight together; a slot is reused only after
// its previous launch completed.
constexpr int RING = 64;
struct LaunchRec {
  hipEvent_t ev0 = nullptr, ev1 = nullptr, done = nullptr;
  hipEvent_t hot_fork = nullptr, hot_join = nullptr;  // the hot rays' side launch (art::HotSide)
  unsigned long long* host_stats = nullptr;  // N_STATS_DEV words (pinned): statistics, then the clock stamps
  int grid = 0;
  hipStream_t stream = nullptr;
  bool pending = false;
  // an asynchronous host call holds its record from its launch until it latches it at its end
  // (latch_launch / finish_timing_slot): take_slot skips a held record, so the ring wrapping
  // under other launches cannot hand it out twice
  std::atomic<bool> held{false};
};

struct Pinned {
  void* p = nullptr;
  size_t bytes = 0;
  unsigned flags = 0;
};
using PoolVec = std::vector<std::pair<void*, size_t>>;

// One set of the maskless streamed pipeline's resources (propagate_host_maskless): the
// integrator's and the helpers' CU-masked streams (a hardware queue each), the two copy
// streams, the host words the GPU polls and raises, the pinned and device staging and the
// events. A context has HOST_LANES of them, so that many host calls can be in flight at once
// (art_propagate_host_flux_async: the next batch's uploads and first rays overlap this one's
// drain); lane 0 also serves the synchronous calls, which first wait for every async call.
constexpr int HOST_LANES = 2;
struct HostLane {
  hipStream_t m_comp = nullptr, m_up = nullptr, m_dn = nullptr, m_help = nullptr;
  unsigned long long* hsig = nullptr;  // [0] ready | [8, 8 + 64) piece flags | [72] helper blocks started
  unsigned long long* hsig_dev = nullptr;
  unsigned int* abort_host = nullptr;  // the word the waves and helpers raise (or read) when a call gives up
  unsigned int* abort_dev = nullptr;
  std::vector<hipEvent_t> pev;
  std::vector<Pinned> pinned;  // [0] gathered inputs, [1] output blobs
  PoolVec pool;                // [0] inputs, [1] output blobs, [2] scratch, [3] flux; [4..] the single-launch fallback
  // the asynchronous calls' worker: one job at a time, results kept by ticket until waited for
  std::thread worker;
  std::mutex m;
  std::condition_variable cv;
  std::function<int()> job;
  bool busy = false, stop = false;
};

struct DeviceCtx {
  int device = -1;
  hipStream_t stream = nullptr;  // the *_host entry points' stream
  LaunchRec ring[RING];
  int next = 0, last = -1;       // next ring slot; the most recent propagate launch
  int64_t launches = 0;          // propagate launches issued so far
  int32_t donate = -1;           // tail donation (art_set_tail_donation): lanes per wave, 0 = off, -1 = by geometry
  int32_t graduate = -1;         // graduation (art_set_graduation): attempts, 0 = off, -1 = the default (2048)
  int32_t sampler_waves = 0;     // art_set_sampler_waves: 0 = by line length, 2 or 3
  // the side stream of each stream that propagate launches ran on (the hot rays' tail launch,
  // art::HotSide): one per caller stream, so a launch waits on no other stream's hot rays
  std::map<hipStream_t, hipStream_t> hot_side;
  std::vector<std::pair<void*, size_t>> pool;  // host-entry staging buffers (grow-only, used under g_mu by the
                                               // synchronous *_host calls only)
  // the chunked host pipeline of art_propagate_host (propagate_host_chunked): its compute
  // streams, one stream for the uploads and one for the chunks' finalize kernels, its pinned
  // input and output staging (grow-only) and two events per chunk (inputs in HBM, outputs in
  // pinned memory)
  std::vector<hipStream_t> pstreams;
  hipStream_t h2d = nullptr, fin = nullptr;
  std::vector<Pinned> pinned;
  std::vector<hipEvent_t> pev;
  HostLane lanes[HOST_LANES];
  // asynchronous host calls: tickets in submission order (ticket t runs on lane t % HOST_LANES);
  // finished calls' results until art_host_wait takes them
  std::atomic<int64_t> next_ticket{0};
  std::atomic<int64_t> done_ticket{-1};  // the highest ticket whose call has ended
  std::mutex res_m;
  std::condition_variable res_cv;
  std::set<int64_t> pending;  // submitted, not yet waited for
  std::map<int64_t, std::pair<int, std::string>> results;
};
// (pointers: a context never moves, so a worker thread may hold one while another device's is created)
std::vector<std::unique_ptr<DeviceCtx>> g_ctx;
std::mutex g_ctx_mu;

int fail(int code, const char* fmt, const char* a = "", const char* b = "") {
  char buf[512];
  std::snprintf(buf, sizeof buf, fmt, a, b);
  g_err = buf;
  return code;
}

#define HIP_OK(expr)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) return fail(ART_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

void shutdown_at_exit();

int current_ctx(DeviceCtx** out) {
  // Release every HIP object of the library at exit, before the HIP runtime tears itself down:
  // handlers registered with atexit run in reverse order, and the runtime (loaded and
  // initialised before libart's first call) registered its teardown earlier. Left to static
  // destruction, the library's streams, signal memory and pinned buffers outlived the runtime
  // (and a profiler's finalisation), DESIGN.md §4 "exit".
  static bool at_exit = false;
  if (!at_exit) {
#ifndef ART_NO_EXIT_RELEASE  // (dev A/B: the round-3 behaviour, static destruction only)
    std::atexit(shutdown_at_exit);
#endif
    at_exit = true;
  }
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  DeviceCtx* cp = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    if ((int)g_ctx.size() <= dev) g_ctx.resize(dev + 1);
    if (!g_ctx[dev]) g_ctx[dev].reset(new DeviceCtx());
    cp = g_ctx[dev].get();
  }
  DeviceCtx& c = *cp;
  if (c.device < 0) {
    HIP_OK(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    unsigned long long* hs = nullptr;
    HIP_OK(hipHostMalloc((void**)&hs, sizeof(unsigned long long) * art::N_STATS_DEV * RING, hipHostMallocDefault));
    for (int i = 0; i < RING; ++i) {
      HIP_OK(hipEventCreate(&c.ring[i].ev0));
      HIP_OK(hipEventCreate(&c.ring[i].ev1));
      HIP_OK(hipEventCreateWithFlags(&c.ring[i].done, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&c.ring[i].hot_fork, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&c.ring[i].hot_join, hipEventDisableTiming));
      c.ring[i].host_stats = hs + i * art::N_STATS_DEV;
    }
    // per-launch scratch comes from the stream-ordered allocator: keep what it frees cached
    // so a steady stream of launches does not go back to the driver
    hipMemPool_t mp;
    if (hipDeviceGetDefaultMemPool(&mp, dev) == hipSuccess) {
      uint64_t thr = ~0ull;
      (void)hipMemPoolSetAttribute(mp, hipMemPoolAttrReleaseThreshold, &thr);
    }
    c.device = dev;
  }
  *out = &c;
  return ART_OK;
}

// The next launch record: waits for the launch that used the slot RING launches ago.
int take_slot(DeviceCtx* c, LaunchRec** out) {
  for (int k = 0; k < RING && c->ring[c->next].held.load(std::memory_order_acquire); ++k) c->next = (c->next + 1) % RING;
  LaunchRec& L = c->ring[c->next];
  if (L.pending) {
    HIP_OK(hipEventSynchronize(L.done));
    L.pending = false;
  }
  *out = &L;
  return ART_OK;
}

int pool_get_v(PoolVec& pool, size_t slot, size_t bytes, void** p) {
  if (pool.size() <= slot) pool.resize(slot + 1, {nullptr, 0});
  auto& e = pool[slot];
  if (e.second < bytes) {
    if (e.first) HIP_OK(hipFree(e.first));
    e.first = nullptr;
    e.second = 0;
    if (hipMalloc(&e.first, bytes) != hipSuccess) return fail(ART_E_NOMEM, "hipMalloc of %s bytes failed", std::to_string(bytes).c_str());
    e.second = bytes;
  }
  *p = e.first;
  return ART_OK;
}

int pool_get(DeviceCtx* c, size_t slot, size_t bytes, void** p) { return pool_get_v(c->pool, slot, bytes, p); }

int pinned_get_v(std::vector<Pinned>& pinned, size_t slot, size_t bytes, void** p, unsigned flags = hipHostMallocDefault) {
  if (pinned.size() <= slot) pinned.resize(slot + 1);
  auto& e = pinned[slot];
  if (e.bytes < bytes || e.flags != flags) {
    if (e.p) HIP_OK(hipHostFree(e.p));
    e.p = nullptr;
    e.bytes = 0;
    e.flags = flags;
    if (hipHostMalloc(&e.p, bytes, flags) != hipSuccess)
      return fail(ART_E_NOMEM, "hipHostMalloc of %s bytes failed", std::to_string(bytes).c_str());
    e.bytes = bytes;
  }
  *p = e.p;
  return ART_OK;
}

int pinned_get(DeviceCtx* c, size_t slot, size_t bytes, void** p, unsigned flags = hipHostMallocDefault) {
  return pinned_get_v(c->pinned, slot, bytes, p, flags);
}

// Host-side copies of the chunked host pipeline (caller arrays <-> pinned staging): a few
// persistent worker threads share each batch of row segments, so gathering one chunk's inputs
// and scattering another's outputs runs at the host's memory bandwidth, not one core's.
class CopyPool {
 public:
  struct Seg {
    void* dst;
    const void* src;
    size_t bytes;
  };
  explicit CopyPool(int nthreads) {
    for (int i = 0; i < nthreads; ++i) th_.emplace_back([this] { loop(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // copies every segment; pieces of at most 1 MiB are shared by the workers and the caller (one
  // caller at a time: the asynchronous calls' workers take turns)
  void run(const std::vector<Seg>& segs) {
    std::lock_guard<std::mutex> one(run_m_);
    pieces_.clear();
    for (const Seg& g : segs)
      for (size_t o = 0; o < g.bytes; o += PIECE)
        pieces_.push_back({(char*)g.dst + o, (const char*)g.src + o, std::min(PIECE, g.bytes - o)});
    if (pieces_.empty()) return;
    next_.store(0);
    {
      std::lock_guard<std::mutex> lk(m_);
      busy_ = (int)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [this] { return busy_ == 0; });
  }

 private:
  static constexpr size_t PIECE = size_t(1) << 20;
  void work() {
    for (size_t i; (i = next_.fetch_add(1)) < pieces_.size();) std::memcpy(pieces_[i].dst, pieces_[i].src, pieces_[i].bytes);
  }
  void loop() {
    unsigned long long seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
      std::lock_guard<std::mutex> lk(m_);
      if (--busy_ == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex run_m_;
  std::vector<Seg> pieces_;
  std::atomic<size_t> next_{0};
  std::mutex m_;
  std::condition_variable cv_, done_;
  unsigned long long gen_ = 0;
  int busy_ = 0;
  bool stop_ = false;
};

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return (e && *e) ? std::atoi(e) : dflt;
}
double env_double(const char* name, double dflt) {
  const char* e = std::getenv(name);
  return (e && *e) ? std::atof(e) : dflt;
}
constexpr size_t HOT_CAP = 1024;  // early-graduation records of one launch (SegOut::hot)

// (a heap object, not a function-local static: art_shutdown joins its threads before the HIP
// runtime's own teardown, and no static destructor of libart is left to run after it)
// Created under its own lock: the gatherer threads of two asynchronous calls may ask for it
// at the same time, outside g_mu.
std::atomic<CopyPool*> g_copy_pool{nullptr};
std::mutex g_copy_pool_mu;
CopyPool& copy_pool() {
  CopyPool* cp = g_copy_pool.load(std::memory_order_acquire);
  if (cp) return *cp;
  std::lock_guard<std::mutex> lk(g_copy_pool_mu);
  cp = g_copy_pool.load(std::memory_order_relaxed);
  // ART_HOST_THREADS: worker threads besides the caller (default 7)
  if (!cp) {
    cp = new CopyPool(std::max(0, env_int("ART_HOST_THREADS", 7)));
    g_copy_pool.store(cp, std::memory_order_release);
  }
  return *cp;
}

// Every HIP object a device context holds, released in dependency order (the streams drained
// first). Used by art_shutdown, which runs at exit ahead of the HIP runtime's teardown.
void stop_workers(DeviceCtx& c) {
  for (HostLane& H : c.lanes) {
    if (!H.worker.joinable()) continue;
    {
      std::lock_guard<std::mutex> lk(H.m);
      H.stop = true;
    }
    H.cv.notify_all();
    H.worker.join();
  }
}

void release_ctx(DeviceCtx& c) {
  if (c.device < 0) return;
  stop_workers(c);  // (each finishes its call first)
  (void)hipSetDevice(c.device);
  (void)hipDeviceSynchronize();
  for (LaunchRec& L : c.ring) {
    if (L.ev0) (void)hipEventDestroy(L.ev0);
    if (L.ev1) (void)hipEventDestroy(L.ev1);
    if (L.done) (void)hipEventDestroy(L.done);
    for (hipEvent_t e : {L.hot_fork, L.hot_join})
      if (e) (void)hipEventDestroy(e);
  }
  for (auto& e : c.hot_side) (void)hipStreamDestroy(e.second);
  if (c.ring[0].host_stats) (void)hipHostFree(c.ring[0].host_stats);  // one block for the ring
  for (auto& e : c.pool)
    if (e.first) (void)hipFree(e.first);
  for (auto& e : c.pinned)
    if (e.p) (void)hipHostFree(e.p);
  for (hipEvent_t e : c.pev) (void)hipEventDestroy(e);
  for (hipStream_t s : c.pstreams)
    if (s && s != c.stream) (void)hipStreamDestroy(s);
  for (hipStream_t s : {c.h2d, c.fin})
    if (s) (void)hipStreamDestroy(s);
  for (HostLane& H : c.lanes) {
    for (auto& e : H.pool)
      if (e.first) (void)hipFree(e.first);
    for (auto& e : H.pinned)
      if (e.p) (void)hipHostFree(e.p);
    for (hipEvent_t e : H.pev) (void)hipEventDestroy(e);
    for (hipStream_t s : {H.m_comp, H.m_up, H.m_dn, H.m_help})
      if (s) (void)hipStreamDestroy(s);
    if (H.hsig) (void)hipHostFree(H.hsig);
    if (H.abort_host) (void)hipHostFree(H.abort_host);
  }
  if (c.stream) (void)hipStreamDestroy(c.stream);
}

void shutdown_locked() {
  std::vector<std::unique_ptr<DeviceCtx>> all;
  {
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    all.swap(g_ctx);
  }
  for (auto& c : all)
    if (c) release_ctx(*c);
  all.clear();
  std::lock_guard<std::mutex> lk(g_copy_pool_mu);
  delete g_copy_pool.exchange(nullptr);
}

void shutdown_at_exit() {
  // (a call still running on another thread at exit keeps its objects: releasing them under it
  // would be worse than leaving them to the runtime)
  if (!g_mu.try_lock()) return;
  shutdown_locked();
  g_mu.unlock();
}

// Device scratch of ONE launch, allocated and freed in the order of its stream (hipMallocAsync /
// hipFreeAsync), so concurrent launches never share a work-queue word or a state buffer.
int scratch_alloc(hipStream_t s, size_t bytes, void** p) {
  if (hipMallocAsync(p, bytes, s) != hipSuccess)
    return fail(ART_E_NOMEM, "hipMallocAsync of %s bytes failed", std::to_string(bytes).c_str());
  return ART_OK;
}

int validate(const art_params* p) {
  if (!p) return fail(ART_E_INVALID, "params is NULL");
  if (!p->melrose) return fail(ART_E_UNSUPPORTED, "melrose=0 (Ctheta_B_sphere form) is not supported; the reference hard-codes melrose=true (Gen_Samples.jl:167)");
  if (p->integrator != ART_VERN6 && p->integrator != ART_RK4) return fail(ART_E_INVALID, "unknown integrator");
  if (p->integrator == ART_RK4 && p->n_fixed < 1) return fail(ART_E_INVALID, "RK4 needs n_fixed >= 1");
  if (!(p->rNS > 0) || !(p->mass_a > 0) || !(p->omega_pul != 0)) return fail(ART_E_INVALID, "rNS, mass_a must be > 0 and omega_pul != 0");
  if (!(p->abstol > 0) || !(p->reltol >= 0)) return fail(ART_E_INVALID, "bad tolerances");
  if (p->maxiters < 1) return fail(ART_E_INVALID, "maxiters must be >= 1");
  if (p->interp_points > 65) return fail(ART_E_INVALID, "interp_points must be <= 65 (the reference uses 50)");
  return ART_OK;
}

// Kernel parameters. ART_SCAN_CERT=0 switches the certified scan steps of the integrator and
// of the sampler off (A/B tests: the results are bit-identical either way,
// tests/test_gpu_scan_cert.py).
art::KParams kparams(const art_params& p) {
  art::KParams K = art::make_kparams(p);
  if (const char* e = std::getenv("ART_SCAN_CERT"))
    if (e[0] == '0') K.cert_fac = __builtin_inf();
  return K;
}

// *_device entry points run on the caller's stream exactly as given: NULL is the HIP null
// stream (torch's default stream), so the library orders correctly with the caller's
// work. Only the *_host entry points use the library's own stream.
hipStream_t pick(DeviceCtx*, void* stream) { return (hipStream_t)stream; }

// saveat outputs (art_propagate_traj_*): ntimes >= 2 points per ray, or none (ntimes = 0)
struct TrajArgs {
  int32_t ntimes = 0;
  double *traj = nullptr, *t = nullptr;
  int32_t* count = nullptr;
};

// art_propagate_host_flux: the batch's binned radiated flux (flux_kernel over the outputs while
// they are still in HBM), 2 * nbins doubles into the caller's `hist`; nbins = 0: none
struct FluxArgs {
  int32_t nbins = 0;
  double* hist = nullptr;
};

// Argument checks shared by the host and device entry points, before any device call (the
// host path stages buffers of n elements, so a bad n or a NULL buffer must stop it first).
// Returns ART_OK with *empty set for n == 0 (nothing to do, nothing written).
int check_segment_args(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                       const double* dw, const double* ln_t0, const int8_t* species, const art_segment_out* out,
                       const art_crossing_buf* xc, const TrajArgs& tr, bool* empty) {
  int rc = validate(p);
  if (rc) return rc;
  if (n < 0 || n > 2147483647LL) return fail(ART_E_INVALID, "n must be in [0, 2^31)");
  if (!out || !out->x_end || !out->k_end || !out->u7_end || !out->tau_end || !out->status || !out->n_accept || !out->n_reject)
    return fail(ART_E_INVALID, "segment output buffers must be non-NULL");
  *empty = n == 0;
  if (n == 0) return ART_OK;
  if (!x0 || !k0 || !erg || !dw || !ln_t0 || !species) return fail(ART_E_INVALID, "input buffers must be non-NULL");
  const int cap = (xc && xc->count) ? xc->capacity : 0;
  if (cap && (cap < 1 || !xc->pos || !xc->k || !xc->t || !xc->dw || !xc->p_nonad))
    return fail(ART_E_INVALID, "crossing buffer incomplete");
  if (tr.ntimes != 0 && (tr.ntimes < 2 || !tr.traj || !tr.t || !tr.count))
    return fail(ART_E_INVALID, "saveat needs ntimes >= 2 and buffers");
  return ART_OK;
}

// Options of one propagate launch beyond the entry points' arguments (the host paths' own
// use): the tail-donation lanes (-1: the device's setting), caller-provided scratch of
// propagate_scratch_bytes() bytes (null: from the stream-ordered pool), and NaN in the
// crossing slots without a crossing (finalize_kernel writes them, the *_host contract).
struct LaunchOpts {
  int donate = -1;
  void* scratch = nullptr;
  size_t scratch_bytes = 0;  // the size of `scratch` (checked against the launch's layout)
  bool nan_fill = false;
  hipStream_t finalize_stream = nullptr;  // finalize_kernel on this stream (after the integrator)
  LaunchRec** launch_out = nullptr;       // the launch's ring entry (finish_timing_slot)
};

// Tail donation of a launch: the caller's choice, else the device's setting, else (-1, the
// default) by geometry. A Schwarzschild batch is bound by its few longest rays (configs[3]: ray
// 717277 takes 23 592 attempts), which a lone pass would run on one lane of a draining wave
// (13.5 us per attempt); donated, they finish on the one-wave-per-ray tail kernel (7.7 us). A
// flat lone pass has no such ray, and donation costs its drain 0.5-1.3%.
int launch_donate(DeviceCtx* c, const LaunchOpts& o, const art_params* p, const TrajArgs& tr) {
  if (o.donate >= 0) return o.donate;
  if (c->donate >= 0) return c->donate;
  const bool sch = !p->flat && !(p->bndry_lyr > 0.0) && !p->isotropic;
  return (sch && p->integrator == ART_VERN6 && tr.ntimes == 0) ? 16 : 0;
}

// A small Vern6 batch without saveat runs every ray on a wave of its own (tail_kernel): the
// latency of a Julia host's per-event calls (its rays run ~40% faster per attempt than a lone
// lane of the persistent integrator), bit-identical results. One decision for the launch and
// for every caller that lays out a launch's scratch ahead of it (the chunked host pipeline).
bool use_small_tail(const art_params* p, int64_t n, const TrajArgs& tr) {
  return tr.ntimes == 0 && p->integrator == ART_VERN6 && n <= art::small_tail_limit();
}

// this launch's scratch: [queue head + statistics (256 B) | u0: U0_REC n doubles of fresh state
// (init_kernel -> the integrator) | END_REC n doubles of end records | X_REC cap n doubles of
// crossing records (the integrator -> finalize_kernel) | donation records of two levels, the
// graduation and early-graduation records (and the latter's ready words) | the claim order's sort]
struct ScratchLayout {
  size_t head = 256, u0b = 0, recb = 0, xrb = 0, ncont = 0, nhot = 0, contb = 0, ordb = 0;
  size_t total() const { return head + u0b + recb + xrb + contb + ordb; }
};
int scratch_layout(DeviceCtx* c, int64_t n, int cap, int32_t donate, ScratchLayout* L, bool small_tail = false) {
  const size_t nd = (size_t)n;
  L->u0b = nd * art::U0_REC * sizeof(double);
  L->recb = nd * art::END_REC * sizeof(double);
  L->xrb = (size_t)cap * nd * art::X_REC * sizeof(double);
  // tail donation: at most (resident waves) x donate records of CONT_REC doubles; a small batch
  // sent to the tail kernel: one record per ray
  L->ncont = 0;
  if (small_tail) {
    L->ncont = nd;
  } else if (donate > 0) {
    int ncu = 0;
    HIP_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device));
    L->ncont = std::min(nd, (size_t)ncu * 32 * (size_t)donate);
  }
  // the second level (the packed continuation's own donations, resumed by the tail kernel):
  // never more than the first level's; then as many graduation records (SegOut::grad) and the
  // early-graduation records (SegOut::hot)
  // early-graduation records (SegOut::hot) and their ready words
  L->nhot = small_tail ? 0 : std::min(L->ncont, (size_t)HOT_CAP);
  L->contb = ((small_tail ? 2 : 3) * L->ncont + L->nhot) * art::CONT_REC * sizeof(double) + L->nhot * sizeof(unsigned);
  // (then the claim order's sort, SegOut::order)
  L->ordb = L->nhot ? art::claim_order_bytes(n) + 256 : 0;
  return ART_OK;
}

int propagate_device_impl(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                          const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                          art_segment_out* out, art_crossing_buf* xc, void* stream, const TrajArgs& tr = TrajArgs(),
                          const LaunchOpts& opt = LaunchOpts(), DeviceCtx* cx = nullptr) {
  bool empty = false;
  int rc = check_segment_args(p, n, x0, k0, erg, dw, ln_t0, species, out, xc, tr, &empty);
  if (rc || empty) return rc;
  DeviceCtx* c = cx;
  if (!c && (rc = current_ctx(&c))) return rc;
  hipStream_t s = pick(c, stream);
  const art::KParams K = kparams(*p);
  const int cap = (xc && xc->count) ? xc->capacity : 0;
  const bool small_tail = use_small_tail(p, n, tr);
  const int32_t donate = small_tail ? 0 : launch_donate(c, opt, p, tr);
  ScratchLayout SL;
  if ((rc = scratch_layout(c, n, cap, donate, &SL, small_tail))) return rc;
  if (opt.scratch && SL.total() > opt.scratch_bytes)
    return fail(ART_E_INVALID, "caller scratch of %s bytes is smaller than the launch needs (%s)",
                std::to_string(opt.scratch_bytes).c_str(), std::to_string(SL.total()).c_str());
  const size_t head = SL.head, u0b = SL.u0b, recb = SL.recb, xrb = SL.xrb, ncont = SL.ncont;
  std::lock_guard<std::mutex> rlk(g_ring_mu);  // (the ring, up to this launch's entry in it)
  LaunchRec* L;
  if ((rc = take_slot(c, &L))) return rc;
  if (opt.launch_out) *opt.launch_out = L;
  void* blk = opt.scratch;
  if (!blk && (rc = scratch_alloc(s, SL.total(), &blk))) return rc;
  unsigned long long* words = (unsigned long long*)blk;
  double* u0 = (double*)((char*)blk + head);
  double* rec = (double*)((char*)blk + head + u0b);
  art::SegIn in{x0, k0, erg, dw, ln_t0, species, u0};
  art::SegOut so{out->x_end, out->k_end, out->u7_end, out->tau_end, out->status, out->n_accept, out->n_reject,
                 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  if (cap) {
    so.cap = cap;
    so.xcount = xc->count;
    so.xpos = xc->pos; so.xk = xc->k; so.xt = xc->t; so.xdw = xc->dw; so.xp = xc->p_nonad;
    so.xrec = (double*)((char*)blk + head + u0b + recb);
    so.nan_fill = opt.nan_fill ? 1 : 0;
  }
  if (tr.ntimes != 0) {
    so.ntimes = tr.ntimes;
    so.traj = tr.traj;
    so.traj_t = tr.t;
    so.traj_n = tr.count;
  }
  so.rec = rec;
  art::HotSide hot;
  if (ncont) {
    so.cont = (double*)((char*)blk + head + u0b + recb + xrb);
    so.cont_count = words + 16;  // head words 16 .. 19 (zeroed with the head)
    so.cont_queue = words + 17;
    so.cont2 = so.cont + ncont * art::CONT_REC;
    so.cont2_count = words + 18;
    so.cont2_queue = words + 19;
    if (!small_tail && tr.ntimes == 0 && p->integrator == ART_VERN6) {
      // graduation of a pass's outlier rays to the tail kernel (ART_GRADUATE attempts, default
      // 2048 -- about 23x the mean GR ray, never reached by a flat one; 0 = off;
      // profiles/r04av_graduation_threshold.txt)
      so.grad = so.cont2 + ncont * art::CONT_REC;
      so.grad_count = words + 20;
      so.grad_queue = words + 21;
      so.grad_cap = (int32_t)std::min(ncont, (size_t)INT32_MAX);
      // (the caller's setting, art_set_graduation: a host that keeps several passes in flight turns
      // it off -- each graduated ray then holds a whole tail wave while the other passes fill the
      // CUs it would free, profiles/r04al_graduation_in_flight.txt; round 4 decided this per launch
      // from the other streams' events, which made it depend on host timing)
      so.graduate = c->graduate >= 0 ? c->graduate : std::max(0, env_int("ART_GRADUATE", 2048));
      // early graduation (SegOut::hot), with graduation only: from ART_HOT_AT attempts (default
      // 128) a ray whose progress in ln t is below ART_HOT_DTAU + ART_HOT_SLOPE log2(attempts /
      // 256) (defaults 15.95, 0.75): on configs[3] 102 rays, 90 of them past 5000 attempts, among
      // them every one of the 20 longest (tools/exp_gr_predict.py)
      // (only on a non-blocking stream: the side stream below is a blocking one, and work on a
      // blocking stream -- the null stream above all -- would wait for the hot launch, which waits
      // for this launch's own kernels)
      unsigned sflags = 0;
      const bool nonblocking = s != nullptr && hipStreamGetFlags(s, &sflags) == hipSuccess && (sflags & hipStreamNonBlocking);
      if (SL.nhot && so.graduate > 0 && nonblocking) {
        so.hot = so.grad + ncont * art::CONT_REC;
        so.hot_ready = (unsigned*)(so.hot + SL.nhot * art::CONT_REC);
        so.hot_count = words + 22;
        so.hot_queue = words + 23;
        so.hot_done = (unsigned*)(words + 26);
        so.hot_cap = (int32_t)SL.nhot;
        so.hot_at = std::max(0, env_int("ART_HOT_AT", 128));
        so.hot_dtau = env_double("ART_HOT_DTAU", 15.95);
        so.hot_slope = env_double("ART_HOT_SLOPE", 0.75);
        if (SL.ordb && env_int("ART_HOT_ORDER", 1)) {  // (256-byte aligned)
          const uintptr_t o = (uintptr_t)blk + SL.total() - SL.ordb;
          so.order_tmp = (void*)((o + 255) & ~(uintptr_t)255);
        }
        auto it = c->hot_side.find(s);
        if (it == c->hot_side.end()) {
          // a hardware queue of its own (a stream with a CU mask gets one; the mask holds every CU):
          // a plain stream may share one with s, and s's kernels would then queue behind the hot
          // launch that waits for them (lane_setup, profiles/r04p_maskless_hwqueue.txt)
          int ncu_all = 0;
          HIP_OK(hipDeviceGetAttribute(&ncu_all, hipDeviceAttributeMultiprocessorCount, c->device));
          std::vector<uint32_t> all((ncu_all + 31) / 32, 0u);
          for (int i = 0; i < ncu_all; ++i) all[i / 32] |= 1u << (i % 32);
          hipStream_t hsd = nullptr;
          HIP_OK(hipExtStreamCreateWithCUMask(&hsd, (uint32_t)all.size(), all.data()));
          it = c->hot_side.emplace(s, hsd).first;
        }
        hot.stream = it->second;
        hot.fork = L->hot_fork;
        hot.join = L->hot_join;
        hot.zero_word = words + 24;  // (words 22 .. 26: zeroed with the head)
      }
    }
    so.donate = donate;
    so.small_tail = small_tail ? 1 : 0;
  }
  HIP_OK(hipMemsetAsync(words, 0, head, s));
  if (so.hot_ready) HIP_OK(hipMemsetAsync(so.hot_ready, 0, SL.nhot * sizeof(unsigned), s));
  HIP_OK(art::launch_propagate(K, n, in, so, max_crossings, words, words + 1, s, &L->grid, L->ev0, L->ev1,
                               opt.finalize_stream, hot));
  HIP_OK(hipMemcpyAsync(L->host_stats, words + 1, sizeof(unsigned long long) * art::N_STATS_DEV, hipMemcpyDeviceToHost, s));
  HIP_OK(hipEventRecord(L->done, s));
  if (!opt.scratch) HIP_OK(hipFreeAsync(blk, s));
  L->stream = s;
  L->pending = true;
  c->last = c->next;
  c->next = (c->next + 1) % RING;
  c->launches += 1;
  return ART_OK;
}

// Latch one propagate launch (L; null: the most recent): its integrator kernel's duration and
// statistics, once it has completed.
int finish_timing_slot(DeviceCtx* c, LaunchRec* Lp) {
  std::lock_guard<std::mutex> rlk(g_ring_mu);
  if (!Lp && c->last < 0) return ART_OK;
  LaunchRec& L = Lp ? *Lp : c->ring[c->last];
  HIP_OK(hipEventSynchronize(L.done));
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, L.ev0, L.ev1));
  g_last_ms = ms;
  g_last_grid = L.grid;
  for (int i = 0; i < art::N_STATS; ++i) g_last_stats[i] = L.host_stats[i];
  L.held.store(false, std::memory_order_release);
  return ART_OK;
}
int finish_timing(DeviceCtx* c) { return finish_timing_slot(c, nullptr); }

// Latch several propagate launches (the chunks of one host call) as one: their integrator
// kernels' summed durations and summed statistics.
int finish_timing_sum(DeviceCtx* c, const std::vector<int>& slots) {
  std::lock_guard<std::mutex> rlk(g_ring_mu);
  double ms_sum = 0.0;
  unsigned long long st[art::N_STATS] = {0};
  int grid = 0;
  for (int i : slots) {
    LaunchRec& L = c->ring[i];
    HIP_OK(hipEventSynchronize(L.done));
    float ms = 0.f;
    HIP_OK(hipEventElapsedTime(&ms, L.ev0, L.ev1));
    ms_sum += ms;
    for (int k = 0; k < art::N_STATS; ++k) st[k] += L.host_stats[k];
    grid = std::max(grid, L.grid);
  }
  g_last_ms = ms_sum;
  g_last_grid = grid;
  for (int k = 0; k < art::N_STATS; ++k) g_last_stats[k] = st[k];
  return ART_OK;
}

}  // namespace

extern "C" {

int art_abi_version(void) { return ART_ABI_VERSION; }
const char* art_last_error(void) { return g_err.c_str(); }

int art_device_count(int32_t* count) {
  int n = 0;
  HIP_OK(hipGetDeviceCount(&n));
  if (count) *count = n;
  return ART_OK;
}

int art_set_device(int32_t device) {
  std::lock_guard<std::mutex> lk(g_mu);
  HIP_OK(hipSetDevice(device));
  return ART_OK;
}

int art_set_tail_donation(int32_t lanes) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (lanes < -1 || lanes > 63) return fail(ART_E_INVALID, "tail donation lanes must be in [-1, 63]");
  DeviceCtx* c;
  int rc = current_ctx(&c);
  if (rc) return rc;
  c->donate = lanes;
  return ART_OK;
}

int art_set_graduation(int32_t attempts) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (attempts < -1) return fail(ART_E_INVALID, "graduation attempts must be >= -1");
  DeviceCtx* c;
  int rc = current_ctx(&c);
  if (rc) return rc;
  c->graduate = attempts;
  return ART_OK;
}

int art_set_sampler_waves(int32_t waves) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (waves != 0 && waves != 2 && waves != 3) return fail(ART_E_INVALID, "sampler waves must be 0, 2 or 3");
  DeviceCtx* c;
  int rc = current_ctx(&c);
  if (rc) return rc;
  c->sampler_waves = waves;
  return ART_OK;
}

int art_synchronize(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceCtx* c;
  int rc = current_ctx(&c);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(c->stream));
  HIP_OK(hipDeviceSynchronize());
  return finish_timing(c);
}

double art_last_kernel_ms(void) { return g_last_ms; }

// Statistics of the last propagate launch (after art_synchronize / a host entry point):
// [attempts, accepted, root re-steps, scan condition evals, interpolant-root evals, rays,
//  init RHS evals, reserved]; grid = persistent grid size.
int art_last_stats(uint64_t* stats, int32_t* grid) {
  for (int i = 0; i < art::N_STATS; ++i) stats[i] = g_last_stats[i];
  if (grid) *grid = g_last_grid;
  return ART_OK;
}

// Integrator-kernel durations [ms] of the last min(n, issued, RING) propagate launches on the
// current device, oldest first (each from the HIP events around that launch on its own
// stream); waits for them. Returns the count written, or a negative ART_E* code.
int art_recent_kernel_ms(int32_t n, double* ms) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceCtx* c;
  int rc = current_ctx(&c);
  if (rc) return rc;
  if (n < 0 || (n > 0 && !ms)) return fail(ART_E_INVALID, "bad buffer");
  std::lock_guard<std::mutex> rlk(g_ring_mu);
  int64_t m = n;
  if (m > c->launches) m = c->launches;
  if (m > RING) m = RING;
  for (int64_t j = 0; j < m; ++j) {
    LaunchRec& L = c->ring[(int)(((int64_t)c->last - (m - 1 - j) + RING) % RING)];
    HIP_OK(hipEventSynchronize(L.done));
    float f = 0.f;
    HIP_OK(hipEventElapsedTime(&f, L.ev0, L.ev1));
    ms[j] = f;
  }
  return (int)m;
}

// The same launches' integrator spans [ms] from in-kernel clock stamps (first wave start to last
// wave end, s_memrealtime at 100 MHz; -1 where a launch left none). Returns the count written.
int art_recent_kernel_span_ms(int32_t n, double* ms) {
  std::lock_guard<std::mutex> lk(g_mu);
  DeviceCtx* c;
  int rc = current_ctx(&c);
  if (rc) return rc;
  if (n < 0 || (n > 0 && !ms)) return fail(ART_E_INVALID, "bad buffer");
  std::lock_guard<std::mutex> rlk(g_ring_mu);
  int64_t m = n;
  if (m > c->launches) m = c->launches;
  if (m > RING) m = RING;
  for (int64_t j = 0; j < m; ++j) {
    LaunchRec& L = c->ring[(int)(((int64_t)c->last - (m - 1 - j) + RING) % RING)];
    HIP_OK(hipEventSynchronize(L.done));
    const unsigned long long t0 = ~L.host_stats[art::ST_T0], t1 = L.host_stats[art::ST_T1];
    // (-1 also for an asynchronous call still in flight: its stamps are latched at its end)
    ms[j] = (L.held.load(std::memory_order_acquire) || L.host_stats[art::ST_T0] == 0ull || t1 < t0)
                ? -1.0
                : (double)(t1 - t0) / art::STAMP_TICKS_PER_MS;
  }
  return (int)m;
}

int art_vern6_tableau(double* c, double* A, double* b, double* bhat) {
  using V = art::Vern6;
  const double cc[9] = {0.0, V::c2, V::c3, V::c4, V::c5, V::c6, V::c7, 1.0, 1.0};
  double AA[9][9] = {{0}};
  AA[1][0] = V::a21;
  AA[2][0] = V::a31; AA[2][1] = V::a32;
  AA[3][0] = V::a41; AA[3][2] = V::a43;
  AA[4][0] = V::a51; AA[4][2] = V::a53; AA[4][3] = V::a54;
  AA[5][0] = V::a61; AA[5][2] = V::a63; AA[5][3] = V::a64; AA[5][4] = V::a65;
  AA[6][0] = V::a71; AA[6][2] = V::a73; AA[6][3] = V::a74; AA[6][4] = V::a75; AA[6][5] = V::a76;
  AA[7][0] = V::a81; AA[7][2] = V::a83; AA[7][3] = V::a84; AA[7][4] = V::a85; AA[7][5] = V::a86; AA[7][6] = V::a87;
  AA[8][0] = V::a91; AA[8][3] = V::a94; AA[8][4] = V::a95; AA[8][5] = V::a96; AA[8][6] = V::a97; AA[8][7] = V::a98;
  const double bh[9] = {V::bh1, 0, 0, V::bh4, V::bh5, V::bh6, 0, V::bh8, V::bh9};
  for (int i = 0; i < 9; ++i) {
    c[i] = cc[i];
    b[i] = AA[8][i];
    bhat[i] = bh[i];
    for (int j = 0; j < 9; ++j) A[9 * i + j] = AA[i][j];
  }
  return ART_OK;
}

double art_find_conversion_surface(const art_params* p) {
  // Find_Conversion_Surface (RayTracer.jl:1250-1263) with fix_time = 0: ωp at the surface
  // point in the plane of the magnetic axis, then rNS (ωp/m_a)^(2/3) * 1.01.
  const double th = p->theta_m < art::PI / 2.0 ? p->theta_m / 2.0 : (p->theta_m + art::PI) / 2.0;
  const double x[3] = {p->rNS * std::sin(th), 0.0, p->rNS * std::cos(th)};
  const double r = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  const double ph = std::atan2(x[1], x[0]);
  const double t = std::acos(x[2] / r);
  const double psi = ph;
  const double Bn = p->B0 * std::pow(p->rNS / r, 3) / 2.0;
  const double Br = 2.0 * Bn * (std::cos(p->theta_m) * std::cos(t) + std::sin(p->theta_m) * std::sin(t) * std::cos(psi));
  const double Bt = Bn * (std::cos(p->theta_m) * std::sin(t) - std::sin(p->theta_m) * std::cos(t) * std::cos(psi));
  const double Bz = Br * std::cos(t) - Bt * std::sin(t);
  const double ne = std::fabs(2.0 * p->omega_pul * Bz / std::sqrt(4 * art::PI / 137) * 1.95e-2 * art::HBAR);
  const double wp = std::sqrt(4 * art::PI * ne / 137 / 5.0e5);
  return p->rNS * std::pow(wp / p->mass_a, 2.0 / 3.0) * 1.01;
}

int art_propagate_device(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                         const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                         art_segment_out* out, art_crossing_buf* xc, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  return propagate_device_impl(p, n, x0, k0, erg, dw, ln_t0, species, max_crossings, out, xc, stream);
}

int art_propagate_traj_device(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                              const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                              art_segment_out* out, art_crossing_buf* xc, int32_t ntimes, double* traj,
                              double* traj_t, int32_t* traj_n, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (ntimes < 2) return fail(ART_E_INVALID, "ntimes must be >= 2");
  TrajArgs tr;
  tr.ntimes = ntimes; tr.traj = traj; tr.t = traj_t; tr.count = traj_n;
  return propagate_device_impl(p, n, x0, k0, erg, dw, ln_t0, species, max_crossings, out, xc, stream, tr);
}

}  // extern "C"

namespace {
// The chunked pipeline's output staging: coarse-grained (non-coherent) mapped host memory
// lets the L2 combine finalize_kernel's 8-byte stores into full-line PCIe writes; the stream
// event the host waits on makes them visible. ART_HOST_COHERENT=1: fine-grained memory (A/B).
unsigned out_coherence() {
  return env_int("ART_HOST_COHERENT", 0) ? hipHostMallocCoherent : hipHostMallocNonCoherent;
}

// art_propagate_host for large batches: a pipeline of chunks (the reference call
// site MainRunner.jl:179-190 hands over host arrays).
//   * uploads: chunk k's inputs, gathered from the caller's arrays into pinned staging by the
//     copy pool, go to HBM on one stream, all submitted up front;
//   * compute: `slots` streams, chunk k on stream k % slots, each launch waiting for its own
//     upload only, so two chunks in flight fill each other's drain tails (tail donation);
//   * downloads: none. Each chunk's finalize_kernel writes its outputs straight into mapped
//     pinned memory over PCIe (coalesced 8-byte-per-lane stores), on a stream of its own
//     after the chunk's integrator kernels, so the outputs leave while the compute stream
//     goes on with its next chunk, and no copy waits behind a kernel.
// The host scatters the chunks' outputs into the caller's arrays in order while the later
// ones still compute. Only the first chunk's upload and the last chunk's finalize and
// scatter are not hidden behind compute, so those two chunks are a quarter of the others.
// Each chunk's scratch is carved from one preallocated buffer (a stream-ordered allocation
// per chunk blocked the submitting thread once several chunks were in flight).
// Earlier versions and why they lost (profiles/r03o_host_timeline.txt,
// profiles/r03p_host_timeline.txt, profiles/r03q_host_timeline.txt): copies on the compute
// streams (an upload waited behind the previous chunk's download on its stream), then on
// their own streams but submitted per chunk (the runtime keeps copies in submission order, so
// a download held the next uploads back until its chunk was computed), then downloads as
// copies after all uploads (the downloads ran as blit kernels competing with the compute for
// CUs, 4-15 ms per chunk). Per-ray results do not depend on the batch split
// (tests/test_edges.py), so the outputs equal the single launch's bit for bit. The statistics
// and kernel time of the call are the sums over its chunks.
int propagate_host_chunked(DeviceCtx* c, const art_params* p, int64_t n, const double* x0, const double* k0,
                           const double* erg, const double* dw, const double* ln_t0, const int8_t* species,
                           int32_t max_crossings, art_segment_out* out, art_crossing_buf* xc, int nchunks,
                           int nslots, const FluxArgs& fx) {
  const int cap = (xc && xc->count) ? xc->capacity : 0;
  const int64_t K = std::max(2, nchunks);
  const art::KParams KP = kparams(*p);
  auto up = [](size_t b) { return (b + 255) & ~size_t(255); };
  // blob layouts of a chunk of m rays (inputs: pinned staging and HBM; outputs: pinned)
  auto in_bytes = [&](int64_t m) { return up((size_t)m * 9 * sizeof(double)) + up((size_t)m); };
  auto cnt_off = [&](int64_t m) { return up((size_t)m * 8 * sizeof(double) + (size_t)m * 3 * sizeof(int32_t)); };
  auto xd_off = [&](int64_t m) { return cnt_off(m) + up((size_t)m * sizeof(int32_t)); };
  auto out_bytes = [&](int64_t m) { return cap ? xd_off(m) + (size_t)cap * m * 9 * sizeof(double) : cnt_off(m); };
  // chunk boundaries: weights 1/4, 1, ..., 1, 1/4
  std::vector<int64_t> lo(K + 1);
  const double wsum = 0.5 + double(K - 2);
  for (int64_t k = 0; k <= K; ++k) {
    const double wk = k == 0 ? 0.0 : (k == K ? wsum : 0.25 + double(k - 1));
    lo[k] = (int64_t)((double)n * (wk / wsum));
  }
  lo[K] = n;
  const int32_t donate = nslots > 1 ? 16 : 0;
  std::vector<size_t> ioff(K + 1, 0), ooff(K + 1, 0), soff(K + 1, 0);
  for (int64_t k = 0; k < K; ++k) {
    const int64_t m = lo[k + 1] - lo[k];
    // the same layout propagate_device_impl will carve out of this chunk's slice (a chunk small
    // enough for the tail kernel keeps one donation record per ray, whatever `donate` says)
    const bool st = use_small_tail(p, m, TrajArgs());
    ScratchLayout SL;
    int rc0 = scratch_layout(c, m, cap, st ? 0 : donate, &SL, st);
    if (rc0) return rc0;
    ioff[k + 1] = ioff[k] + in_bytes(m);
    ooff[k + 1] = ooff[k] + out_bytes(m);
    soff[k + 1] = soff[k] + up(SL.total());
  }
  while ((int)c->pstreams.size() < nslots) {
    hipStream_t st = c->stream;
    if (!c->pstreams.empty()) HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    c->pstreams.push_back(st);
  }
  if (!c->h2d) HIP_OK(hipStreamCreateWithFlags(&c->h2d, hipStreamNonBlocking));
  if (!c->fin) HIP_OK(hipStreamCreateWithFlags(&c->fin, hipStreamNonBlocking));
  while ((int64_t)c->pev.size() < 2 * K) {
    hipEvent_t ev;
    HIP_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    c->pev.push_back(ev);
  }
  hipEvent_t *ev_in = c->pev.data(), *ev_done = ev_in + K;
  int rc;
  void *pi, *po, *di_, *sc_;
  if ((rc = pinned_get(c, 0, ioff[K], &pi)) ||
      (rc = pinned_get(c, 1, ooff[K], &po, hipHostMallocMapped | out_coherence())) ||
      (rc = pool_get(c, 16, ioff[K], &di_)) || (rc = pool_get(c, 17, soff[K], &sc_)))
    return rc;
  void* po_dev = nullptr;
  HIP_OK(hipHostGetDevicePointer(&po_dev, po, 0));
  char *pin_in = (char*)pi, *pin_out = (char*)po, *out_dev = (char*)po_dev, *dev_in = (char*)di_, *scratch = (char*)sc_;
  double* hist_dev = nullptr;
  if (fx.nbins) {
    if ((rc = pool_get(c, 23, 2 * (size_t)fx.nbins * sizeof(double), (void**)&hist_dev))) return rc;
    HIP_OK(hipMemsetAsync(hist_dev, 0, 2 * (size_t)fx.nbins * sizeof(double), c->fin));
  }
  using Seg = CopyPool::Seg;
  std::vector<int> rings;
  // ART_HOST_TRACE=1: the host side of every chunk to stderr (gathers, submits, waits, scatters)
  const bool trace = env_int("ART_HOST_TRACE", 0) != 0;
  auto clk = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t_start = clk();
  // Submission order: upload 0, compute 0, the other uploads, the other computes (the
  // runtime keeps copies in submission order, so no upload waits behind anything).
  auto upload = [&](int64_t k) -> int {
    const int64_t l0 = lo[k], m = lo[k + 1] - lo[k];
    char* bi = pin_in + ioff[k];
    double* d = (double*)bi;
    std::vector<Seg> g;
    for (int q = 0; q < 3; ++q) {
      g.push_back({d + q * m, x0 + q * n + l0, m * sizeof(double)});
      g.push_back({d + (3 + q) * m, k0 + q * n + l0, m * sizeof(double)});
    }
    g.push_back({d + 6 * m, erg + l0, m * sizeof(double)});
    g.push_back({d + 7 * m, dw + l0, m * sizeof(double)});
    g.push_back({d + 8 * m, ln_t0 + l0, m * sizeof(double)});
    g.push_back({bi + up((size_t)m * 9 * sizeof(double)), species + l0, (size_t)m});
    const double tg0 = clk();
    copy_pool().run(g);
    const double tg1 = clk();
    HIP_OK(hipMemcpyAsync(dev_in + ioff[k], bi, in_bytes(m), hipMemcpyHostToDevice, c->h2d));
    HIP_OK(hipEventRecord(ev_in[k], c->h2d));
    if (trace)
      std::fprintf(stderr, "[art-host] t=%.2f upload lo=%lld m=%lld gather %.2f ms submit %.2f ms\n", tg0 - t_start,
                   (long long)l0, (long long)m, tg1 - tg0, clk() - tg1);
    return ART_OK;
  };
  auto compute = [&](int64_t k) -> int {
    const double t0 = clk();
    hipStream_t st = c->pstreams[k % nslots];
    const int64_t m = lo[k + 1] - lo[k];
    const double* di = (const double*)(dev_in + ioff[k]);
    char* dbo = out_dev + ooff[k];  // device view of the chunk's pinned outputs
    HIP_OK(hipStreamWaitEvent(st, ev_in[k], 0));
    double* dd = (double*)dbo;
    int32_t* di32 = (int32_t*)(dd + 8 * m);
    art_segment_out dso{dd, dd + 3 * m, dd + 6 * m, dd + 7 * m, di32, di32 + m, di32 + 2 * m};
    art_crossing_buf dxb{};
    art_crossing_buf* dxbp = nullptr;
    if (cap) {
      int32_t* cnt = (int32_t*)(dbo + cnt_off(m));
      double* x = (double*)(dbo + xd_off(m));
      dxb = art_crossing_buf{cap, cnt, x, x + 3 * cap * m, x + 6 * cap * m, x + 7 * cap * m, x + 8 * cap * m};
      dxbp = &dxb;
    }
    LaunchOpts lo_;
    lo_.donate = donate;
    lo_.scratch = scratch + soff[k];
    lo_.scratch_bytes = soff[k + 1] - soff[k];
    lo_.nan_fill = true;
    lo_.finalize_stream = c->fin;
    const int8_t* dsp = (const int8_t*)((const char*)di + up((size_t)m * 9 * sizeof(double)));
    int rc2 = propagate_device_impl(p, m, di, di + 3 * m, di + 6 * m, di + 7 * m, di + 8 * m, dsp, max_crossings,
                                    &dso, dxbp, st, TrajArgs(), lo_);
    if (rc2) return rc2;
    if (fx.nbins)  // the chunk's flux from its outputs (mapped pinned memory), behind its finalize
      HIP_OK(art::launch_flux(KP, m, dso.x_end, dso.k_end, dso.status, dsp, nullptr, fx.nbins, hist_dev, c->fin));
    rings.push_back(c->last);
    HIP_OK(hipEventRecord(ev_done[k], c->fin));
    if (trace) std::fprintf(stderr, "[art-host] t=%.2f compute k=%lld submit %.2f ms\n", t0 - t_start, (long long)k, clk() - t0);
    return ART_OK;
  };
  if ((rc = upload(0)) || (rc = compute(0))) return rc;
  for (int64_t k = 1; k < K; ++k)
    if ((rc = upload(k))) return rc;
  for (int64_t k = 1; k < K; ++k)
    if ((rc = compute(k))) return rc;
  // the chunks' outputs, in order: pinned staging -> the caller's arrays
  for (int64_t k = 0; k < K; ++k) {
    const double tw0 = clk();
    HIP_OK(hipEventSynchronize(ev_done[k]));
    const double tw1 = clk();
    const int64_t l0 = lo[k], m = lo[k + 1] - lo[k];
    const char* bo = pin_out + ooff[k];
    const double* d = (const double*)bo;
    const int32_t* i32 = (const int32_t*)(d + 8 * m);
    std::vector<Seg> g;
    for (int q = 0; q < 3; ++q) {
      g.push_back({out->x_end + q * n + l0, d + q * m, m * sizeof(double)});
      g.push_back({out->k_end + q * n + l0, d + (3 + q) * m, m * sizeof(double)});
    }
    g.push_back({out->u7_end + l0, d + 6 * m, m * sizeof(double)});
    g.push_back({out->tau_end + l0, d + 7 * m, m * sizeof(double)});
    g.push_back({out->status + l0, i32, m * sizeof(int32_t)});
    g.push_back({out->n_accept + l0, i32 + m, m * sizeof(int32_t)});
    g.push_back({out->n_reject + l0, i32 + 2 * m, m * sizeof(int32_t)});
    if (cap) {
      g.push_back({xc->count + l0, bo + cnt_off(m), m * sizeof(int32_t)});
      const double* x = (const double*)(bo + xd_off(m));
      // rows of [(comp * cap + j) * n + ray]: 3 cap rows of pos, of k, cap rows of t, dw, P
      for (int r = 0; r < 3 * cap; ++r) {
        g.push_back({xc->pos + r * n + l0, x + r * m, m * sizeof(double)});
        g.push_back({xc->k + r * n + l0, x + (3 * cap + r) * m, m * sizeof(double)});
      }
      for (int r = 0; r < cap; ++r) {
        g.push_back({xc->t + r * n + l0, x + (6 * cap + r) * m, m * sizeof(double)});
        g.push_back({xc->dw + r * n + l0, x + (7 * cap + r) * m, m * sizeof(double)});
        g.push_back({xc->p_nonad + r * n + l0, x + (8 * cap + r) * m, m * sizeof(double)});
      }
    }
    copy_pool().run(g);
    if (trace)
      std::fprintf(stderr, "[art-host] t=%.2f drain lo=%lld wait %.2f ms scatter %.2f ms\n", tw0 - t_start,
                   (long long)l0, tw1 - tw0, clk() - tw1);
  }
  if (trace) std::fprintf(stderr, "[art-host] total %.2f ms\n", clk() - t_start);
  if (fx.nbins) {
    HIP_OK(hipMemcpyAsync(fx.hist, hist_dev, 2 * (size_t)fx.nbins * sizeof(double), hipMemcpyDeviceToHost, c->fin));
    HIP_OK(hipStreamSynchronize(c->fin));
  }
  return finish_timing_sum(c, rings);
}

// The streamed pipeline gave up (a wave waited too long for its inputs, or a piece for its
// signal): the call's results are discarded and the batch runs again on another path.
constexpr int STREAM_FALLBACK = 1 << 20;

// art_propagate_host for large batches, streamed with no CU reserved (the default; SURVEY §8b,
// the reference call site MainRunner.jl:179-190 hands over host arrays). ONE integrator launch
// (propagate_kernel<..., DON = 3>) holds every CU for the whole batch; nothing else needs a CU
// while it runs:
//   * the host gathers piece k from the caller's arrays into pinned staging (copy pool) and
//     copies it to HBM on the upload stream (DMA engines:
//     profiles/r04k_probe_*.jsonl -- 64 MB copies finish at 56 GB/s under a kernel holding
//     every CU); a host thread raises the ready counter (host memory) as each piece lands;
//   * persistent helper blocks (helper_kernel HK_TILES, a separate kernel on a stream of its own,
//     resident beside the integrator) initialise 1024-ray tiles whose inputs have landed
//     (init_one, the init_kernel arithmetic) and flag their chunks; a wave that claims a
//     chunk of 64 rays waits for its flag. Once every ray of a piece has finished, helpers
//     finalize its tiles (finalize_one) into the piece's SoA blob in HBM, and the block that
//     finalizes its last tile raises the piece's flag (host memory);
//   * the host polls the flags, copies each finished blob to pinned memory (DMA engines) and
//     scatters it into the caller's arrays.
// Before the integrator, one helper_kernel pass on the integrator's stream initialises the first
// rays with every block slot; after it, one more pass finalizes what is left.
// Round 3's CU-masked pipeline ran the init and finalize kernels on 8 reserved CUs, which cost
// ~10% of the integrator (profiles/r04g_stream_anatomy.jsonl); it is gone. Per-ray results
// equal the single launch's bit for bit.
// The HostLane words the GPU reads and writes over PCIe: [0] the ready counter | [8, 8 + 64)
// the piece flags | [72] helper blocks started | [76] the last integrator fully resident on the
// GPU (ticket + 1; never reset) | [HSIG_DONE, ...) SegOut::done_host (the flag, the statistics,
// the flux)
constexpr int HSIG_NFLAG = 64, HSIG_RESIDENT = 76, HSIG_DONE = 80;
constexpr size_t HSIG_WORDS = HSIG_DONE + art::DONE_FLUX + 2 * art::FLUX_HELPER_BINS;

int lane_setup(DeviceCtx* c, HostLane* H) {
  if (!H->m_comp) {
    // the integrator's and the persistent helpers' streams each on a hardware queue of its own
    // (a stream with a CU mask gets one; here the mask holds every CU): plain streams share the
    // process's few queues (GPU_MAX_HW_QUEUES), and a stream queued behind a persistent kernel
    // waits for that kernel to end -- the integrator behind the helpers never started
    // (profiles/r04p_maskless_hwqueue.txt)
    int ncu_all = 0;
    HIP_OK(hipDeviceGetAttribute(&ncu_all, hipDeviceAttributeMultiprocessorCount, c->device));
    std::vector<uint32_t> all((ncu_all + 31) / 32, 0u);
    for (int i = 0; i < ncu_all; ++i) all[i / 32] |= 1u << (i % 32);
    HIP_OK(hipExtStreamCreateWithCUMask(&H->m_comp, (uint32_t)all.size(), all.data()));
    HIP_OK(hipExtStreamCreateWithCUMask(&H->m_help, (uint32_t)all.size(), all.data()));
    HIP_OK(hipStreamCreateWithFlags(&H->m_up, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&H->m_dn, hipStreamNonBlocking));
  }
  if (!H->hsig) {
    unsigned long long* hs = nullptr;
    HIP_OK(hipHostMalloc((void**)&hs, sizeof(unsigned long long) * HSIG_WORDS, hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(hs, 0, sizeof(unsigned long long) * HSIG_WORDS);  // ([HSIG_RESIDENT] is never reset)
    HIP_OK(hipHostGetDevicePointer((void**)&H->hsig_dev, hs, 0));
    // (published last, with release: another lane's worker reads the pointer in prev_resident)
    __atomic_store_n(&H->hsig, hs, __ATOMIC_RELEASE);
  }
  if (!H->abort_host) {
    HIP_OK(hipHostMalloc((void**)&H->abort_host, 64, hipHostMallocCoherent | hipHostMallocMapped));
    HIP_OK(hipHostGetDevicePointer((void**)&H->abort_dev, H->abort_host, 0));
  }
  return ART_OK;
}

// Latch one launch's statistics (the ring entry's, for art_recent_kernel_*; and the "last
// launch" figures of art_last_stats / art_last_kernel_ms) from words the host already holds.
int latch_launch(DeviceCtx* c, LaunchRec* L, const unsigned long long* st) {
  std::lock_guard<std::mutex> rlk(g_ring_mu);
  for (int i = 0; i < art::N_STATS_DEV; ++i) L->host_stats[i] = st[i];
  HIP_OK(hipEventSynchronize(L->ev1));
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, L->ev0, L->ev1));
  g_last_ms = ms;
  g_last_grid = L->grid;
  for (int i = 0; i < art::N_STATS; ++i) g_last_stats[i] = st[i];
  L->held.store(false, std::memory_order_release);
  return ART_OK;
}

int propagate_host_maskless(DeviceCtx* c, HostLane* H, bool overlap, int64_t ticket, const art_params* p, int64_t n,
                            const double* x0,
                            const double* k0, const double* erg, const double* dw, const double* ln_t0,
                            const int8_t* species, int32_t max_crossings, art_segment_out* out, art_crossing_buf* xc,
                            const FluxArgs& fx) {
  const int cap = (xc && xc->count) ? xc->capacity : 0;
  const art::KParams K = kparams(*p);
  int shift = 16;
  while (((int64_t)1 << (shift + 1)) * 32 <= n) ++shift;  // 32..64 pieces (2^18 rays for 10^7: the last
  // piece's finalize, copy and scatter are the call's tail, 95.3-96.5 ms against 98.4-101 with 2^19,
  // profiles/r04ag_piece_shift.jsonl)
  if (const int e = env_int("ART_HOST_PIECE_SHIFT", 0)) shift = std::max(10, e);  // (tests: many small pieces)
  while (((n + ((int64_t)1 << shift) - 1) >> shift) > HSIG_NFLAG) ++shift;  // 64 piece counters and flags
  const int np = (int)((n + ((int64_t)1 << shift) - 1) >> shift);
  int rc;
  if ((rc = lane_setup(c, H))) return rc;
  const size_t nd = (size_t)n;
  auto up = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t in_bytes = nd * 9 * sizeof(double) + nd;  // x0 (3n) k0 (3n) erg dw lnt0 | species
  // per-piece SoA output blobs, pinned and in HBM: the layout piece_blob (art_kernels.hip) computes
  auto piece_lo = [&](int k) { return std::min((int64_t)k << shift, n); };
  auto cnt_off = [&](int64_t m) { return up((size_t)m * 8 * sizeof(double) + (size_t)m * 3 * sizeof(int32_t)); };
  auto xd_off = [&](int64_t m) { return cnt_off(m) + up((size_t)m * sizeof(int32_t)); };
  auto out_bytes = [&](int64_t m) { return cap ? xd_off(m) + (size_t)cap * m * 9 * sizeof(double) : cnt_off(m); };
  const size_t stride = up(out_bytes((int64_t)1 << shift));
  // scratch: head [queue | stats (10) | init_next (16) fin_next (17) chunk misses (18) exit count (19) waves done (20)
  // waves started (21) |
  // finished rays per piece from word 32 | finalized tiles per piece from word 96] | chunk flags | u0 U0_REC n | rec 16n | xrec
  const size_t nchunk = (nd + art::CHUNK - 1) / art::CHUNK;
  const size_t head = 2048, ccb = up(nchunk * sizeof(unsigned)), u0b = nd * art::U0_REC * sizeof(double),
               recb = nd * art::END_REC * sizeof(double);
  const size_t xrb = (size_t)cap * nd * art::X_REC * sizeof(double);
  // ART_HOST_DIRECT=1: the pieces' output blobs in pinned host memory (fine-grained), written by the
  // helpers over PCIe and scattered as soon as a piece is flagged -- no download copies (which a
  // profiler's tracing turns into blit kernels competing for CU slots)
  const bool direct = env_int("ART_HOST_DIRECT", 0) != 0;
  void *pi, *po, *din, *dout, *dsc;
  if ((rc = pinned_get_v(H->pinned, 0, in_bytes, &pi)) ||
      (rc = pinned_get_v(H->pinned, 1, stride * np, &po,
                         direct ? (hipHostMallocMapped | hipHostMallocCoherent) : hipHostMallocDefault)) ||
      (rc = pool_get_v(H->pool, 0, in_bytes, &din)) ||
      (!direct && (rc = pool_get_v(H->pool, 1, stride * np, &dout))) ||
      (rc = pool_get_v(H->pool, 2, head + ccb + u0b + recb + xrb, &dsc)))
    return rc;
  if (direct) HIP_OK(hipHostGetDevicePointer(&dout, po, 0));
  double* pin = (double*)pi;
  double* di = (double*)din;
  unsigned long long* words = (unsigned long long*)dsc;
  unsigned* ccnt = (unsigned*)((char*)dsc + head);
  double* u0 = (double*)((char*)dsc + head + ccb);
  double* rec = (double*)((char*)dsc + head + ccb + u0b);
  double* xrec = cap ? (double*)((char*)dsc + head + ccb + u0b + recb) : nullptr;
  const art::SegIn in{di, di + 3 * nd, di + 6 * nd, di + 7 * nd, di + 8 * nd, (const int8_t*)(di + 9 * nd), u0};
  // upload units (independent of the output pieces): a small first one (2^16 rays, the
  // integrator starts soon), then units of max(2^18 rays, a piece) -- each unit costs ~0.2 ms of
  // host-side submission, which small pieces made the bound of a 1.25e6-ray call's uploads
  // (ART_HOST_FIRST_UNIT / ART_HOST_UNIT: tests, other sizes in rays)
  std::vector<int64_t> ulo{0};
  const int64_t ustep = std::max(1, env_int("ART_HOST_UNIT", (int)std::max((int64_t)1 << 18, (int64_t)1 << shift)));
  for (int64_t lo = std::min(n, (int64_t)std::max(1, env_int("ART_HOST_FIRST_UNIT", 1 << 16))); ;
       lo = std::min(n, lo + ustep)) {
    ulo.push_back(lo);
    if (lo >= n) break;
  }
  const int nu = (int)ulo.size() - 1;
  while ((int64_t)H->pev.size() < nu + np + 2) {
    hipEvent_t ev;
    HIP_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    H->pev.push_back(ev);
  }
  hipEvent_t* ev_up = H->pev.data();
  hipEvent_t* ev_dn = H->pev.data() + nu;
  const bool trace = env_int("ART_HOST_TRACE", 0) != 0;
  auto clk = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t_start = clk();
  unsigned long long* hready = H->hsig;
  unsigned long long* hflag = H->hsig + 8;
  unsigned long long* hdone = H->hsig + HSIG_DONE;
  __atomic_store_n(hready, 0ull, __ATOMIC_RELEASE);
  for (int k = 0; k <= HSIG_NFLAG; ++k) __atomic_store_n(hflag + k, 0ull, __ATOMIC_RELEASE);  // (+ the started count)
  __atomic_store_n(hdone, 0ull, __ATOMIC_RELEASE);
  __atomic_store_n(H->abort_host, 0u, __ATOMIC_RELEASE);
  // The host gathers the upload units from the caller's arrays into pinned staging on a thread of
  // its own, from the call's first moment: the set-up and launches below (~1.5 ms at 1.25e6 rays)
  // and the first units' gathers overlap instead of adding up (profiles/r05d_shard_if1_trace.err).
  // (tests: ART_HOST_UPLOAD_DELAY_MS holds back the second upload unit, so the integrator's
  // waves outwait their 2 s bound and the device side gives the call up)
  const int delay_ms = env_int("ART_HOST_UPLOAD_DELAY_MS", 0);
  std::atomic<int> gathered{0};
  std::atomic<bool> gstop{false};
  std::thread gatherer([&] {
    using Seg = CopyPool::Seg;
    for (int u = 0; u < nu && !gstop.load(); ++u) {
      if (delay_ms > 0 && u == 1)
        for (int w = 0; w < delay_ms && !gstop.load(); ++w) std::this_thread::sleep_for(std::chrono::milliseconds(1));
      const int64_t lo = ulo[u], m = ulo[u + 1] - lo;
      const double* src[9] = {x0, x0 + n, x0 + 2 * n, k0, k0 + n, k0 + 2 * n, erg, dw, ln_t0};
      std::vector<Seg> g;
      for (int r = 0; r < 9; ++r) g.push_back({pin + r * nd + lo, src[r] + lo, (size_t)m * sizeof(double)});
      g.push_back({(int8_t*)(pin + 9 * nd) + lo, species + lo, (size_t)m});
      const double tg0 = clk();
      copy_pool().run(g);
      gathered.store(u + 1, std::memory_order_release);
      if (trace) std::fprintf(stderr, "[art-host] t=%.2f unit %d gathered in %.2f ms\n", tg0 - t_start, u, clk() - tg0);
    }
  });
  // (every return below, the early ones of HIP_OK included, stops and joins the gatherer first)
  struct JoinOnExit {
    std::atomic<bool>& stop;
    std::thread& t;
    ~JoinOnExit() {
      stop = true;
      if (t.joinable()) t.join();
    }
  } gjoin{gstop, gatherer};
  HIP_OK(hipMemsetAsync(words, 0, head + ccb, H->m_comp));
  // the batch's flux: binned by the helpers as they finalize (bins <= FLUX_HELPER_BINS), else by
  // flux kernels over the pieces' blobs after the integrator
  const bool hflux = fx.nbins > 0 && fx.nbins <= art::FLUX_HELPER_BINS;
  double* hist_dev = nullptr;
  if (fx.nbins) {
    if ((rc = pool_get_v(H->pool, 3, 2 * (size_t)fx.nbins * sizeof(double), (void**)&hist_dev))) return rc;
    HIP_OK(hipMemsetAsync(hist_dev, 0, 2 * (size_t)fx.nbins * sizeof(double), H->m_comp));
  }
  art::SegOut so{};
  so.rec = rec;
  so.cap = cap;
  so.xrec = xrec;
  so.xcount = cap ? (int32_t*)((char*)dout + cnt_off(piece_lo(1) - piece_lo(0))) : nullptr;  // (tested for null only)
  so.piece_cnt = words + 32;
  so.abort_word = H->abort_dev;
  so.queue_word = words;
  // (tests: ART_HOST_WAVE_WAIT_MS shortens a wave's bound on its chunk, s_memrealtime at 100 MHz)
  so.wait_ticks = env_int("ART_HOST_WAVE_WAIT_MS", 0) > 0 ? (unsigned long long)env_int("ART_HOST_WAVE_WAIT_MS", 0) * 100000ull
                                                         : art::STREAM_WAIT_TICKS;
  so.piece_shift = shift;
  so.host_ready = H->hsig_dev;
  so.host_flags = H->hsig_dev + 8;
  so.init_next = words + 16;
  so.fin_next = words + 17;
  so.piece_fin = words + 96;
  so.chunk_ready = ccnt;
  so.blob = (char*)dout;
  so.blob_host = direct ? 1 : 0;
  so.blob_stride = (int64_t)stride;
  so.flux_hist = hflux ? hist_dev : nullptr;
  so.flux_nbins = hflux ? fx.nbins : 0;
  so.done_host = H->hsig_dev + HSIG_DONE;
  so.exit_count = words + 19;
  so.waves_done = words + 20;
  so.waves_started = words + 21;
  int ncu = 0;
  HIP_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device));
  const int slots = std::max(2, env_int("ART_HOST_BLOCKS", 2 * ncu));  // block slots: 2 per CU
  // helper blocks beside the integrator (ART_HOST_HELPERS, default 16): launched first, and the
  // integrator only once every one of them is resident, so it cannot take their slots. Each helper
  // block (2 waves per SIMD, the top issue priority) shares a CU with one integrator block, so it
  // costs one integrator block slot, not a CU: 1e7 rays, 3 rounds on one box, the integrator 92.1-
  // 93.4 -> 88.2-89.0 ms and the call 95.3-96.0 -> 91.1-92.1 ms with 16 helpers; 8 helpers let the
  // finalize lag (109 ms calls), 12 and 24 are between (profiles/r06j_helpers.jsonl)
  const int hw = art::helper_waves_per_simd(K);
  const int helpers = std::min(slots - 1, std::max(1, env_int("ART_HOST_HELPERS", hw == 2 ? 16 : 8)));
  so.helpers = helpers;
  // (dev, ART_HOST_STREAM_SERIAL=1: no persistent helpers -- every tile initialised before the
  // integrator and finalized after it, kernel by kernel: for a counter-collection run, which
  // serialises kernels; the integrator's code and traffic are the same)
  const bool serial = env_int("ART_HOST_STREAM_SERIAL", 0) != 0;
  // After the integrator, one pass of every block slot finalizes what is left -- unless this call
  // overlaps the next one (art_propagate_host_flux_async): then the next call's integrator would
  // hold those slots, and the helpers finalize alone
  const bool final_pass = serial || !overlap;
  // (a 1-wave/SIMD helper block holds a whole CU: two integrator block slots)
  const int iblocks = serial ? slots : slots - (hw == 2 ? helpers : 2 * helpers);
  so.exit_expected = (serial ? 0 : helpers) + (final_pass ? slots : 0);
  hipEvent_t ev_zero = H->pev[nu + np];  // (the helpers start on zeroed counters)
  HIP_OK(hipEventRecord(ev_zero, H->m_comp));
  HIP_OK(hipStreamWaitEvent(H->m_help, ev_zero, 0));
  if (!serial) HIP_OK(art::launch_helpers(K, n, in, so, helpers, -1, 1, words + 1, H->m_help));
  if (trace) std::fprintf(stderr, "[art-host] t=%.2f counters zeroed, helpers launched\n", clk() - t_start);
  // the integrator, once every helper block is resident: before the uploads when they are at once
  // (a lone call), else from the upload loop as soon as they are (a call overlapping the previous
  // one, whose blocks hold the slots until its drain)
  LaunchRec* L = nullptr;
  struct ReleaseRec {  // a call that leaves before latching its record frees it for take_slot
    LaunchRec*& L;
    ~ReleaseRec() {
      if (L) L->held.store(false, std::memory_order_release);
    }
  } release_rec{L};
  bool launched = false;
  auto helpers_in = [&] { return serial || __atomic_load_n(hflag + HSIG_NFLAG, __ATOMIC_ACQUIRE) >= (unsigned long long)helpers; };
  // A call in flight launches its init pass and integrator only once the previous call's integrator
  // is fully resident (its last-starting wave stores ticket + 1 into its lane's word) or that call
  // has ended: launched earlier, both integrators' blocks took the slots the call before them freed,
  // ran side by side at half speed each, and their downloads and scatters piled up at the end
  // (1.25e6 rays: calls of 28 instead of 14 ms, profiles/r05t_ab_helpers.txt). Bounded: 200 ms.
  auto prev_resident = [&] {
    if (!overlap || ticket <= 0 || c->done_ticket.load() >= ticket - 1 || clk() - t_start > 200.0) return true;
    for (const HostLane& O : c->lanes) {
      unsigned long long* const os = __atomic_load_n(&O.hsig, __ATOMIC_ACQUIRE);
      if (&O != H && os && __atomic_load_n(os + HSIG_RESIDENT, __ATOMIC_ACQUIRE) >= (unsigned long long)ticket)
        return true;
    }
    return false;
  };
  auto launch_main = [&]() -> int {
    std::lock_guard<std::mutex> rlk(g_ring_mu);
    int r = take_slot(c, &L);
    if (r) return r;
    L->held.store(true, std::memory_order_release);  // until this call latches it (or leaves early)
    // every block slot initialises the first upload unit's rays before the integrator starts, then
    // the helpers keep ahead. (Round 4 took 258k rays, two per integrator lane: the first unit alone
    // left the integrator waiting on 8 helpers, 33 ms against 18 per 1.25e6-ray call. With the
    // units gathered from the call's start, the helpers keep up, and the first unit alone starts
    // the integrator ~1 ms sooner: 1.25e6 rays 17.2 -> 16.2 ms, 1e7 95.3 -> 94.1 ms, two boxes,
    // profiles/r05l_init_pass_sweep.txt. ART_HOST_INIT_RAYS: tests and A/B, another amount)
    const int64_t first =
        serial ? n : std::min(n, (int64_t)std::max(1, env_int("ART_HOST_INIT_RAYS", (int)(ulo[1] - ulo[0]))));
    if (env_int("ART_HOST_INITPASS", 1))  // (dev: 0 leaves the first piece to the helpers)
      HIP_OK(art::launch_helpers(K, n, in, so, iblocks, first, 0, words + 1, H->m_comp));
    HIP_OK(hipEventRecord(L->ev0, H->m_comp));
    int grid = 0;
    if (overlap && ticket >= 0) {  // (see prev_resident)
      so.resident_host = H->hsig_dev + HSIG_RESIDENT;
      so.resident_value = (unsigned long long)ticket + 1ull;
      so.waves_total = (int32_t)std::min((n + 255) / 256, (int64_t)iblocks) * 4;
    }
    HIP_OK(art::launch_integrator_streamed(K, n, in, so, max_crossings, words, words + 1, iblocks, H->m_comp, &grid));
    L->grid = grid;
    HIP_OK(hipEventRecord(L->ev1, H->m_comp));
    if (final_pass) {
      HIP_OK(art::launch_helpers(K, n, in, so, slots, -1, 0, words + 1, H->m_comp));
      hipEvent_t ev_help = H->pev[nu + np + 1];  // (the persistent helpers' init counts, in the statistics)
      HIP_OK(hipEventRecord(ev_help, H->m_help));
      HIP_OK(hipStreamWaitEvent(H->m_comp, ev_help, 0));
      HIP_OK(hipMemcpyAsync(L->host_stats, words + 1, sizeof(unsigned long long) * art::N_STATS_DEV,
                            hipMemcpyDeviceToHost, H->m_comp));
    }
    // (overlapping calls: the statistics come from the helpers' completion words, and nothing
    // after the integrator waits on this stream for CU slots the next call holds)
    HIP_OK(hipEventRecord(L->done, H->m_comp));
    L->stream = H->m_comp;
    L->pending = true;
    c->last = c->next;
    c->next = (c->next + 1) % RING;
    c->launches += 1;
    launched = true;
    return ART_OK;
  };
  if ((helpers_in() && prev_resident()) || !overlap) {
    const double tw = clk();
    while (!helpers_in()) {
      if (clk() - tw > 5000.0) break;  // (never seen: the device is shared or wedged; handled below)
      std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
    if (helpers_in() && (rc = launch_main())) return rc;
    if (trace) std::fprintf(stderr, "[art-host] t=%.2f helpers resident (%.2f ms), integrator launched\n", clk() - t_start,
                            clk() - tw);
  }
  // a host thread raises the ready counter as each unit's copies land
  std::atomic<int> recorded{0};
  std::atomic<bool> stop{false};
  std::atomic<int> ready_err{0};
  std::thread readier([&] {
    for (int u = 0; u < nu && !stop.load(); ++u) {
      while (recorded.load(std::memory_order_acquire) <= u && !stop.load()) std::this_thread::sleep_for(std::chrono::microseconds(5));
      if (stop.load()) break;
      hipError_t q;  // (polled every 5 us, as the piece flags are)
      while ((q = hipEventQuery(ev_up[u])) == hipErrorNotReady && !stop.load())
        std::this_thread::sleep_for(std::chrono::microseconds(5));
      if (stop.load()) break;
      if (q != hipSuccess) {
        ready_err = 1;
        break;
      }
      __atomic_store_n(hready, (unsigned long long)ulo[u + 1], __ATOMIC_RELEASE);
      if (trace) std::fprintf(stderr, "[art-host] t=%.2f unit %d ready\n", clk() - t_start, u);
    }
  });
  using Seg = CopyPool::Seg;
  int dk = 0, sk = 0;  // pieces whose download is queued / scattered
  auto scatter = [&](int k) {
    const int64_t lo = piece_lo(k), m = piece_lo(k + 1) - lo;
    const char* bo = (const char*)po + stride * k;
    const double* d = (const double*)bo;
    const int32_t* i32 = (const int32_t*)(d + 8 * m);
    std::vector<Seg> g;
    for (int q = 0; q < 3; ++q) {
      g.push_back({out->x_end + q * n + lo, d + q * m, m * sizeof(double)});
      g.push_back({out->k_end + q * n + lo, d + (3 + q) * m, m * sizeof(double)});
    }
    g.push_back({out->u7_end + lo, d + 6 * m, m * sizeof(double)});
    g.push_back({out->tau_end + lo, d + 7 * m, m * sizeof(double)});
    g.push_back({out->status + lo, i32, m * sizeof(int32_t)});
    g.push_back({out->n_accept + lo, i32 + m, m * sizeof(int32_t)});
    g.push_back({out->n_reject + lo, i32 + 2 * m, m * sizeof(int32_t)});
    if (cap) {
      g.push_back({xc->count + lo, bo + cnt_off(m), m * sizeof(int32_t)});
      const double* x = (const double*)(bo + xd_off(m));
      for (int r = 0; r < 3 * cap; ++r) {
        g.push_back({xc->pos + r * n + lo, x + r * m, m * sizeof(double)});
        g.push_back({xc->k + r * n + lo, x + (3 * cap + r) * m, m * sizeof(double)});
      }
      for (int r = 0; r < cap; ++r) {
        g.push_back({xc->t + r * n + lo, x + (6 * cap + r) * m, m * sizeof(double)});
        g.push_back({xc->dw + r * n + lo, x + (7 * cap + r) * m, m * sizeof(double)});
        g.push_back({xc->p_nonad + r * n + lo, x + (8 * cap + r) * m, m * sizeof(double)});
      }
    }
    copy_pool().run(g);
  };
  // downloads of the finished pieces, in order; scatters of the landed ones
  auto progress = [&]() -> int {
    int moved = 0;
    while (direct && dk < np && __atomic_load_n(hflag + dk, __ATOMIC_ACQUIRE) != 0ull) {
      if (trace) std::fprintf(stderr, "[art-host] t=%.2f piece %d done\n", clk() - t_start, dk);
      ++dk;
      ++moved;
    }
    while (!direct && dk < np && __atomic_load_n(hflag + dk, __ATOMIC_ACQUIRE) != 0ull) {
      const int64_t m = piece_lo(dk + 1) - piece_lo(dk);
      if (hipMemcpyAsync((char*)po + stride * dk, (char*)dout + stride * dk, out_bytes(m), hipMemcpyDeviceToHost,
                         H->m_dn) != hipSuccess ||
          hipEventRecord(ev_dn[dk], H->m_dn) != hipSuccess)
        return -1;
      if (trace) std::fprintf(stderr, "[art-host] t=%.2f piece %d done\n", clk() - t_start, dk);
      ++dk;
      ++moved;
    }
    while (sk < dk) {
      const hipError_t q = direct ? hipSuccess : hipEventQuery(ev_dn[sk]);
      if (q == hipErrorNotReady) break;
      if (q != hipSuccess) return -1;
      const double t0 = clk();
      scatter(sk);
      if (trace) std::fprintf(stderr, "[art-host] t=%.2f piece %d scattered (%.2f ms)\n", t0 - t_start, sk, clk() - t0);
      ++sk;
      ++moved;
    }
    return moved;
  };
  int perr = 0;
  bool int_logged = false;  // (trace)
  for (int u = 0; u < nu && !perr; ++u) {
    if (!launched && helpers_in() && prev_resident() && launch_main() != ART_OK) perr = 1;
    while (!perr && gathered.load(std::memory_order_acquire) <= u) {  // (the gatherer is ahead of the H2D copies)
      if (progress() < 0) perr = 1;
      if (!launched && helpers_in() && prev_resident() && launch_main() != ART_OK) perr = 1;
      std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
    if (perr) break;
    const int64_t lo = ulo[u], m = ulo[u + 1] - lo;
    // the nine double rows of the unit in one strided copy (one DMA command instead of nine)
    perr |= hipMemcpy2DAsync(di + lo, nd * sizeof(double), pin + lo, nd * sizeof(double), (size_t)m * sizeof(double), 9,
                             hipMemcpyHostToDevice, H->m_up) != hipSuccess;
    perr |= hipMemcpyAsync((int8_t*)(di + 9 * nd) + lo, (int8_t*)(pin + 9 * nd) + lo, (size_t)m, hipMemcpyHostToDevice,
                           H->m_up) != hipSuccess;
    perr |= hipEventRecord(ev_up[u], H->m_up) != hipSuccess;
    recorded.store(u + 1, std::memory_order_release);
    if (trace) std::fprintf(stderr, "[art-host] t=%.2f unit %d submitted%s\n", clk() - t_start, u,
                            launched ? "" : " (integrator not launched yet)");
    if (!perr && progress() < 0) perr = 1;
  }
  if (!perr && !launched) {  // the helpers wait for CU slots the previous call still holds
    const double tw = clk();
    while (!(helpers_in() && prev_resident()) && clk() - tw < 5000.0) {
      if (progress() < 0) break;
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    if (!helpers_in()) {
      std::fprintf(stderr, "[art] maskless streamed pipeline: helper blocks did not start; running the batch again\n");
      perr = 1;
    } else if (launch_main() != ART_OK) {
      perr = 1;
    }
  }
  if (trace) std::fprintf(stderr, "[art-host] t=%.2f uploads submitted\n", clk() - t_start);
  const double limit_ms = (double)env_int("ART_HOST_STREAM_TIMEOUT_MS", 30000);
  double t_last = clk(), t_peek = clk();
  bool gave_up = perr != 0;
  unsigned long long* peek = nullptr;  // (trace) the device counters, copied out every 100 ms
  if (trace && hipHostMalloc((void**)&peek, 160 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess)
    peek = nullptr;  // (no HIP_OK between the readier thread's start and its join)
  while (!gave_up && sk < np) {
    if (peek && clk() - t_peek > (double)env_int("ART_HOST_PEEK_MS", 100)) {
      t_peek = clk();
      if (hipMemcpyAsync(peek, words, 160 * sizeof(unsigned long long), hipMemcpyDeviceToHost, H->m_dn) == hipSuccess &&
          hipStreamSynchronize(H->m_dn) == hipSuccess) {
        unsigned long long fin = 0, tiles = 0;
        for (int k = 0; k < np; ++k) {
          fin += peek[32 + k];
          tiles += peek[96 + k];
        }
        std::fprintf(stderr, "[art-host] t=%.1f queue %llu init_next %llu fin_next %llu misses %llu finished %llu tiles %llu flags:",
                     clk() - t_start, peek[0], peek[16], peek[17], peek[18], fin, tiles);
        for (int k = 0; k < np; ++k) std::fprintf(stderr, "%llu", hflag[k]);
        std::fprintf(stderr, " ready %llu started %llu abort %u init-pass %s integrator %s\n", *hready, hflag[HSIG_NFLAG],
                     *H->abort_host, hipEventQuery(L->ev0) == hipSuccess ? "done" : "running",
                     hipEventQuery(L->ev1) == hipSuccess ? "done" : "running");
      }
    }
    if (trace && !int_logged && launched && hipEventQuery(L->ev1) == hipSuccess) {
      int_logged = true;
      std::fprintf(stderr, "[art-host] t=%.2f integrator done\n", clk() - t_start);
    }
    const int mv = progress();
    if (mv < 0 || ready_err.load()) {
      gave_up = true;
      break;
    }
    if (mv > 0) {
      t_last = clk();
      continue;
    }
    if (__atomic_load_n(H->abort_host, __ATOMIC_ACQUIRE) != 0u || clk() - t_last > limit_ms) {
      gave_up = true;
      break;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  // the call's end: the helpers' completion words (the statistics, the flux), raised by the last
  // serving helper block once every integrator wave has counted itself (bounded like the pieces)
  if (!gave_up) {
    while (__atomic_load_n(hdone, __ATOMIC_ACQUIRE) == 0ull) {
      if (__atomic_load_n(H->abort_host, __ATOMIC_ACQUIRE) != 0u || clk() - t_last > limit_ms) {
        gave_up = true;
        break;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(10));
    }
  }
  stop = true;
  if (peek) (void)hipHostFree(peek);
  if (gave_up) {
    // stop the launch, then leave the batch to another path: every wait of the helpers and the
    // waves ends on the abort word, and a helper that sees it drains the work queue (queue_word),
    // so the integrator stops at each wave's next chunk claim. (The ready counter is NOT raised:
    // helpers would initialise tiles whose inputs never landed)
    __atomic_store_n(H->abort_host, 1u, __ATOMIC_RELEASE);
    readier.join();
    (void)hipStreamSynchronize(H->m_up);
    (void)hipStreamSynchronize(H->m_comp);
    (void)hipStreamSynchronize(H->m_help);
    (void)hipStreamSynchronize(H->m_dn);
    (void)hipGetLastError();
    if (trace) {  // the device counters at the give-up
      std::vector<unsigned long long> w(160);
      if (hipMemcpy(w.data(), words, w.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost) == hipSuccess) {
        std::fprintf(stderr, "[art-host] queue %llu init_next %llu fin_next %llu\n", w[0], w[16], w[17]);
        for (int k = 0; k < np; ++k)
          std::fprintf(stderr, "[art-host] piece %d finished %llu finalized tiles %llu flag %llu\n", k, w[32 + k], w[96 + k],
                       hflag[k]);
      }
    }
    std::fprintf(stderr, "[art] maskless streamed pipeline gave up at piece %d of %d (abort=%u); running the batch again\n",
                 sk, np, *H->abort_host);
    return STREAM_FALLBACK;
  }
  readier.join();
  if (trace) std::fprintf(stderr, "[art-host] maskless total %.2f ms (%d pieces of 2^%d)\n", clk() - t_start, np, shift);
  const bool complete = __atomic_load_n(hdone, __ATOMIC_ACQUIRE) == 1ull;
  if (fx.nbins && hflux && complete) {
    for (int b = 0; b < 2 * fx.nbins; ++b) {
      const unsigned long long v = __atomic_load_n(hdone + art::DONE_FLUX + b, __ATOMIC_ACQUIRE);
      std::memcpy(fx.hist + b, &v, sizeof(double));
    }
  } else if (fx.nbins) {  // flux kernels over the pieces' blobs, once the integrator is done
    if (hflux) HIP_OK(hipMemsetAsync(hist_dev, 0, 2 * (size_t)fx.nbins * sizeof(double), H->m_comp));
    for (int k = 0; k < np; ++k) {
      const int64_t lo = piece_lo(k), m = piece_lo(k + 1) - lo;
      double* dd = (double*)((char*)dout + stride * k);
      const int32_t* st = (const int32_t*)(dd + 8 * m);
      HIP_OK(art::launch_flux(K, m, dd, dd + 3 * m, st, in.species + lo, nullptr, fx.nbins, hist_dev, H->m_comp));
    }
    HIP_OK(hipMemcpyAsync(fx.hist, hist_dev, 2 * (size_t)fx.nbins * sizeof(double), hipMemcpyDeviceToHost, H->m_comp));
    HIP_OK(hipStreamSynchronize(H->m_comp));
  }
  if (complete && !final_pass) {  // the statistics from the completion words
    unsigned long long st[art::N_STATS_DEV];
    for (int i = 0; i < art::N_STATS_DEV; ++i) st[i] = __atomic_load_n(hdone + art::DONE_STATS + i, __ATOMIC_ACQUIRE);
    return latch_launch(c, L, st);
  }
  if (!final_pass) {  // (the helpers' copy timed out: the statistics as the stream has them)
    HIP_OK(hipMemcpyAsync(L->host_stats, words + 1, sizeof(unsigned long long) * art::N_STATS_DEV, hipMemcpyDeviceToHost,
                          H->m_comp));
    HIP_OK(hipStreamSynchronize(H->m_comp));
  }
  return finish_timing_slot(c, L);
}

// The single-launch host path: the inputs up, one propagate launch (init, integrator, finalize),
// the outputs back, all on stream s with device staging from `pool` (slots pb .. pb + 4): the
// context's own for synchronous calls, a host lane's for an asynchronous call's fallback.
int propagate_host_single(DeviceCtx* c, hipStream_t s, PoolVec& pool, size_t pb, const art_params* p, int64_t n,
                          const double* x0, const double* k0, const double* erg, const double* dw, const double* ln_t0,
                          const int8_t* species, int32_t max_crossings, art_segment_out* out, art_crossing_buf* xc,
                          const TrajArgs& htr, const FluxArgs& fx) {
  int rc;
  const int cap = (xc && xc->count) ? xc->capacity : 0;
  const size_t nd = (size_t)n;
  // staging layout: inputs 3n+3n+n+n+n doubles + n int8; outputs 3n+3n+n+n doubles + 3n int32 (+ crossings)
  void *din, *dout, *dxc = nullptr;
  const size_t in_bytes = nd * 9 * sizeof(double) + nd;
  const size_t out_bytes = nd * 8 * sizeof(double) + nd * 3 * sizeof(int32_t);
  const size_t cnt_bytes = ((nd * sizeof(int32_t) + 15) / 16) * 16;
  const size_t xc_bytes = cap ? cnt_bytes + (size_t)cap * nd * 9 * sizeof(double) : 0;
  if ((rc = pool_get_v(pool, pb + 0, in_bytes, &din))) return rc;
  if ((rc = pool_get_v(pool, pb + 1, out_bytes, &dout))) return rc;
  if (cap && (rc = pool_get_v(pool, pb + 2, xc_bytes, &dxc))) return rc;
  double* di = (double*)din;
  HIP_OK(hipMemcpyAsync(di, x0, nd * 3 * sizeof(double), hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(di + 3 * nd, k0, nd * 3 * sizeof(double), hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(di + 6 * nd, erg, nd * sizeof(double), hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(di + 7 * nd, dw, nd * sizeof(double), hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(di + 8 * nd, ln_t0, nd * sizeof(double), hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync((int8_t*)(di + 9 * nd), species, nd, hipMemcpyHostToDevice, s));
  double* dd = (double*)dout;
  int32_t* di32 = (int32_t*)(dd + 8 * nd);
  art_segment_out dso{dd, dd + 3 * nd, dd + 6 * nd, dd + 7 * nd, di32, di32 + nd, di32 + 2 * nd};
  art_crossing_buf dxb{};
  art_crossing_buf* dxbp = nullptr;
  if (cap) {
    int32_t* cnt = (int32_t*)dxc;
    double* xd = (double*)((char*)dxc + cnt_bytes);
    dxb = art_crossing_buf{cap, cnt, xd, xd + 3 * cap * nd, xd + 6 * cap * nd, xd + 7 * cap * nd, xd + 8 * cap * nd};
    dxbp = &dxb;
  }
  TrajArgs dtr;
  if (htr.ntimes != 0) {
    void* dt_ = nullptr;
    const size_t nt = (size_t)htr.ntimes * nd;
    if ((rc = pool_get_v(pool, pb + 3, nt * 4 * sizeof(double) + nd * sizeof(int32_t), &dt_))) return rc;
    dtr.ntimes = htr.ntimes;
    dtr.traj = (double*)dt_;
    dtr.t = dtr.traj + 3 * nt;
    dtr.count = (int32_t*)(dtr.t + nt);
  }
  // slots without a crossing come back as NaN, not as whatever the pooled staging buffer last
  // held: finalize_kernel writes them (LaunchOpts::nan_fill)
  LaunchOpts opt;
  opt.nan_fill = true;
  LaunchRec* L = nullptr;
  opt.launch_out = &L;
  rc = propagate_device_impl(p, n, di, di + 3 * nd, di + 6 * nd, di + 7 * nd, di + 8 * nd, (const int8_t*)(di + 9 * nd),
                             max_crossings, &dso, dxbp, s, dtr, opt, c);
  if (rc) return rc;
  if (fx.nbins) {  // the batch's flux from its outputs in HBM
    double* hist_dev = nullptr;
    if ((rc = pool_get_v(pool, pb + 4, 2 * (size_t)fx.nbins * sizeof(double), (void**)&hist_dev))) return rc;
    HIP_OK(hipMemsetAsync(hist_dev, 0, 2 * (size_t)fx.nbins * sizeof(double), s));
    HIP_OK(art::launch_flux(kparams(*p), n, dso.x_end, dso.k_end, dso.status, (const int8_t*)(di + 9 * nd), nullptr,
                            fx.nbins, hist_dev, s));
    HIP_OK(hipMemcpyAsync(fx.hist, hist_dev, 2 * (size_t)fx.nbins * sizeof(double), hipMemcpyDeviceToHost, s));
  }
  if (htr.ntimes != 0) {
    const size_t nt = (size_t)htr.ntimes * nd;
    HIP_OK(hipMemcpyAsync(htr.traj, dtr.traj, nt * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(htr.t, dtr.t, nt * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(htr.count, dtr.count, nd * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  }
  HIP_OK(hipMemcpyAsync(out->x_end, dso.x_end, nd * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(out->k_end, dso.k_end, nd * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(out->u7_end, dso.u7_end, nd * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(out->tau_end, dso.tau_end, nd * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(out->status, dso.status, nd * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(out->n_accept, dso.n_accept, nd * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(out->n_reject, dso.n_reject, nd * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  if (cap) {
    HIP_OK(hipMemcpyAsync(xc->count, dxb.count, nd * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(xc->pos, dxb.pos, (size_t)cap * nd * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(xc->k, dxb.k, (size_t)cap * nd * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(xc->t, dxb.t, (size_t)cap * nd * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(xc->dw, dxb.dw, (size_t)cap * nd * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(xc->p_nonad, dxb.p_nonad, (size_t)cap * nd * sizeof(double), hipMemcpyDeviceToHost, s));
  }
  HIP_OK(hipStreamSynchronize(s));
  return finish_timing_slot(c, L);
}

// Synchronous host calls wait for every asynchronous one first: they share lane 0 and the
// context's staging (art_propagate_host_flux_async).
void drain_async(DeviceCtx* c) {
  for (HostLane& H : c->lanes) {
    std::unique_lock<std::mutex> lk(H.m);
    H.cv.wait(lk, [&] { return !H.busy; });
  }
}

// Which path a host call of n rays takes: the streamed pipeline for large Vern6 batches without
// saveat (ART_HOST_CHUNK_MIN rays and more, default 2^20, so the 1.25e6-ray shard of 8 GPUs
// streams: 18.3 ms against 20.0 in one launch, profiles/r04x_shard_sizes.jsonl), the chunked one
// with ART_HOST_MODE=chunked; the single launch otherwise (and after a streamed call gave up)
enum HostPath { HP_STREAM, HP_CHUNKED, HP_SINGLE };
HostPath host_path(const art_params* p, int64_t n, const TrajArgs& htr) {
  const char* mode_env = std::getenv("ART_HOST_MODE");
  const std::string mode = (mode_env && *mode_env) ? mode_env : "stream";
  if (htr.ntimes == 0 && n >= env_int("ART_HOST_CHUNK_MIN", 1 << 20)) {
    if (mode == "stream" && p->integrator == ART_VERN6) return HP_STREAM;
    if (mode == "chunked") return HP_CHUNKED;
  }
  return HP_SINGLE;
}

int host_args(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg, const double* dw,
              const double* ln_t0, const int8_t* species, art_segment_out* out, art_crossing_buf* xc, const TrajArgs& htr,
              const FluxArgs& fx, bool* empty) {
  int rc = check_segment_args(p, n, x0, k0, erg, dw, ln_t0, species, out, xc, htr, empty);
  if (rc) return rc;
  if (fx.nbins && (fx.nbins < 1 || fx.nbins > 4096 || !fx.hist)) return fail(ART_E_INVALID, "flux needs nbins in [1, 4096] and hist");
  if (fx.nbins) std::fill(fx.hist, fx.hist + 2 * (size_t)fx.nbins, 0.0);
  return ART_OK;
}

int propagate_host_impl(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                        const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                        art_segment_out* out, art_crossing_buf* xc, const TrajArgs& htr,
                        const FluxArgs& fx = FluxArgs()) {
  bool empty = false;
  int rc = host_args(p, n, x0, k0, erg, dw, ln_t0, species, out, xc, htr, fx, &empty);
  if (rc || empty) return rc;
  DeviceCtx* c;
  if ((rc = current_ctx(&c))) return rc;
  drain_async(c);
  g_host_cnt[HC_CALLS] += 1;
  const HostPath hp = host_path(p, n, htr);
  if (hp == HP_STREAM) {
    rc = propagate_host_maskless(c, &c->lanes[0], false, -1, p, n, x0, k0, erg, dw, ln_t0, species, max_crossings, out, xc, fx);
    if (rc != STREAM_FALLBACK) {
      if (rc == ART_OK) g_host_cnt[HC_STREAMED] += 1;
      return rc;
    }
    g_host_cnt[HC_GIVEUPS] += 1;
  } else if (hp == HP_CHUNKED) {
    g_host_cnt[HC_CHUNKED] += 1;
    return propagate_host_chunked(c, p, n, x0, k0, erg, dw, ln_t0, species, max_crossings, out, xc,
                                  std::max(2, env_int("ART_HOST_CHUNKS", 4)), std::max(1, env_int("ART_HOST_SLOTS", 2)), fx);
  }
  g_host_cnt[HC_SINGLE] += 1;
  return propagate_host_single(c, c->stream, c->pool, 0, p, n, x0, k0, erg, dw, ln_t0, species, max_crossings, out, xc,
                               htr, fx);
}

// The asynchronous calls' workers: one thread per host lane, one call at a time.
void lane_worker(DeviceCtx* c, HostLane* H) {
  (void)hipSetDevice(c->device);
  for (;;) {
    std::function<int()> job;
    {
      std::unique_lock<std::mutex> lk(H->m);
      H->cv.wait(lk, [&] { return H->stop || (bool)H->job; });
      if (!H->job) return;  // (stop, nothing left)
      job = std::move(H->job);
      H->job = nullptr;
    }
    job();
    {
      std::lock_guard<std::mutex> lk(H->m);
      H->busy = false;
    }
    H->cv.notify_all();
  }
}

// Ticket t runs on lane t % HOST_LANES once that lane's previous call has ended; its result waits
// in c->results for art_host_wait.
int64_t submit_async(DeviceCtx* c, std::function<int(HostLane*, int64_t)> body) {
  const int64_t t = c->next_ticket++;
  HostLane* H = &c->lanes[t % HOST_LANES];
  {
    std::lock_guard<std::mutex> lk(c->res_m);
    c->pending.insert(t);
  }
  {
    std::unique_lock<std::mutex> lk(H->m);
    H->cv.wait(lk, [&] { return !H->busy; });
    H->busy = true;
    H->job = [c, H, t, body] {
      g_err.clear();
      const int rc = body(H, t);
      for (int64_t d = c->done_ticket.load(); d < t && !c->done_ticket.compare_exchange_weak(d, t);) {
      }
      std::lock_guard<std::mutex> lk2(c->res_m);
      c->results[t] = {rc, g_err};
      c->res_cv.notify_all();
      return rc;
    };
    if (!H->worker.joinable()) H->worker = std::thread(lane_worker, c, H);
  }
  H->cv.notify_all();
  return t;
}
}  // namespace

extern "C" {

int art_propagate_host(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                       const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                       art_segment_out* out, art_crossing_buf* xc) {
  std::lock_guard<std::mutex> lk(g_mu);
  return propagate_host_impl(p, n, x0, k0, erg, dw, ln_t0, species, max_crossings, out, xc, TrajArgs());
}

int art_propagate_host_flux(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                            const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                            art_segment_out* out, art_crossing_buf* xc, int32_t nbins, double* hist) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (nbins < 1) return fail(ART_E_INVALID, "nbins must be >= 1");
  FluxArgs fx;
  fx.nbins = nbins;
  fx.hist = hist;
  return propagate_host_impl(p, n, x0, k0, erg, dw, ln_t0, species, max_crossings, out, xc, TrajArgs(), fx);
}

int art_propagate_host_flux_async(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                                  const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                                  art_segment_out* out, art_crossing_buf* xc, int32_t nbins, double* hist, int64_t* ticket) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!ticket) return fail(ART_E_INVALID, "ticket is NULL");
  if (nbins < 1) return fail(ART_E_INVALID, "nbins must be >= 1");
  FluxArgs fx;
  fx.nbins = nbins;
  fx.hist = hist;
  bool empty = false;
  int rc = host_args(p, n, x0, k0, erg, dw, ln_t0, species, out, xc, TrajArgs(), fx, &empty);
  if (rc) return rc;
  DeviceCtx* c;
  if ((rc = current_ctx(&c))) return rc;
  if (empty || host_path(p, n, TrajArgs()) != HP_STREAM) {
    // (a batch the streamed pipeline does not take runs now, in this thread; its ticket is complete)
    const int rc1 = empty ? ART_OK : propagate_host_impl(p, n, x0, k0, erg, dw, ln_t0, species, max_crossings, out, xc,
                                                          TrajArgs(), fx);
    const std::string e1 = g_err;
    *ticket = submit_async(c, [rc1, e1](HostLane*, int64_t) {
      g_err = e1;
      return rc1;
    });
    return ART_OK;
  }
  g_host_cnt[HC_CALLS] += 1;
  const art_params pc = *p;  // (the caller's structs by value: they may go out of scope before the call ends)
  art_segment_out oc = *out;
  const bool has_xc = xc != nullptr;
  art_crossing_buf xcc = has_xc ? *xc : art_crossing_buf{};
  *ticket = submit_async(c, [=](HostLane* H, int64_t t) mutable {
    int r = propagate_host_maskless(c, H, true, t, &pc, n, x0, k0, erg, dw, ln_t0, species, max_crossings, &oc,
                                    has_xc ? &xcc : nullptr, fx);
    if (r == STREAM_FALLBACK) {  // the batch again as one launch, on this lane's stream and staging
      g_host_cnt[HC_GIVEUPS] += 1;
      g_host_cnt[HC_SINGLE] += 1;
      if (fx.nbins) std::fill(fx.hist, fx.hist + 2 * (size_t)fx.nbins, 0.0);
      r = propagate_host_single(c, H->m_comp, H->pool, 4, &pc, n, x0, k0, erg, dw, ln_t0, species, max_crossings, &oc,
                                has_xc ? &xcc : nullptr, TrajArgs(), fx);
    } else if (r == ART_OK) {
      g_host_cnt[HC_STREAMED] += 1;
    }
    return r;
  });
  return ART_OK;
}

int art_host_wait(int64_t ticket) {
  DeviceCtx* c;
  int rc = current_ctx(&c);
  if (rc) return rc;
  std::unique_lock<std::mutex> lk(c->res_m);
  if (!c->pending.count(ticket)) return fail(ART_E_INVALID, "unknown ticket, or one already waited for");
  c->res_cv.wait(lk, [&] { return c->results.count(ticket) > 0; });
  const std::pair<int, std::string> r = c->results[ticket];
  c->results.erase(ticket);
  c->pending.erase(ticket);
  if (r.first != ART_OK) g_err = r.second;
  return r.first;
}

int art_host_path_counters(uint64_t* counters, int32_t n, int32_t reset) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (n < 0 || (n > 0 && !counters)) return fail(ART_E_INVALID, "bad buffer");
  for (int i = 0; i < n && i < HC_N; ++i) counters[i] = g_host_cnt[i];
  for (int i = HC_N; i < n; ++i) counters[i] = 0;
  if (reset)
    for (auto& v : g_host_cnt) v = 0;
  return HC_N;
}

int art_propagate_traj_host(const art_params* p, int64_t n, const double* x0, const double* k0, const double* erg,
                            const double* dw, const double* ln_t0, const int8_t* species, int32_t max_crossings,
                            art_segment_out* out, art_crossing_buf* xc, int32_t ntimes, double* traj, double* traj_t,
                            int32_t* traj_n) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (ntimes < 2) return fail(ART_E_INVALID, "ntimes must be >= 2");
  TrajArgs tr;
  tr.ntimes = ntimes; tr.traj = traj; tr.t = traj_t; tr.count = traj_n;
  return propagate_host_impl(p, n, x0, k0, erg, dw, ln_t0, species, max_crossings, out, xc, tr);
}

int art_get_prob_nonad_device(const art_params* p, int64_t nc, const double* pos, const double* kpos,
                              const double* erg_eff, int64_t n_groups, const int64_t* group_start, double* out,
                              void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = validate(p);
  if (rc) return rc;
  if (nc == 0) return ART_OK;
  if (nc < 0 || nc > 2147483647LL) return fail(ART_E_INVALID, "nc must be in [0, 2^31)");
  if (!pos || !kpos || !erg_eff || !out) return fail(ART_E_INVALID, "NULL buffer");
  if (!group_start) n_groups = nc;
  DeviceCtx* c;
  if ((rc = current_ctx(&c))) return rc;
  HIP_OK(art::launch_prob(art::make_kparams(*p), nc, pos, kpos, erg_eff, n_groups, group_start, out, pick(c, stream)));
  return ART_OK;
}

int art_get_prob_nonad_host(const art_params* p, int64_t nc, const double* pos, const double* kpos,
                            const double* erg_eff, int64_t n_groups, const int64_t* group_start, double* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = validate(p);
  if (rc) return rc;
  if (nc == 0) return ART_OK;
  if (nc < 0 || nc > 2147483647LL) return fail(ART_E_INVALID, "nc must be in [0, 2^31)");
  if (!pos || !kpos || !erg_eff || !out) return fail(ART_E_INVALID, "NULL buffer");
  if (!group_start) n_groups = nc;
  if (group_start) {  // groups must tile [0, nc)
    if (n_groups < 1) return fail(ART_E_INVALID, "n_groups must be >= 1");
    if (group_start[0] != 0 || group_start[n_groups] != nc) return fail(ART_E_INVALID, "group_start must span [0, nc]");
    for (int64_t g = 0; g < n_groups; ++g)
      if (group_start[g + 1] <= group_start[g]) return fail(ART_E_INVALID, "empty or unsorted group");
  }
  DeviceCtx* c;
  if ((rc = current_ctx(&c))) return rc;
  void* d;
  const size_t nd = (size_t)nc;
  const size_t bytes = nd * 8 * sizeof(double) + (size_t)(n_groups + 1) * sizeof(int64_t);
  if ((rc = pool_get(c, 3, bytes, &d))) return rc;
  double* dd = (double*)d;
  int64_t* dg = group_start ? (int64_t*)(dd + 8 * nd) : nullptr;
  hipStream_t s = c->stream;
  HIP_OK(hipMemcpyAsync(dd, pos, nd * 3 * sizeof(double), hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(dd + 3 * nd, kpos, nd * 3 * sizeof(double), hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(dd + 6 * nd, erg_eff, nd * sizeof(double), hipMemcpyHostToDevice, s));
  if (dg) HIP_OK(hipMemcpyAsync(dg, group_start, (size_t)(n_groups + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  HIP_OK(art::launch_prob(art::make_kparams(*p), nc, dd, dd + 3 * nd, dd + 6 * nd, n_groups, dg, dd + 7 * nd, s));
  HIP_OK(hipMemcpyAsync(out, dd + 7 * nd, nd * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return ART_OK;
}

}  // extern "C"

namespace {
int sample_device_impl(const art_params* p, double max_r, uint64_t seed, int64_t ray_offset, int64_t n, double* x,
                       double* k_init, double* erg_inf, double* vifty, int32_t* weights, int32_t* attempts,
                       hipStream_t s) {
  int rc = validate(p);
  if (rc) return rc;
  if (n == 0) return ART_OK;
  if (n < 0 || n > 2147483647LL) return fail(ART_E_INVALID, "n must be in [0, 2^31)");
  if (!(max_r > p->rNS)) return fail(ART_E_INVALID, "max_r must exceed rNS (MainRunner.jl:389-396 quits otherwise)");
  if (!x || !k_init || !erg_inf || !vifty || !weights || !attempts) return fail(ART_E_INVALID, "NULL buffer");
  DeviceCtx* c;
  if ((rc = current_ctx(&c))) return rc;
  void* q = nullptr;  // this launch's work-queue word
  if ((rc = scratch_alloc(s, 256, &q))) return rc;
  HIP_OK(hipMemsetAsync(q, 0, sizeof(unsigned long long), s));
  HIP_OK(hipMemsetAsync(q, 0, 256, s));
  HIP_OK(art::launch_sample(kparams(*p), max_r, seed, ray_offset, n, x, k_init, erg_inf, vifty, weights,
                            attempts, (unsigned long long*)q, s, c->sampler_waves));
#ifdef ART_SAMPLER_SECTIONS  // (dev build: the sampler's section cycles to stderr)
  {
    unsigned long long w[16];
    HIP_OK(hipMemcpyAsync(w, q, sizeof w, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    std::fprintf(stderr, "[sampler-sections] n=%lld setup %llu control %llu cert %llu grid %llu brackets %llu out %llu "
                 "grid_steps %llu steps %llu\n", (long long)n, w[8], w[9], w[10], w[11], w[12], w[13], w[14], w[15]);
  }
#endif
  HIP_OK(hipFreeAsync(q, s));
  return ART_OK;
}

int event_weight_device_impl(const art_params* p, double max_r, double rho_dm, double mcmc_weight, int64_t n,
                             const double* x, const double* k_init, const double* vifty, double* out, hipStream_t s) {
  int rc = validate(p);
  if (rc) return rc;
  if (n == 0) return ART_OK;
  if (n < 0) return fail(ART_E_INVALID, "n must be >= 0");
  if (!x || !k_init || !vifty || !out) return fail(ART_E_INVALID, "NULL buffer");
  DeviceCtx* c;
  if ((rc = current_ctx(&c))) return rc;
  HIP_OK(art::launch_event_weight(art::make_kparams(*p), n, x, k_init, vifty, max_r, rho_dm, mcmc_weight, out, s));
  return ART_OK;
}
}  // namespace

extern "C" {

int art_sample_conversion_points_device(const art_params* p, double max_r, uint64_t seed, int64_t ray_offset,
                                        int64_t n, double* x, double* k_init, double* erg_inf, double* vifty,
                                        int32_t* weights, int32_t* attempts, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  return sample_device_impl(p, max_r, seed, ray_offset, n, x, k_init, erg_inf, vifty, weights, attempts,
                            (hipStream_t)stream);
}

// The whole stage-run-copy sequence holds the mutex, so no other thread can regrow the staging
// buffer in between.
int art_sample_conversion_points_host(const art_params* p, double max_r, uint64_t seed, int64_t ray_offset, int64_t n,
                                      double* x, double* k_init, double* erg_inf, double* vifty, int32_t* weights,
                                      int32_t* attempts) {
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = validate(p);
  if (rc) return rc;
  if (n == 0) return ART_OK;
  if (n < 0 || n > 2147483647LL) return fail(ART_E_INVALID, "n must be in [0, 2^31)");
  if (!(max_r > p->rNS)) return fail(ART_E_INVALID, "max_r must exceed rNS (MainRunner.jl:389-396 quits otherwise)");
  if (!x || !k_init || !erg_inf || !vifty || !weights || !attempts) return fail(ART_E_INVALID, "NULL buffer");
  DeviceCtx* c;
  if ((rc = current_ctx(&c))) return rc;
  void* d;
  const size_t nd = (size_t)n;
  if ((rc = pool_get(c, 4, nd * 10 * sizeof(double) + nd * 2 * sizeof(int32_t), &d))) return rc;
  double* dd = (double*)d;
  int32_t* di = (int32_t*)(dd + 10 * nd);
  hipStream_t s = c->stream;
  if ((rc = sample_device_impl(p, max_r, seed, ray_offset, n, dd, dd + 3 * nd, dd + 6 * nd, dd + 7 * nd, di, di + nd,
                               s)))
    return rc;
  HIP_OK(hipMemcpyAsync(x, dd, nd * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(k_init, dd + 3 * nd, nd * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(erg_inf, dd + 6 * nd, nd * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(vifty, dd + 7 * nd, nd * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(weights, di, nd * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(attempts, di + nd, nd * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return ART_OK;
}

int art_event_weight_device(const art_params* p, double max_r, double rho_dm, double mcmc_weight, int64_t n,
                            const double* x, const double* k_init, const double* vifty, double* out, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  return event_weight_device_impl(p, max_r, rho_dm, mcmc_weight, n, x, k_init, vifty, out, (hipStream_t)stream);
}

int art_event_weight_host(const art_params* p, double max_r, double rho_dm, double mcmc_weight, int64_t n,
                          const double* x, const double* k_init, const double* vifty, double* out) {
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = validate(p);
  if (rc) return rc;
  if (n == 0) return ART_OK;
  if (n < 0 || n > 2147483647LL) return fail(ART_E_INVALID, "n must be in [0, 2^31)");
  if (!x || !k_init || !vifty || !out) return fail(ART_E_INVALID, "NULL buffer");
  DeviceCtx* c;
  if ((rc = current_ctx(&c))) return rc;
  void* d;
  const size_t nd = (size_t)n;
  if ((rc = pool_get(c, 5, nd * 14 * sizeof(double), &d))) return rc;
  double* dd = (double*)d;
  hipStream_t s = c->stream;
  HIP_OK(hipMemcpyAsync(dd, x, nd * 3 * sizeof(double), hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(dd + 3 * nd, k_init, nd * 3 * sizeof(double), hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(dd + 6 * nd, vifty, nd * 3 * sizeof(double), hipMemcpyHostToDevice, s));
  if ((rc = event_weight_device_impl(p, max_r, rho_dm, mcmc_weight, n, dd, dd + 3 * nd, dd + 6 * nd, dd + 9 * nd, s)))
    return rc;
  HIP_OK(hipMemcpyAsync(out, dd + 9 * nd, nd * 5 * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return ART_OK;
}

int art_flux_histogram_device(const art_params* p, int64_t n, const double* x_end, const double* k_end,
                              const int32_t* status, const int8_t* species, const double* w, int32_t nbins,
                              double* hist, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = validate(p);
  if (rc) return rc;
  if (nbins < 1 || nbins > 4096) return fail(ART_E_INVALID, "nbins must be in [1, 4096]");
  if (n == 0) return ART_OK;
  DeviceCtx* c;
  if ((rc = current_ctx(&c))) return rc;
  HIP_OK(art::launch_flux(art::make_kparams(*p), n, x_end, k_end, status, species, w, nbins, hist, pick(c, stream)));
  return ART_OK;
}

int art_flux_histogram_phi_device(int64_t n, const double* phi, const int8_t* species, const double* w, int32_t nbins,
                                  double* hist, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (nbins < 1 || nbins > 4096) return fail(ART_E_INVALID, "nbins must be in [1, 4096]");
  if (n < 0) return fail(ART_E_INVALID, "n must be >= 0");
  if (n == 0) return ART_OK;
  if (!phi || !hist) return fail(ART_E_INVALID, "NULL buffer");
  DeviceCtx* c;
  int rc = current_ctx(&c);
  if (rc) return rc;
  HIP_OK(art::launch_flux_phi(n, phi, species, w, nbins, -art::PI, art::PI, hist, (hipStream_t)stream));
  return ART_OK;
}

int art_flux_histogram_phi_range_device(int64_t n, const double* phi, const int8_t* species, const double* w,
                                        int32_t nbins, double lo, double hi, double* hist, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (nbins < 1 || nbins > 4096) return fail(ART_E_INVALID, "nbins must be in [1, 4096]");
  if (n < 0) return fail(ART_E_INVALID, "n must be >= 0");
  if (!(lo < hi) || !std::isfinite(lo) || !std::isfinite(hi)) return fail(ART_E_INVALID, "need finite lo < hi");
  if (n == 0) return ART_OK;
  if (!phi || !hist) return fail(ART_E_INVALID, "NULL buffer");
  DeviceCtx* c;
  int rc = current_ctx(&c);
  if (rc) return rc;
  HIP_OK(art::launch_flux_phi(n, phi, species, w, nbins, lo, hi, hist, (hipStream_t)stream));
  return ART_OK;
}

int art_eval_rhs_device(const art_params* p, int64_t n, const double* u, const double* tau, const double* erg,
                        const int8_t* species, double* du, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = validate(p);
  if (rc) return rc;
  if (n == 0) return ART_OK;
  DeviceCtx* c;
  if ((rc = current_ctx(&c))) return rc;
  HIP_OK(art::launch_eval_rhs(art::make_kparams(*p), n, u, tau, erg, species, du, pick(c, stream)));
  return ART_OK;
}

int art_eval_hamiltonian_device(const art_params* p, int64_t n, const double* x, const double* k, const double* T,
                                const double* E, double* H, double* dHdx, double* dHdk, double* dHdT, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = validate(p);
  if (rc) return rc;
  if (n == 0) return ART_OK;
  DeviceCtx* c;
  if ((rc = current_ctx(&c))) return rc;
  HIP_OK(art::launch_eval_hamiltonian(art::make_kparams(*p), n, x, k, T, E, H, dHdx, dHdk, dHdT, pick(c, stream)));
  return ART_OK;
}

int art_eval_condition_device(const art_params* p, int64_t n, const double* u, const double* tau, double* out,
                              void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  int rc = validate(p);
  if (rc) return rc;
  if (n == 0) return ART_OK;
  DeviceCtx* c;
  if ((rc = current_ctx(&c))) return rc;
  HIP_OK(art::launch_eval_condition(art::make_kparams(*p), n, u, tau, out, pick(c, stream)));
  return ART_OK;
}

// ---- the radiated-flux reduction across ranks: one RCCL all-reduce ----
// RCCL is opened at first use (dlopen), so libart.so loads and runs single-GPU work where it
// is absent; a process that already loaded librccl.so.1 (e.g. PyTorch's) shares that copy.
}  // extern "C"

namespace {
typedef int (*nccl_get_id_t)(void*);
typedef int (*nccl_init_rank_t)(void**, int, art_rccl_id, int);
typedef int (*nccl_allreduce_t)(const void*, void*, size_t, int, int, void*, hipStream_t);
typedef int (*nccl_destroy_t)(void*);
typedef const char* (*nccl_err_t)(int);
struct Rccl {
  void* h = nullptr;
  nccl_get_id_t get_id = nullptr;
  nccl_init_rank_t init_rank = nullptr;
  nccl_allreduce_t allreduce = nullptr;
  nccl_destroy_t destroy = nullptr;
  nccl_err_t err = nullptr;
  void* comm = nullptr;
  int device = -1;
};
Rccl g_rccl;
constexpr int NCCL_FLOAT64 = 8;  // ncclFloat64 (rccl.h)
constexpr int NCCL_SUM = 0;      // ncclSum

int rccl_open() {
  if (g_rccl.h) return ART_OK;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (!h) return fail(ART_E_UNSUPPORTED, "RCCL (librccl.so.1) is not available: %s", dlerror());
  g_rccl.get_id = (nccl_get_id_t)dlsym(h, "ncclGetUniqueId");
  g_rccl.init_rank = (nccl_init_rank_t)dlsym(h, "ncclCommInitRank");
  g_rccl.allreduce = (nccl_allreduce_t)dlsym(h, "ncclAllReduce");
  g_rccl.destroy = (nccl_destroy_t)dlsym(h, "ncclCommDestroy");
  g_rccl.err = (nccl_err_t)dlsym(h, "ncclGetErrorString");
  if (!g_rccl.get_id || !g_rccl.init_rank || !g_rccl.allreduce || !g_rccl.destroy || !g_rccl.err)
    return fail(ART_E_UNSUPPORTED, "librccl.so.1 lacks the nccl* entry points");
  g_rccl.h = h;
  return ART_OK;
}

int rccl_fail(int r, const char* what) {
  return fail(ART_E_HIP, "%s: %s", what, g_rccl.err ? g_rccl.err(r) : "RCCL error");
}
}  // namespace

extern "C" {

int art_comm_unique_id(art_rccl_id* id) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!id) return fail(ART_E_INVALID, "id is NULL");
  int rc = rccl_open();
  if (rc) return rc;
  const int r = g_rccl.get_id(id);
  return r ? rccl_fail(r, "ncclGetUniqueId") : ART_OK;
}

int art_comm_init(int32_t rank, int32_t world, const art_rccl_id* id) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!id || world < 1 || rank < 0 || rank >= world) return fail(ART_E_INVALID, "bad rank/world/id");
  if (g_rccl.comm) return fail(ART_E_INVALID, "communicator already initialised (art_comm_destroy first)");
  int rc = rccl_open();
  if (rc) return rc;
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  void* comm = nullptr;
  const int r = g_rccl.init_rank(&comm, world, *id, rank);
  if (r) return rccl_fail(r, "ncclCommInitRank");
  g_rccl.comm = comm;
  g_rccl.device = dev;
  return ART_OK;
}

int art_flux_allreduce(double* buf, int64_t count, void* stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_rccl.comm) return fail(ART_E_INVALID, "no communicator: art_comm_init first");
  if (count < 0 || (count > 0 && !buf)) return fail(ART_E_INVALID, "bad buffer");
  if (count == 0) return ART_OK;
  const int r = g_rccl.allreduce(buf, buf, (size_t)count, NCCL_FLOAT64, NCCL_SUM, g_rccl.comm, (hipStream_t)stream);
  return r ? rccl_fail(r, "ncclAllReduce") : ART_OK;
}

// The same for a host buffer (a Julia host's Vector{Float64}): staged through HBM on the
// library's stream, reduced, copied back; synchronous.
int art_flux_allreduce_host(double* buf, int64_t count) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_rccl.comm) return fail(ART_E_INVALID, "no communicator: art_comm_init first");
  if (count < 0 || (count > 0 && !buf)) return fail(ART_E_INVALID, "bad buffer");
  if (count == 0) return ART_OK;
  DeviceCtx* c;
  int rc = current_ctx(&c);
  if (rc) return rc;
  void* d;
  if ((rc = pool_get(c, 8, (size_t)count * sizeof(double), &d))) return rc;
  HIP_OK(hipMemcpyAsync(d, buf, (size_t)count * sizeof(double), hipMemcpyHostToDevice, c->stream));
  const int r = g_rccl.allreduce(d, d, (size_t)count, NCCL_FLOAT64, NCCL_SUM, g_rccl.comm, c->stream);
  if (r) return rccl_fail(r, "ncclAllReduce");
  HIP_OK(hipMemcpyAsync(buf, d, (size_t)count * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  return ART_OK;
}

int art_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  shutdown_locked();
  return ART_OK;
}

int art_comm_destroy(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_rccl.comm) return ART_OK;
  const int r = g_rccl.destroy(g_rccl.comm);
  g_rccl.comm = nullptr;
  return r ? rccl_fail(r, "ncclCommDestroy") : ART_OK;
}

}  // extern "C"
