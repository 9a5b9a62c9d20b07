// art_internal.h -- launch wrappers shared by art_kernels.hip and art_capi.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include "art_core.h"

namespace art {
// Segment inputs / outputs (device pointers, SoA), see art_segment_out / art_crossing_buf.
struct SegIn {
  const double *x0, *k0, *erg, *dw, *lnt0;
  const int8_t* species;
  // device scratch filled by the init pass: one U0_REC-double fresh-state record per ray
  // (fresh_rec below), so a refilling lane reads its ray with 10 16-byte loads from two lines
  double* u0;
};

struct SegOut {
  double *x_end, *k_end, *u7_end, *tau_end;
  int32_t *status, *n_acc, *n_rej;
  int32_t cap;
  int32_t* xcount;
  double *xpos, *xk, *xt, *xdw, *xp;
  // saveat (RayTracer.jl:176, 383), only with ntimes >= 2: ntimes points per ray, positions
  // [(c * ntimes + k) * n + ray] (spherical from the integrator, Cartesian after finalize),
  // ln t [k * n + ray], and the number of points of each ray
  int32_t ntimes;
  double *traj, *traj_t;
  int32_t* traj_n;
  // END_REC doubles of device scratch per ray: the integrator's raw end state as one AoS
  // record per ray, [u (7) | tau | int4 {status, n_acc, n_rej, ncross} | int4 {traj_n, 0, 0, 0}],
  // which finalize_kernel spreads into the SoA outputs above with coalesced stores. A finishing
  // lane then writes 5 (saveat: 6) 16-byte stores into its own 128-byte line instead of 12
  // 4/8-byte stores into as many partly written lines.
  double* rec;
  // X_REC doubles of device scratch per (ray, crossing j < cap), the same idea for the
  // crossings affect! records: [x (3) | k (3) | t | Δω] at ((ray cap + j) X_REC), spread into
  // xpos / xk / xt / xdw by finalize_kernel
  double* xrec;
  // Tail donation (art_set_tail_donation): once the queue is drained, a wave whose live rays
  // (all at a step boundary) number at most `donate` writes their complete integrator state
  // as CONT_REC-double records to cont[] (count in *cont_count) and retires, so its CU slot
  // goes to the next launch in flight; a continuation launch (cont_mode = 1) then integrates
  // those rays packed into full waves, bit for bit as if they had never moved.
  double* cont;
  unsigned long long* cont_count;
  unsigned long long* cont_queue;
  int32_t donate, cont_mode;
  // the continuation launch (cont_mode = 1) reads the records from cont_src (count
  // *cont_src_count) and may itself donate its own drained waves' last rays into cont /
  // cont_count: the second level, which tail_kernel resumes one ray per wave
  const double* cont_src;
  const unsigned long long* cont_src_count;
  double* cont2;  // the second-level records (set on the launch's SegOut; read by launch_propagate)
  unsigned long long *cont2_count, *cont2_queue;
  // 1: finalize_kernel writes NaN into the crossing slots j >= min(count, cap) (the *_host
  // entry points' contract, include/art.h), so no fill of the outputs is needed beforehand
  int32_t nan_fill;
  // The streamed host pipeline (propagate_kernel<..., DON = 3>, art_propagate_host): piece
  // p = ray >> piece_shift; every finished ray counts into piece_cnt[p]; a wave that waits too
  // long (STREAM_WAIT_TICKS of s_memrealtime) raises *abort_word and stops taking rays.
  unsigned long long* piece_cnt;
  unsigned int* abort_word;
  // the launch's work-queue word: a helper that sees the call given up adds 2^40 to it, so every
  // integrator wave's next chunk claim finds the queue drained and the launch runs out at once
  unsigned long long* queue_word;
  unsigned long long wait_ticks;  // a wave's bound on a chunk flag (STREAM_WAIT_TICKS; tests set less)
  int32_t piece_shift;
  // The maskless streamed pipeline (DON = 3, art_capi.cpp propagate_host_maskless): one launch
  // over the whole batch holds every CU; its first `helpers` blocks are helpers, not
  // integrators. *host_ready (host memory, raised by the host as each piece's copies land)
  // counts rays whose inputs are in HBM. Helpers claim 1024-ray tiles (HELPER_TILE) to initialise
  // (*init_next, init_one) and set chunk_ready[c] for each 64-ray chunk they finish; an
  // integrator wave that claims a chunk waits for its flag. Finished rays count into
  // piece_cnt[p] as in DON = 2; once a piece is complete, helpers claim its tiles to finalize
  // (*fin_next, finalize_one) into the piece's SoA blob (blob + p blob_stride, piece_blob), and
  // the block that finalizes a piece's last tile sets host_flags[p] (host memory the host
  // polls, then copies the blob out). The helpers are a separate persistent kernel on a stream of
  // their own; one helper pass over every block slot initialises the first rays before the
  // integrator starts, and another finalizes the rest after it.
  const unsigned long long* host_ready;
  unsigned long long* host_flags;
  unsigned long long *init_next, *fin_next;
  unsigned long long* piece_fin;
  unsigned* chunk_ready;
  char* blob;
  int64_t blob_stride;
  int32_t blob_host;  // 1: the blobs are pinned host memory the helpers write over PCIe (no download copies)
  int32_t helpers;
  // The end of a streamed call without the integrator's stream (art_capi.cpp, HostLane): the
  // helpers bin the radiated flux of the rays they finalize (flux_hist, 2 flux_nbins doubles of
  // device memory, flux_nbins <= FLUX_HELPER_BINS; 0 = none), every integrator wave counts itself
  // into *waves_started as it starts and into *waves_done after its statistics, and the last of the
  // exit_expected serving helper blocks to leave (*exit_count) -- every ray is done by then -- waits
  // until every started wave is done (blocks the next call's kernels kept from starting find the
  // queue drained and add nothing), then copies the statistics (stats[0, N_STATS_DEV)) and the flux
  // into host memory (done_host[DONE_STATS...], [DONE_FLUX...]) and raises done_host[0]. The host
  // then has the call's results without waiting on a stream.
  double* flux_hist;
  int32_t flux_nbins;
  unsigned long long* done_host;
  unsigned long long *exit_count, *waves_started, *waves_done;
  int32_t exit_expected;
  // (calls in flight) the wave that starts last of the integrator's waves_total stores
  // resident_value into host-mapped *resident_host: the next call launches its own init pass and
  // integrator only then, so its blocks queue behind this launch's instead of sharing the GPU with it
  unsigned long long* resident_host;
  unsigned long long resident_value;
  int32_t waves_total;
  // Small batches (art_capi.cpp, propagate_device_impl): 1 = every fresh ray goes straight to
  // tail_kernel, one wave per ray (pack_fresh_kernel writes their CONT_REC records to cont),
  // instead of one lane per ray of the persistent integrator
  int32_t small_tail;
  // Graduation (DON = 1 launches with tail_kernel): a ray that has taken `graduate` step
  // attempts leaves its lane for the tail kernel at its next step boundary -- one wave per ray
  // from then on -- without waiting for its wave to drain: CONT_REC records in grad[0, grad_cap)
  // (count in *grad_count, which may pass grad_cap: a ray that finds no slot stays where it is),
  // taken by tail_kernel ahead of the drained waves' records. 0 = off.
  double* grad;
  unsigned long long *grad_count, *grad_queue;
  int32_t grad_cap, graduate;
  // Early graduation (DON = 1 launches with tail_kernel, art_capi.cpp): a ray whose progress
  // in ln t since its start is below hot_dtau + hot_slope log2(attempts / 256) -- tested at every
  // power-of-two attempt count >= hot_at, and when its drained wave donates it -- leaves for
  // hot[0, hot_cap) at once: the count in *hot_count (it may pass hot_cap: a ray that finds no
  // slot stays where it is), each record's hot_ready word raised once it is written.
  // configs[3]'s longest rays crawl along the star's surface and are singled out this way
  // (tail_kernel "hot rays"). A tail_kernel launch beside the bulk pass and the
  // continuation claims them through *hot_queue as they arrive, until *hot_done (raised after
  // the continuation) and none is left. hot_at 0 = off.
  double* hot;
  unsigned long long *hot_count, *hot_queue;
  unsigned* hot_ready;
  unsigned* hot_done;
  int32_t hot_cap, hot_at;
  double hot_dtau, hot_slope;
  // The bulk pass's claim order with early graduation (launch_propagate sorts it; null: ray index
  // order): the rays by their initial step size, smallest first -- configs[3]'s 20 longest rays
  // are among the 1066 with the smallest (tools/exp_gr_predict.py), so they start at once and reach
  // their hot test within the first few milliseconds. order_tmp: claim_order_bytes(n) of scratch.
  const int32_t* order;
  void* order_tmp;
};
constexpr unsigned long long STREAM_WAIT_TICKS = 200000000ull;  // 2 s at 100 MHz
constexpr int FLUX_HELPER_BINS = 256;  // flux bins the helpers bin themselves (2 x 256 doubles of LDS)
constexpr int DONE_STATS = 1, DONE_FLUX = 16;  // done_host layout: [0] flag | [1, 11) statistics | [16, 16 + 2 nbins) flux
constexpr int CHUNK = 64;  // rays a persistent wave claims from the queue at once
constexpr int HELPER_TILE = 1024;  // rays a helper block initialises or finalizes per claim
// The fresh state of ray i at u0 + i U0_REC (init_one writes it, a refilling integrator lane
// reads it): [u0 (7) | f(u0) (7) | dt | c0 | erg | ln t0 | species | 0], 160 bytes, 32-byte aligned.
constexpr int U0_REC = 20;
constexpr int END_REC = 16;
constexpr int X_REC = 8;
constexpr int CONT_REC = 24;  // [u (7) | f (7) | τ, dt, qpow, cprev, bstart, erg | int4 {ray, n_acc, n_rej, ncross} | int4 {iter, sprev, flags, save_k}]
constexpr int N_STATS = 8;  // propagate statistics: attempts, accepted, root re-steps, scan evals,
                            // interpolant-root evals, rays, init RHS, certified steps (art_last_stats)
// ... followed by the integrator's span from in-kernel clock stamps (s_memrealtime, the device's
// 100 MHz constant clock): [8] the max over waves of ~(start), [9] the max of the end
constexpr int ST_T0 = 8, ST_T1 = 9, N_STATS_DEV = 10;
constexpr double STAMP_TICKS_PER_MS = 1e5;
int persistent_blocks(const void* func, int64_t work, int block, int fallback_per_cu);
// propagate = init (u0 of every ray) -> the persistent integrator -> finalize (Cartesian
// end state, conversion probability at the crossings); ev0/ev1 (may be null) bracket the
// integrator kernels alone. With fs (and ev1) given, finalize runs on stream fs after ev1,
// so s can go on with its next launch while the outputs are written (the chunked host
// pipeline writes them over PCIe into pinned memory).
// hs: the side stream of the hot rays' tail launch (SegOut::hot), its fork and join events and two
// zeroed device words; without them the launch does not graduate early.
struct HotSide {
  hipStream_t stream = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  unsigned long long* zero_word = nullptr;
};
size_t claim_order_bytes(int64_t n);
// 200 ms at 100 MHz: a hot wave that has waited this long for a record leaves (the records still
// to come, if any, go to the tail launch after the continuation). In a 10^6-ray GR launch the
// hot records arrive within the first ~70 ms; a profiler that serialises kernels runs the
// continuation, and so the raising of *hot_done, only after this launch has ended.
constexpr unsigned long long HOT_WAIT_TICKS = 20000000ull;
constexpr int HOT_BLOCKS = 32;  // the hot rays' tail launch: 32 blocks of 4 waves (one ray a wave)
hipError_t launch_propagate(const KParams& P, int64_t n, const SegIn& in, const SegOut& out, int32_t max_crossings,
                            unsigned long long* queue, unsigned long long* stats, hipStream_t s, int* grid_out,
                            hipEvent_t ev0, hipEvent_t ev1, hipStream_t fs = nullptr, const HotSide& hs = HotSide());
// The streamed host pipeline's integrator (DON = 3) with at most `blocks` persistent blocks.
hipError_t launch_integrator_streamed(const KParams& P, int64_t n, const SegIn& in, const SegOut& out,
                                      int32_t max_crossings, unsigned long long* queue, unsigned long long* stats,
                                      int blocks, hipStream_t s, int* grid_out);
// The maskless streamed pipeline's helper duty (helper_kernel HK_TILES, SegOut::host_ready ...):
// `blocks` blocks; init_limit >= 0 initialises only (tiles below it), -1 serves to the end;
// announce counts each block into host_flags[64] as it starts.
hipError_t launch_helpers(const KParams& P, int64_t n, const SegIn& in, const SegOut& out, int blocks, int64_t init_limit,
                          int announce, unsigned long long* stats, hipStream_t s);
// The helper kernel (art_kernels_nolicm.hip, its own translation unit): the instantiation for these
// parameters' geometry, and its waves per SIMD (2: a helper block shares its CU with one
// integrator block; 1: it takes the whole CU).
using HFn = void (*)(const KParams, const int64_t, const SegIn, const SegOut, const int, const int64_t, const int64_t,
                     const int64_t, const int, unsigned long long*);
HFn pick_helper(const KParams& P);
// The integrator (propagate_kernel) and tail kernel builds of art_kernels_nolicm.hip: every geometry
// but flat's (nullptr for a combination no path launches). integ: ART_VERN6 / ART_RK4; geom: the
// GEOM_* of art_kernels.hip (0 any, 1 flat, 2 GR); don: the donation mode; wps: waves per SIMD.
using KFn = void (*)(const KParams, const int64_t, const SegIn, const SegOut, const int32_t, unsigned long long*,
                     unsigned long long*);
using TFn = void (*)(const KParams, const int64_t, const SegIn, const SegOut, const int32_t, const int32_t,
                     unsigned long long*);
KFn nl_propagate(int integ, int geom, bool save, int don, int wps);
TFn nl_tail(int geom);
// the sampler (find_samples_new) builds, also in art_kernels_nolicm.hip: wps 2 or 3 waves per SIMD,
// blocks: the blocks-of-steps line scan
using SFn = void (*)(const KParams, const double, const uint64_t, const int64_t, const int64_t, double*, double*,
                     double*, double*, int32_t*, int32_t*, unsigned long long*);
SFn nl_sample(int wps, bool blocks);
int helper_waves_per_simd(const KParams& P);
// The batch size up to which launch_propagate runs every ray on a wave of its own (tail_kernel):
// ART_SMALL_TAIL, default one ray per SIMD of the device; 0 switches it off.
int64_t small_tail_limit();
hipError_t launch_sample(const KParams& P, double maxR, uint64_t seed, int64_t ray_offset, int64_t n, double* x,
                         double* k, double* erg, double* vifty, int32_t* w, int32_t* att, unsigned long long* queue,
                         hipStream_t s, int waves);
hipError_t launch_prob(const KParams& P, int64_t nc, const double* pos, const double* kpos, const double* erg,
                       int64_t n_groups, const int64_t* gstart, double* out, hipStream_t s);
hipError_t launch_flux(const KParams& P, int64_t n, const double* x_end, const double* k_end, const int32_t* status,
                       const int8_t* species, const double* w, int32_t nbins, double* hist, hipStream_t s);
hipError_t launch_flux_phi(int64_t n, const double* phi, const int8_t* species, const double* w, int32_t nbins,
                           double lo, double hi, double* hist, hipStream_t s);
hipError_t launch_eval_rhs(const KParams& P, int64_t n, const double* u, const double* tau, const double* erg,
                           const int8_t* species, double* du, hipStream_t s);
hipError_t launch_eval_hamiltonian(const KParams& P, int64_t n, const double* x, const double* k, const double* T,
                                   const double* E, double* H, double* dHdx, double* dHdk, double* dHdT,
                                   hipStream_t s);
hipError_t launch_event_weight(const KParams& P, int64_t n, const double* x, const double* k, const double* v,
                               double maxR, double rho, double mcmc, double* out, hipStream_t s);
hipError_t launch_eval_condition(const KParams& P, int64_t n, const double* u, const double* tau, double* out,
                                 hipStream_t s);
}  // namespace art
