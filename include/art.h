/*
 * art.h -- C ABI of libart.so, the MI355X (gfx950) engine for the hot path of
 * SamWitte/Adiabatic_RayTracer: the per-ray Hamiltonian ODE of a photon/axion
 * segment around a neutron star (Goldreich-Julian plasma, rotating dipole,
 * Schwarzschild metric), its Vern6/RK4 integration, resonance detection and the
 * conversion probability at each crossing.
 *
 * Every entry point replaces a reference interface (file:line under
 * /root/reference/src):
 *
 *   art_propagate_host / _device   RT.propagate              RayTracer.jl:171-452
 *       (callers MainRunner.jl:179-182 photon, :187-190 axion)
 *   art_propagate_traj_host/_dev   RT.propagate with saveat points (RayTracer.jl:176,383,444)
 *   art_get_prob_nonad_host/_dev   get_Prob_nonAD            MainRunner.jl:67-124
 *       (-> RT.conversion_prob RayTracer.jl:1405-1473; callers MainRunner.jl:134,265)
 *   art_sample_conversion_points_* RT.find_samples_new + k_norm_Cart
 *                                  RayTracer.jl:1480-1653, MainRunner.jl:463-529
 *   art_find_conversion_surface    RT.Find_Conversion_Surface RayTracer.jl:1250-1263
 *   art_flux_histogram_device      plot/flux.py:38-48 (binned flux of segment end states)
 *   art_flux_histogram_phi_device  plot/flux.py:38-48 (binned flux of the npy rows' φf;
 *   art_flux_histogram_phi_range_device  _range: over flux.py's data-dependent bins)
 *   art_propagate_host_flux        RT.propagate + the batch's binned flux (bench.py's step)
 *   art_propagate_host_flux_async  the same, two batches in flight; art_host_wait
 *   art_comm_* / art_flux_allreduce  the reduction of the flux and counters over the GPUs of
 *                                  a node (the reference merges files instead,
 *                                  Combine_Files.py, Gen_Samples.jl:195-239)
 *   art_grow_trees[_traj]          get_tree (MainRunner.jl:126-352) for n trees, batched
 *                                  (_traj: + saveNode data, MainRunner.jl:17-65)
 *   art_event_weight_*             sln_prob of a sampled point: dwp_ds cos_w + g_det
 *                                  (MainRunner.jl:498-557, RayTracer.jl:734-754,1327-1403)
 *   art_eval_*_device              pointwise physics (func!, func_axion!, hamiltonian,
 *                                  GJ_Model_ωp_vecSPH, condition) for parity tests
 *
 * Conventions
 *   - All arrays are caller-owned. Position/momentum arrays are structure-of-arrays,
 *     exactly the memory of a Julia column-major N x 3 Matrix{Float64}:
 *     x[0..n) = x-column, x[n..2n) = y-column, x[2n..3n) = z-column.
 *   - *_host entry points take host pointers and do H2D/kernel/D2H on the library's
 *     own HIP stream (a Julia ccall passes Vector/Matrix pointers straight through).
 *     *_device entry points take device (HBM) pointers plus a hipStream_t passed as
 *     void*, used exactly as given (NULL = the HIP null stream, which is also
 *     PyTorch's default stream); they are asynchronous on that stream.
 *   - Return 0 on success or a negative ART_E* code; art_last_error() describes it.
 *   - Thread safety: calls are issued under an internal mutex; one device per call
 *     (art_set_device). *_host calls are synchronous. *_device calls only enqueue work:
 *     every propagate / sampler launch allocates its own scratch (work-queue word,
 *     statistics, fresh-state and end-record buffers) from the stream-ordered allocator
 *     and frees it in stream order, so launches on different streams may run
 *     concurrently and never share device state.
 */
#ifndef ART_H
#define ART_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ART_ABI_VERSION 1

/* error codes */
#define ART_OK 0
#define ART_E_INVALID (-1)     /* bad argument / unsupported option */
#define ART_E_HIP (-2)         /* HIP runtime error */
#define ART_E_NOMEM (-3)       /* device allocation failed */
#define ART_E_UNSUPPORTED (-4) /* melrose=0 (dead code at the reference's fixed flags) */

/* integrators */
#define ART_VERN6 0 /* adaptive Verner 6(5), the reference's Vern6() (RayTracer.jl:383) */
#define ART_RK4 1   /* fixed-step classical RK4 in ln t (BASELINE config 1) */

/* per-ray segment status (the reference's sol.retcode, refined) */
#define ART_STATUS_SUCCESS 0    /* reached ln_t_end                      (:Success)    */
#define ART_STATUS_CROSSING 1   /* terminate! after max_crossings         (:Terminated) */
#define ART_STATUS_HIT_NS 2     /* photon r < 1.01 rNS (cb_r, :352-368)   (:Terminated) */
#define ART_STATUS_MAXITERS 3   /* maxiters step attempts                 (:MaxIters)   */
#define ART_STATUS_NONFINITE 4  /* NaN/Inf in state or error estimate     (:Unstable)   */

/* max_crossings of art_propagate_*: no callbacks (RT.propagate with make_tree = false) */
#define ART_NO_CALLBACKS (-2147483647 - 1)

/* species (RT.node.species; MainRunner.jl:175-191) */
#define ART_AXION 0
#define ART_PHOTON 1

typedef struct art_params {
  /* physics: Gen_Samples.jl:139-170, Mvars of MainRunner.jl:177-178,185-186 */
  double theta_m;   /* θm misalignment angle [rad]                                  */
  double omega_pul; /* ωPul rotation frequency [1/s]                                */
  double B0;        /* surface dipole field [G]                                     */
  double rNS;       /* neutron-star radius [km]                                     */
  double mass_ns;   /* Mass_NS [solar masses]; get_Prob_nonAD always uses this GR   */
                    /* mass, even when flat != 0 (MainRunner.jl:75, global)         */
  double mass_a;    /* axion mass [eV]                                              */
  double g_agg;     /* axion-photon coupling Ax_g [1/GeV]                          */
  double bndry_lyr; /* boundary-layer index; <= 0 disables (Gen_Samples.jl:130)    */
  /* numerics: NumerP = [ln_tstart, ln_tend, ode_err] (MainRunner.jl:411-413),       */
  /* solve(...) keywords RayTracer.jl:383-384                                        */
  double ln_t_end;  /* log(1/ωPul)                                                  */
  double abstol;    /* ode_err = 1e-6                                               */
  double reltol;    /* 1e-7                                                         */
  double dtmin;     /* 1e-13 with force_dtmin = true                                */
  int64_t maxiters; /* 1e5 step attempts                                            */
  int32_t flat;     /* 1: Mass_NS -> 0 in the ray equations (RayTracer.jl:77,187)   */
  int32_t isotropic;/* 1: k_par -> 0                                                */
  int32_t melrose;  /* must be 1 (Gen_Samples.jl:167)                               */
  int32_t integrator;    /* ART_VERN6 or ART_RK4                                    */
  int32_t n_fixed;       /* RK4: steps per segment                                  */
  int32_t interp_points; /* ContinuousCallback interp_points (RayTracer.jl:358 = 50),*/
                         /* at most 65                                             */
} art_params;

/* Outputs of one batch of segments (the 14-tuple of RayTracer.jl:448, per ray). */
typedef struct art_segment_out {
  double* x_end;     /* 3n  final Cartesian position [km]       (x_reshaped[:, :, end]) */
  double* k_end;     /* 3n  final Cartesian momentum [eV]       (v_reshaped[:, :, end]) */
  double* u7_end;    /* n   final u[7] = erg*Δω                 (dt[:, end], :431)      */
  double* tau_end;   /* n   final ln t                          (times[end], :444)      */
  int32_t* status;   /* n   ART_STATUS_*                                               */
  int32_t* n_accept; /* n   accepted steps                                             */
  int32_t* n_reject; /* n   rejected steps                                             */
} art_segment_out;

/* Resonance crossings (xc..Δωc of RayTracer.jl:325-342), layout [(c*cap + j)*n + i]
 * for component c, crossing j < capacity, ray i. Slots j >= min(count[i], capacity) hold no
 * crossing (the reference's arrays simply end there): the *_device entry points leave them
 * unwritten, the *_host entry points fill them with NaN. */
typedef struct art_crossing_buf {
  int32_t capacity; /* crossings stored per ray (1 for forward trees)               */
  int32_t* count;   /* n  crossings recorded (> capacity means overflow)            */
  double* pos;      /* 3*cap*n  xc, yc, zc [km]                                     */
  double* k;        /* 3*cap*n  kxc, kyc, kzc [eV]                                  */
  double* t;        /* cap*n    tc = exp(τ) [s]                                     */
  double* dw;       /* cap*n    Δωc = u7/erg                                        */
  double* p_nonad;  /* cap*n    get_Prob_nonAD at the crossing, Nc = 1 semantics   */
} art_crossing_buf;

/* ---- library / device ---- */
int art_abi_version(void);
const char* art_last_error(void);
int art_device_count(int32_t* count);
int art_set_device(int32_t device);
int art_synchronize(void);
/* Releases every device object the library holds (streams, events, pooled HBM and pinned
 * staging, the host-mapped flags of the streamed pipeline, the host copy threads) after
 * draining its work; the next call re-creates what it needs. The library registers this to run at process exit, before the HIP
 * runtime's own teardown; a host may also call it itself. */
int art_shutdown(void);
/* Duration [ms] of the last propagate kernel, from HIP events recorded on the stream
 * the kernel ran on. */
double art_last_kernel_ms(void);
/* Counters of the last propagate launch: [step attempts, accepted steps, root re-steps,
 * scan condition evals, interpolant-root condition evals, rays, init RHS evals, 0] and the
 * persistent grid size; they feed the roofline accounting of bench.py. */
int art_last_stats(uint64_t* stats, int32_t* grid);
/* Integrator-kernel durations [ms] of the last min(n, 64) propagate launches on the current
 * device, oldest first, each from the HIP events around that launch on its own stream (waits
 * for them). Returns the number written (>= 0) or a negative ART_E* code. */
int art_recent_kernel_ms(int32_t n, double* ms);
/* The same launches' integrator spans [ms] from in-kernel clock stamps: the first wave's start
 * to the last wave's end on the device's 100 MHz constant clock (s_memrealtime), so free of a
 * profiler's per-dispatch completion signals; -1 where a launch left none. Returns the number
 * written (>= 0) or a negative ART_E* code. (No reference counterpart: measurement) */
int art_recent_kernel_span_ms(int32_t n, double* ms);
/* Tail donation for propagate launches that are pipelined with others (several batches in
 * flight on different streams): once a launch's work queue is drained, a wave with at most
 * `lanes` live rays (all between steps) hands them to a continuation launch on the same
 * stream and retires, so its CU slot goes to the next batch instead of idling behind one
 * long ray. The continuation launch integrates the donated rays packed into full waves, and
 * its own last rays finish one per wave (the tail kernel); results are bit-identical to
 * lanes = 0 (off). -1 (the default) chooses by geometry: 16 for Schwarzschild Vern6 batches,
 * whose few longest rays set a lone batch's wall time (configs[3]), 0 otherwise. Applies to
 * the current device's subsequent launches (the streamed host pipeline never donates). No
 * reference counterpart (an execution policy). */
int art_set_tail_donation(int32_t lanes);
/* Graduation for Vern6 launches with tail donation (the Schwarzschild default): a ray still
 * stepping after `attempts` step attempts leaves its lane at its next step boundary for the
 * one-wave-per-ray tail kernel, so a batch's longest rays run at lone-wave speed without waiting
 * for their waves to drain (configs[3] as one batch: 260-297 -> 230 ms). 0 switches it off -- for
 * a host that keeps several batches in flight, where each graduated ray would hold a whole tail
 * wave while the other batches fill the CUs it frees; -1 (the default) = 2048 attempts (or
 * ART_GRADUATE). Per device; results are bit-identical either way.
 * With graduation on, a launch on a non-blocking stream also graduates early: from 128 attempts
 * on, a ray whose progress in ln t lags 15.95 + 0.75 log2(attempts / 256) (ART_HOT_AT,
 * ART_HOT_DTAU, ART_HOT_SLOPE) -- on configs[3] the rays that crawl along the star's surface,
 * every one of its 20 longest among them -- leaves at once for a tail-kernel launch that runs on
 * a side stream beside the bulk pass, and the bulk pass claims its rays smallest initial step
 * first (configs[3] as one batch: 226 -> 188 ms). Not on the null stream or another blocking
 * stream, whose work would wait for that side launch. */
int art_set_graduation(int32_t attempts);
/* Waves per SIMD of the conversion-point sampler (art_sample_conversion_points*): 0 (the default)
 * chooses by line length -- 3 for lines up to 2.2 x 60 km, walked step by step, else 2 with blocks
 * of 3 steps, the faster builds for one launch at a time; 3 takes the 3-wave build for every line,
 * which packs better beside other sampler launches in flight on other streams (the 32-point scan's
 * sampling on 8 streams: 0.503-0.508 -> 0.484 s, profiles/r05ah_scan_sampler_waves.txt). Per
 * device; samples are bit-identical either way. No reference counterpart (an execution policy). */
int art_set_sampler_waves(int32_t waves);
/* The Vern6 tableau the kernel uses: c[9], A[81] row-major, b[9], bhat[9]. */
int art_vern6_tableau(double* c, double* A, double* b, double* bhat);

/* ---- RT.Find_Conversion_Surface (RayTracer.jl:1250-1263), pure host math ---- */
double art_find_conversion_surface(const art_params* p);

/* ---- RT.propagate for a batch of n segments (RayTracer.jl:171-452) ----
 * x0, k0   : 3n Cartesian start position [km] / momentum (rescaled onto the axion
 *            mass shell in-kernel exactly as k_norm_Cart, RayTracer.jl:179-186)
 * erg      : n  Mvars erg (erg_inf_ini) [eV]
 * dw       : n  Δω (u0[7] = erg*Δω, RayTracer.jl:216)
 * ln_t0    : n  NumerP[1] = log(max(event.t, e^-30)) (MainRunner.jl:166)
 * species  : n  ART_PHOTON (func!) or ART_AXION (func_axion!)
 * max_crossings : terminate! once this many crossings are recorded (RayTracer.jl:346);
 *            <= 0 means "stop at the first new crossing" exactly like the reference's
 *            splittings_cutoff = -1 (MainRunner.jl:128). ART_NO_CALLBACKS integrates the
 *            plain ODE with no callbacks, as the reference does for make_tree = false
 *            (RayTracer.jl:361-377): no crossing is recorded and photons are not stopped
 *            at 1.01 rNS.
 * xc may be NULL when crossings are not wanted (the segment still stops on them).
 * art_propagate_host streams Vern6 batches of 2^20 rays and more: one
 * integrator launch while the inputs are still being copied in and finished pieces already
 * copied out; the outputs are those of one launch bit for bit, and a streamed call that outlasts
 * its bounds runs again as one launch (counted by art_host_path_counters). */
int art_propagate_host(const art_params* p, int64_t n, const double* x0, const double* k0,
                       const double* erg, const double* dw, const double* ln_t0,
                       const int8_t* species, int32_t max_crossings,
                       art_segment_out* out, art_crossing_buf* xc);
int art_propagate_device(const art_params* p, int64_t n, const double* x0, const double* k0,
                         const double* erg, const double* dw, const double* ln_t0,
                         const int8_t* species, int32_t max_crossings,
                         art_segment_out* out, art_crossing_buf* xc, void* stream);
/* art_propagate_host plus the batch's binned radiated flux (plot/flux.py:38-48, the quantity
 * MainRunner.jl:749 normalises): hist[2*nbins] (host, overwritten; row 0 axions, row 1
 * photons) counts the segments that end without a crossing beyond 1.1 rNS (MainRunner.jl:
 * 203-209) by the azimuth atan2(k_y, k_x) of their final momentum, in nbins equal bins of
 * [-pi, pi] with np.histogram's bin assignment. It is binned on the device while the outputs
 * are still in HBM, so it costs no second pass over them; a multi-process run sums hist over
 * its ranks (art_flux_allreduce_host). */
int art_propagate_host_flux(const art_params* p, int64_t n, const double* x0, const double* k0,
                            const double* erg, const double* dw, const double* ln_t0,
                            const int8_t* species, int32_t max_crossings, art_segment_out* out,
                            art_crossing_buf* xc, int32_t nbins, double* hist);
/* art_propagate_host_flux, asynchronous: checks the arguments, returns at once with *ticket, and
 * runs the call on a library worker thread; art_host_wait(ticket) returns the call's result code.
 * Two calls per device can be in flight (a third waits for the lane of the one two before it),
 * each with its own streams and staging, so the next batch's uploads and first rays overlap this
 * batch's drain (MainRunner.jl:179-190 calls RT.propagate batch after batch; a host that has the
 * next batch ready submits it before waiting for this one). Every buffer of a call must stay
 * valid and untouched until its art_host_wait returns; wait on the device the call was submitted
 * on. A batch the streamed pipeline does not take (below ART_HOST_CHUNK_MIN rays, default 2^20)
 * runs inside the submitting call and its ticket is complete. Synchronous host calls first wait
 * for every asynchronous one. Results equal art_propagate_host_flux's bit for bit. */
int art_propagate_host_flux_async(const art_params* p, int64_t n, const double* x0, const double* k0,
                                  const double* erg, const double* dw, const double* ln_t0,
                                  const int8_t* species, int32_t max_crossings, art_segment_out* out,
                                  art_crossing_buf* xc, int32_t nbins, double* hist, int64_t* ticket);
/* Waits for an asynchronous host call and returns its result (ART_OK or the ART_E* code it
 * failed with; art_last_error() then says why). Each ticket is waited for once. */
int art_host_wait(int64_t ticket);
/* What the art_propagate_host* calls of this process ran as, since load or the last reset:
 * [0] calls, [1] streamed-pipeline completions, [2] streamed-pipeline give-ups (a wait
 * outlasted its bound; the batch then ran again as one launch, same results), [3] chunked-
 * pipeline calls, [4] single-launch calls (a give-up counts there too). Writes min(n, 5)
 * counters (0 beyond), resets them when reset != 0, and returns 5. No reference counterpart
 * (execution-path bookkeeping; bench.py asserts no give-up inside its timed passes). */
int art_host_path_counters(uint64_t* counters, int32_t n, int32_t reset);

/* ---- RT.propagate with its saved points (saveat, RayTracer.jl:176, 383, 427-444) ----
 * As art_propagate_*, plus up to ntimes (>= 2) saved points per ray: the start, the
 * interior times ln_t0 + k (ln_t_end - ln_t0)/(ntimes - 1) that the segment reached before
 * it ended (from the step's cubic Hermite interpolant), and the end state -- the
 * reference's x_reshaped[:, :, k] and times = sol.t, without the duplicate points DiffEq
 * adds at callback events. Used by saveMode 3 tree dumps (saveNode, MainRunner.jl:17-65).
 * traj: 3*ntimes*n Cartesian positions [(c*ntimes + k)*n + i]; traj_t: ntimes*n ln t
 * [k*n + i]; traj_n: n points per ray (2 .. ntimes). */
int art_propagate_traj_host(const art_params* p, int64_t n, const double* x0, const double* k0,
                            const double* erg, const double* dw, const double* ln_t0,
                            const int8_t* species, int32_t max_crossings, art_segment_out* out,
                            art_crossing_buf* xc, int32_t ntimes, double* traj, double* traj_t,
                            int32_t* traj_n);
int art_propagate_traj_device(const art_params* p, int64_t n, const double* x0, const double* k0,
                              const double* erg, const double* dw, const double* ln_t0,
                              const int8_t* species, int32_t max_crossings, art_segment_out* out,
                              art_crossing_buf* xc, int32_t ntimes, double* traj, double* traj_t,
                              int32_t* traj_n, void* stream);

/* ---- get_Prob_nonAD (MainRunner.jl:67-124) ----
 * One call of the reference per group: group g covers crossings
 * [group_start[g], group_start[g+1]) and reproduces the reference's column-major
 * linear indexing of ksphere/Bsphere inside conversion_prob (RayTracer.jl:1432-1443)
 * for groups with more than one crossing. group_start == NULL means n_groups == nc
 * groups of one crossing each (forward-tree semantics).
 * pos, kpos: 3nc Cartesian; erg_eff: nc = erg_inf_ini .* abs.(Δωc). out: nc P_nonAD. */
int art_get_prob_nonad_host(const art_params* p, int64_t nc, const double* pos,
                            const double* kpos, const double* erg_eff,
                            int64_t n_groups, const int64_t* group_start, double* out);
int art_get_prob_nonad_device(const art_params* p, int64_t nc, const double* pos,
                              const double* kpos, const double* erg_eff,
                              int64_t n_groups, const int64_t* group_start, double* out,
                              void* stream);

/* ---- conversion-surface sampler (find_samples_new, RayTracer.jl:1480-1653) ----
 * Draws one accepted sample per ray i in [0, n) with a Philox4x32-10 stream keyed by
 * (seed, ray_offset + i): attempts are repeated until accepted (MainRunner.jl:463-495).
 * Outputs (n or 3n, SoA): x [km], k_init (k_norm_Cart onto the axion shell, :529),
 * erg_inf_ini [eV] (:526), vifty = vIfty/c (unitless, :1651), weights (# crossings on
 * the accepted line, :1636), attempts (# find_samples_new calls, feeds f_inx :469). */
int art_sample_conversion_points_host(const art_params* p, double max_r, uint64_t seed,
                                      int64_t ray_offset, int64_t n, double* x, double* k_init,
                                      double* erg_inf, double* vifty, int32_t* weights,
                                      int32_t* attempts);
int art_sample_conversion_points_device(const art_params* p, double max_r, uint64_t seed,
                                        int64_t ray_offset, int64_t n, double* x,
                                        double* k_init, double* erg_inf, double* vifty,
                                        int32_t* weights, int32_t* attempts, void* stream);

/* ---- batched tree driver: get_tree (MainRunner.jl:126-352) for n trees at once ----
 * Roots are RT.node(x0, k0, t = 0, Δω = -1, species, prob = 1, weight = 1, -1, -1, -1) with
 * root.prob replaced by 1 - exp(-P_nonAD) at the root (:132-137), as main_runner_tree
 * builds both its backtrace (axion, -k, -B0: pass p with B0 negated) and its forward
 * (photon) trees (:578-590, :653-667). Every round propagates the next node of every
 * active tree in one batched launch. Per tree the reference's rules are kept: pop the
 * highest-weight event (stable sort by weight), stop each segment at its first crossing
 * when splittings_cutoff <= 0, full splitting while count <= mc_nodes and one
 * Monte-Carlo branch after (Philox4x32-10 keyed by (seed, tree, count) in place of
 * rand(Float64)), the |kc| > 1 rule, the 1e-5 km crossing merge, the stop rules and the
 * info codes 1..4 (negative once Monte-Carlo). */
typedef struct art_tree_opts {
  int32_t num_cutoff;        /* 5   (Gen_Samples.jl default)                       */
  int32_t mc_nodes;          /* 5                                                  */
  int32_t max_nodes;         /* 50                                                 */
  int32_t splittings_cutoff; /* -1: forward trees; 100000: backtrace (:588)        */
  int32_t crossing_cap;      /* crossings stored per segment when splittings > 0   */
  int32_t tree_offset;       /* global id of tree 0: the Monte-Carlo draws are keyed */
                             /* by (seed, tree_offset + i, count), so a run sharded */
                             /* over ranks by event id draws what one process would */
  double prob_cutoff;        /* 1e-10                                              */
  uint64_t seed;             /* key of the Monte-Carlo draws                        */
} art_tree_opts;

/* One RT.node of a finished tree, in the order get_tree pushed it onto `tree`. */
typedef struct art_tree_node {
  int32_t tree;      /* index of its root                                          */
  int32_t species;   /* ART_AXION / ART_PHOTON                                     */
  int32_t is_final;  /* no crossing and |x_end| > 1.1 rNS (:200-207)               */
  int32_t n_cross;   /* crossings kept on its segment (after the 1e-5 km merge)    */
  int32_t status;    /* ART_STATUS_* of its segment                                */
  int32_t pad;
  double weight, prob, parent_weight, prob_conv, prob_conv0;
  double x0[3], k0[3], t0, dw0;               /* node.x .. node.Δω (start)          */
  double x_end[3], k_end[3], u7_end, tau_end; /* traj[end], mom[end], erg[end], ln t */
  double xc[3], kc[3], tc, dwc, pc;           /* first crossing, Pc = 1 - e^-P_nonAD */
} art_tree_node;

/* x0, k0: 3n SoA; erg: n erg_inf_ini; species: n. nodes: caller-owned, node_capacity
 * records; *n_nodes receives the number of nodes (returns ART_E_NOMEM with the needed
 * count when node_capacity is too small). counts, infos (n, may be NULL): get_tree's
 * `count` and `info`. Host pointers; synchronous. */
int art_grow_trees(const art_params* p, int64_t n, const double* x0, const double* k0,
                   const double* erg, const int8_t* species, const art_tree_opts* opts,
                   int64_t node_capacity, art_tree_node* nodes, int64_t* n_nodes,
                   int32_t* counts, int32_t* infos);

/* saveMode 3 tree dumps (saveNode, MainRunner.jl:17-65, called at :612 and :671): per node,
 * its saved trajectory points (art_propagate_traj_*) and all of its crossings after the
 * 1e-5 km merge. Arrays are caller-owned, node_capacity records each. */
typedef struct art_tree_traj {
  int32_t ntimes;       /* saved points per segment, >= 2 (Gen_Samples.jl:164: 3)            */
  int32_t crossing_cap; /* crossings kept per node in xc                                      */
  double* traj;         /* node_capacity*ntimes*3 Cartesian positions [node][k][c]            */
  double* times;        /* node_capacity*ntimes   ln t of each point (sol.t, RayTracer.jl:444) */
  int32_t* count;       /* node_capacity          points of each node                         */
  double* xc;           /* node_capacity*crossing_cap*4 (x, y, z, tc) [node][j][c]             */
} art_tree_traj;
/* art_grow_trees plus the saveNode data of every node. */
int art_grow_trees_traj(const art_params* p, int64_t n, const double* x0, const double* k0,
                        const double* erg, const int8_t* species, const art_tree_opts* opts,
                        int64_t node_capacity, art_tree_node* nodes, int64_t* n_nodes,
                        int32_t* counts, int32_t* infos, const art_tree_traj* traj);

/* ---- event weight of sampled points (MainRunner.jl:498-557) ----
 * For n sampled conversion points (x, k_init, vifty: 3n SoA, as returned by the
 * sampler) computes out (5n SoA): cos_w of dwp_ds (RayTracer.jl:1327-1403),
 * jacobian_GR = g_det (:734-754, 1 when flat), sln_prob (the incoming axion rate,
 * npy column 8 before the division by f_inx, :549-552), erg_inf_ini (:517) and
 * vel_eng (:513). rho_dm [GeV/cm^3] defaults to 0.45 and mcmc_weight = n_maxSample = 6
 * in the reference (MainRunner.jl:356-362,480). */
int art_event_weight_host(const art_params* p, double max_r, double rho_dm, double mcmc_weight, int64_t n,
                          const double* x, const double* k_init, const double* vifty, double* out);
int art_event_weight_device(const art_params* p, double max_r, double rho_dm, double mcmc_weight, int64_t n,
                            const double* x, const double* k_init, const double* vifty, double* out,
                            void* stream);

/* ---- binned flux (plot/flux.py:38-48): histogram of the final momentum azimuth
 * φf = atan2(ky, kx) over [-π, π) in nbins bins, separately for axions (row 0) and
 * photons (row 1), weight w[i] (NULL = 1), only rays that ended without a crossing
 * (status != ART_STATUS_CROSSING) and whose final radius exceeds 1.1 rNS -- the
 * reference's is_final (MainRunner.jl:200-207), whatever the retcode. hist (2*nbins, device,
 * float64) is ACCUMULATED into (zero it first). */
int art_flux_histogram_device(const art_params* p, int64_t n, const double* x_end,
                              const double* k_end, const int32_t* status,
                              const int8_t* species, const double* w, int32_t nbins,
                              double* hist, void* stream);

/* ---- binned flux of the npy rows (plot/flux.py:38-48): np.histogram(phif, nbins,
 * range = (-π, π), weights = w) of the given azimuths φf (npy column 4, MainRunner.jl:715),
 * axions (species 0) into row 0 and photons into row 1 of hist (2*nbins, device, float64),
 * with numpy's bin assignment (edges linspace(-π, π, nbins + 1), the right edge in the last
 * bin, values outside [-π, π] dropped). hist is ACCUMULATED into. The reference's radiated
 * flux is row 1 with w = weight * sln_prob (columns 9 and 8). */
int art_flux_histogram_phi_device(int64_t n, const double* phi, const int8_t* species, const double* w,
                                  int32_t nbins, double* hist, void* stream);
/* The same over [lo, hi] (finite, lo < hi): plot/flux.py:43-47 itself calls np.histogram(phif,
 * bins=50) without a range, i.e. over [min φf, max φf] of the rows, and this reproduces those
 * bins (edges linspace(lo, hi, nbins + 1), numpy's bin assignment). */
int art_flux_histogram_phi_range_device(int64_t n, const double* phi, const int8_t* species, const double* w,
                                        int32_t nbins, double lo, double hi, double* hist, void* stream);

/* ---- reduction over the GPUs of a node (RCCL over xGMI) ----
 * One process per GPU. Rank 0 calls art_comm_unique_id and shares the 128 bytes with the
 * other ranks (a file, MPI, the launcher); every rank then calls art_comm_init on its device.
 * art_flux_allreduce sums count float64 values of a device buffer in place over all ranks,
 * asynchronously on `stream` (the binned flux and the run's counters f_inx, Σ weight, ...).
 * RCCL is opened on first use; without it these return ART_E_UNSUPPORTED. */
typedef struct art_rccl_id {
  char internal[128]; /* ncclUniqueId */
} art_rccl_id;
int art_comm_unique_id(art_rccl_id* id);
int art_comm_init(int32_t rank, int32_t world, const art_rccl_id* id);
int art_flux_allreduce(double* buf, int64_t count, void* stream);
/* the same for a host buffer (staged through HBM; synchronous) */
int art_flux_allreduce_host(double* buf, int64_t count);
int art_comm_destroy(void);

/* ---- pointwise physics on device, for parity tests (u: 7n SoA r,θ,φ,w_r,w_θ,w_φ,u7) */
/* func!/func_axion! (RayTracer.jl:71-123): du (7n) */
int art_eval_rhs_device(const art_params* p, int64_t n, const double* u, const double* tau,
                        const double* erg, const int8_t* species, double* du, void* stream);
/* hamiltonian (RayTracer.jl:530-556) at spherical x (3n), covariant k (3n), time T (n),
 * energy E (n): H (n), dH/dx (3n), dH/dk (3n), dH/dT (n). bndry_lyr applies to all. */
int art_eval_hamiltonian_device(const art_params* p, int64_t n, const double* x,
                                const double* k, const double* T, const double* E,
                                double* H, double* dHdx, double* dHdk, double* dHdT,
                                void* stream);
/* resonance condition (RayTracer.jl:254-298): value (n) */
int art_eval_condition_device(const art_params* p, int64_t n, const double* u,
                              const double* tau, double* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ART_H */
