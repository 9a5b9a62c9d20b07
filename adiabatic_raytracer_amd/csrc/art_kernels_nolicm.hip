// art_kernels_nolicm.hip -- the kernels compiled without MachineLICM (build.py adds
// -disable-machine-licm to this translation unit only): the helper kernel (init_one / finalize_one,
// the streamed pipeline's helper duty), the integrator for every geometry but flat's (GR, boundary
// layer, isotropic, RK4 with saveat) and the one-wave-per-ray tail kernel. MachineLICM hoists the
// loop bodies' polynomial and tableau constants (exp, sincos, acos, atan2, the Vern6 coefficients:
// ~150 v_mov_b32) out of the loops into registers live across them:
//   * the helper kernel then spilled 74-95 VGPRs to scratch at 2 waves per SIMD, and a persistent
//     helper using scratch stalled the next launch on another queue for seconds;
//   * the GR integrator spilled 60 VGPRs (226 without the pass, no spill): its bulk launch runs
//     3.4% faster without it, the lone tail ray 2% (profiles/r06q_gr_licm.jsonl).
// The flat integrator keeps the pass (art_kernels.hip): without it it spills nothing either but
// rematerialises the constants inside the step loop and runs 3% slower
// (profiles/r06o_ab_device_licm_off_everywhere.jsonl). The pass moves instructions and changes no
// arithmetic: the outputs are bit-identical (profiles/r06n_bitident_licm.log).
#define ART_NOLICM_TU 1
#include "art_kernels.hip"
