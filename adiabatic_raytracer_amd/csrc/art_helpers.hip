// art_helpers.hip -- the helper kernel (init_one / finalize_one, the streamed pipeline's helper
// duty) as a translation unit of its own, so it can be compiled with -disable-machine-licm
// (build.py): MachineLICM hoisted the polynomial constants of its ray loop (exp, sincos, acos,
// atan2: ~150 v_mov_b32) into VGPRs live across the loop, and at 2 waves per SIMD the kernel
// then spilled 74-95 VGPRs to scratch. The integrator kernels keep MachineLICM: without it they
// spill nothing either, but rematerialise those constants inside the step loop and run 3% slower
// (profiles/r06o_ab_device.jsonl). The arithmetic is the same either way (bit-identical outputs,
// profiles/r06n_bitident.log): the pass moves instructions, it does not change them.
#define ART_HELPER_TU 1
#include "art_kernels.hip"
