// Fence around the timing experiments that compile deliberately WRONG verdicts into the
// kernels (DESIGN.md "Roofline"):
//   CPZ_EXP_SLAB_MOD  k_verify_each threads share table slots (an L2-sized slab)
//   CPZ_EXP_NOSPLIT   verify_proof skips the challenge split and the recodings
//   CPZ_CLOCK_PROBE   k_verify_each writes clock stamps over its statuses
//   CPZ_EXP_NIELS_TABLES  the Straus loop adds its table entries as affine Niels points
//                     (Z taken as 1, 7 M instead of 8 M, Z never loaded): the best case of
//                     affine per-proof tables, without the normalisation they would need
//   CPZ_EXP_EXTRA_INV one extra field inversion per equation (the normalisation's price)
// Such a build must say so: it does not compile unless CPZ_TIMING_ONLY is defined too, and
// then cpz_ctx_create refuses (CPZ_EINVAL, naming the flag) -- only the timing harness's
// cpz_ctx_create_timing_only (exported by these builds alone) opens a context.  The product
// library defines none of them.
#pragma once

#if defined(CPZ_EXP_SLAB_MOD)
#define CPZ_WRONG_VERDICT_FLAG "CPZ_EXP_SLAB_MOD"
#elif defined(CPZ_EXP_NOSPLIT)
#define CPZ_WRONG_VERDICT_FLAG "CPZ_EXP_NOSPLIT"
#elif defined(CPZ_CLOCK_PROBE)
#define CPZ_WRONG_VERDICT_FLAG "CPZ_CLOCK_PROBE"
#elif defined(CPZ_EXP_NIELS_TABLES)
#define CPZ_WRONG_VERDICT_FLAG "CPZ_EXP_NIELS_TABLES"
#elif defined(CPZ_EXP_EXTRA_INV)
#define CPZ_WRONG_VERDICT_FLAG "CPZ_EXP_EXTRA_INV"
#endif

#if defined(CPZ_WRONG_VERDICT_FLAG) && !defined(CPZ_TIMING_ONLY)
#error "CPZ_EXP_SLAB_MOD / CPZ_EXP_NOSPLIT / CPZ_CLOCK_PROBE / CPZ_EXP_NIELS_TABLES / CPZ_EXP_EXTRA_INV give wrong verdicts: build them with -DCPZ_TIMING_ONLY"
#endif
