// mtgp_ab.h -- build-time knobs of the kernel library, kept out of the kernel source.
//
// Two kinds:
//  * tunables, whose defaults ARE the shipped configuration (each chosen by an A/B measurement
//    recorded in DESIGN.md); __graft_entry__.build_hip() never overrides them;
//  * diagnostics (MTGP_AB_*), 0 in the shipped build.  A non-zero value removes or replaces a
//    section of a kernel so that its cost can be measured by difference (scripts/kvariants.py,
//    __graft_entry__.build_variant, libraries under multitreegp_amd/lib/variants/).  Results
//    of such builds are wrong by construction and never compared against the oracle.
#ifndef MTGP_AB_H
#define MTGP_AB_H

// ---- tunables (shipped values)
#ifndef MTGP_COLD_INTERP
#define MTGP_COLD_INTERP 0  // fixed-step kernels: interpreter fallback out of line (1) or inline (0)
#endif
#ifndef MTGP_DP_COLD
#define MTGP_DP_COLD 0      // the same for the Dopri5 kernels
#endif
#ifndef MTGP_DP_WAVES
#define MTGP_DP_WAVES 2     // register budget of the Dopri5 control kernels (waves per SIMD)
#endif
#ifndef MTGP_FLAT_LANES
#define MTGP_FLAT_LANES 16  // lanes per program of the lane-per-program flattener (A/B kernel)
#endif

// ---- diagnostics (0 = shipped)
#ifndef MTGP_AB_NOPROG
#define MTGP_AB_NOPROG 0      // no program call at all (the environment and integrator alone)
#endif
#ifndef MTGP_AB_NOFALLBACK
#define MTGP_AB_NOFALLBACK 0  // ignore the JIT's slow-lane report (no interpreter re-run)
#endif
#ifndef MTGP_AB_FBCOUNT
#define MTGP_AB_FBCOUNT 0     // count JIT calls that report slow sin/cos lanes (mtgp_ab_fb_count)
#endif
#ifndef MTGP_AB_NOINTERP
#define MTGP_AB_NOINTERP 0    // JIT kernels without the interpreter (with NOFALLBACK: a readable ISA of the hot loop)
#endif
#ifndef MTGP_AB_FLAT_LANE
#define MTGP_AB_FLAT_LANE 0   // compile the lane-per-program flattener (MTGP_FLAT_MODE=lane selects it)
#endif
// Per-section cost of the fixed-step dynamic / static Acrobot kernels (DESIGN.md "C3 VALU budget"):
#ifndef MTGP_AB_NOTRIG
#define MTGP_AB_NOTRIG 0      // the drift's five sin/cos values replaced by one multiply each
#endif
#ifndef MTGP_AB_NODIV
#define MTGP_AB_NODIV 0       // the drift's four IEEE divisions replaced by multiplications
#endif
#ifndef MTGP_AB_SLOWDIV
#define MTGP_AB_SLOWDIV 0     // the drift's divisions always by the compiler's `/` sequence (no shared reciprocal)
#endif
#ifndef MTGP_AB_NODRIFT
#define MTGP_AB_NODRIFT 0     // the whole Acrobot drift replaced by dx = (thd1, thd2, u, -u)
#endif
#ifndef MTGP_AB_NOOBS
#define MTGP_AB_NOOBS 0       // observation = state (no angle wraps)
#endif
#ifndef MTGP_AB_NOSTORE
#define MTGP_AB_NOSTORE 0     // no trajectory stores
#endif
#ifndef MTGP_AB_NOFIT
#define MTGP_AB_NOFIT 0       // no online fitness update at the save points
#endif
// Save-point sections of the fixed-step static kernel (C2, round 5 ConstantStepSize cost):
#ifndef MTGP_AB_NOHERMITE
#define MTGP_AB_NOHERMITE 0   // the saved state is the step end y1 (no dense-output evaluation, no theta)
#endif
#ifndef MTGP_AB_NOSAVECALL
#define MTGP_AB_NOSAVECALL 0  // no policy call at a save point (us = the last stage's u)
#endif
// Debug build (round 5, never shipped): bounds checks on every trajectory-row store and on the
// Acrobot mask's fit_hist row index; a violation is counted (mtgp_debug_violations_tuN) and the
// access skipped instead of trapping, so a bad offset can never fault the GPU or hide silently.
#ifndef MTGP_DEBUG_CHECKS
#define MTGP_DEBUG_CHECKS 0
#endif

#ifndef MTGP_AB_WAVETIME
#define MTGP_AB_WAVETIME 0    // record each k_ctl_dynamic wave's start / end clock and HW_ID (mtgp_ab_wave_times)
#endif

#endif  // MTGP_AB_H
