// forward_diag.hpp — timing proxies of the fused forward kernel (diagnostic builds only).
//
// Included by forward_wg.hpp only under -DMIB_DIAG, which no library build sets: tools/build_diag.sh,
// tools/build_clock.sh and tools/energy_budget.py builds add it together with one of the switches
// below.  Every proxy gives WRONG results; they exist to time or weigh a part of the kernel by
// removing it (DESIGN.md §3 energy and clock tables).  The finer proxies of rounds 1-4 (layer-1
// requant or MFMAs removed, pooling removed, 16x16 layer-2 tiles, extra VALU/MFMA/LDS work, the
// channel-major load patterns) are in git history (tools/build_base.sh 8da2a87 name -DMIB_DIAG_...).
//   MIB_DIAG_NOBAR       no barriers in the trial loop
//   MIB_DIAG_SAME_TRIAL  every trial reads trial 0 (no HBM traffic after the first)
//   MIB_DIAG_NOL2 / NOTAIL / NOL3 / NOL45  skip layer 2 / the layer-2 tail / layer 3 / layers 4-5
//   MIB_DIAG_L2_TWO      layer 2's full tiles run 2 of their 3 MFMAs (the upper bound of a 2:4
//                        sparse form: two smfmac_32x32x64 in place of three dense 32x32x32)
#pragma once

namespace mib {
namespace wg {

#ifdef MIB_DIAG_L2_TWO
constexpr int DIAG_L2_STEPS = 2;
#else
constexpr int DIAG_L2_STEPS = 3;
#endif

#ifdef MIB_DIAG_NOL2
constexpr bool DIAG_NOL2 = true;
#else
constexpr bool DIAG_NOL2 = false;
#endif
#ifdef MIB_DIAG_NOTAIL
constexpr bool DIAG_NOTAIL = true;
#else
constexpr bool DIAG_NOTAIL = false;
#endif
#ifdef MIB_DIAG_NOL3
constexpr bool DIAG_NOL3 = true;
#else
constexpr bool DIAG_NOL3 = false;
#endif
#ifdef MIB_DIAG_NOL45
constexpr bool DIAG_NOL45 = true;
#else
constexpr bool DIAG_NOL45 = false;
#endif

}  // namespace wg
}  // namespace mib

#ifdef MIB_DIAG_NOBAR
#define MIB_LOOP_BARRIER() ((void)0)
#else
#define MIB_LOOP_BARRIER() __syncthreads()
#endif
#ifdef MIB_DIAG_SAME_TRIAL
#define MIB_TRIAL_OFF(b) ((size_t)0 * (size_t)(b))
#define MIB_TRIALS_LEFT(b) ((int)(b) < B ? 1 : 0)
#else
#define MIB_TRIAL_OFF(b) ((size_t)(b) * K::XTRIAL)
#define MIB_TRIALS_LEFT(b) (B - (int)(b))
#endif
