// step_tu.h — body of one k_step translation unit (step_*.hip): instantiates
// k_step<GPA_STEP_HT> and exports it with the upload of this code object's
// engine constants. A step_*_z12.hip unit first sets the 4096-actor zone
// geometry and renames the namespace (gpa -> gpa_z12), so both geometries'
// kernels link into one library.
#define GPA_STEP_TU 1
#include "zone_dev.h"
#include "step_entry.h"

namespace gpa {

// A/B experiment builds (-DGPA_STEP_ONLY=<table>) compile one instantiation;
// the others become stubs the host refuses to launch (GPU_ACTOR_EINVAL).
// Two-pass tables also compile the step as two launches (zone_dev.h k_step PM).
#if defined(GPA_STEP_ONLY) && (GPA_STEP_ONLY != GPA_STEP_HT)
#define GPA_STEP_STUB 1
template <int HT> __global__ void k_step_stub(uint32_t, uint32_t, uint32_t) {}
template __global__ void k_step_stub<GPA_STEP_HT>(uint32_t, uint32_t, uint32_t);
#else
#define GPA_STEP_STUB 0
template __global__ void k_step<GPA_STEP_HT, 0>(uint32_t, uint32_t, uint32_t);
// split for the two-pass table and for the general-path tables whose plain
// zones spill least without the cold paths (measured: C2-det, the storm)
// PM 3 (one launch, the rest through a call) for the two-pass table only:
// C2 70.4-71.0 us against 72.3-72.7 as two launches; C2-det 177-178 against
// 175.6 (profiles/r05w_fused_ab.txt)
template <int HT, int PM> constexpr step_kernel_t split_kernel()
{
  if constexpr(PM == 3 && !(HT >= 0 && two_pass<HT>()))
    return nullptr;
  else if constexpr(HT >= 0 && (two_pass<HT>() || HT == GPU_ACTOR_HT_PINGER_DET || HT == GPU_ACTOR_HT_STORM ||
                                HT == GPU_ACTOR_HT_PROGRAM ||
                                HT == kHtFifoPair))
    return k_step<HT, PM>;
  else return nullptr;
}
#endif

namespace {
hipError_t step_upload(const void* types, const void* eng, hipStream_t s)
{
  const hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_types), types,
    sizeof(TypeDev) * GPU_ACTOR_MAX_TYPES, 0, hipMemcpyHostToDevice, s);
  if(e != hipSuccess) return e;
  return hipMemcpyToSymbolAsync(HIP_SYMBOL(c_eng), eng, sizeof(EngDev), 0, hipMemcpyHostToDevice, s);
}
} // namespace

#if GPA_STEP_STUB
StepEntry GPA_STEP_ENTRY() { return { k_step_stub<GPA_STEP_HT>, step_upload, true, (uint32_t)kZoneBits,
                                      (uint32_t)kZoneThreads, kSortWork, 4u, false, nullptr, nullptr, nullptr }; }
#else
StepEntry GPA_STEP_ENTRY() { return { k_step<GPA_STEP_HT, 0>, step_upload, false, (uint32_t)kZoneBits,
                                      (uint32_t)kZoneThreads, kSortWork,
                                      (two_pass<GPA_STEP_HT>() || dp_table<GPA_STEP_HT>()) ? 6u : 4u,
                                      GPA_STEP_HT < 0 || GPA_STEP_HT == kHtFifoPair,
                                      split_kernel<GPA_STEP_HT, 1>(), split_kernel<GPA_STEP_HT, 2>(),
                                      split_kernel<GPA_STEP_HT, 3>() }; }
#endif

} // namespace gpa
