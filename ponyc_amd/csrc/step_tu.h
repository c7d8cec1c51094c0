// step_tu.h — body of one k_step translation unit (step_*.hip): instantiates
// k_step<GPA_STEP_HT> and exports it with the upload of this code object's
// engine constants.
#define GPA_STEP_TU 1
#include "zone_dev.h"
#include "step_entry.h"

namespace gpa {

template __global__ void k_step<GPA_STEP_HT>(uint32_t, uint32_t, uint32_t);

namespace {
hipError_t step_upload(const TypeDev* types, const EngDev* eng, hipStream_t s)
{
  const hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_types), types,
    sizeof(TypeDev) * GPU_ACTOR_MAX_TYPES, 0, hipMemcpyHostToDevice, s);
  if(e != hipSuccess) return e;
  return hipMemcpyToSymbolAsync(HIP_SYMBOL(c_eng), eng, sizeof(EngDev), 0, hipMemcpyHostToDevice, s);
}
} // namespace

StepEntry GPA_STEP_ENTRY() { return { k_step<GPA_STEP_HT>, step_upload }; }

} // namespace gpa
