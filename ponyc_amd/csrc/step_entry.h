// step_entry.h — the compiled instantiations of k_step (zone_dev.h).
//
// Each instantiation lives in a translation unit of its own (step_*.hip), so
// the library builds them in parallel; each such unit is its own code object
// with its own copy of the engine constants (c_types, c_eng), which the host
// uploads to every unit (engine.hip: upload_types).
#pragma once
#include "engine_dev.h"

namespace gpa {

typedef void (*step_kernel_t)(uint32_t, uint32_t, uint32_t);

struct StepEntry {
  step_kernel_t kernel;
  hipError_t (*upload)(const TypeDev* types, const EngDev* eng, hipStream_t s);
  bool stub;               // not compiled in this (experiment) build
};

StepEntry step_entry_any();             // any mix of handler tables
StepEntry step_entry_ring();
StepEntry step_entry_pinger();
StepEntry step_entry_pinger_det();
StepEntry step_entry_fanin_sender();
StepEntry step_entry_gups_streamer();
StepEntry step_entry_storm();
StepEntry step_entry_spreader();

} // namespace gpa
