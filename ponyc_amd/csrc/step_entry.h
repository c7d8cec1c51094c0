// step_entry.h — the compiled instantiations of k_step (zone_dev.h).
//
// Each instantiation lives in a translation unit of its own (step_*.hip), so
// the library builds them in parallel; each such unit is its own code object
// with its own copy of the engine constants (c_types, c_eng), which the host
// uploads to every unit (engine.hip: upload_types).
//
// Two zone geometries are compiled: 2048-actor zones with 512-thread
// workgroups (namespace gpa, step_*.hip) and 4096-actor zones with 1024-thread
// workgroups (namespace gpa_z12, step_*_z12.hip: the same sources with the
// namespace renamed). The host picks one per engine (engine.hip: relayout_zones).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef void (*step_kernel_t)(uint32_t, uint32_t, uint32_t);

// Geometry-neutral (outside the renamed namespace): the host holds entries of
// both geometries. upload() takes the host's TypeDev[GPU_ACTOR_MAX_TYPES] and
// EngDev, whose layout both geometries share.
struct StepEntry {
  step_kernel_t kernel;
  hipError_t (*upload)(const void* types, const void* eng, hipStream_t s);
  bool stub;               // not compiled in this (experiment) build
  uint32_t zone_bits;      // actors per zone = 1 << zone_bits
  uint32_t threads;        // workgroup size
  uint32_t sort_work;      // u32 of dynamic LDS the hot-group sort borrows
  uint32_t bucket_words;   // u32 of dynamic LDS per destination bucket (6: a two-pass table)
  bool hot;                // takes zones prepared by k_hot (hot_dev.h): any-mix and FIFO pair
  // split tables: the step as two launches (zone_dev.h k_step PM 1, 2), or
  // as one that calls the second's code (PM 3); nullptr for the other tables
  step_kernel_t plan, rest, fused;
};

namespace gpa {

StepEntry step_entry_any();             // any mix of handler tables
StepEntry step_entry_ring();
StepEntry step_entry_pinger();
StepEntry step_entry_pinger_det();
StepEntry step_entry_fanin_sender();
StepEntry step_entry_gups_streamer();
StepEntry step_entry_storm();
StepEntry step_entry_spreader();
StepEntry step_entry_fifo_pair();       // FIFO sources + sinks (zone_dev.h kHtFifoPair)
StepEntry step_entry_program();         // behaviours as programs (GPU_ACTOR_HT_PROGRAM)

} // namespace gpa
