// k_step<GPU_ACTOR_HT_SPREADER> at 1024-actor zones, 1024-thread workgroups (step_entry.h).
#define GPA_STAGED_TU 1   // mail staged in LDS before the behaviours run (engine_dev.h)
#define GPA_ZONE_BITS 10
#define GPA_ZONE_THREADS 1024
#define GPA_IDX_CAP 8192
#define gpa gpa_z10
#define GPA_STEP_HT GPU_ACTOR_HT_SPREADER
#define GPA_STEP_ENTRY step_entry_spreader
#include "step_tu.h"
