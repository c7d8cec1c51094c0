// k_step<GPU_ACTOR_HT_PROGRAM> at 4096-actor zones, 1024-thread workgroups (step_entry.h).
#define GPA_ZONE_BITS 12
#define GPA_ZONE_THREADS 1024
#define GPA_IDX_CAP 24576
#define GPA_TILE 7168
#define gpa gpa_z12
#define GPA_STEP_HT GPU_ACTOR_HT_PROGRAM
#define GPA_STEP_ENTRY step_entry_program
#include "step_tu.h"
