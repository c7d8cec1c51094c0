// k_step for any mix of handler tables at 1024-actor zones, 1024-thread workgroups (step_entry.h).
#define GPA_ZONE_BITS 10
#define GPA_ZONE_THREADS 1024
#define GPA_IDX_CAP 8192
#define gpa gpa_z10
#define GPA_STEP_HT -1
#define GPA_STEP_ENTRY step_entry_any
#include "step_tu.h"
