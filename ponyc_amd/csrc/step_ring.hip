// k_step for engines whose serial actors all run GPU_ACTOR_HT_RING (step_tu.h).
#define GPA_STEP_HT GPU_ACTOR_HT_RING
#define GPA_STEP_ENTRY step_entry_ring
#include "step_tu.h"
