// k_step for engines whose serial actors all run GPU_ACTOR_HT_STORM (step_tu.h).
#define GPA_STEP_HT GPU_ACTOR_HT_STORM
#define GPA_STEP_ENTRY step_entry_storm
#include "step_tu.h"
