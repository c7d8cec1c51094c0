// k_step for engines whose serial actors all run GPU_ACTOR_HT_SPREADER (step_tu.h).
#define GPA_STEP_HT GPU_ACTOR_HT_SPREADER
#define GPA_STEP_ENTRY step_entry_spreader
#include "step_tu.h"
