// k_step for engines whose serial actors all run GPU_ACTOR_HT_PINGER (step_tu.h).
#define GPA_STEP_HT GPU_ACTOR_HT_PINGER
#define GPA_STEP_ENTRY step_entry_pinger
#include "step_tu.h"
