// k_step for engines whose serial actors all run GPU_ACTOR_HT_PINGER_DET (step_tu.h).
#define GPA_STEP_HT GPU_ACTOR_HT_PINGER_DET
#define GPA_STEP_ENTRY step_entry_pinger_det
#include "step_tu.h"
