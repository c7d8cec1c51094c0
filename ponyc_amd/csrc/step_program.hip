// k_step for engines whose serial actors all run GPU_ACTOR_HT_PROGRAM (step_tu.h).
#define GPA_STEP_HT GPU_ACTOR_HT_PROGRAM
#define GPA_STEP_ENTRY step_entry_program
#include "step_tu.h"
