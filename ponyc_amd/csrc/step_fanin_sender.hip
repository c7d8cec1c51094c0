// k_step for engines whose serial actors all run GPU_ACTOR_HT_FANIN_SENDER (step_tu.h).
#define GPA_STEP_HT GPU_ACTOR_HT_FANIN_SENDER
#define GPA_STEP_ENTRY step_entry_fanin_sender
#include "step_tu.h"
