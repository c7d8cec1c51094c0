// k_step for engines whose serial actors all run GPU_ACTOR_HT_GUPS_STREAMER (step_tu.h).
#define GPA_STEP_HT GPU_ACTOR_HT_GUPS_STREAMER
#define GPA_STEP_ENTRY step_entry_gups_streamer
#include "step_tu.h"
